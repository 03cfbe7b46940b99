// Launches of the finishing kernel with every key's score on MFMA (mxa_finish_qk.hpp).
// Compiled twice (build_native.py): MXA_FQ_XDT=0 the float32 instantiations
// (launch_finish_qk_x0), MXA_FQ_XDT=1 the float16 / bfloat16 ones (launch_finish_qk_x1),
// so that the two build in parallel.
#include <algorithm>
#include <atomic>

#include "mxa_finish_qk.hpp"
#include "mxa_launch.hpp"

#ifndef MXA_FQ_XDT
#define MXA_FQ_XDT 0
#endif
#if MXA_FQ_XDT
#define MXA_FQ_FN launch_finish_qk_x1
#else
#define MXA_FQ_FN launch_finish_qk_x0
#endif

namespace mxa {

constexpr bool kXdt = MXA_FQ_XDT != 0;

// ---- finishing kernel, every key's score on MFMA (mxa_finish_qk.hpp) ------------------
// key blocks the kernel's registers hold (template NTB): 4 or 8
static int fq_ntb_max(int ntb) { return ntb <= 4 ? 4 : 8; }
// waves per workgroup as finish16_plan (LDS per workgroup only, none per wave)
static int finish_qk_plan(const Rows2Args& ra, int nb, int BH, int regs_waves_per_simd, int* waves, int* rows_per_wg) {
  const int tiles = (ra.N + kFqRows - 1) / kFqRows;
  const size_t t = fq_lds(ra.ntb, nb, fq_ntb_max(ra.ntb), ra.D).total;
  if (t > 160 * 1024) return MXA_ERR_UNSUPPORTED;
  int chunks = 1;
  while ((int64_t)BH * chunks < 512 && chunks < tiles) ++chunks;
  const int tpc = (tiles + chunks - 1) / chunks;
  const int64_t wgs_per_cu = ((int64_t)BH * chunks + 255) / 256;
  const int wave_cap = 4 * std::max(1, std::min(8, regs_waves_per_simd));
  int w = 1;
  int64_t best = -1;
  for (int c = 1; c <= std::min(8, tpc); ++c) {
    const int64_t conc = std::max<int64_t>(1, std::min<int64_t>(160 * 1024 / t, wave_cap / c));
    const int64_t score = (wgs_per_cu + conc - 1) / conc * ((tpc + c - 1) / c);
    if (best < 0 || score < best) best = score, w = c;
  }
  *waves = w;
  *rows_per_wg = kFqRows * ((tiles + chunks - 1) / chunks);
  return MXA_OK;
}
template <int NB, int NTB, bool XDT>
static int launch_finish_qk_xdt(const Rows2Args& ra0, int BH, hipStream_t stream) {
  Rows2Args ra = ra0;
  if ((!ra.mask_out && !ra.dense) || fq_ntb_max(ra.ntb) != NTB || ra.nbd != NB || ra.dpad != 32 * NB) return MXA_ERR_ARG;
  const bool extra = ra.bias || ra.true_out || (ra.bfloat != 0 && ra.bfloat != 32);
  const void* fn = extra ? reinterpret_cast<const void*>(&finish_qk_kernel<NB, NTB, XDT, true>)
                         : reinterpret_cast<const void*>(&finish_qk_kernel<NB, NTB, XDT, false>);
  // waves per SIMD the registers allow: a property of the code object (gfx950 only), cached
  // per instantiation; concurrent first launches compute the same value
  static std::atomic<int> regs_wps[2] = {0, 0};
  int wps = regs_wps[extra].load(std::memory_order_relaxed);
  if (!wps) {
    hipFuncAttributes fa{};
    wps = hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.numRegs > 0 ? 512 / ((fa.numRegs + 7) / 8 * 8) : 2;
    regs_wps[extra].store(wps, std::memory_order_relaxed);
  }
  int rc = finish_qk_plan(ra, NB, BH, wps, &ra.waves, &ra.rows_per_wg);
  if (rc) return rc;
  const size_t lds = fq_lds(ra.ntb, NB, NTB, ra.D).total;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  if (extra)
    hipLaunchKernelGGL((finish_qk_kernel<NB, NTB, XDT, true>), dim3((unsigned)BH, gy), dim3(64 * ra.waves), lds, stream, ra);
  else
    hipLaunchKernelGGL((finish_qk_kernel<NB, NTB, XDT, false>), dim3((unsigned)BH, gy), dim3(64 * ra.waves), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
template <int NB>
static int launch_finish_qk_nb(const Rows2Args& ra, int BH, hipStream_t stream) {
  if (ra.ntb <= 4) return launch_finish_qk_xdt<NB, 4, kXdt>(ra, BH, stream);
  return launch_finish_qk_xdt<NB, 8, kXdt>(ra, BH, stream);
}

int MXA_FQ_FN(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (plan) {
    int w, r;
    return finish_qk_plan(ra, ra.nbd, BH, 2, &w, &r);
  }
  switch (ra.nbd) {
    case 1: return launch_finish_qk_nb<1>(ra, BH, stream);
    case 2: return launch_finish_qk_nb<2>(ra, BH, stream);
    case 3: return launch_finish_qk_nb<3>(ra, BH, stream);
    default: return launch_finish_qk_nb<4>(ra, BH, stream);
  }
}


}  // namespace mxa
