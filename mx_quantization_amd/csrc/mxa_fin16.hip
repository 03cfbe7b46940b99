// Launches of the 16-row finishing kernel (mxa_finish16.hpp: k <= 64).  Compiled twice
// (build_native.py): MXA_F16_XDT=0 the float32 instantiations (launch_finish16_x0),
// MXA_F16_XDT=1 the float16 / bfloat16 ones (launch_finish16_x1), so that they build in
// parallel with the other finishing kernels.
#include <algorithm>
#include <atomic>

#include "mxa_finish16.hpp"
#include "mxa_launch.hpp"

#ifndef MXA_F16_XDT
#define MXA_F16_XDT 0
#endif
#if MXA_F16_XDT
#define MXA_F16_FN launch_finish16_x1
#else
#define MXA_F16_FN launch_finish16_x0
#endif

namespace mxa {

constexpr bool kF16Xdt = MXA_F16_XDT != 0;

// waves per workgroup: the fewest sequential tile rounds per CU -- workgroups per CU over
// the concurrency the LDS and the kernel's registers allow, times each workgroup's rounds
// over its tiles (a head's tiles round-robin over the waves: the K table staged once)
static int finish16_plan(const Rows2Args& ra, int BH, int regs_waves_per_simd, int* waves, int* rows_per_wg) {
  const int tiles = (ra.N + kFin16 - 1) / kFin16;
  const bool xo = ra.xo_codes != nullptr;
  auto lds = [&](int w) { return fin16_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, w, xo).total; };
  if (lds(1) > 160 * 1024) return MXA_ERR_UNSUPPORTED;
  int chunks = 1;
  while ((int64_t)BH * chunks < 512 && chunks < tiles) ++chunks;
  const int tpc = (tiles + chunks - 1) / chunks;
  const int64_t wgs_per_cu = ((int64_t)BH * chunks + 255) / 256;
  const int wave_cap = 4 * std::max(1, std::min(8, regs_waves_per_simd));
  int w = 1;
  int64_t best = -1;
  for (int c = 1; c <= std::min(8, tpc); ++c) {
    const size_t t = lds(c);
    if (t > 160 * 1024) break;
    const int64_t conc = std::max<int64_t>(1, std::min<int64_t>(160 * 1024 / t, wave_cap / c));
    const int64_t score = (wgs_per_cu + conc - 1) / conc * ((tpc + c - 1) / c);
    if (best < 0 || score < best) best = score, w = c;
  }
  *waves = w;
  *rows_per_wg = kFin16 * ((tiles + chunks - 1) / chunks);
  return MXA_OK;
}
template <int NB, int KS, bool EXTRA, bool XO = false>
static int launch_finish16_x(const Rows2Args& ra0, int BH, hipStream_t stream) {
  Rows2Args ra = ra0;
  const void* fn = reinterpret_cast<const void*>(&finish16_kernel<NB, KS, kF16Xdt, EXTRA, XO>);
  // waves per SIMD the kernel's registers allow: a property of the code object (gfx950
  // only), cached per instantiation; concurrent first launches compute the same value
  static std::atomic<int> regs_wps{0};
  int wps = regs_wps.load(std::memory_order_relaxed);
  if (!wps) {
    hipFuncAttributes fa{};
    wps = hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.numRegs > 0 ? 512 / ((fa.numRegs + 7) / 8 * 8) : 2;
    regs_wps.store(wps, std::memory_order_relaxed);
  }
  int rc = finish16_plan(ra, BH, wps, &ra.waves, &ra.rows_per_wg);
  if (rc) return rc;
  const size_t lds = fin16_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, ra.waves, XO).total;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  hipLaunchKernelGGL((finish16_kernel<NB, KS, kF16Xdt, EXTRA, XO>), dim3((unsigned)BH, gy), dim3(64 * ra.waves), lds,
                     stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
template <int NB, int KS>
static int launch_finish16_ks(const Rows2Args& ra, int BH, hipStream_t stream) {
  // EXTRA: a bias, the debug true scores or bfloatX rounding (float16 / bfloat16 always round)
  const bool extra = kF16Xdt || ra.bias || ra.true_out || (ra.bfloat != 0 && ra.bfloat != 32);
  if (ra.xo_codes) {  // the proj Linear's MX input codes: float32, D % 32 == 0, k <= 32
    if constexpr (!kF16Xdt && KS <= 8) {
      if (ra.D % 32) return MXA_ERR_UNSUPPORTED;
      return extra ? launch_finish16_x<NB, KS, true, true>(ra, BH, stream) : launch_finish16_x<NB, KS, false, true>(ra, BH, stream);
    }
    return MXA_ERR_UNSUPPORTED;
  }
  if (extra) return launch_finish16_x<NB, KS, true>(ra, BH, stream);
  if constexpr (!kF16Xdt) return launch_finish16_x<NB, KS, false>(ra, BH, stream);
  return MXA_ERR_UNSUPPORTED;
}
template <int NB>
static int launch_finish16_nb(const Rows2Args& ra, int BH, hipStream_t stream) {
  // four lanes per row: slots ceil(k / 4) (DeiT / PixArt k = 20: 5, DeiT k = 30: 8)
  const int ks = (ra.k_top + 3) / 4;
  if (ks <= 5) return launch_finish16_ks<NB, 5>(ra, BH, stream);
  if (ks <= 8) return launch_finish16_ks<NB, 8>(ra, BH, stream);
  if (ks <= 12) return launch_finish16_ks<NB, 12>(ra, BH, stream);
  if (ks <= 16) return launch_finish16_ks<NB, 16>(ra, BH, stream);
  return MXA_ERR_UNSUPPORTED;  // k > 64: the 32-row kernel
}

int MXA_F16_FN(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (ra.xo_codes && (kF16Xdt || ra.k_top > 32 || ra.D % 32)) return MXA_ERR_UNSUPPORTED;
  if (plan) {
    int w, r;
    return ra.k_top <= 64 ? finish16_plan(ra, BH, 2, &w, &r) : MXA_ERR_UNSUPPORTED;
  }
  switch (ra.nbd) {
    case 1: return launch_finish16_nb<1>(ra, BH, stream);
    case 2: return launch_finish16_nb<2>(ra, BH, stream);
    case 3: return launch_finish16_nb<3>(ra, BH, stream);
    default: return launch_finish16_nb<4>(ra, BH, stream);
  }
}

}  // namespace mxa
