// Row-kernel launches: the finishing kernel of the top-k path (mxa_finish.hpp) and the
// dense (top_k=False) branch: the MFMA finishing kernel with every key kept
// (mxa_finish_qk.hpp, T <= 256), else the row kernel (mxa_rows2.hpp).
#include <algorithm>
#include <atomic>

#include "mxa_finish.hpp"
#include "mxa_launch.hpp"

// Compiled five times (build_native.py, MXA_FIN_PART): part 0 the dispatch (launch_rows) and
// the dense row kernel, parts 1..4 the 32-row finishing kernel for NB = 1..4 blocks per head
// dim (launch_finish32_p<NB>), so that the instantiations build in parallel.
#ifndef MXA_FIN_PART
#define MXA_FIN_PART 0
#endif

namespace mxa {

#if MXA_FIN_PART == 0

// ---- the dense row kernel (mxa_rows2.hpp) ------------------------------------------
static size_t rows2_total(const Rows2Args& ra, int W) {
  return rows2_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, ra.tpad, W).total;
}
// waves per workgroup: the size (8 or 16) that keeps the most waves resident per CU
// (LDS-limited workgroups x waves, capped by the kernel's 7-waves-per-SIMD register use)
static int rows2_waves(const Rows2Args& ra) {
  auto resident = [&](int w) {
    const size_t t = rows2_total(ra, w);
    return t > 160 * 1024 ? 0 : std::min((int)(160 * 1024 / t) * w, 28);
  };
  const int r8 = resident(8), r16 = resident(16);
  if (r8 > 0 || r16 > 0) return r16 > r8 ? 16 : 8;
  return rows2_total(ra, 4) <= 160 * 1024 ? 4 : 0;
}

template <int S>
static int launch_dense_s(const Rows2Args& ra0, int BH, hipStream_t stream, bool plan) {
  Rows2Args ra = ra0;
  ra.waves = rows2_waves(ra);
  if (ra.waves <= 0) return MXA_ERR_UNSUPPORTED;
  if (plan) return MXA_OK;
  const size_t lds = rows2_total(ra, ra.waves);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&dense_rows_kernel<S>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  // few heads: split each head's rows over grid.y so that the launch still has ~4
  // workgroups per CU
  const int chunks = std::max(1, std::min((ra.N + ra.waves - 1) / ra.waves, 1024 / std::max(BH, 1)));
  ra.rows_per_wg = (ra.N + chunks - 1) / chunks;
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  hipLaunchKernelGGL(dense_rows_kernel<S>, dim3((unsigned)BH, gy), dim3(64 * ra.waves), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

#endif  // MXA_FIN_PART == 0

// ---- finishing kernel (mxa_finish.hpp): 32-row MFMA tiles, one per wave ------------
// two lanes per query row (one pass per tile) when every row's kept keys fit 2 x 16 slots
static bool finish_pair(const Rows2Args& ra) { return ra.k_top <= 32; }
static int finish_plan(const Rows2Args& ra, int BH, int* waves, int* rows_per_wg) {
  const int tiles = (ra.N + kFinTile - 1) / kFinTile;
  const bool pair = finish_pair(ra);
  const bool xo = ra.xo_codes != nullptr;
  auto lds = [&](int w) { return fin_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, w, pair, xo).total; };
  if (lds(1) > 160 * 1024) return MXA_ERR_UNSUPPORTED;
  // a head's tiles round-robin over the waves of one workgroup (the K / V tables
  // staged once per head); few heads (PixArt cross-attention): the tiles split over
  // grid.y so that the grid still has ~2 workgroups per CU
  int chunks = 1;
  while ((int64_t)BH * chunks < 512 && chunks < tiles) ++chunks;
  // waves per workgroup: the fewest sequential tile rounds per CU -- workgroups per
  // CU over the LDS-limited concurrency, times each workgroup's rounds over its
  // tiles; ties to the smaller workgroup (measured: DeiT-base 4 waves, 2 workgroups
  // per CU, 0.29 ms vs 0.36 ms with 5; DiT 8 waves, 0.36 ms vs 0.61 ms with 4)
  const int tpc = (tiles + chunks - 1) / chunks;
  const int64_t wgs_per_cu = ((int64_t)BH * chunks + 255) / 256;
  int w = 1;
  int64_t best = -1;
  for (int c = 1; c <= std::min(8, tpc); ++c) {
    const size_t t = lds(c);
    if (t > 160 * 1024) break;
    const int64_t conc = std::min<int64_t>(160 * 1024 / t, 12 / c > 0 ? 12 / c : 1);
    const int64_t score = (wgs_per_cu + conc - 1) / conc * ((tpc + c - 1) / c);
    if (best < 0 || score < best) best = score, w = c;
  }
  *waves = w;
  *rows_per_wg = kFinTile * ((tiles + chunks - 1) / chunks);
  return MXA_OK;
}
template <int NB, int KS, bool PAIR, bool XDT, bool XO = false>
static int launch_finish_xdt(const Rows2Args& ra0, int BH, hipStream_t stream) {
  Rows2Args ra = ra0;
  int rc = finish_plan(ra, BH, &ra.waves, &ra.rows_per_wg);
  if (rc) return rc;
  const size_t lds = fin_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, ra.waves, PAIR, XO).total;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&finish_kernel<NB, KS, PAIR, XDT, XO>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  hipLaunchKernelGGL((finish_kernel<NB, KS, PAIR, XDT, XO>), dim3((unsigned)BH, gy), dim3(64 * ra.waves), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
template <int NB, int KS, bool PAIR>
static int launch_finish_ks(const Rows2Args& ra, int BH, hipStream_t stream) {
  if (ra.xo_codes) {  // output MX codes for the proj Linear: float32, D % 32 == 0
    if (ra.s_dt != kF32 || ra.in_dt != kF32 || ra.D % 32) return MXA_ERR_UNSUPPORTED;
    return launch_finish_xdt<NB, KS, PAIR, false, true>(ra, BH, stream);
  }
  if (ra.s_dt != kF32 || ra.in_dt != kF32) return launch_finish_xdt<NB, KS, PAIR, true>(ra, BH, stream);
  return launch_finish_xdt<NB, KS, PAIR, false>(ra, BH, stream);
}
template <int NB>
static int launch_finish_nb(const Rows2Args& ra, int BH, hipStream_t stream) {
  if (finish_pair(ra)) {  // slots per lane: ceil(k / 2)
    const int kp = (ra.k_top + 1) / 2;
    if (kp <= 2) return launch_finish_ks<NB, 2, true>(ra, BH, stream);
    if (kp <= 4) return launch_finish_ks<NB, 4, true>(ra, BH, stream);
    if (kp <= 8) return launch_finish_ks<NB, 8, true>(ra, BH, stream);
    if (kp <= 12) return launch_finish_ks<NB, 12, true>(ra, BH, stream);
    return launch_finish_ks<NB, 16, true>(ra, BH, stream);
  }
  const int ks = (ra.k_top + 15) / 16;
  if (ks <= 1) return launch_finish_ks<NB, 1, false>(ra, BH, stream);
  if (ks <= 2) return launch_finish_ks<NB, 2, false>(ra, BH, stream);
  if (ks <= 4) return launch_finish_ks<NB, 4, false>(ra, BH, stream);
  if (ks <= 8) return launch_finish_ks<NB, 8, false>(ra, BH, stream);
  if (ks <= 16) return launch_finish_ks<NB, 16, false>(ra, BH, stream);
  return launch_finish_ks<NB, 32, false>(ra, BH, stream);
}
#if MXA_FIN_PART > 0
#define MXA_FIN_FN2(i) launch_finish32_p##i
#define MXA_FIN_FN(i) MXA_FIN_FN2(i)
int MXA_FIN_FN(MXA_FIN_PART)(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (plan) {
    int w, r;
    return finish_plan(ra, BH, &w, &r);
  }
  return launch_finish_nb<MXA_FIN_PART>(ra, BH, stream);
}
#else
static int launch_finish(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  const int kind = rows_kernel_kind(true, ra.k_top, ra.T, ra.nbd, ra.xo_codes != nullptr);
  const bool xdt = ra.s_dt != kF32 || ra.in_dt != kF32;
  if (kind == MXA_FIN_MFMA) return xdt ? launch_finish_qk_x1(ra, BH, stream, plan) : launch_finish_qk_x0(ra, BH, stream, plan);
  // k <= 64 (DeiT's 20 / 30, PixArt's 20): 16-row tiles, four lanes per row (also with the
  // proj's MX input codes for k <= 32); larger k with T > 256: the 32-row kernel.
  if (kind == MXA_FIN_GATHER16) return xdt ? launch_finish16_x1(ra, BH, stream, plan) : launch_finish16_x0(ra, BH, stream, plan);
  switch (ra.nbd) {
    case 1: return launch_finish32_p1(ra, BH, stream, plan);
    case 2: return launch_finish32_p2(ra, BH, stream, plan);
    case 3: return launch_finish32_p3(ra, BH, stream, plan);
    default: return launch_finish32_p4(ra, BH, stream, plan);
  }
}

// the row kernel of the path: the finishing kernel (top-k) or the dense kernel
int launch_rows(const Rows2Args& ra, bool topk, bool true_mode, int S, int BH, hipStream_t stream, bool plan) {
  if (topk) {
    // the selection kernel already wrote the true scores when it ranked them
    Rows2Args rf = ra;
    if (true_mode) rf.true_out = nullptr;
    return launch_finish(rf, BH, stream, plan);
  }
  // the dense branch: the MFMA finishing kernel with every key kept (T <= 256: a row's scores
  // in registers); longer rows: the v_dot4 row kernel
  if (rows_kernel_kind(false, 0, ra.T, ra.nbd, false) == MXA_FIN_DENSE_MFMA) {
    Rows2Args rd = ra;
    rd.dense = 1;
    rd.mask_out = nullptr;
    if (rd.s_dt != kF32 || rd.in_dt != kF32) return launch_finish_qk_x1(rd, BH, stream, plan);
    return launch_finish_qk_x0(rd, BH, stream, plan);
  }
  switch (S) {
    case 1: return launch_dense_s<1>(ra, BH, stream, plan);
    case 2: return launch_dense_s<2>(ra, BH, stream, plan);
    case 4: return launch_dense_s<4>(ra, BH, stream, plan);
    default: return launch_dense_s<8>(ra, BH, stream, plan);
  }
}
#endif  // MXA_FIN_PART


}  // namespace mxa
