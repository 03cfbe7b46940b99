// Selection kernel launches (mxa_select.hpp): the attention path's approximate scores +
// exact-order top-k, and the standalone mxa_topk entry point of include/mxa.h.
#include "mxa_launch.hpp"
#include "mxa_select.hpp"

namespace mxa {

// ---- selection kernel (mxa_select.hpp): four query rows per wave -------------------
template <int NP, int MODE, int W, typename El>
static size_t select_lds(const Rows2Args& ra) {
  return sel_lds(MODE, ra.T, ra.D, ra.kst, ra.nbd).rows + (size_t)4 * W * grp_row_bytes(grp_alloc(ra.T), NP, sizeof(El));
}
// query rows per selection workgroup: few heads (PixArt cross-attention) take shorter row
// chunks so that the grid still fills the chip
inline int sel_rows_per_wg(int BH, int N) {
  int rows = kSelRows;
  while (rows > 16 && (int64_t)BH * ((N + rows - 1) / rows) < 2048) rows -= 16;
  return rows;
}
template <int NP, int MODE, int W, typename El = uint64_t, int QM = 0, int TW = 0>
static int launch_select_w(const Rows2Args& ra0, int BH, hipStream_t stream, bool plan) {
  Rows2Args ra = ra0;
  const size_t lds = select_lds<NP, MODE, W, El>(ra);
  if (lds > 160 * 1024) return MXA_ERR_UNSUPPORTED;
  if (plan) return MXA_OK;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&select_kernel<NP, MODE, W, El, QM, TW>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  ra.rows_per_wg = sel_rows_per_wg(BH, ra.N);
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  dim3 grid((unsigned)BH, gy);
  if (sizeof(El) == 8 && ra.fb_only) {  // one workgroup per kFbItems flags of the packed pass
    ra.fb_gy = (int)gy;
    grid = dim3((unsigned)(((int64_t)BH * gy + kFbItems - 1) / kFbItems), 1);
  }
  hipLaunchKernelGGL((select_kernel<NP, MODE, W, El, QM, TW>), grid, dim3(64 * W), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
// the one-lane tail (mxa_tail.hpp) over every row of the call: the rows the packed pass
// handed over
template <int TW>
static int launch_tail(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (plan) return MXA_OK;
  TailArgs ta{ra.tail_rec, (int64_t)BH * ra.N, ra.k_top, (ra.T + 31) / 32, ra.idx_out, ra.idx16, ra.mask_out};
  const size_t lds = tail_lds(TW);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_tail_kernel<TW>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const int64_t per = 64 * kTailWaves;
  hipLaunchKernelGGL(topk_tail_kernel<TW>, dim3((unsigned)((ta.rows + per - 1) / per)), dim3(64 * kTailWaves), lds, stream, ta);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
template <int NP, int MODE, int W>
static int launch_select_packed(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  const int tw = sel_tail_width(MODE, ra.T, ra.k_top, ra.bias != nullptr);
  int rc;
  if (tw == kTailPref) {
    rc = launch_select_w<NP, MODE, W, uint32_t, 1, kTailPref>(ra, BH, stream, plan);
    if (rc == MXA_OK) rc = launch_tail<kTailPref>(ra, BH, stream, plan);
  } else {
    rc = launch_select_w<NP, MODE, W, uint32_t, 0, 0>(ra, BH, stream, plan);
  }
  return rc;
}
template <int NP, int MODE>
static int launch_select_np(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  const int wsel = sel_waves_for(ra.T, BH, ra.N);
  // packed elements (rows of <= 256 keys) for the approximators whose scores are sums of
  // small integers times powers of two (the one-lane tail behind it for small k); then the
  // 64-bit kernel on the rows whose scores do not pack (fb_only: its workgroups without
  // such rows return at once).  The true scores, ELSA and longer rows: the 64-bit kernel.
  if constexpr (NP <= 256) {
    if (sel_packs(MODE, ra.T, ra.bias != nullptr) && ra.k_top > 0 && ra.fb_flags) {
      const int rc = wsel == 2 ? launch_select_packed<NP, MODE, 2>(ra, BH, stream, plan)
                               : launch_select_packed<NP, MODE, 4>(ra, BH, stream, plan);
      if (rc != MXA_OK) return rc;
      Rows2Args fb = ra;
      fb.fb_only = 1;
      return wsel == 2 ? launch_select_w<NP, MODE, 2>(fb, BH, stream, plan) : launch_select_w<NP, MODE, 4>(fb, BH, stream, plan);
    }
  }
  return wsel == 2 ? launch_select_w<NP, MODE, 2>(ra, BH, stream, plan) : launch_select_w<NP, MODE, 4>(ra, BH, stream, plan);
}
template <int MODE>
static int launch_select_m(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (ra.T <= 128) return launch_select_np<128, MODE>(ra, BH, stream, plan);
  if (ra.T <= 256) return launch_select_np<256, MODE>(ra, BH, stream, plan);
  return launch_select_np<512, MODE>(ra, BH, stream, plan);
}
// The selection kernel's instantiations are split over one compilation of this file per
// score mode (MXA_SEL_PART 1..6; part 0 holds the dispatcher and the standalone top-k:
// build_native.py) so that hipcc builds them in parallel.
#ifndef MXA_SEL_PART
#define MXA_SEL_PART 0
#endif
#if MXA_SEL_PART == 0
int launch_select(const Rows2Args& ra, int mode, int BH, hipStream_t stream, bool plan) {
  return launch_select_mode(ra, mode, BH, stream, plan);
}
#else
constexpr int kPartMode[7] = {0, kModeExSign, kModeOpMul, kModeOpExp, kModeTrueEx, kModeElsa, kModeTrue};
#define MXA_SEL_FN2(i) launch_select_p##i
#define MXA_SEL_FN(i) MXA_SEL_FN2(i)
int MXA_SEL_FN(MXA_SEL_PART)(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  return launch_select_m<kPartMode[MXA_SEL_PART]>(ra, BH, stream, plan);
}
#endif

}  // namespace mxa

#if MXA_SEL_PART == 0
using namespace mxa;

// ---- standalone top-k: one DPP row per row (mxa_topk_grp.hpp) -----------------------
template <int NP>
static int launch_topk_wave(const GrpTopkArgs& ga, hipStream_t stream) {
  const size_t lds = (size_t)4 * wrow_bytes(ga.n);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_wave_kernel<NP>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  hipLaunchKernelGGL(topk_wave_kernel<NP>, dim3((unsigned)((ga.rows + 3) / 4)), dim3(256), lds, stream, ga);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
template <int NP, typename El = uint64_t, int QM = 0, int TW = 0>
static int launch_topk_grp(const GrpTopkArgs& ga, const TopkWs& w, unsigned grid, hipStream_t stream) {
  const size_t lds = (size_t)16 * grp_row_bytes(grp_alloc(ga.n), NP, sizeof(El));
  const void* fn = reinterpret_cast<const void*>(&topk_grp_kernel<NP, El, QM, TW>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return MXA_ERR_LAUNCH;
  hipLaunchKernelGGL((topk_grp_kernel<NP, El, QM, TW>), dim3(grid), dim3(256), lds, stream, ga, w);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

// the workspace path of the standalone top-k: the packed pass for rows of <= 256 values
// (mxa_select.hpp topk_rows16), the one-lane tail for k <= 33 (mxa_tail.hpp), the 64-bit
// pass over the rows it leaves
static int topk_ws_tw(int n, int k) { return tail_width_for(n, k); }
static bool topk_ws_packs(int n, int k) { return n <= 256 && k > 0; }
static int64_t topk_ws_bytes(int64_t rows, int n, int k) {
  if (!topk_ws_packs(n, k)) return 0;
  const int tw = topk_ws_tw(n, k);
  const int64_t nwg = (rows + 15) / 16;
  return ((nwg * 4 + 255) / 256) * 256 + (tw ? rows * (int64_t)tail_rec_words(tw) * 4 : 0);
}
template <int NP, int TW>
static int launch_topk_packed(const GrpTopkArgs& ga, const TopkWs& w, unsigned grid, hipStream_t stream) {
  const int m = ga.k - 1;
  int rc;
  if (TW > 0 || m <= 64) rc = launch_topk_grp<NP, uint32_t, 1, TW>(ga, w, grid, stream);
  else rc = launch_topk_grp<NP, uint32_t, 2, 0>(ga, w, grid, stream);
  if (rc) return rc;
  if constexpr (TW > 0) {
    TailArgs ta{w.tail_rec, ga.rows, ga.k, (ga.n + 31) / 32, ga.out_idx, nullptr, ga.out_mask, ga.vals, ga.ld, ga.dt,
                ga.out_vals};
    const size_t lds = tail_lds(TW);
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_tail_kernel<TW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return MXA_ERR_LAUNCH;
    hipLaunchKernelGGL(topk_tail_kernel<TW>, dim3((unsigned)((ga.rows + 64 * kTailWaves - 1) / (64 * kTailWaves))),
                       dim3(64 * kTailWaves), lds, stream, ta);
    if (hipGetLastError() != hipSuccess) return MXA_ERR_LAUNCH;
  }
  TopkWs f = w;
  f.fb_only = 1;
  return launch_topk_grp<NP>(ga, f, (unsigned)((w.n_wg + kFbItems - 1) / kFbItems), stream);
}

static int topk_check(const void* vals, int64_t rows, int32_t n, int64_t ld, int32_t k, int64_t* out_idx, int32_t dtype) {
  if (!vals || !out_idx || rows < 0 || n <= 0 || ld < n || k < 0 || k > n) return MXA_ERR_ARG;
  if (dtype != kF32 && dtype != kF16 && dtype != kBF16) return MXA_ERR_ARG;
  if (n > kWMaxN) return MXA_ERR_UNSUPPORTED;
  return MXA_OK;
}

extern "C" int64_t mxa_topk_workspace_bytes(int64_t rows, int32_t n, int32_t k) {
  if (rows < 0 || n <= 0 || k < 0 || k > n) return -1;
  return topk_ws_bytes(rows, n, k);
}

extern "C" int mxa_topk(const void* vals, int64_t rows, int32_t n, int64_t ld, int32_t k, int64_t* out_idx,
                        void* out_vals, uint32_t* out_mask, int32_t dtype, hipStream_t stream) {
  int rc = topk_check(vals, rows, n, ld, k, out_idx, dtype);
  if (rc) return rc;
  if (rows == 0) return MXA_OK;
  if (k == 0) {
    if (out_mask) return hipMemsetAsync(out_mask, 0, (size_t)rows * ((n + 31) / 32) * 4, stream) == hipSuccess
                             ? MXA_OK : MXA_ERR_LAUNCH;
    return MXA_OK;
  }
  const GrpTopkArgs ga{vals, rows, ld, n, k, out_idx, out_vals, out_mask, dtype};
  // rows of 513..1024 (PixArt 512x512 self-attention): one wave per row (mxa_topk_wave.hpp);
  // shorter rows: four rows per wave (mxa_topk_grp.hpp, measured faster)
  if (n > 512) return launch_topk_wave<1024>(ga, stream);
  const unsigned grid = (unsigned)((rows + 15) / 16);
  const TopkWs w{};
  if (n <= 128) return launch_topk_grp<128>(ga, w, grid, stream);
  if (n <= 256) return launch_topk_grp<256>(ga, w, grid, stream);
  return launch_topk_grp<512>(ga, w, grid, stream);
}

extern "C" int mxa_topk_ws(const void* vals, int64_t rows, int32_t n, int64_t ld, int32_t k, int64_t* out_idx,
                           void* out_vals, uint32_t* out_mask, int32_t dtype, void* workspace, int64_t workspace_bytes,
                           hipStream_t stream) {
  int rc = topk_check(vals, rows, n, ld, k, out_idx, dtype);
  if (rc) return rc;
  const int64_t need = topk_ws_bytes(rows, n, k);
  if (rows == 0 || need == 0) return mxa_topk(vals, rows, n, ld, k, out_idx, out_vals, out_mask, dtype, stream);
  if (!workspace || workspace_bytes < need) return MXA_ERR_WORKSPACE;
  if ((reinterpret_cast<uintptr_t>(workspace) & 15u) != 0) return MXA_ERR_ARG;
  const GrpTopkArgs ga{vals, rows, ld, n, k, out_idx, out_vals, out_mask, dtype};
  TopkWs w{};
  w.n_wg = (rows + 15) / 16;
  w.fb_flags = static_cast<uint32_t*>(workspace);
  w.tail_rec = reinterpret_cast<uint32_t*>(static_cast<unsigned char*>(workspace) + ((w.n_wg * 4 + 255) / 256) * 256);
  const unsigned grid = (unsigned)w.n_wg;
  const int tw = topk_ws_tw(n, k);
  if (n <= 128) {
    if (tw == kTailPref) return launch_topk_packed<128, kTailPref>(ga, w, grid, stream);
    return launch_topk_packed<128, 0>(ga, w, grid, stream);
  }
  if (tw == kTailPref) return launch_topk_packed<256, kTailPref>(ga, w, grid, stream);
  return launch_topk_packed<256, 0>(ga, w, grid, stream);
}

#endif  // MXA_SEL_PART == 0
