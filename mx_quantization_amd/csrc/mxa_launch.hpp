// Host-side launchers shared across the library's translation units (one TU per
// kernel family, so that hipcc compiles them in parallel).
#pragma once
#include "mxa_proj_args.hpp"
#include "mxa_rows2.hpp"

namespace mxa {

inline bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }

// selection kernel (mxa_sel.hip); plan: only check the LDS budget, launch nothing
int launch_select(const Rows2Args& ra, int mode, int BH, hipStream_t stream, bool plan);
// the one-lane tail's prefix (measured, DeiT-base: 48 positions 0.575-0.583 ms against 0.585-0.599
// for 64 -- 12 KB of LDS per wave, 3 waves per SIMD instead of 2, outweighs the selection kernel's
// extra step -- and 0.573-0.584 for 56; a 32-position prefix is slower: the selection kernel then
// runs one more lockstep step per row).  MXA_TAIL_PREF: a tools-only
// build of another width for same-box A/Bs (build_native defines)
#ifndef MXA_TAIL_PREF
#define MXA_TAIL_PREF 48
#endif
constexpr int kTailPref = MXA_TAIL_PREF;
// the selection's packed pass: rows of <= 256 keys, the approximators whose scores pack
// (sums of a few small integers times powers of two), no bias (a bias of -10000 next to
// small scores needs the key's low byte: PixArt's masked cross-attention would fall back
// for every row)
inline bool sel_packs(int mode, int T, bool bias) {
  return !bias && T <= 256 && (mode == kModeExSign || mode == kModeOpExp || mode == kModeOpMul || mode == kModeTrueEx);
}
// the prefix the one-lane tail takes over (mxa_tail.hpp), 0 = none: k + 2 <= TW (the
// introselect's last range and the sort of [0, k-1) lie in it), not partial_sort (k*64 <= T)
// (k - 1 <= 32: the final stable rank of [0, k-1) in at most 32 registers per lane; k + ntw
// <= TW: the prune-mask words are set in the prefix's free positions)
inline int tail_width_for(int n, int k) {
  if (k <= 0 || k > 33 || (int64_t)k * 64 <= n) return 0;
  return k + 2 <= kTailPref && k + (n + 31) / 32 <= kTailPref ? kTailPref : 0;
}
inline int sel_tail_width(int mode, int T, int k, bool bias) { return sel_packs(mode, T, bias) ? tail_width_for(T, k) : 0; }

// one score mode per translation unit of mxa_sel.hip (MXA_SEL_PART 1..6)
int launch_select_p1(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);  // ex_pred
int launch_select_p2(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);  // EXION
int launch_select_p3(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);  // MXINT4 / partial
int launch_select_p4(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);  // true_ex
int launch_select_p5(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);  // ELSA
int launch_select_p6(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);  // the true scores
inline int launch_select_mode(const Rows2Args& ra, int mode, int BH, hipStream_t stream, bool plan) {
  switch (mode) {
    case kModeExSign: return launch_select_p1(ra, BH, stream, plan);
    case kModeOpMul: return launch_select_p2(ra, BH, stream, plan);
    case kModeOpExp: return launch_select_p3(ra, BH, stream, plan);
    case kModeTrueEx: return launch_select_p4(ra, BH, stream, plan);
    case kModeElsa: return launch_select_p5(ra, BH, stream, plan);
    default: return launch_select_p6(ra, BH, stream, plan);
  }
}
// the finishing kernel with the scores of every key on MFMA (mxa_finish_qk.hpp): k a large
// share of T (above the 16-row gather kernel's k <= 64), T <= 256 (the scores of a row in
// registers); not with the proj Linear's MX input codes (xo).  It reads the selection's
// prune-mask words (the caller's mask_out, else a workspace copy), not the kept indices.
// (MXA_FQ_KMIN: a tools-only build of the threshold for same-box A/Bs, build_native defines)
#ifndef MXA_FQ_KMIN
#define MXA_FQ_KMIN 65
#endif
inline bool finish_qk_wanted(int k, int T, int nbd, bool xo) { return k >= MXA_FQ_KMIN && T <= 256 && nbd <= 4 && !xo; }
// the dense branch (top_k=False) on the same kernel with every key kept (Rows2Args::dense)
inline bool finish_qk_dense_ok(int T, int nbd) { return T <= 256 && nbd <= 4; }
// the finishing kernel of a call (include/mxa.h MXA_FIN_*): the single decision launch_rows
// (mxa_fin.hip) dispatches on and mxa_attention_finish_kernel reports
inline int rows_kernel_kind(bool topk, int k, int T, int nbd, bool xo) {
  if (!topk) return finish_qk_dense_ok(T, nbd) ? MXA_FIN_DENSE_MFMA : MXA_FIN_DENSE_ROWS;
  if (finish_qk_wanted(k, T, nbd, xo)) return MXA_FIN_MFMA;
  // k <= 64 (DeiT's 20 / 30, PixArt's 20): 16-row tiles, four lanes per row (with the proj's
  // MX input codes: k <= 32); larger k: the 32-row kernel
  return k <= (xo ? 32 : 64) ? MXA_FIN_GATHER16 : MXA_FIN_GATHER32;
}
// its launches (mxa_fin_qk.hip): float32 inputs and scores (x0), float16 / bfloat16 (x1)
int launch_finish_qk_x0(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
int launch_finish_qk_x1(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
// the 16-row finishing kernel (mxa_fin16.hip): float32 (x0), float16 / bfloat16 (x1)
int launch_finish16_x0(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
int launch_finish16_x1(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
// the 32-row finishing kernel for NB blocks per head dim (mxa_fin.hip parts 1..4)
int launch_finish32_p1(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
int launch_finish32_p2(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
int launch_finish32_p3(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
int launch_finish32_p4(const Rows2Args& ra, int BH, hipStream_t stream, bool plan);
// the row kernel of the path: finishing kernel (top-k) or dense row kernel (mxa_fin.hip)
int launch_rows(const Rows2Args& ra, bool topk, bool true_mode, int S, int BH, hipStream_t stream, bool plan);
// fused qkv projection kernel (mxa_proj.hip)
int launch_proj(const ProjArgs& pa, hipStream_t stream);
// does the prepared weight at wq carry this header?  Buffers prepared in this process
// are looked up host-side; others have their header read once (not under stream capture)
LinearWeightHeader linear_weight_header(int out_f, int in_f, int gw, int flush, int bfloat);
bool linear_weight_verify(const void* wq, const LinearWeightHeader& want, hipStream_t stream);

// does the prepared weight carry (out_f, in_f, flush, bfloat), whatever its group width?
bool linear_weight_verify_any_group(const void* wq, int out_f, int in_f, int flush, int bfloat, hipStream_t stream);
// the header of a prepared weight this process has seen (verified or prepared)
bool linear_weight_known_header(const void* wq, LinearWeightHeader* h);
// block-scaled MX GEMM (mxa_gemm.hip); mx.Linear on MX rows with a prepared weight
// (slow: gemm_slow_bytes of device scratch for the list of waves the fp64 kernel takes)
int launch_gemm(const GemmArgs& ga, int64_t batch, hipStream_t stream);
int launch_linear_codes(const int8_t* xc, const int16_t* xs, int64_t rows, int in_f, const void* wq, int out_f,
                        const float* bias, float* out, int64_t out_row_stride, int bfloat, int autocast,
                        hipStream_t stream, bool x_mfma);

}  // namespace mxa
