// The MX top-k attention hot path on gfx950, and the mx.matmul drop-in.
//
//   rows_prep(Q), rows_prep(K)  MXINT8 codes + block exponents + approximator operands
//                               (mxa_quant.hip)
//   cols_prep(V)                MXINT8 codes of V along tokens, stored [d][t]
//   select_kernel               approximate scores + torch-CPU-order top-k, four query
//                               rows per wave (mxa_select.hpp, mxa_topk_grp.hpp), the
//                               one-lane tail (mxa_tail.hpp)
//   finish16_kernel / finish_kernel / finish_qk_kernel
//                               the kept keys' true scores, softmax, MX(P), P.V on int8
//                               MFMA (mxa_finish16.hpp, mxa_finish.hpp, mxa_finish_qk.hpp)
//   dense (top_k=False)         finish_qk_kernel with every key kept (T <= 256), else
//                               dense_rows_kernel (mxa_rows2.hpp)
//
// This is the mx_quant branch of the patched attention forward:
//   workloads/deit/scripts/main.py:100-152, workloads/DiT/models.py:168-225,
//   workloads/PixArt/models/MX_transformer_block.py:648-717, :792-859.
#include "mxa_launch.hpp"

#include <algorithm>
#include <cstdlib>
#include <vector>



namespace mxa {

typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v4i_ __attribute__((ext_vector_type(4)));

// Self-test of the v_mfma_i32_32x32x32_i8 lane maps of the finishing kernel's P.V: A (32x32 row-major
// M x K), B (32x32 row-major K x N) -> C (32x32 row-major) through the same maps.
__global__ void selftest_mfma32_kernel(const int8_t* A, const int8_t* B, int32_t* C) {
  const int lane = threadIdx.x, ln = lane & 31, kh = 16 * (lane >> 5), m0 = 4 * (lane >> 5);
  v4i_ a4, b4;
  for (int w = 0; w < 4; ++w) {
    uint32_t x = 0, y = 0;
    for (int j = 0; j < 4; ++j) {
      x |= (uint32_t)(uint8_t)A[ln * 32 + kh + 4 * w + j] << (8 * j);
      y |= (uint32_t)(uint8_t)B[(kh + 4 * w + j) * 32 + ln] << (8 * j);
    }
    a4[w] = (int)x;
    b4[w] = (int)y;
  }
  const v16i zero = {};
  const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, zero, 0, 0, 0);
  for (int i = 0; i < 16; ++i) C[(8 * (i >> 2) + m0 + (i & 3)) * 32 + ln] = c[i];
}

__global__ void selftest_mfma_kernel(const int8_t* A, const int8_t* B, int32_t* C) {
  // A row-major 16x32, B row-major 32x16 (k-major), C row-major 16x16
  const int lane = threadIdx.x;
  const int r = lane & 15, kg = lane >> 4;
  long av = 0, bv = 0;
  for (int j = 0; j < 8; ++j) {
    av |= (long)(uint8_t)A[r * 32 + kg * 8 + j] << (8 * j);
    bv |= (long)(uint8_t)B[(kg * 8 + j) * 16 + r] << (8 * j);
  }
  const v4i zero = {0, 0, 0, 0};
  const v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, zero, 0, 0, 0);
  for (int i = 0; i < 4; ++i) C[(4 * kg + i) * 16 + r] = c[i];
}

}  // namespace mxa

using namespace mxa;

namespace {

constexpr int64_t kAlign = 256;
inline int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// workspace regions, 256-B aligned
struct AttnLayout {
  int nbd, dpad, ntb, tpad;
  int64_t qc, qop, qz, qsT, qsA, qsg, kc, kop, kz, ksT, ksA, ksg, knorm, vt, vs, idx16, tail, fbf, mask;
  int64_t xc, xs;  // fused qkv projection: x codes / exponents
  int64_t yc, ys, yf;  // fused proj Linear: its input codes / exponents, the fp32 output
                              // copy (D % 32 != 0 only), the GEMM's fp64 wave list
  int64_t total;
};

// the selection kernel's score mode of a call (ranked: the selection kernel runs)
int score_mode(const mxa_attn_params* p, bool ranked) {
  if (!(p->approx && ranked)) return kModeTrue;
  switch (p->pred_mode) {
    case MXA_PRED_EX_PRED: return kModeExSign;
    case MXA_PRED_EXION: return kModeOpMul;
    case MXA_PRED_TRUE_EX: return kModeTrueEx;
    case MXA_PRED_ELSA: return kModeElsa;
    default: return kModeOpExp;
  }
}

// the proj Linear's input comes MX-quantized out of the finishing kernel
bool proj_codes_direct(const mxa_attn_params* p) {
  return p->D % 32 == 0 && p->dtype == MXA_DT_F32 && p->score_dtype <= MXA_DT_F32;
}

AttnLayout attn_layout(const mxa_attn_params* p, int mode, const mxa_qkv_params* xq = nullptr,
                       const mxa_proj_params* pj = nullptr) {
  AttnLayout L{};
  const int64_t BH = (int64_t)p->B * p->H;
  L.nbd = (p->D + 31) / 32;
  L.dpad = L.nbd * 32;
  L.ntb = (p->T + 31) / 32;
  L.tpad = L.ntb * 32;
  const bool need_pred = mode != kModeTrue;
  const bool op = mode == kModeOpExp || mode == kModeOpMul || mode == kModeTrueEx;  // approximator codes
  const bool sg = mode == kModeExSign || mode == kModeElsa;                         // sign / hash words
  const bool sa = need_pred && mode != kModeElsa;                                   // approximator scales
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    const int64_t o = off;
    off += align_up(bytes);
    return o;
  };
  const int64_t qrows = BH * p->N, krows = BH * p->T;
  L.qc = take(qrows * L.dpad);
  L.qop = take(op ? qrows * L.dpad : 0);
  L.qz = take(mode == kModeTrueEx ? qrows * L.dpad : 0);
  L.qsT = take(qrows * L.nbd * 2);
  L.qsA = take(sa ? qrows * L.nbd * 2 : 0);
  L.qsg = take(sg ? qrows * L.nbd * 4 : 0);
  L.kc = take(krows * L.dpad);
  L.kop = take(op ? krows * L.dpad : 0);
  L.kz = take(mode == kModeTrueEx ? krows * L.dpad : 0);
  L.ksT = take(krows * L.nbd * 2);
  L.ksA = take(sa ? krows * L.nbd * 2 : 0);
  L.ksg = take(sg ? krows * L.nbd * 4 : 0);
  L.knorm = take(mode == kModeElsa ? krows * 4 : 0);
  L.vt = take(BH * p->D * (int64_t)L.tpad);
  L.vs = take(BH * L.ntb * (int64_t)p->D * 2);
  L.idx16 = take(p->top_k ? qrows * (int64_t)p->k_top * 2 : 0);  // used when the caller takes no idx
  {  // the one-lane top-k tail's staging records (mxa_tail.hpp); the packed selection
     // pass's per-workgroup flags (at most one workgroup per 16 query rows of a head)
    const bool pk = p->top_k && sel_packs(mode, p->T, p->bias != nullptr);
    const int tw = p->top_k ? sel_tail_width(mode, p->T, p->k_top, p->bias != nullptr) : 0;
    L.tail = take(tw ? qrows * (int64_t)tail_rec_words(tw) * 4 : 0);
    L.fbf = take(pk ? BH * (int64_t)((p->N + 15) / 16) * 4 : 0);
  }
  // the prune-mask words for the MFMA finishing kernel when the caller takes none
  // (reserved whatever mask_out is: the size must not depend on it)
  L.mask = take(p->top_k && finish_qk_wanted(p->k_top, p->T, L.nbd, pj && proj_codes_direct(p))
                    ? qrows * (int64_t)L.ntb * 4
                    : 0);
  if (xq) {
    const int64_t nbk = (xq->C + 31) / 32, tokens = (int64_t)p->B * p->N;
    L.xc = take(tokens * nbk * 32);
    L.xs = take(tokens * nbk * 2);
  }
  if (pj) {
    const int64_t C = (int64_t)p->H * p->D, nbk = (C + 31) / 32, tokens = (int64_t)p->B * p->N;
    L.yc = take((tokens + 31) / 32 * 32 * nbk * 32);  // MFMA-ready codes: whole 32-row blocks
    L.ys = take(tokens * nbk * 2);
    L.yf = take(proj_codes_direct(p) ? 0 : tokens * C * 4);
  }
  L.total = off;
  return L;
}


}  // namespace

extern "C" int mxa_abi_version(void) { return MXA_ABI_VERSION; }

extern "C" const char* mxa_status_string(int status) {
  switch (status) {
    case MXA_OK: return "ok";
    case MXA_ERR_ARG: return "invalid argument";
    case MXA_ERR_UNSUPPORTED: return "unsupported configuration";
    case MXA_ERR_LAUNCH: return "HIP kernel launch failed";
    case MXA_ERR_WORKSPACE: return "workspace too small";
    default: return "unknown status";
  }
}

extern "C" int64_t mxa_attention_workspace_bytes(const mxa_attn_params* p) {
  if (!p || p->B <= 0 || p->H <= 0 || p->N <= 0 || p->T <= 0 || p->D <= 0) return -1;
  // sized for the approximator whenever it may run (top-k, or the scores alone)
  return attn_layout(p, score_mode(p, p->top_k || p->pred_out)).total;
}

// x -> MX codes along C (rows_prep), then the projection kernel writing the q / k
// operands (rq, rk) and V's transposed codes (cv)
static int launch_qkv_proj(const mxa_attn_params& pp, const mxa_qkv_params& xq, const AttnLayout& L,
                           const RowsPrepArgs& rq, const RowsPrepArgs& rk, const ColsPrepArgs& cv, unsigned char* ws,
                           hipStream_t stream) {
  const int nbk = (xq.C + 31) / 32, Cpad = 32 * nbk;
  const int64_t tokens = (int64_t)pp.B * pp.N;
  RowsPrepArgs rx{};
  rx.x = xq.x; rx.s0 = 0; rx.s1 = 0; rx.s2 = xq.x_row_stride;
  rx.H = 1; rx.R = tokens; rx.rows = tokens; rx.D = xq.C; rx.nb = nbk; rx.dpad = Cpad;
  rx.vec4 = aligned16(xq.x) && xq.x_row_stride % 4 == 0;
  rx.op_kind = MXA_OP_MXINT8; rx.flush = pp.flush_subnormals; rx.bfloat = pp.bfloat; rx.dt = MXA_DT_F32;
  rx.codes = reinterpret_cast<int8_t*>(ws + L.xc);
  rx.sT = reinterpret_cast<int16_t*>(ws + L.xs);
  int rc = launch_rows_prep(rx, stream);
  if (rc) return rc;
  const LinearLayout W = linear_layout(3 * pp.H * pp.D, xq.C, pp.D);
  const unsigned char* wb = static_cast<const unsigned char*>(xq.wq);
  ProjArgs pa{};
  pa.xc = rx.codes; pa.xs = rx.sT;
  pa.pk = reinterpret_cast<const int8_t*>(wb + W.pk);
  pa.pe = reinterpret_cast<const int16_t*>(wb + W.pe);
  pa.ps = reinterpret_cast<const int16_t*>(wb + W.ps);
  pa.gs = reinterpret_cast<const int16_t*>(wb + W.gs);
  pa.pn = reinterpret_cast<const int16_t*>(wb + W.pn);
  pa.pd = reinterpret_cast<const int8_t*>(wb + W.pd);
  if (W.ps - W.pk >= ((int64_t)1 << 31) || W.total - W.pd >= ((int64_t)1 << 31))
    return MXA_ERR_UNSUPPORTED;  // 32-bit buffer offsets
  pa.pk_bytes = (int)(W.pe - W.pk);
  pa.pe_bytes = (int)(W.ps - W.pe);
  pa.pd_bytes = (int)(W.total - W.pd);
  pa.ntb = (pp.N + 31) / 32;
  pa.bias = xq.bias; pa.qkv_out = xq.qkv_out;
  pa.autocast = xq.autocast_dtype;
  pa.B = pp.B; pa.N = pp.N; pa.H = pp.H; pa.D = pp.D; pa.nbk = nbk; pa.Cpad = Cpad; pa.bfloat = pp.bfloat;
  // shifted int32 block sums stay exact while nbk * 32 * 127^2 * 2^smax < 2^31
  pa.smax = -1;
  while ((int64_t)nbk * 516128 * ((int64_t)1 << (pa.smax + 1)) < ((int64_t)1 << 31)) ++pa.smax;
  pa.rq = rq; pa.rk = rk; pa.cv = cv;
  return launch_proj(pa, stream);
}

// plan != nullptr: only report the kernel path (MXA_PATH_*), launch nothing;
// scores_only: the approximate (or true) scores into p->pred_out / true_out, no top-k
// xq: the fused qkv projection (q, k, v produced from x and the prepared weight)
// pj: the proj Linear behind the attention (y = mx.Linear(out.transpose(1,2).reshape(B,N,C)))
// fin (with plan): the finishing kernel (MXA_FIN_*, 0 for the scores alone)
static int attention_impl(const mxa_attn_params* p, hipStream_t stream, hipEvent_t* ev, int* plan = nullptr,
                          bool scores_only = false, const mxa_qkv_params* xq = nullptr,
                          const mxa_proj_params* pj = nullptr, int* fin = nullptr) {
  if (!p) return MXA_ERR_ARG;
  if (pj) {
    if (scores_only || !p->top_k || !pj->wq || !pj->y || pj->out_features <= 0 || pj->y_row_stride < pj->out_features)
      return MXA_ERR_ARG;
    if ((int64_t)p->B * p->N > INT32_MAX) return MXA_ERR_UNSUPPORTED;
  }
  if (xq) {
    if (!xq->x || !xq->wq || xq->C <= 0 || xq->x_row_stride < xq->C || p->N != p->T || scores_only) return MXA_ERR_ARG;
  } else if (!p->q || !p->k) {
    return MXA_ERR_ARG;
  }
  if (!scores_only && ((!p->v && !xq) || (!p->out && !pj))) return MXA_ERR_ARG;
  if (scores_only && !(p->approx ? p->pred_out : p->true_out)) return MXA_ERR_ARG;
  if (p->B <= 0 || p->H <= 0 || p->N <= 0 || p->T <= 0 || p->D <= 0) return MXA_ERR_ARG;
  if (!scores_only && p->top_k && (p->k_top <= 0 || p->k_top > p->T)) return MXA_ERR_ARG;
  if (p->pred_mode < MXA_PRED_EX_PRED || p->pred_mode > MXA_PRED_ELSA) return MXA_ERR_ARG;
  if (p->dtype < MXA_DT_F32 || p->dtype > MXA_DT_BF16 || p->score_dtype < 0 || p->score_dtype > MXA_DT_BF16)
    return MXA_ERR_ARG;
  if (xq && (p->dtype != MXA_DT_F32 || (xq->autocast_dtype != 0 && xq->autocast_dtype != p->score_dtype)))
    return MXA_ERR_ARG;  // the fused projection reads fp32 x; under autocast its scores follow autocast
  // approximators whose operands are not exact in float16 / bfloat16 (EXION's e*(2^l1+2^l2),
  // true_ex's per-element exponents, ELSA's fp32 projections): float32 only
  if ((p->dtype != MXA_DT_F32 || p->score_dtype > MXA_DT_F32) && p->approx &&
      (p->pred_mode == MXA_PRED_EXION || p->pred_mode == MXA_PRED_TRUE_EX || p->pred_mode == MXA_PRED_ELSA))
    return MXA_ERR_UNSUPPORTED;
  if (p->bfloat != 0 && p->bfloat != 32 && (p->bfloat < 10 || p->bfloat > 31)) return MXA_ERR_ARG;
  if (p->T > 512 || p->D > 32 * kMaxNB) return MXA_ERR_UNSUPPORTED;
  // the prepared weight must have been prepared for this geometry and these settings
  if (xq && !linear_weight_verify(xq->wq, linear_weight_header(3 * p->H * p->D, xq->C, p->D, p->flush_subnormals,
                                                                p->bfloat),
                                  stream))
    return MXA_ERR_ARG;
  if (pj && !linear_weight_verify_any_group(pj->wq, pj->out_features, p->H * p->D, p->flush_subnormals, p->bfloat,
                                            stream))
    return MXA_ERR_ARG;
  mxa_attn_params pp = *p;
  if (scores_only) {  // the selection kernel alone, with no kept keys
    pp.top_k = 0;
    pp.k_top = 0;
    pp.idx_out = nullptr;
    pp.mask_out = nullptr;
  }
  const bool topk = pp.top_k != 0;
  const bool ranked = topk || scores_only;  // the selection kernel runs
  const int mode = score_mode(&pp, ranked);
  if (mode == kModeElsa && (!pp.elsa_proj || pp.N != pp.T)) return MXA_ERR_ARG;  // elsa_approximation.py:126, :142
  const AttnLayout L = attn_layout(&pp, mode, xq, pj);
  const int64_t BH = (int64_t)pp.B * pp.H;

  int opq = MXA_OP_SIGN, opk = MXA_OP_SIGN;
  switch (pp.pred_mode) {
    case MXA_PRED_PARTIAL_Q: opq = MXA_OP_MXINT8; break;  // Q = MXINT8, K = exp-sign
    case MXA_PRED_PARTIAL_K: opk = MXA_OP_MXINT8; break;  // Q = exp-sign, K = MXINT8
    case MXA_PRED_MXINT4: opq = opk = MXA_OP_MXINT4; break;
    case MXA_PRED_EXION: opq = opk = MXA_OP_EXION; break;
    case MXA_PRED_TRUE_EX: opq = opk = MXA_OP_TRUE_EX; break;
    default: break;
  }
  const int S0 = (pp.T + 63) / 64;
  const int S = S0 <= 1 ? 1 : (S0 <= 2 ? 2 : (S0 <= 4 ? 4 : 8));
  Rows2Args r2{};
  r2.B = pp.B; r2.H = pp.H; r2.N = pp.N; r2.T = pp.T; r2.D = pp.D;
  r2.nbd = L.nbd; r2.dpad = L.dpad; r2.ntb = L.ntb; r2.tpad = L.tpad; r2.k_top = topk ? pp.k_top : 0;
  r2.kst = L.dpad + 16;  // conflict-free b128 reads of the LDS code tables
  r2.vst = L.tpad + 16;
  // feasibility of the path's kernels (LDS budgets)
  int rc = scores_only ? MXA_OK : launch_rows(r2, topk, mode == kModeTrue, S, (int)BH, stream, true);
  if (!rc && ranked) rc = launch_select(r2, mode, (int)BH, stream, true);
  if (rc) return rc;
  if (plan) {
    *plan = topk ? MXA_PATH_ROWS_SPLIT : MXA_PATH_ROWS_FUSED;
    if (fin)
      *fin = scores_only ? 0 : rows_kernel_kind(topk, r2.k_top, r2.T, r2.nbd, pj && proj_codes_direct(&pp));
    return MXA_OK;
  }
  if (!pp.workspace || pp.workspace_bytes < L.total) return MXA_ERR_WORKSPACE;
  unsigned char* ws = static_cast<unsigned char*>(pp.workspace);
  if (!aligned16(ws)) return MXA_ERR_ARG;
  const bool need_op = mode == kModeOpExp || mode == kModeOpMul || mode == kModeTrueEx;
  const bool need_sa = mode != kModeTrue && mode != kModeElsa;

  RowsPrepArgs rq{};
  rq.x = pp.q; rq.s0 = pp.q_strides[0]; rq.s1 = pp.q_strides[1]; rq.s2 = pp.q_strides[2];
  rq.H = pp.H; rq.R = pp.N; rq.rows = BH * pp.N; rq.D = pp.D; rq.nb = L.nbd; rq.dpad = L.dpad;
  const int64_t vpe = pp.dtype == MXA_DT_F32 ? 4 : 8;  // elements per 16 B
  rq.vec4 = aligned16(pp.q) && (pp.q_strides[0] % vpe == 0) && (pp.q_strides[1] % vpe == 0) && (pp.q_strides[2] % vpe == 0);
  rq.op_kind = opq; rq.flush = pp.flush_subnormals; rq.bfloat = pp.bfloat; rq.dt = xq ? MXA_DT_F32 : pp.dtype;
  rq.codes = reinterpret_cast<int8_t*>(ws + L.qc);
  rq.sT = reinterpret_cast<int16_t*>(ws + L.qsT);
  rq.op = need_op ? reinterpret_cast<int8_t*>(ws + L.qop) : nullptr;
  rq.zind = mode == kModeTrueEx ? reinterpret_cast<int8_t*>(ws + L.qz) : nullptr;
  rq.signs = mode == kModeExSign ? reinterpret_cast<uint32_t*>(ws + L.qsg) : nullptr;
  rq.sA = need_sa ? reinterpret_cast<int16_t*>(ws + L.qsA) : nullptr;
  if (ev) (void)hipEventRecord(ev[0], stream);

  RowsPrepArgs rk = rq;
  rk.x = pp.k; rk.s0 = pp.k_strides[0]; rk.s1 = pp.k_strides[1]; rk.s2 = pp.k_strides[2];
  rk.R = pp.T; rk.rows = BH * pp.T;
  rk.vec4 = aligned16(pp.k) && (pp.k_strides[0] % vpe == 0) && (pp.k_strides[1] % vpe == 0) && (pp.k_strides[2] % vpe == 0);
  rk.op_kind = opk;
  rk.codes = reinterpret_cast<int8_t*>(ws + L.kc);
  rk.sT = reinterpret_cast<int16_t*>(ws + L.ksT);
  rk.op = need_op ? reinterpret_cast<int8_t*>(ws + L.kop) : nullptr;
  rk.zind = mode == kModeTrueEx ? reinterpret_cast<int8_t*>(ws + L.kz) : nullptr;
  rk.signs = mode == kModeExSign ? reinterpret_cast<uint32_t*>(ws + L.ksg) : nullptr;
  rk.sA = need_sa ? reinterpret_cast<int16_t*>(ws + L.ksA) : nullptr;
  ColsPrepArgs cv{};
  cv.x = pp.v; cv.s0 = pp.v_strides[0]; cv.s1 = pp.v_strides[1]; cv.s2 = pp.v_strides[2];
  cv.H = pp.H; cv.mats = BH; cv.R = pp.T; cv.C = pp.D; cv.nb = L.ntb; cv.rpad = L.tpad;
  cv.mbits = 8; cv.flush = pp.flush_subnormals; cv.bfloat = pp.bfloat; cv.dt = rq.dt;
  cv.codes_t = reinterpret_cast<int8_t*>(ws + L.vt);
  cv.tb_major = 1;
  cv.scale = reinterpret_cast<int16_t*>(ws + L.vs);
  if (xq) {
    rc = launch_qkv_proj(pp, *xq, L, rq, rk, cv, ws, stream);
  } else if (scores_only) {
    rc = launch_rows_prep(rq, stream);
    if (!rc) rc = launch_rows_prep(rk, stream);
  } else {
    rc = launch_attn_prep(rq, rk, cv, stream);  // Q, K and V in one launch
  }
  if (rc) return rc;
  if (mode == kModeElsa) {  // hashes of MX(Q), MX(K); norms of MX(K) rows
    ElsaPrepArgs eq{};
    eq.codes = rq.codes; eq.sT = rq.sT; eq.proj = pp.elsa_proj; eq.rows = rq.rows;
    eq.D = pp.D; eq.nb = L.nbd; eq.dpad = L.dpad;
    eq.hash = reinterpret_cast<uint32_t*>(ws + L.qsg);
    rc = launch_elsa_prep(eq, stream);
    if (rc) return rc;
    ElsaPrepArgs ek = eq;
    ek.codes = rk.codes; ek.sT = rk.sT; ek.rows = rk.rows;
    ek.hash = reinterpret_cast<uint32_t*>(ws + L.ksg);
    ek.norm = reinterpret_cast<float*>(ws + L.knorm);
    rc = launch_elsa_prep(ek, stream);
    if (rc) return rc;
  }
  if (ev) {  // stages 1 and 2 are empty: the operand builders run as stage 0
    (void)hipEventRecord(ev[1], stream);
    (void)hipEventRecord(ev[2], stream);
    (void)hipEventRecord(ev[3], stream);
  }

  r2.qc = reinterpret_cast<const int8_t*>(ws + L.qc);
  r2.qop = reinterpret_cast<const int8_t*>(ws + L.qop);
  r2.qz = reinterpret_cast<const int8_t*>(ws + L.qz);
  r2.qsT = reinterpret_cast<const int16_t*>(ws + L.qsT);
  r2.qsA = reinterpret_cast<const int16_t*>(ws + L.qsA);
  r2.qsg = reinterpret_cast<const uint32_t*>(ws + L.qsg);
  r2.kc = reinterpret_cast<const int8_t*>(ws + L.kc);
  r2.kop = reinterpret_cast<const int8_t*>(ws + L.kop);
  r2.kz = reinterpret_cast<const int8_t*>(ws + L.kz);
  r2.ksT = reinterpret_cast<const int16_t*>(ws + L.ksT);
  r2.ksA = reinterpret_cast<const int16_t*>(ws + L.ksA);
  r2.ksg = reinterpret_cast<const uint32_t*>(ws + L.ksg);
  r2.knorm = reinterpret_cast<const float*>(ws + L.knorm);
  r2.elsa_cos = pp.elsa_cos;
  r2.vt = reinterpret_cast<const int8_t*>(ws + L.vt);
  r2.vs = reinterpret_cast<const int16_t*>(ws + L.vs);
  r2.bfloat = pp.bfloat; r2.flush_p = pp.flush_subnormals; r2.scale = pp.scale;
  r2.in_dt = pp.dtype;
  r2.s_dt = pp.score_dtype > MXA_DT_F32 ? pp.score_dtype : pp.dtype;
  r2.bias = pp.bias;
  r2.bs0 = pp.bias_strides[0]; r2.bs1 = pp.bias_strides[1]; r2.bs2 = pp.bias_strides[2]; r2.bs3 = pp.bias_strides[3];
  r2.out = pp.out; r2.os0 = pp.out_strides[0]; r2.os1 = pp.out_strides[1]; r2.os2 = pp.out_strides[2];
  r2.idx_out = pp.idx_out; r2.true_out = pp.true_out; r2.pred_out = pp.pred_out; r2.mask_out = pp.mask_out;
  r2.idx16 = reinterpret_cast<uint16_t*>(ws + L.idx16);
  r2.tail_rec = reinterpret_cast<uint32_t*>(ws + L.tail);
  r2.fb_flags = reinterpret_cast<uint32_t*>(ws + L.fbf);
  const bool direct = pj && proj_codes_direct(&pp);
  if (topk && !r2.mask_out && finish_qk_wanted(r2.k_top, r2.T, r2.nbd, direct))
    r2.mask_out = reinterpret_cast<uint32_t*>(ws + L.mask);
  if (direct) {  // the finishing kernel writes the proj's input codes
    r2.xo_codes = reinterpret_cast<int8_t*>(ws + L.yc);
    r2.xo_exps = reinterpret_cast<int16_t*>(ws + L.ys);
  } else if (pj) {  // fp32 (B, N, H*D) into the workspace, then the row quantizer
    r2.out = ws + L.yf;
    r2.os0 = (int64_t)pp.N * pp.H * pp.D; r2.os1 = pp.D; r2.os2 = (int64_t)pp.H * pp.D;
    r2.s_dt = MXA_DT_F32;
    if (pp.dtype != MXA_DT_F32 || pp.score_dtype > MXA_DT_F32) return MXA_ERR_UNSUPPORTED;
  }
  if (ranked) {
    rc = launch_select(r2, mode, (int)BH, stream, false);
    if (rc) return rc;
  }
  if (ev) (void)hipEventRecord(ev[4], stream);
  if (!scores_only) {
    rc = launch_rows(r2, topk, mode == kModeTrue, S, (int)BH, stream, false);
    if (rc) return rc;
  }
  if (ev) (void)hipEventRecord(ev[5], stream);
  if (pj) {
    const int C = pp.H * pp.D, nbk = (C + 31) / 32;
    const int64_t tokens = (int64_t)pp.B * pp.N;
    int8_t* yc = reinterpret_cast<int8_t*>(ws + L.yc);
    int16_t* ys = reinterpret_cast<int16_t*>(ws + L.ys);
    if (!direct) {
      RowsPrepArgs ry{};
      ry.x = ws + L.yf; ry.s0 = 0; ry.s1 = 0; ry.s2 = C;
      ry.H = 1; ry.R = tokens; ry.rows = tokens; ry.D = C; ry.nb = nbk; ry.dpad = 32 * nbk;
      ry.vec4 = C % 4 == 0;
      ry.op_kind = MXA_OP_MXINT8; ry.flush = pp.flush_subnormals; ry.bfloat = pp.bfloat; ry.dt = MXA_DT_F32;
      ry.codes = yc; ry.sT = ys; ry.mfma_rows = 1;
      rc = launch_rows_prep(ry, stream);
      if (rc) return rc;
    }
    rc = launch_linear_codes(yc, ys, tokens, C, pj->wq, pj->out_features, pj->bias, pj->y, pj->y_row_stride,
                             pp.bfloat, 0, stream, true);
    if (rc) return rc;
    if (ev) (void)hipEventRecord(ev[6], stream);
  }
  return MXA_OK;
}

extern "C" int64_t mxa_qkv_attention_workspace_bytes(const mxa_attn_params* p, const mxa_qkv_params* xq) {
  if (!p || !xq || p->B <= 0 || p->H <= 0 || p->N <= 0 || p->T <= 0 || p->D <= 0 || xq->C <= 0) return -1;
  return attn_layout(p, score_mode(p, p->top_k || p->pred_out), xq).total;
}

extern "C" int mxa_qkv_attention(const mxa_attn_params* p, const mxa_qkv_params* xq, hipStream_t stream) {
  if (!xq) return MXA_ERR_ARG;
  return attention_impl(p, stream, nullptr, nullptr, false, xq);
}

static int timed_impl(const mxa_attn_params* p, const mxa_qkv_params* xq, hipStream_t stream, int32_t iters,
                      float* stage_ms, const mxa_proj_params* pj);

extern "C" int64_t mxa_attention_proj_workspace_bytes(const mxa_attn_params* p, const mxa_qkv_params* xq,
                                                      const mxa_proj_params* pj) {
  if (!p || !pj || p->B <= 0 || p->H <= 0 || p->N <= 0 || p->T <= 0 || p->D <= 0 || pj->out_features <= 0) return -1;
  if (xq && xq->C <= 0) return -1;
  return attn_layout(p, score_mode(p, true), xq, pj).total;
}

extern "C" int mxa_attention_proj(const mxa_attn_params* p, const mxa_qkv_params* xq, const mxa_proj_params* pj,
                                  hipStream_t stream) {
  if (!pj) return MXA_ERR_ARG;
  return attention_impl(p, stream, nullptr, nullptr, false, xq, pj);
}

extern "C" int mxa_attention_proj_timed(const mxa_attn_params* p, const mxa_qkv_params* xq, const mxa_proj_params* pj,
                                        hipStream_t stream, int32_t iters, float* stage_ms) {
  if (!pj) return MXA_ERR_ARG;
  return timed_impl(p, xq, stream, iters, stage_ms, pj);
}

extern "C" int mxa_approx_scores(const mxa_attn_params* p, hipStream_t stream) {
  return attention_impl(p, stream, nullptr, nullptr, true);
}

extern "C" int mxa_attention(const mxa_attn_params* p, hipStream_t stream) {
  return attention_impl(p, stream, nullptr);
}

extern "C" int mxa_attention_path(const mxa_attn_params* p) {
  int plan = -1;
  const int rc = attention_impl(p, nullptr, nullptr, &plan);
  return rc ? rc : plan;
}

extern "C" int mxa_attention_finish_kernel(const mxa_attn_params* p) {
  int plan = -1, fin = -1;
  const int rc = attention_impl(p, nullptr, nullptr, &plan, false, nullptr, nullptr, &fin);
  return rc ? rc : fin;
}

static int timed_impl(const mxa_attn_params* p, const mxa_qkv_params* xq, hipStream_t stream, int32_t iters,
                      float* stage_ms, const mxa_proj_params* pj) {
  if (iters <= 0 || !stage_ms) return MXA_ERR_ARG;
  const int ns = pj ? MXA_PROJ_STAGES : MXA_ATTN_STAGES, ne = ns + 1;
  std::vector<hipEvent_t> ev((size_t)iters * ne);
  for (auto& e : ev)
    if (hipEventCreate(&e) != hipSuccess) return MXA_ERR_LAUNCH;
  int rc = MXA_OK;
  for (int i = 0; i < iters && rc == MXA_OK; ++i)
    rc = attention_impl(p, stream, &ev[(size_t)i * ne], nullptr, false, xq, pj);
  if (rc == MXA_OK && hipStreamSynchronize(stream) != hipSuccess) rc = MXA_ERR_LAUNCH;
  if (rc == MXA_OK) {
    for (int s = 0; s < ns; ++s) {
      double acc = 0.0;
      for (int i = 0; i < iters; ++i) {
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, ev[(size_t)i * ne + s], ev[(size_t)i * ne + s + 1]);
        acc += ms;
      }
      stage_ms[s] = (float)(acc / iters);
    }
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return rc;
}

extern "C" int mxa_attention_timed(const mxa_attn_params* p, hipStream_t stream, int32_t iters, float* stage_ms) {
  return timed_impl(p, nullptr, stream, iters, stage_ms, nullptr);
}

extern "C" int mxa_qkv_attention_timed(const mxa_attn_params* p, const mxa_qkv_params* xq, hipStream_t stream,
                                       int32_t iters, float* stage_ms) {
  if (!xq) return MXA_ERR_ARG;
  return timed_impl(p, xq, stream, iters, stage_ms, nullptr);
}

extern "C" int64_t mxa_matmul_workspace_bytes(int64_t batch, int32_t M, int32_t K, int32_t Nc) {
  if (batch <= 0 || M <= 0 || K <= 0 || Nc <= 0) return -1;
  const int64_t nbk = (K + 31) / 32, kpad = nbk * 32;
  return align_up(batch * M * kpad) + align_up(batch * M * nbk * 2) + align_up(batch * Nc * kpad) +
         align_up(batch * nbk * Nc * 2);
}

// in2 given as b (batch, K, Nc) row-major (cols_prep: codes transposed to [Nc][kpad],
// exponents [nbk][Nc]) or, bt_rows, as its transpose bt (batch, Nc, K) row-major (rows_prep:
// the same codes and blocks along K, exponents [Nc][nbk]) -- the k.transpose(-2, -1) view of
// the callers needs no copy
static int matmul_impl(const void* a, const void* b, bool bt_rows, void* c, int64_t batch, int32_t M, int32_t K,
                       int32_t Nc, int64_t a_batch_stride, int64_t b_batch_stride, int32_t elem_mbits_a,
                       int32_t elem_mbits_b, int32_t flush_subnormals, int32_t bfloat, int32_t a_dtype, int32_t b_dtype,
                       int32_t c_dtype, void* workspace, int64_t workspace_bytes, hipStream_t stream) {
  if (!a || !b || !c || batch <= 0 || M <= 0 || K <= 0 || Nc <= 0) return MXA_ERR_ARG;
  for (int dt : {a_dtype, b_dtype, c_dtype})
    if (dt < MXA_DT_F32 || dt > MXA_DT_BF16) return MXA_ERR_ARG;
  if ((elem_mbits_a != 8 && elem_mbits_a != 4) || (elem_mbits_b != 8 && elem_mbits_b != 4))
    return MXA_ERR_UNSUPPORTED;
  if (bfloat != 0 && bfloat != 32 && (bfloat < 10 || bfloat > 31)) return MXA_ERR_ARG;
  const int64_t need = mxa_matmul_workspace_bytes(batch, M, K, Nc);
  if (!workspace || workspace_bytes < need) return MXA_ERR_WORKSPACE;
  const int nbk = (K + 31) / 32, kpad = nbk * 32;
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  int8_t* ac = reinterpret_cast<int8_t*>(ws);
  int16_t* as = reinterpret_cast<int16_t*>(ws + align_up(batch * M * kpad));
  int8_t* bt = reinterpret_cast<int8_t*>(ws + align_up(batch * M * kpad) + align_up(batch * M * nbk * 2));
  int16_t* bsc = reinterpret_cast<int16_t*>(ws + align_up(batch * M * kpad) + align_up(batch * M * nbk * 2) +
                                            align_up(batch * Nc * kpad));
  // MX rows along K (rows_prep): a, and b's transpose when given so
  auto rows_mx = [&](const void* x, int64_t bstride, int R, int mbits, int dt, int8_t* codes, int16_t* exps) {
    RowsPrepArgs ra{};
    ra.x = x; ra.s0 = bstride; ra.s1 = 0; ra.s2 = K; ra.H = 1; ra.R = R; ra.rows = batch * R;
    ra.D = K; ra.nb = nbk; ra.dpad = kpad;
    const int64_t vpe = dt == MXA_DT_F32 ? 4 : 8;
    ra.vec4 = aligned16(x) && (bstride % vpe == 0) && (K % vpe == 0);
    ra.op_kind = mbits == 8 ? MXA_OP_MXINT8 : MXA_OP_MXINT4;
    ra.flush = flush_subnormals; ra.bfloat = bfloat; ra.dt = dt;
    ra.codes = nullptr; ra.sT = nullptr; ra.op = codes; ra.sA = exps;
    return launch_rows_prep(ra, stream);
  };
  int rc = rows_mx(a, a_batch_stride, M, elem_mbits_a, a_dtype, ac, as);
  if (rc) return rc;
  if (bt_rows) {
    rc = rows_mx(b, b_batch_stride, Nc, elem_mbits_b, b_dtype, bt, bsc);
  } else {
    ColsPrepArgs cb{};
    cb.x = b; cb.s0 = b_batch_stride; cb.s1 = 0; cb.s2 = Nc; cb.H = 1; cb.mats = batch; cb.R = K; cb.C = Nc;
    cb.nb = nbk; cb.rpad = kpad; cb.mbits = elem_mbits_b; cb.flush = flush_subnormals; cb.bfloat = bfloat; cb.dt = b_dtype;
    cb.codes_t = bt; cb.scale = bsc;
    rc = launch_cols_prep(cb, stream);
  }
  if (rc) return rc;
  // C[b] = MX(A[b]) @ MX(B[b]) on the block-scaled GEMM (mxa_gemm.hpp): A's MX codes
  // row-major along K, B's transposed codes [Nc][kpad], exponents [nbk][Nc] or [Nc][nbk]
  GemmArgs g{};
  g.a = ac; g.ae = as; g.a_bat = (int64_t)M * kpad; g.ae_bat = (int64_t)M * nbk; g.lda = kpad;
  g.b = bt; g.b_bat = (int64_t)Nc * kpad; g.ldb = kpad;
  g.be = bsc; g.be_bat = (int64_t)nbk * Nc;
  g.be_n = bt_rows ? nbk : 1; g.be_k = bt_rows ? 1 : Nc;
  g.M = M; g.Nc = Nc; g.nbk = nbk;
  g.linear = 0; g.dt = c_dtype; g.bfloat = bfloat;
  g.c = c; g.c_bat = (int64_t)M * Nc; g.ldc = Nc;
  return launch_gemm(g, batch, stream);
}

extern "C" int mxa_matmul(const void* a, const void* b, void* c, int64_t batch, int32_t M, int32_t K, int32_t Nc,
                          int64_t a_batch_stride, int64_t b_batch_stride, int32_t elem_mbits_a, int32_t elem_mbits_b,
                          int32_t flush_subnormals, int32_t bfloat, int32_t a_dtype, int32_t b_dtype,
                          int32_t c_dtype, void* workspace, int64_t workspace_bytes, hipStream_t stream) {
  return matmul_impl(a, b, false, c, batch, M, K, Nc, a_batch_stride, b_batch_stride, elem_mbits_a, elem_mbits_b,
                     flush_subnormals, bfloat, a_dtype, b_dtype, c_dtype, workspace, workspace_bytes, stream);
}

extern "C" int mxa_matmul_bt(const void* a, const void* bt, void* c, int64_t batch, int32_t M, int32_t K, int32_t Nc,
                             int64_t a_batch_stride, int64_t bt_batch_stride, int32_t elem_mbits_a, int32_t elem_mbits_b,
                             int32_t flush_subnormals, int32_t bfloat, int32_t a_dtype, int32_t b_dtype,
                             int32_t c_dtype, void* workspace, int64_t workspace_bytes, hipStream_t stream) {
  return matmul_impl(a, bt, true, c, batch, M, K, Nc, a_batch_stride, bt_batch_stride, elem_mbits_a, elem_mbits_b,
                     flush_subnormals, bfloat, a_dtype, b_dtype, c_dtype, workspace, workspace_bytes, stream);
}

extern "C" int mxa_selftest_mfma32(const int8_t* a, const int8_t* b, int32_t* c, hipStream_t stream) {
  if (!a || !b || !c) return MXA_ERR_ARG;
  hipLaunchKernelGGL(selftest_mfma32_kernel, dim3(1), dim3(64), 0, stream, a, b, c);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

extern "C" int mxa_selftest_mfma(const int8_t* a, const int8_t* b, int32_t* c, hipStream_t stream) {
  if (!a || !b || !c) return MXA_ERR_ARG;
  hipLaunchKernelGGL(selftest_mfma_kernel, dim3(1), dim3(64), 0, stream, a, b, c);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
