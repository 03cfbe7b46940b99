// The MX top-k attention hot path on gfx950, and the mx.matmul drop-in.
//
//   rows_prep(Q), rows_prep(K)  MXINT8 codes + block exponents + approximator operands
//                               (mxa_quant.hip)
//   cols_prep(V)                MXINT8 codes of V along tokens, stored [d][t]
//   select_kernel               approximate scores + torch-CPU-order top-k, four query
//                               rows per wave (mxa_select.hpp, mxa_topk_grp.hpp)
//   finish_kernel               the kept keys' true scores, softmax, MX(P), P.V on int8
//                               MFMA (mxa_finish.hpp)
//   attn_rows2_kernel<..., 0>   the dense (top_k=False) branch (mxa_rows2.hpp)
//
// This is the mx_quant branch of the patched attention forward:
//   workloads/deit/scripts/main.py:100-152, workloads/DiT/models.py:168-225,
//   workloads/PixArt/models/MX_transformer_block.py:648-717, :792-859.
#include "mxa_kernels.hpp"
#include "mxa_order.hpp"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace mxa {

constexpr int kMaxNB = 4;  // head dim <= 128

enum RowsMode : int {
  kModeTrue = 0,   // row values are the true scores (approx off, or dense)
  kModeOpExp = 1,  // approximator codes, block scale 2^(sa + sb)
  kModeOpMul = 2,  // approximator codes, block scale sa * sb / 4096 (EXION)
  kModeExSign = 3,  // ex_pred: sign words + block exponents
  kModeTrueEx = 4,  // true_ex: power-of-two codes + zero indicators + block exponents
  kModeElsa = 5     // ELSA: hash words, key norms, cosine table
};

// scalar (uniform-address) loads of a wave's query row
typedef __attribute__((address_space(4))) const uint32_t* cu32;
__device__ __forceinline__ int s_exp16(const int16_t* base, int64_t i) {
  const uint32_t d = ((cu32)(base + (i & ~(int64_t)1)))[0];
  return exp_from16((int16_t)(i & 1 ? d >> 16 : d & 0xFFFFu));
}

}  // namespace mxa

#include "mxa_rows2.hpp"
#include "mxa_finish.hpp"
#include "mxa_proj.hpp"

namespace mxa {

// ---- mx.matmul: C[b] = MX(A[b], along K) @ MX(B[b], along K) ---------------
struct MatmulArgs {
  const int8_t* ac;
  const int16_t* as;
  const int8_t* bt;
  const int16_t* bsc;
  int M, Nc, nbk, kpad, bfloat;
  float* c;
};

__global__ __launch_bounds__(256) void matmul_kernel(MatmulArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t bt = blockIdx.z;
  const int row0 = blockIdx.y * 16;
  const int col0 = (blockIdx.x * 4 + wave) * 16;
  if (col0 >= a.Nc) return;
  const int rows_valid = min(16, a.M - row0);
  const int cols_valid = min(16, a.Nc - col0);
  const int64_t arow0 = bt * a.M + row0;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  scaled_tile<false>(a.ac + arow0 * a.kpad, a.kpad, rows_valid, a.as + arow0 * a.nbk, a.nbk, 1,
                     a.bt + (bt * a.Nc + col0) * a.kpad, a.kpad, cols_valid, a.bsc + bt * a.nbk * a.Nc + col0,
                     1, a.Nc, a.nbk, acc);
  const int col = col0 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 4 * (lane >> 4) + i;
    if (r < rows_valid && col < a.Nc)
      a.c[(arow0 + r) * a.Nc + col] = round_bfloat((float)acc[i], a.bfloat, kRoundNearest, 1);
  }
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
  int64_t qc, qop, qz, qsT, qsA, qsg, kc, kop, kz, ksT, ksA, ksg, knorm, vt, vs, idx32;
  int64_t xc, xs;  // fused qkv projection: x codes / exponents
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

AttnLayout attn_layout(const mxa_attn_params* p, int mode, const mxa_qkv_params* xq = nullptr) {
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
  L.idx32 = take(p->top_k ? qrows * (int64_t)p->k_top * 4 : 0);
  if (xq) {
    const int64_t nbk = (xq->C + 31) / 32, tokens = (int64_t)p->B * p->N;
    L.xc = take(tokens * nbk * 32);
    L.xs = take(tokens * nbk * 2);
  }
  L.total = off;
  return L;
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }

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

// ---- selection kernel (mxa_select.hpp): four query rows per wave -------------------
template <int NP, int MODE, int W>
static size_t select_lds(const Rows2Args& ra) {
  return sel_lds(MODE, ra.T, ra.D, ra.kst, ra.nbd).rows + (size_t)4 * W * grp_row_bytes(grp_alloc(ra.T), NP);
}
template <int NP, int MODE, int W>
static int launch_select_w(const Rows2Args& ra0, int BH, hipStream_t stream, bool plan) {
  Rows2Args ra = ra0;
  const size_t lds = select_lds<NP, MODE, W>(ra);
  if (lds > 160 * 1024) return MXA_ERR_UNSUPPORTED;
  if (plan) return MXA_OK;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&select_kernel<NP, MODE, W>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  // few heads (PixArt cross-attention): shorter row chunks so that the grid still fills the chip
  int rows = kSelRows;
  while (rows > 16 && (int64_t)BH * ((ra.N + rows - 1) / rows) < 2048) rows -= 16;
  ra.rows_per_wg = rows;
  const unsigned gy = (unsigned)((ra.N + rows - 1) / rows);
  hipLaunchKernelGGL((select_kernel<NP, MODE, W>), dim3((unsigned)BH, gy), dim3(64 * W), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
template <int NP, int MODE>
static int launch_select_np(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (sel_waves_for(ra.T, BH, ra.N) == 2) return launch_select_w<NP, MODE, 2>(ra, BH, stream, plan);
  return launch_select_w<NP, MODE, 4>(ra, BH, stream, plan);
}
template <int MODE>
static int launch_select_m(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (ra.T <= 128) return launch_select_np<128, MODE>(ra, BH, stream, plan);
  if (ra.T <= 256) return launch_select_np<256, MODE>(ra, BH, stream, plan);
  return launch_select_np<512, MODE>(ra, BH, stream, plan);
}
static int launch_select(const Rows2Args& ra, int mode, int BH, hipStream_t stream, bool plan) {
  switch (mode) {
    case kModeOpExp: return launch_select_m<kModeOpExp>(ra, BH, stream, plan);
    case kModeOpMul: return launch_select_m<kModeOpMul>(ra, BH, stream, plan);
    case kModeExSign: return launch_select_m<kModeExSign>(ra, BH, stream, plan);
    case kModeTrueEx: return launch_select_m<kModeTrueEx>(ra, BH, stream, plan);
    case kModeElsa: return launch_select_m<kModeElsa>(ra, BH, stream, plan);
    default: return launch_select_m<kModeTrue>(ra, BH, stream, plan);
  }
}

// ---- finishing kernel (mxa_finish.hpp): 32-row MFMA tiles, one per wave ------------
// two lanes per query row (one pass per tile) when every row's kept keys fit 2 x 16 slots
static bool finish_pair(const Rows2Args& ra) { return ra.k_top <= 32; }
static int finish_plan(const Rows2Args& ra, int BH, int* waves, int* rows_per_wg) {
  const int tiles = (ra.N + kFinTile - 1) / kFinTile;
  const bool pair = finish_pair(ra);
  auto lds = [&](int w) { return fin_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, w, pair).total; };
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
template <int NB, int KS, bool PAIR>
static int launch_finish_ks(const Rows2Args& ra0, int BH, hipStream_t stream) {
  Rows2Args ra = ra0;
  int rc = finish_plan(ra, BH, &ra.waves, &ra.rows_per_wg);
  if (rc) return rc;
  const size_t lds = fin_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, ra.waves, PAIR).total;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&finish_kernel<NB, KS, PAIR>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  hipLaunchKernelGGL((finish_kernel<NB, KS, PAIR>), dim3((unsigned)BH, gy), dim3(64 * ra.waves), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
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
static int launch_finish(const Rows2Args& ra, int BH, hipStream_t stream, bool plan) {
  if (plan) {
    int w, r;
    return finish_plan(ra, BH, &w, &r);
  }
  switch (ra.nbd) {
    case 1: return launch_finish_nb<1>(ra, BH, stream);
    case 2: return launch_finish_nb<2>(ra, BH, stream);
    case 3: return launch_finish_nb<3>(ra, BH, stream);
    default: return launch_finish_nb<4>(ra, BH, stream);
  }
}

// the row kernel of the path: the finishing kernel (top-k) or the dense kernel
static int launch_rows(const Rows2Args& ra, bool topk, bool true_mode, int S, int BH, hipStream_t stream, bool plan) {
  if (topk) {
    // the selection kernel already wrote the true scores when it ranked them
    Rows2Args rf = ra;
    if (true_mode) rf.true_out = nullptr;
    return launch_finish(rf, BH, stream, plan);
  }
  switch (S) {
    case 1: return launch_dense_s<1>(ra, BH, stream, plan);
    case 2: return launch_dense_s<2>(ra, BH, stream, plan);
    case 4: return launch_dense_s<4>(ra, BH, stream, plan);
    default: return launch_dense_s<8>(ra, BH, stream, plan);
  }
}

// ---- fused qkv projection (mxa_proj.hpp) ------------------------------------------
template <int NBD>
static int launch_proj_nbd(const ProjArgs& pa, hipStream_t stream) {
  const size_t lds = proj_lds(pa.Cpad, pa.nbk, pa.D).total;
  if (lds > 160 * 1024) return MXA_ERR_UNSUPPORTED;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&qkv_proj_kernel<NBD>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  // head groups: a workgroup loops over hpg heads after staging its x tile once; the
  // group count minimises (rounds of resident workgroups) x (heads + ~1/4 head of x
  // staging) -- with all heads per workgroup DeiT-base's 1,792 workgroups ran 3.5
  // rounds of 512 resident ones, the last half empty
  static int per_cu = -1, cus = -1;
  static size_t lds_q = 0;  // the LDS size the occupancy was queried for
  if (per_cu < 0 || lds_q != lds) {
    lds_q = lds;
    int dev = 0, n = 0, c = 0;
    (void)hipGetDevice(&dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&qkv_proj_kernel<NBD>),
                                                     64 * 3 * NBD, lds) != hipSuccess || n < 1)
      n = 1;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) c = 256;
    per_cu = n;
    cus = c;
  }
  ProjArgs p = pa;
  const int64_t wg0 = (int64_t)((pa.N + 31) / 32) * pa.B, slots = (int64_t)per_cu * cus;
  int best_g = 1;
  double best = 1e300;
  for (int g = 1; g <= pa.H; ++g) {
    const int hpg = (pa.H + g - 1) / g;
    if (g > 1 && (pa.H + hpg - 1) / hpg != g) continue;  // same hpg as a smaller g
    const double cost = (double)((wg0 * g + slots - 1) / slots) * (hpg + 0.25);
    if (cost < best - 1e-9) {
      best = cost;
      best_g = g;
    }
  }
  p.hpg = (pa.H + best_g - 1) / best_g;
  const int ng = (pa.H + p.hpg - 1) / p.hpg;
  hipLaunchKernelGGL(qkv_proj_kernel<NBD>, dim3((unsigned)((pa.N + 31) / 32), (unsigned)pa.B, (unsigned)ng),
                     dim3(64 * 3 * NBD), lds, stream, p);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
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
  rx.op_kind = MXA_OP_MXINT8; rx.flush = pp.flush_subnormals; rx.bfloat = pp.bfloat;
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
  pa.bias = xq.bias; pa.qkv_out = xq.qkv_out;
  pa.B = pp.B; pa.N = pp.N; pa.H = pp.H; pa.D = pp.D; pa.nbk = nbk; pa.Cpad = Cpad; pa.bfloat = pp.bfloat;
  // shifted int32 block sums stay exact while nbk * 32 * 127^2 * 2^smax < 2^31
  pa.smax = -1;
  while ((int64_t)nbk * 516128 * ((int64_t)1 << (pa.smax + 1)) < ((int64_t)1 << 31)) ++pa.smax;
  pa.rq = rq; pa.rk = rk; pa.cv = cv;
  switch ((pp.D + 31) / 32) {
    case 1: return launch_proj_nbd<1>(pa, stream);
    case 2: return launch_proj_nbd<2>(pa, stream);
    case 3: return launch_proj_nbd<3>(pa, stream);
    default: return launch_proj_nbd<4>(pa, stream);
  }
}

// plan != nullptr: only report the kernel path (MXA_PATH_*), launch nothing;
// scores_only: the approximate (or true) scores into p->pred_out / true_out, no top-k
// xq: the fused qkv projection (q, k, v produced from x and the prepared weight)
static int attention_impl(const mxa_attn_params* p, hipStream_t stream, hipEvent_t* ev, int* plan = nullptr,
                          bool scores_only = false, const mxa_qkv_params* xq = nullptr) {
  if (!p) return MXA_ERR_ARG;
  if (xq) {
    if (!xq->x || !xq->wq || xq->C <= 0 || xq->x_row_stride < xq->C || p->N != p->T || scores_only) return MXA_ERR_ARG;
  } else if (!p->q || !p->k) {
    return MXA_ERR_ARG;
  }
  if (!scores_only && ((!p->v && !xq) || !p->out)) return MXA_ERR_ARG;
  if (scores_only && !(p->approx ? p->pred_out : p->true_out)) return MXA_ERR_ARG;
  if (p->B <= 0 || p->H <= 0 || p->N <= 0 || p->T <= 0 || p->D <= 0) return MXA_ERR_ARG;
  if (!scores_only && p->top_k && (p->k_top <= 0 || p->k_top > p->T)) return MXA_ERR_ARG;
  if (p->pred_mode < MXA_PRED_EX_PRED || p->pred_mode > MXA_PRED_ELSA) return MXA_ERR_ARG;
  if (p->bfloat != 0 && p->bfloat != 32 && (p->bfloat < 10 || p->bfloat > 31)) return MXA_ERR_ARG;
  if (p->T > 512 || p->D > 32 * kMaxNB) return MXA_ERR_UNSUPPORTED;
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
  const AttnLayout L = attn_layout(&pp, mode, xq);
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
  rq.vec4 = aligned16(pp.q) && (pp.q_strides[0] % 4 == 0) && (pp.q_strides[1] % 4 == 0) && (pp.q_strides[2] % 4 == 0);
  rq.op_kind = opq; rq.flush = pp.flush_subnormals; rq.bfloat = pp.bfloat;
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
  rk.vec4 = aligned16(pp.k) && (pp.k_strides[0] % 4 == 0) && (pp.k_strides[1] % 4 == 0) && (pp.k_strides[2] % 4 == 0);
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
  cv.mbits = 8; cv.flush = pp.flush_subnormals; cv.bfloat = pp.bfloat;
  cv.codes_t = reinterpret_cast<int8_t*>(ws + L.vt);
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
  r2.bias = pp.bias;
  r2.bs0 = pp.bias_strides[0]; r2.bs1 = pp.bias_strides[1]; r2.bs2 = pp.bias_strides[2]; r2.bs3 = pp.bias_strides[3];
  r2.out = pp.out; r2.os0 = pp.out_strides[0]; r2.os1 = pp.out_strides[1]; r2.os2 = pp.out_strides[2];
  r2.idx_out = pp.idx_out; r2.true_out = pp.true_out; r2.pred_out = pp.pred_out; r2.mask_out = pp.mask_out;
  r2.idx32 = reinterpret_cast<int32_t*>(ws + L.idx32);
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
  return MXA_OK;
}

extern "C" int64_t mxa_linear_weight_bytes(int32_t out_features, int32_t in_features, int32_t group_width) {
  if (out_features <= 0 || in_features <= 0 || group_width <= 0 || out_features % group_width) return -1;
  return linear_layout(out_features, in_features, group_width).total;
}

extern "C" int mxa_linear_weight_prep(const float* w, int32_t out_features, int32_t in_features, int32_t group_width,
                                      int32_t flush_subnormals, int32_t bfloat, void* wq, hipStream_t stream) {
  if (!w || !wq || out_features <= 0 || in_features <= 0 || group_width <= 0 || out_features % group_width)
    return MXA_ERR_ARG;
  if (bfloat != 0 && bfloat != 32 && (bfloat < 10 || bfloat > 31)) return MXA_ERR_ARG;
  if (!aligned16(wq)) return MXA_ERR_ARG;
  const LinearLayout W = linear_layout(out_features, in_features, group_width);
  unsigned char* wb = static_cast<unsigned char*>(wq);
  RowsPrepArgs rw{};
  rw.x = w; rw.s0 = 0; rw.s1 = 0; rw.s2 = in_features;
  rw.H = 1; rw.R = out_features; rw.rows = out_features; rw.D = in_features; rw.nb = W.nbk; rw.dpad = W.Cpad;
  rw.vec4 = aligned16(w) && in_features % 4 == 0;
  rw.op_kind = MXA_OP_MXINT8; rw.flush = flush_subnormals; rw.bfloat = bfloat;
  rw.codes = reinterpret_cast<int8_t*>(wb + W.rawc);
  rw.sT = reinterpret_cast<int16_t*>(wb + W.rawe);
  int rc = launch_rows_prep(rw, stream);
  if (rc) return rc;
  const int64_t pcols = (int64_t)W.G * W.NB32 * 32;
  hipLaunchKernelGGL(linear_pack_kernel, dim3((unsigned)((pcols * W.nbk + 255) / 256)), dim3(256), 0, stream,
                     rw.codes, rw.sT, out_features, group_width, W.NB32, W.nbk, W.Cpad, pcols,
                     reinterpret_cast<int8_t*>(wb + W.pk), reinterpret_cast<int16_t*>(wb + W.pe));
  if (hipGetLastError() != hipSuccess) return MXA_ERR_LAUNCH;
  hipLaunchKernelGGL(linear_stats_kernel, dim3((unsigned)((pcols + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const int16_t*>(wb + W.pe), pcols, W.nbk, reinterpret_cast<int16_t*>(wb + W.ps));
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

extern "C" int64_t mxa_qkv_attention_workspace_bytes(const mxa_attn_params* p, const mxa_qkv_params* xq) {
  if (!p || !xq || p->B <= 0 || p->H <= 0 || p->N <= 0 || p->T <= 0 || p->D <= 0 || xq->C <= 0) return -1;
  return attn_layout(p, score_mode(p, p->top_k || p->pred_out), xq).total;
}

extern "C" int mxa_qkv_attention(const mxa_attn_params* p, const mxa_qkv_params* xq, hipStream_t stream) {
  if (!xq) return MXA_ERR_ARG;
  return attention_impl(p, stream, nullptr, nullptr, false, xq);
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

static int timed_impl(const mxa_attn_params* p, const mxa_qkv_params* xq, hipStream_t stream, int32_t iters,
                      float* stage_ms) {
  if (iters <= 0 || !stage_ms) return MXA_ERR_ARG;
  std::vector<hipEvent_t> ev((size_t)iters * MXA_ATTN_STAGES_PLUS1);
  for (auto& e : ev)
    if (hipEventCreate(&e) != hipSuccess) return MXA_ERR_LAUNCH;
  int rc = MXA_OK;
  for (int i = 0; i < iters && rc == MXA_OK; ++i)
    rc = attention_impl(p, stream, &ev[(size_t)i * MXA_ATTN_STAGES_PLUS1], nullptr, false, xq);
  if (rc == MXA_OK && hipStreamSynchronize(stream) != hipSuccess) rc = MXA_ERR_LAUNCH;
  if (rc == MXA_OK) {
    for (int s = 0; s < MXA_ATTN_STAGES; ++s) {
      double acc = 0.0;
      for (int i = 0; i < iters; ++i) {
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, ev[(size_t)i * MXA_ATTN_STAGES_PLUS1 + s], ev[(size_t)i * MXA_ATTN_STAGES_PLUS1 + s + 1]);
        acc += ms;
      }
      stage_ms[s] = (float)(acc / iters);
    }
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  return rc;
}

extern "C" int mxa_attention_timed(const mxa_attn_params* p, hipStream_t stream, int32_t iters, float* stage_ms) {
  return timed_impl(p, nullptr, stream, iters, stage_ms);
}

extern "C" int mxa_qkv_attention_timed(const mxa_attn_params* p, const mxa_qkv_params* xq, hipStream_t stream,
                                       int32_t iters, float* stage_ms) {
  if (!xq) return MXA_ERR_ARG;
  return timed_impl(p, xq, stream, iters, stage_ms);
}

// ---- standalone top-k: one DPP row per row (mxa_topk_grp.hpp) -----------------------
template <int NP>
static int launch_topk_grp(const GrpTopkArgs& ga, unsigned grid, hipStream_t stream) {
  const size_t lds = (size_t)16 * grp_row_bytes(grp_alloc(ga.n), NP);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_grp_kernel<NP>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  hipLaunchKernelGGL(topk_grp_kernel<NP>, dim3(grid), dim3(256), lds, stream, ga);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

extern "C" int mxa_topk(const float* vals, int64_t rows, int32_t n, int64_t ld, int32_t k, int64_t* out_idx,
                        float* out_vals, uint32_t* out_mask, hipStream_t stream) {
  if (!vals || !out_idx || rows < 0 || n <= 0 || ld < n || k < 0 || k > n) return MXA_ERR_ARG;
  if (n > 512) return MXA_ERR_UNSUPPORTED;
  if (rows == 0) return MXA_OK;
  if (k == 0) {
    if (out_mask) return hipMemsetAsync(out_mask, 0, (size_t)rows * ((n + 31) / 32) * 4, stream) == hipSuccess
                             ? MXA_OK : MXA_ERR_LAUNCH;
    return MXA_OK;
  }
  const GrpTopkArgs ga{vals, rows, ld, n, k, out_idx, out_vals, out_mask};
  const unsigned grid = (unsigned)((rows + 15) / 16);
  if (n <= 128) return launch_topk_grp<128>(ga, grid, stream);
  if (n <= 256) return launch_topk_grp<256>(ga, grid, stream);
  return launch_topk_grp<512>(ga, grid, stream);
}

extern "C" int64_t mxa_matmul_workspace_bytes(int64_t batch, int32_t M, int32_t K, int32_t Nc) {
  if (batch <= 0 || M <= 0 || K <= 0 || Nc <= 0) return -1;
  const int64_t nbk = (K + 31) / 32, kpad = nbk * 32;
  return align_up(batch * M * kpad) + align_up(batch * M * nbk * 2) + align_up(batch * Nc * kpad) +
         align_up(batch * nbk * Nc * 2);
}

extern "C" int mxa_matmul(const float* a, const float* b, float* c, int64_t batch, int32_t M, int32_t K, int32_t Nc,
                          int64_t a_batch_stride, int64_t b_batch_stride, int32_t elem_mbits_a, int32_t elem_mbits_b,
                          int32_t flush_subnormals, int32_t bfloat, void* workspace, int64_t workspace_bytes,
                          hipStream_t stream) {
  if (!a || !b || !c || batch <= 0 || M <= 0 || K <= 0 || Nc <= 0) return MXA_ERR_ARG;
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
  RowsPrepArgs ra{};
  ra.x = a; ra.s0 = a_batch_stride; ra.s1 = 0; ra.s2 = K; ra.H = 1; ra.R = M; ra.rows = batch * M;
  ra.D = K; ra.nb = nbk; ra.dpad = kpad;
  ra.vec4 = aligned16(a) && (a_batch_stride % 4 == 0) && (K % 4 == 0);
  ra.op_kind = elem_mbits_a == 8 ? MXA_OP_MXINT8 : MXA_OP_MXINT4;
  ra.flush = flush_subnormals; ra.bfloat = bfloat;
  ra.codes = nullptr; ra.sT = nullptr; ra.op = ac; ra.sA = as;
  int rc = launch_rows_prep(ra, stream);
  if (rc) return rc;
  ColsPrepArgs cb{};
  cb.x = b; cb.s0 = b_batch_stride; cb.s1 = 0; cb.s2 = Nc; cb.H = 1; cb.mats = batch; cb.R = K; cb.C = Nc;
  cb.nb = nbk; cb.rpad = kpad; cb.mbits = elem_mbits_b; cb.flush = flush_subnormals; cb.bfloat = bfloat;
  cb.codes_t = bt; cb.scale = bsc;
  rc = launch_cols_prep(cb, stream);
  if (rc) return rc;
  MatmulArgs ma{ac, as, bt, bsc, M, Nc, nbk, kpad, bfloat, c};
  dim3 grid((unsigned)((Nc + 63) / 64), (unsigned)((M + 15) / 16), (unsigned)batch);
  hipLaunchKernelGGL(matmul_kernel, grid, dim3(256), 0, stream, ma);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
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
