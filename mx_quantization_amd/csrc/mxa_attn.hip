// The MX top-k attention hot path on gfx950.
//
//   rows_prep(Q), rows_prep(K)  MXINT8 codes + block exponents + approximator operands
//   cols_prep(V)                MXINT8 codes of V along tokens, stored [d][t]
//   scores_topk_kernel          per (head, 16 query rows): true + approximate scores on
//                               int8 MFMA with exact block epilogues, wave-per-row top-k
//                               in torch's CPU order, softmax over the kept scores,
//                               scatter, MX quantization of P along keys
//   pv_kernel                   P.V on int8 MFMA (per-block scales 2^(eP + eV))
//
// This is the mx_quant branch of the patched attention forward:
//   workloads/deit/scripts/main.py:100-152, workloads/DiT/models.py:168-225,
//   workloads/PixArt/models/MX_transformer_block.py:648-717, :792-859.
#include "mxa_kernels.hpp"
#include "mxa_topk.hpp"
#include "mxa_topk_lds.hpp"

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

namespace mxa {

constexpr int kRowsPerWG = 16;

struct ScoresArgs {
  const int8_t *qc, *qop, *kc, *kop;
  const int16_t *qsT, *qsA, *ksT, *ksA;
  int B, H, N, T, nbd, dpad, ntb, tpad;
  int k_top, top_k, approx, mul_combine, bfloat, flush_p;
  float scale;
  const float* bias;
  int64_t bs0, bs1, bs2, bs3;
  int64_t* idx_out;
  float* true_out;
  float* pred_out;
  int8_t* pc;   // [B*H*N][tpad]
  int16_t* ps;  // [B*H*N][ntb]
};

// Row tail shared by the fused kernels, one wave per row:
// top-k in torch's CPU order (TopKImpl.h:45-86) on the approximate scores,
// softmax over the kept true scores, scatter, MX quantization of P along keys.
// trow / prow: the row's true and approximate scores in LDS (tpad floats each);
// prow is reused for the dense P row.
template <int S>
__device__ __forceinline__ void finish_row(const ScoresArgs& a, int64_t grow, float* trow, float* prow, const TopkLdsV2& sc,
                           int lane) {
  float pv[S];
  if (a.top_k) {
    const float* src = a.approx ? prow : trow;
    for (int pos = lane; pos < a.T; pos += 64) sc.A[pos] = pack_ki(order_key(src[pos]), (uint32_t)pos);
    wave_lds_sync();
    lds_topk<S>(sc, a.T, a.k_top, lane);
    uint32_t widx[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      widx[s] = pos < a.k_top ? (uint32_t)sc.A[pos] : 0u;
    }
    // vals = true.gather(idx); softmax(vals); zeros.scatter_(idx, softmax)
    float v[S];
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      v[s] = -INFINITY;
      if (pos < a.k_top) {
        if (a.idx_out) a.idx_out[grow * a.k_top + pos] = (int64_t)widx[s];
        v[s] = trow[widx[s]];
        mx = fmaxf(mx, v[s]);
      }
    }
    mx = wave_max_f32(mx);
    float sum = 0.0f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      v[s] = pos < a.k_top ? expf(v[s] - mx) : 0.0f;
      sum += v[s];
    }
    sum = wave_sum_f32(sum);
    wave_lds_sync();
    for (int pos = lane; pos < a.tpad; pos += 64) prow[pos] = 0.0f;
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      if (pos < a.k_top) prow[widx[s]] = v[s] / sum;
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      pv[s] = pos < a.tpad ? prow[pos] : 0.0f;
    }
  } else {
    // dense: attn = softmax(true) (blocks excluded from top-k)
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      pv[s] = pos < a.T ? trow[pos] : -INFINITY;
      mx = fmaxf(mx, pv[s]);
    }
    mx = wave_max_f32(mx);
    float sum = 0.0f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      pv[s] = pos < a.T ? expf(pv[s] - mx) : 0.0f;
      sum += pv[s];
    }
    sum = wave_sum_f32(sum);
#pragma unroll
    for (int s = 0; s < S; ++s) pv[s] = pv[s] / sum;
  }
  // P -> MXINT8 along keys (matmul(attn, v): quantize_mx_op(axes=[-1]), matmul.py:68-76)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = s * 64 + lane;
    if (s * 64 >= a.tpad) break;
    const float x = round_bfloat(pv[s], a.bfloat, kRoundNearest, 1);
    const uint32_t mb = half_reduce(__float_as_uint(x) & 0x7FFFFFFFu,
                                    [](uint32_t u, uint32_t w) { return u > w ? u : w; });
    int e_raw;
    const int es = scale_exponent(mb, 127, &e_raw);
    float xv = x;
    if (a.flush_p && !(e_raw != kExpNaN && e_raw > -127)) xv = xv * 0.0f;
    const int code = es == kExpNaN ? 0 : (int)round_code(xv, es, 8, kRoundNearest);
    if (pos < a.tpad) {
      a.pc[grow * a.tpad + pos] = (int8_t)code;
      if ((lane & 31) == 0) a.ps[grow * a.ntb + (pos >> 5)] = exp_to16(es == kExpNaN ? kExpNaN : es - 6);
    }
  }
}

template <int S>
__global__ __launch_bounds__(256) void scores_topk_kernel(ScoresArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* tileT = reinterpret_cast<float*>(smem);   // [16][tpad] true scores (then P)
  float* tileP = tileT + kRowsPerWG * a.tpad;       // [16][tpad] approximate scores
  unsigned char* scr_base = reinterpret_cast<unsigned char*>(tileP + kRowsPerWG * a.tpad);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.y;
  const int row0 = blockIdx.x * kRowsPerWG;
  const int rows_valid = min(kRowsPerWG, a.N - row0);
  const int b = bh / a.H, h = bh % a.H;
  const bool need_pred = a.top_k && a.approx;

  // ---- block-scaled int8 MFMA scores for 16 rows x T columns ----------------
  const int64_t qrow0 = (int64_t)bh * a.N + row0;
  const int64_t krow0 = (int64_t)bh * a.T;
  const int ntiles = (a.T + 15) / 16;
  for (int ct = wave; ct < ntiles; ct += 4) {
    const int col0 = ct * 16;
    const int cols_valid = min(16, a.T - col0);
    double accT[4] = {0.0, 0.0, 0.0, 0.0};
    double accP[4] = {0.0, 0.0, 0.0, 0.0};
    scaled_tile<false>(a.qc + qrow0 * a.dpad, a.dpad, rows_valid, a.qsT + qrow0 * a.nbd, a.nbd, 1,
                       a.kc + (krow0 + col0) * a.dpad, a.dpad, cols_valid, a.ksT + (krow0 + col0) * a.nbd,
                       a.nbd, 1, a.nbd, accT);
    if (need_pred) {
      if (a.mul_combine)
        scaled_tile<true>(a.qop + qrow0 * a.dpad, a.dpad, rows_valid, a.qsA + qrow0 * a.nbd, a.nbd, 1,
                          a.kop + (krow0 + col0) * a.dpad, a.dpad, cols_valid, a.ksA + (krow0 + col0) * a.nbd,
                          a.nbd, 1, a.nbd, accP);
      else
        scaled_tile<false>(a.qop + qrow0 * a.dpad, a.dpad, rows_valid, a.qsA + qrow0 * a.nbd, a.nbd, 1,
                           a.kop + (krow0 + col0) * a.dpad, a.dpad, cols_valid, a.ksA + (krow0 + col0) * a.nbd,
                           a.nbd, 1, a.nbd, accP);
    }
    const int col = col0 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * (lane >> 4) + i;
      if (r < rows_valid && col < a.T) {
        // true = quantize_elemwise(fl32(QK^T)) * scale (+ bias)   (matmul.py:88-91, caller)
        float t = round_bfloat((float)accT[i], a.bfloat, kRoundNearest, 1);
        t = t * a.scale;
        float bv = 0.0f;
        if (a.bias) {
          bv = a.bias[b * a.bs0 + h * a.bs1 + (int64_t)(row0 + r) * a.bs2 + (int64_t)col * a.bs3];
          t = t + bv;
        }
        tileT[r * a.tpad + col] = t;
        const int64_t go = (qrow0 + r) * a.T + col;
        if (a.true_out) a.true_out[go] = t;
        if (need_pred) {
          float p = (float)accP[i];
          if (a.bias) p = p + bv;
          tileP[r * a.tpad + col] = p;
          if (a.pred_out) a.pred_out[go] = p;
        }
      }
    }
  }
  __syncthreads();

  // ---- per row: top-k, softmax, scatter, MX-quantize P along keys ----------
  const TopkLdsV2 sc = carve_topk(scr_base + (size_t)wave * topk_scratch_bytes(S), S);
  for (int r = wave; r < rows_valid; r += 4)
    finish_row<S>(a, qrow0 + r, tileT + r * a.tpad, tileP + r * a.tpad, sc, lane);
}

// ---- row-oriented fused scores + top-k: one wave per query row -------------
// A workgroup of kRowsWaves waves takes the rows of one head.  The head's K
// tables are staged once in LDS: the MXINT8 codes (true scores) and, for the
// approximate scores, either the approximator codes (MXINT4 / EXION / partial_*
// operands, v_dot4 per 32-element block) or, for ex_pred, one sign word per
// block (pred = sum_b 2^(eq_b + ek_b) (n_b - 2 popc(sq_b ^ sk_b)), exact).  Each
// wave computes its row's T scores with an exact fp64 block epilogue (the floats
// the reference's fp32 matmul gives), writes them as order keys
// into its LDS top-k array, runs the exact-order top-k (mxa_topk_lds.hpp), and
// takes the true scores of the kept keys from the LDS codes.  Softmax, scatter
// and the MX quantization of P along keys follow; P leaves as MXINT8 codes for
// pv_kernel.  Each query row arrives in one vector load (lane i holds dword i),
// prefetched one row ahead.
constexpr int kRowsWaves = 8;
constexpr int kMaxNB = 4;  // head dim <= 128

#ifdef MXA_PHASE_PROF  // instrumented build only (build_native --phase-prof, tools/phase_prof.py)
__device__ unsigned long long g_phase_cycles[16];
// per-wave sums in registers, flushed once per wave (MXA_PHASE_FLUSH)
#define MXA_PHASE_INIT() \
  uint64_t ph_t = clock64(); \
  uint64_t ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define MXA_PHASE(i)                  \
  do {                                \
    const uint64_t ph_n = clock64();  \
    ph_acc[i] += ph_n - ph_t;         \
    ph_t = ph_n;                      \
  } while (0)
#define MXA_PHASE_FLUSH()                                                   \
  do {                                                                      \
    if (lane == 0)                                                          \
      for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_phase_cycles[i_], ph_acc[i_]); \
  } while (0)
#else
#define MXA_PHASE_INIT() (void)0
#define MXA_PHASE(i) (void)0
#define MXA_PHASE_FLUSH() (void)0
#endif

enum RowsMode : int {
  kModeTrue = 0,   // row values are the true scores (approx off, or dense)
  kModeOpExp = 1,  // approximator codes, block scale 2^(sa + sb)
  kModeOpMul = 2,  // approximator codes, block scale sa * sb / 4096 (EXION)
  kModeExSign = 3  // ex_pred: sign words + block exponents
};

struct RowsArgs {
  ScoresArgs s;
  const uint32_t* qsg;  // [B*H*N][nbd] sign words of the Q codes (ex_pred)
  const uint32_t* ksg;  // [B*H*T][nbd] sign words of the K codes (ex_pred)
  int D;
  int kst;  // LDS row stride of the code tables (dpad + 16: conflict-free b128 reads)
  int rows_per_wg;
  int dbg;  // instrumented build only: phases to skip (tools/phase_prof.py), 0 otherwise
};

#ifdef MXA_PHASE_PROF
#define MXA_SKIP(bit) (ra.dbg & (bit))
#else
#define MXA_SKIP(bit) false
#endif

__host__ __device__ inline size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

struct RowsLds {
  size_t mx, sT, op, sA, sg, waves, per_wave, total;
};
__host__ __device__ inline RowsLds rows_lds(int mode, int T, int kst, int nbd, int S, int tpad, bool topk) {
  RowsLds L;
  size_t o = 0;
  L.mx = o;
  o += al16((size_t)T * kst);
  L.sT = o;
  o += al16((size_t)T * nbd * 2);
  L.op = o;
  if (mode == kModeOpExp || mode == kModeOpMul) o += al16((size_t)T * kst);
  L.sA = o;
  if (mode != kModeTrue) o += al16((size_t)T * nbd * 2);
  L.sg = o;
  if (mode == kModeExSign) o += al16((size_t)T * nbd * 4);
  L.waves = o;
  L.per_wave = topk_scratch_bytes(S) + (topk ? al16(tpad) : (size_t)tpad * 4) + 64;
  L.total = o + kRowsWaves * L.per_wave;
  return L;
}

// Block-outer dot products of one uniform query row (codes at qrow, code-unit
// exponents at qs) with up to S LDS key rows per lane (jj[s], where ok[s]):
// acc[s] = exact sum_b I_b * scale_b in fp64 (EXP scale 2^(sa + sb), MUL scale
// sa * sb / 4096).  The query block's 8 words come in by scalar loads, so only 8
// SGPRs are live at a time.
typedef __attribute__((address_space(4))) const uint32_t* cu32;

__device__ __forceinline__ int s_exp16(const int16_t* base, int64_t i) {
  const uint32_t d = ((cu32)(base + (i & ~(int64_t)1)))[0];
  return exp_from16((int16_t)(i & 1 ? d >> 16 : d & 0xFFFFu));
}

template <int S, bool MUL>
__device__ __forceinline__ void dot_slots(const int8_t* qrow, const int16_t* qs, int64_t qs0, int nbd, const int8_t* tab, int kst,
                                          const int16_t* tsc, const int (&jj)[S], const bool (&ok)[S],
                                          double (&acc)[S], bool (&nan)[S]) {
#pragma unroll
  for (int s = 0; s < S; ++s) {
    acc[s] = 0.0;
    nan[s] = false;
  }
#pragma unroll
  for (int b = 0; b < kMaxNB; ++b) {
    if (b < nbd) {
      const cu32 src = (cu32)(qrow + 32 * b);
      uint32_t w[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) w[c] = src[c];
      const int qe = s_exp16(qs, qs0 + b);  // (absolute index: the dword load needs the array's alignment)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (ok[s]) {
          const int8_t* kr = tab + (size_t)jj[s] * kst + 32 * b;
          const uint4 x0 = *reinterpret_cast<const uint4*>(kr);
          const uint4 x1 = *reinterpret_cast<const uint4*>(kr + 16);
          int I = 0;
          I = __builtin_amdgcn_sdot4((int)w[0], (int)x0.x, I, false);
          I = __builtin_amdgcn_sdot4((int)w[1], (int)x0.y, I, false);
          I = __builtin_amdgcn_sdot4((int)w[2], (int)x0.z, I, false);
          I = __builtin_amdgcn_sdot4((int)w[3], (int)x0.w, I, false);
          I = __builtin_amdgcn_sdot4((int)w[4], (int)x1.x, I, false);
          I = __builtin_amdgcn_sdot4((int)w[5], (int)x1.y, I, false);
          I = __builtin_amdgcn_sdot4((int)w[6], (int)x1.z, I, false);
          I = __builtin_amdgcn_sdot4((int)w[7], (int)x1.w, I, false);
          const int e = exp_from16(tsc[jj[s] * nbd + b]);
          if (e == kExpNaN || qe == kExpNaN) nan[s] = true;
          else if (MUL) acc[s] += (double)I * (double)(qe * e) * (1.0 / 4096.0);
          else acc[s] += (double)I * pow2d(qe + e);
        }
      }
    }
  }
}

template <int S, int MODE, bool TOPK>
__global__ __launch_bounds__(64 * kRowsWaves, 4) void attn_rows_kernel(RowsArgs ra) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const ScoresArgs& a = ra.s;
  constexpr bool kOp = MODE == kModeOpExp || MODE == kModeOpMul;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.y;
  const int T = a.T, nbd = a.nbd, kst = ra.kst;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const RowsLds L = rows_lds(MODE, T, kst, nbd, S, a.tpad, TOPK);
  int8_t* tmx = reinterpret_cast<int8_t*>(smem + L.mx);      // [T][kst] K MXINT8 codes
  int16_t* tsT = reinterpret_cast<int16_t*>(smem + L.sT);    // [T][nbd] their code-unit exponents
  int8_t* top = reinterpret_cast<int8_t*>(smem + L.op);      // [T][kst] K approximator codes
  int16_t* tsA = reinterpret_cast<int16_t*>(smem + L.sA);    // [T][nbd] approximator scales
  uint32_t* tsg = reinterpret_cast<uint32_t*>(smem + L.sg);  // [T][nbd] ex_pred sign words
  unsigned char* wbase = smem + L.waves + (size_t)wave * L.per_wave;
  const TopkLdsV2 sc = carve_topk(wbase, S);
  unsigned char* rowbuf = wbase + topk_scratch_bytes(S);  // P code row (top-k) / score row (dense)
  uint32_t* bm = reinterpret_cast<uint32_t*>(rowbuf + (TOPK ? al16(a.tpad) : (size_t)a.tpad * 4));

  // ---- stage the head's K tables -------------------------------------------
  MXA_PHASE_INIT();
  const int64_t kb = (int64_t)bh * T;
  const int cpr = a.dpad / 16;
  for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
    const int j = i / cpr, c = i - j * cpr;
    *reinterpret_cast<uint4*>(tmx + (size_t)j * kst + 16 * c) =
        *reinterpret_cast<const uint4*>(a.kc + (kb + j) * a.dpad + 16 * c);
    if (kOp)
      *reinterpret_cast<uint4*>(top + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(a.kop + (kb + j) * a.dpad + 16 * c);
  }
  for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) {
    tsT[i] = a.ksT[kb * nbd + i];
    if (MODE != kModeTrue) tsA[i] = a.ksA[kb * nbd + i];
    if (MODE == kModeExSign) tsg[i] = ra.ksg[kb * nbd + i];
  }
  __syncthreads();
  MXA_PHASE(0);

  const int r0 = blockIdx.x * ra.rows_per_wg;
  const int r1 = min(a.N, r0 + ra.rows_per_wg);
  for (int r = r0 + __builtin_amdgcn_readfirstlane(wave); r < r1; r += kRowsWaves) {
    const int64_t grow = (int64_t)bh * a.N + r;
    const float* brow = a.bias ? a.bias + b_ * a.bs0 + h_ * a.bs1 + (int64_t)r * a.bs2 : nullptr;
    const int8_t* qmx = a.qc + grow * a.dpad;

    // ---- the row's T values (approximate scores, or true scores) -----------
    float vals[S];
    if (MXA_SKIP(4)) {
#pragma unroll
      for (int s = 0; s < S; ++s) vals[s] = (float)((64 * s + lane) & 7);
    } else if constexpr (MODE == kModeExSign) {
      // pred = sum_b 2^(eq_b + ek_b) (n_b - 2 popc(sq_b ^ sk_b))   (exact)
      uint32_t sq[kMaxNB];
      int eq[kMaxNB];
#pragma unroll
      for (int b = 0; b < kMaxNB; ++b) {
        sq[b] = b < nbd ? ((cu32)(ra.qsg + grow * nbd))[b] : 0u;
        eq[b] = b < nbd ? s_exp16(a.qsA, grow * nbd + b) : 0;
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int j = 64 * s + lane;
        double acc = 0.0;
        bool nan = false;
        if (j < T) {
#pragma unroll
          for (int b = 0; b < kMaxNB; ++b) {
            if (b < nbd) {
              const int e = exp_from16(tsA[j * nbd + b]);
              if (e == kExpNaN || eq[b] == kExpNaN) nan = true;
              const int m = min(32, ra.D - 32 * b) - 2 * (int)__popc(sq[b] ^ tsg[j * nbd + b]);
              acc += (double)m * pow2d(nan ? 0 : eq[b] + e);
            }
          }
        }
        vals[s] = nan ? __uint_as_float(0x7FC00000u) : (float)acc;
      }
    } else {
      int jj[S];
      bool ok[S];
      double acc[S];
      bool nan[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        jj[s] = min(64 * s + lane, T - 1);
        ok[s] = 64 * s + lane < T;
      }
      if (MODE == kModeTrue) dot_slots<S, false>(qmx, a.qsT, grow * nbd, nbd, tmx, kst, tsT, jj, ok, acc, nan);
      else dot_slots<S, MODE == kModeOpMul>(a.qop + grow * a.dpad, a.qsA, grow * nbd, nbd, top, kst, tsA, jj, ok,
                                            acc, nan);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        vals[s] = nan[s] ? __uint_as_float(0x7FC00000u) : (float)acc[s];
        // true = quantize_elemwise(fl32(QK^T)) * scale (+ bias)   (matmul.py:88-91, caller)
        if (MODE == kModeTrue) vals[s] = round_bfloat(vals[s], a.bfloat, kRoundNearest, 1) * a.scale;
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = 64 * s + lane;
      if (j < T) {
        float v = vals[s];
        if (brow) v = v + brow[(int64_t)j * a.bs3];
        if (MODE == kModeTrue) {
          if (a.true_out) a.true_out[grow * T + j] = v;
        } else if (a.pred_out) {
          a.pred_out[grow * T + j] = v;
        }
        if (TOPK) sc.A[j] = pack_ki(order_key(v), (uint32_t)j);
        else reinterpret_cast<float*>(rowbuf)[j] = v;
      }
    }
    if (TOPK) {  // clear the P row and the block maxima off the critical path
      if (lane < 16) bm[lane] = 0u;
      for (int c = lane; c < a.tpad / 4; c += 64) reinterpret_cast<uint32_t*>(rowbuf)[c] = 0u;
    }
    wave_lds_sync();
    MXA_PHASE(1);

    if constexpr (!TOPK) {  // dense: softmax over every key (finish_row's dense branch)
      finish_row<S>(a, grow, reinterpret_cast<float*>(rowbuf), reinterpret_cast<float*>(rowbuf), sc, lane);
      wave_lds_sync();
      continue;
    }
    const bool done = MXA_SKIP(1) ? true : lds_select<S>(sc, T, a.k_top, lane);
    MXA_PHASE(2);
    if (!done && !MXA_SKIP(16)) lds_sort_head<S>(sc, a.k_top - 1, lane, MXA_SKIP(32) ? 32 : 0);
    MXA_PHASE(3);

    // ---- vals = true.gather(idx); softmax(vals) ------------------------------
    auto true_scores = [&](const int (&jj)[S], const bool (&ok)[S], float (&t)[S]) {
      double acc[S];
      bool nan[S];
      dot_slots<S, false>(qmx, a.qsT, grow * nbd, nbd, tmx, kst, tsT, jj, ok, acc, nan);
#pragma unroll
      for (int s = 0; s < S; ++s) {
        t[s] = nan[s] ? __uint_as_float(0x7FC00000u) : (float)acc[s];
        t[s] = round_bfloat(t[s], a.bfloat, kRoundNearest, 1) * a.scale;
        if (brow && ok[s]) t[s] = t[s] + brow[(int64_t)jj[s] * a.bs3];
      }
    };
    if (a.true_out && MODE != kModeTrue) {  // debug output: every key's true score
      int jj[S];
      bool ok[S];
      float t[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        jj[s] = min(64 * s + lane, T - 1);
        ok[s] = 64 * s + lane < T;
      }
      true_scores(jj, ok, t);
#pragma unroll
      for (int s = 0; s < S; ++s)
        if (ok[s]) a.true_out[grow * T + jj[s]] = t[s];
    }
    int ix[S];
    bool kept[S];
    float v[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      kept[s] = pos < a.k_top;
      ix[s] = kept[s] ? (int)(uint32_t)sc.A[pos] : 0;
      if (kept[s] && a.idx_out) a.idx_out[grow * a.k_top + pos] = (int64_t)ix[s];
    }
    if (MXA_SKIP(8)) {
#pragma unroll
      for (int s = 0; s < S; ++s) v[s] = (float)(ix[s] & 3);
    } else {
      true_scores(ix, kept, v);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < S; ++s) mx = kept[s] ? fmaxf(mx, v[s]) : mx;
    mx = wave_max_f32(mx);
    float sum = 0.0f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      v[s] = kept[s] ? expf(v[s] - mx) : 0.0f;
      sum += v[s];
    }
    sum = wave_sum_f32(sum);
    MXA_PHASE(4);

    // ---- zeros.scatter_(idx, softmax) -> MXINT8 along keys ------------------
    if (MXA_SKIP(2)) {
      wave_lds_sync();
      continue;
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (kept[s]) {
        v[s] = round_bfloat(v[s] / sum, a.bfloat, kRoundNearest, 1);
        atomicMax(&bm[ix[s] >> 5], __float_as_uint(v[s]) & 0x7FFFFFFFu);
      }
    }
    wave_lds_sync();
    if (lane < a.ntb) {
      int e_raw;
      const int es = scale_exponent(bm[lane], 127, &e_raw);
      const bool fl = a.flush_p && !(e_raw != kExpNaN && e_raw > -127);
      a.ps[grow * a.ntb + lane] = exp_to16(es == kExpNaN ? kExpNaN : es - 6);
      bm[lane] = (es == kExpNaN ? 0u : (uint32_t)(es + 1024)) | (fl ? 0x10000u : 0u);  // 0: NaN block
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (kept[s]) {
        const uint32_t e = bm[ix[s] >> 5];
        int code = 0;
        if (e & 0xFFFFu) {
          const int es = (int)(e & 0xFFFFu) - 1024;
          const float x = (e & 0x10000u) ? v[s] * 0.0f : v[s];
          code = (int)round_code(x, es, 8, kRoundNearest);
        }
        reinterpret_cast<int8_t*>(rowbuf)[ix[s]] = (int8_t)code;
      }
    }
    wave_lds_sync();
    for (int c = lane; c < a.tpad / 4; c += 64)
      reinterpret_cast<uint32_t*>(a.pc + grow * a.tpad)[c] = reinterpret_cast<const uint32_t*>(rowbuf)[c];
    wave_lds_sync();
    MXA_PHASE(5);
  }
  MXA_PHASE_FLUSH();
}

}  // namespace mxa
#include "mxa_rows2.hpp"
#include "mxa_finish.hpp"
namespace mxa {

struct PVArgs {
  const int8_t* pc;
  const int16_t* ps;
  const int8_t* vt;
  const int16_t* vs;
  int B, H, N, D, ntb, tpad, bfloat;
  float* out;
  int64_t os0, os1, os2;
};

__global__ __launch_bounds__(256) void pv_kernel(PVArgs a) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.y;
  const int row0 = blockIdx.x * kRowsPerWG;
  const int rows_valid = min(kRowsPerWG, a.N - row0);
  const int b = bh / a.H, h = bh % a.H;
  const int64_t prow0 = (int64_t)bh * a.N + row0;
  const int ntiles = (a.D + 15) / 16;
  for (int ct = wave; ct < ntiles; ct += 4) {
    const int col0 = ct * 16;
    const int cols_valid = min(16, a.D - col0);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    scaled_tile<false>(a.pc + prow0 * a.tpad, a.tpad, rows_valid, a.ps + prow0 * a.ntb, a.ntb, 1,
                       a.vt + ((int64_t)bh * a.D + col0) * a.tpad, a.tpad, cols_valid,
                       a.vs + (int64_t)bh * a.ntb * a.D + col0, 1, a.D, a.ntb, acc);
    const int col = col0 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * (lane >> 4) + i;
      if (r < rows_valid && col < a.D)
        a.out[b * a.os0 + h * a.os1 + (int64_t)(row0 + r) * a.os2 + col] =
            round_bfloat((float)acc[i], a.bfloat, kRoundNearest, 1);
    }
  }
}

// ---- standalone exact-order top-k over rows of a float matrix --------------
struct TopkArgs {
  const float* vals;
  int64_t rows, ld;
  int n, k;
  int64_t* out_idx;
  float* out_vals;
  int dbg;  // MXA_TOPK_DBG (tools only): 1 skip the lane tails, 2 skip the wave-wide steps
};

template <int S>
__global__ __launch_bounds__(256) void topk_rows_kernel(TopkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= a.rows) return;  // wave-uniform
  const TopkLdsV2 sc = carve_topk(smem + (size_t)wave * topk_scratch_bytes(S), S);
  const float* src = a.vals + row * a.ld;
  for (int pos = lane; pos < a.n; pos += 64) sc.A[pos] = pack_ki(order_key(src[pos]), (uint32_t)pos);
  wave_lds_sync();
  lds_topk<S>(sc, a.n, a.k, lane);
  for (int pos = lane; pos < a.k; pos += 64) {
    const uint32_t ix = (uint32_t)sc.A[pos];
    a.out_idx[row * a.k + pos] = (int64_t)ix;
    if (a.out_vals) a.out_vals[row * a.k + pos] = src[ix];
  }
}

// register-resident top-k (mxa_topk_reg.hpp)
template <int S>
__global__ __launch_bounds__(256) void topk_reg_kernel(TopkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= a.rows) return;  // wave-uniform
  RegTopk<S> tk;
  tk.init(smem + (size_t)wave * topk_scratch_bytes(S), a.n, lane);
  const float* src = a.vals + row * a.ld;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = 64 * s + lane;
    tk.K[s] = pos < a.n ? order_key(src[pos]) : 0u;
    tk.I[s] = (uint32_t)pos;
  }
  tk.run(a.k);
  tk.finalize();
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = 64 * s + lane;
    if (64 * s < a.k) {
      const uint32_t ix = tk.out_idx(s);
      if (pos < a.k) {
        a.out_idx[row * a.k + pos] = (int64_t)ix;
        if (a.out_vals) a.out_vals[row * a.k + pos] = src[ix];
      }
    }
  }
}

// wave-wide steps while the pending range reaches past W, then one row per lane
// (mxa_topk_lane.hpp).  A workgroup of WAVES waves takes 64 rows: the waves run
// the wave-wide steps of the rows in turn and park each row's window [0, W) in a
// shared pool; then the rows' lanes finish them (rows spread over TAILW waves).
constexpr int kLaneRows = 64;  // rows per workgroup
constexpr int kLaneStk = 16;   // lane stack entries (>= 2 lg W)
template <int W>
__host__ __device__ constexpr int lane_rs() { return W + 1; }  // u64 row stride (odd: spreads the banks)
template <int S, int W, int WAVES>
__host__ __device__ constexpr size_t topk_lane_lds() {
  return (size_t)WAVES * topk_scratch_bytes(S) + (size_t)kLaneRows * (lane_rs<W>() * 8 + sizeof(LaneTask) + kLaneStk * 4);
}

template <int S, int W, int WAVES, int TAILW>
__global__ __launch_bounds__(64 * WAVES) void topk_lane_kernel(TopkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int RS = lane_rs<W>();
  unsigned char* wb = smem + (size_t)wave * topk_scratch_bytes(S);
  unsigned char* pool = smem + (size_t)WAVES * topk_scratch_bytes(S);
  lu64* stage = (lu64*)pool;                                                  // [64][RS]
  LaneTask* tasks = reinterpret_cast<LaneTask*>(pool + kLaneRows * RS * 8);  // [64]
  li32* stks = (li32*)(reinterpret_cast<int*>(tasks + kLaneRows));           // [64][kLaneStk]
  const int64_t row0 = (int64_t)blockIdx.x * kLaneRows;
  const int nrows = (int)min((int64_t)kLaneRows, a.rows - row0);
  for (int r = wave; r < nrows; r += WAVES) {
    RegTopk<S, false> tk;
    tk.init(wb, a.n, lane);
    const float* src = a.vals + (row0 + r) * a.ld;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      tk.K[s] = pos < a.n ? order_key(src[pos]) : 0u;
      tk.I[s] = (uint32_t)pos;
    }
    LaneTask t;
    if (a.dbg & 2) {
      t.first = 0; t.last = min(a.n, W); t.depth = 2 * ilog2(a.n); t.nth = a.k - 1; t.k = a.k;
    } else {
      t = tk.select_big(a.k, W);
    }
    tk.stage_out(stage + r * RS, W);
    if (lane == 0) tasks[r] = t;
    wave_lds_sync();
  }
  __syncthreads();
  {
    // row r -> wave r % TAILW, lane r / TAILW
    const int r = lane * TAILW + wave;
    if (wave < TAILW && r < nrows && !(a.dbg & 1)) lane_topk_tail(stage + r * RS, tasks[r], stks + r * kLaneStk);
  }
  __syncthreads();
  for (int r = wave; r < nrows; r += WAVES) {
    if (lane < a.k) {
      const uint32_t ix = (uint32_t)stage[r * RS + lane];
      a.out_idx[(row0 + r) * a.k + lane] = (int64_t)ix;
      if (a.out_vals) a.out_vals[(row0 + r) * a.k + lane] = a.vals[(row0 + r) * a.ld + ix];
    }
  }
}

template <int S, int W, int WAVES, int TAILW>
static int launch_topk_lane(const TopkArgs& ta, hipStream_t stream) {
  const size_t lds = topk_lane_lds<S, W, WAVES>();
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topk_lane_kernel<S, W, WAVES, TAILW>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const dim3 g((unsigned)((ta.rows + kLaneRows - 1) / kLaneRows));
  hipLaunchKernelGGL((topk_lane_kernel<S, W, WAVES, TAILW>), g, dim3(64 * WAVES), lds, stream, ta);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
template <int S, int W>
static int launch_topk_lane_cfg(const TopkArgs& ta, hipStream_t stream) {
  const char* env = getenv("MXA_LANE_CFG");  // tools only: WAVES x TAILW
  const std::string c = env ? env : "8x8";
  if (c == "4x1") return launch_topk_lane<S, W, 4, 1>(ta, stream);
  if (c == "4x4") return launch_topk_lane<S, W, 4, 4>(ta, stream);
  if (c == "8x1") return launch_topk_lane<S, W, 8, 1>(ta, stream);
  if (c == "8x2") return launch_topk_lane<S, W, 8, 2>(ta, stream);
  if (c == "16x16") return launch_topk_lane<S, W, 16, 16>(ta, stream);
  return launch_topk_lane<S, W, 8, 8>(ta, stream);
}

// previous register-resident form (mxa_topk.hpp), kept for A/B timing (MXA_TOPK_V1)
template <int S>
__global__ __launch_bounds__(256) void topk_rows_v1_kernel(TopkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= a.rows) return;  // wave-uniform
  TopkLds sc;
  sc.a = reinterpret_cast<uint64_t*>(smem) + (size_t)wave * (2 * 64 * S + kTopkStack / 2);
  sc.b = sc.a + 64 * S;
  sc.stk = reinterpret_cast<int*>(sc.b + 64 * S);
  const float* src = a.vals + row * a.ld;
  WaveRow<S> w;
  w.lane = lane;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = s * 64 + lane;
    w.key[s] = pos < a.n ? order_key(src[pos]) : 0u;
    w.idx[s] = (uint32_t)pos;
  }
  wave_topk<S>(w, a.n, a.k, sc);
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = s * 64 + lane;
    if (pos < a.k) {
      a.out_idx[row * a.k + pos] = (int64_t)w.idx[s];
      if (a.out_vals) a.out_vals[row * a.k + pos] = src[w.idx[s]];
    }
  }
}


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

struct AttnLayout {
  int nbd, dpad, ntb, tpad;
  int64_t qc, qop, qsT, qsA, qsg, kc, kop, ksT, ksA, ksg, vt, vs, pc, ps, idx32, total;
};

AttnLayout attn_layout(const mxa_attn_params* p) {
  AttnLayout L{};
  const int64_t BH = (int64_t)p->B * p->H;
  L.nbd = (p->D + 31) / 32;
  L.dpad = L.nbd * 32;
  L.ntb = (p->T + 31) / 32;
  L.tpad = L.ntb * 32;
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    const int64_t o = off;
    off += align_up(bytes);
    return o;
  };
  const int64_t qrows = BH * p->N, krows = BH * p->T;
  L.qc = take(qrows * L.dpad);
  L.qop = take(qrows * L.dpad);
  L.qsT = take(qrows * L.nbd * 2);
  L.qsA = take(qrows * L.nbd * 2);
  L.qsg = take(qrows * L.nbd * 4);
  L.kc = take(krows * L.dpad);
  L.kop = take(krows * L.dpad);
  L.ksT = take(krows * L.nbd * 2);
  L.ksA = take(krows * L.nbd * 2);
  L.ksg = take(krows * L.nbd * 4);
  L.vt = take(BH * p->D * (int64_t)L.tpad);
  L.vs = take(BH * L.ntb * (int64_t)p->D * 2);
  L.pc = take(qrows * L.tpad);
  L.ps = take(qrows * L.ntb * 2);
  L.idx32 = take(p->top_k ? qrows * (int64_t)p->k_top * 4 : 0);
  L.total = off;
  return L;
}

bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }

}  // namespace

extern "C" int mxa_abi_version(void) { return MXA_ABI_VERSION; }

#ifdef MXA_PHASE_PROF
// instrumented build only: per-phase cycle sums of attn_rows_kernel (lane 0 of each wave)
extern "C" int mxa_debug_phase_cycles(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_cycles), sizeof(unsigned long long) * 16) != hipSuccess)
    return MXA_ERR_LAUNCH;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof(z)) != hipSuccess) return MXA_ERR_LAUNCH;
  }
  return MXA_OK;
}
#endif

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
  return attn_layout(p).total;
}

template <int S>
static int launch_scores(const ScoresArgs& sa, int BH, int N, hipStream_t stream) {
  const size_t lds = (size_t)2 * kRowsPerWG * sa.tpad * sizeof(float) +
                     (size_t)4 * topk_scratch_bytes(S);
  dim3 grid((unsigned)((N + kRowsPerWG - 1) / kRowsPerWG), (unsigned)BH);
  if (lds > 65536 &&
      hipFuncSetAttribute(reinterpret_cast<const void*>(&scores_topk_kernel<S>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  hipLaunchKernelGGL(scores_topk_kernel<S>, grid, dim3(256), lds, stream, sa);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

template <int S, int MODE, bool TOPK>
static int launch_rows_s(const RowsArgs& ra, int BH, hipStream_t stream) {
  const size_t lds = rows_lds(MODE, ra.s.T, ra.kst, ra.s.nbd, S, ra.s.tpad, TOPK).total;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_rows_kernel<S, MODE, TOPK>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const dim3 grid((unsigned)((ra.s.N + ra.rows_per_wg - 1) / ra.rows_per_wg), (unsigned)BH);
  hipLaunchKernelGGL((attn_rows_kernel<S, MODE, TOPK>), grid, dim3(64 * kRowsWaves), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

template <int S>
static int launch_rows_mode(const RowsArgs& ra, int mode, int BH, hipStream_t stream) {
  if (!ra.s.top_k) return launch_rows_s<S, kModeTrue, false>(ra, BH, stream);
  switch (mode) {
    case kModeOpExp: return launch_rows_s<S, kModeOpExp, true>(ra, BH, stream);
    case kModeOpMul: return launch_rows_s<S, kModeOpMul, true>(ra, BH, stream);
    case kModeExSign: return launch_rows_s<S, kModeExSign, true>(ra, BH, stream);
    default: return launch_rows_s<S, kModeTrue, true>(ra, BH, stream);
  }
}

static int launch_rows(const RowsArgs& ra, int mode, int S, int BH, hipStream_t stream) {
  switch (S) {
    case 1: return launch_rows_mode<1>(ra, mode, BH, stream);
    case 2: return launch_rows_mode<2>(ra, mode, BH, stream);
    case 4: return launch_rows_mode<4>(ra, mode, BH, stream);
    default: return launch_rows_mode<8>(ra, mode, BH, stream);
  }
}

// ---- row kernels v2 (mxa_rows2.hpp): fused (part 0) or split (parts 1 + 2) ----
static size_t rows2_total(int mode, bool topk, const Rows2Args& ra, int S, int W, int part) {
  return rows2_lds(mode, ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, S, ra.tpad, topk ? ra.k_top : 0, W, part).total;
}
// waves per workgroup.  Fused / finishing kernel: two 8-wave workgroups per CU when
// they fit, else one 16-wave one.  Selection kernel: 4-wave workgroups (its LDS is
// the small score tables and the per-wave top-k scratch), as many per CU as fit.
static int rows2_waves(int mode, bool topk, const Rows2Args& ra, int S, int part) {
  const char* env = getenv(part == 1 ? "MXA_SELECT_WAVES" : "MXA_ROWS2_WAVES");
  if (env) {
    const int w = atoi(env);
    const int wmax = part == 1 ? 4 : 16;
    return w <= wmax && rows2_total(mode, topk, ra, S, w, part) <= 160 * 1024 ? w : 0;
  }
  if (part == 1) return rows2_total(mode, topk, ra, S, 4, part) <= 160 * 1024 ? 4 : 0;
  if (part == 2) {
    // finishing kernel: the workgroup size that keeps the most waves resident per CU
    // (LDS-limited workgroups x waves, capped by its 7-waves-per-SIMD register use):
    // DeiT-base 8 (tie), DiT 16 (larger K / V tables: 2 workgroups per CU either way)
    auto resident = [&](int w) {
      const size_t t = rows2_total(mode, topk, ra, S, w, part);
      return t > 160 * 1024 ? 0 : std::min((int)(160 * 1024 / t) * w, 28);
    };
    const int r8 = resident(8), r16 = resident(16);
    if (r8 > 0 || r16 > 0) return r16 > r8 ? 16 : 8;
  }
  if (rows2_total(mode, topk, ra, S, 8, part) <= 80 * 1024) return 8;
  if (rows2_total(mode, topk, ra, S, 16, part) <= 160 * 1024) return 16;
  if (rows2_total(mode, topk, ra, S, 8, part) <= 160 * 1024) return 8;
  if (rows2_total(mode, topk, ra, S, 4, part) <= 160 * 1024) return 4;
  return 0;
}

template <int S, int MODE, bool TOPK, bool BIG, int PART>
static int launch_rows2_p(const Rows2Args& ra0, int BH, hipStream_t stream) {
  Rows2Args ra = ra0;
  ra.waves = rows2_waves(MODE, TOPK, ra, S, PART);
  if (ra.waves <= 0) return MXA_ERR_UNSUPPORTED;
  const size_t lds = rows2_total(MODE, TOPK, ra, S, ra.waves, PART);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_rows2_kernel<S, MODE, TOPK, BIG, PART>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  // few heads (PixArt cross-attention: 128): split each head's rows over grid.y so
  // that the launch still has ~4 workgroups per CU
  int chunks = std::max(1, std::min((ra.N + ra.waves - 1) / ra.waves, 1024 / std::max(BH, 1)));
  if (PART == 1) {
    // the selection kernel stages only the small score tables, so a head's rows are
    // split over more, shorter workgroups: the last dispatch round of a long grid
    // then leaves less of the chip idle (32 rows: DeiT-base 1.34 -> 1.24 ms, DiT 2.07 -> 1.68 ms)
    const char* env = getenv("MXA_SELECT_ROWS");  // tools only: rows per workgroup
    const int rows = env ? std::max(1, atoi(env)) : 32;
    chunks = std::max(chunks, (ra.N + rows - 1) / rows);
  }
  ra.rows_per_wg = (ra.N + chunks - 1) / chunks;
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  hipLaunchKernelGGL((attn_rows2_kernel<S, MODE, TOPK, BIG, PART>), dim3((unsigned)BH, gy), dim3(64 * ra.waves), lds,
                     stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

// finishing kernel with P.V on int8 MFMA (mxa_finish.hpp): 16-row tiles, <= 8 key blocks
// Opt-in (MXA_FINISH=mfma): measured slower than the per-row v_dot4 finishing kernel
// at the bench shapes (DeiT-base 0.70 vs 0.55 ms: its 16-row P tiles in LDS cut the
// occupancy to 12 waves per CU, and the per-row gather / softmax dominate anyway).
static bool finish_mfma_ok(const Rows2Args& ra) {
  const char* env = getenv("MXA_FINISH");
  if (!env || std::string(env) != "mfma") return false;
  return ra.ntb <= 8 && fin_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, ra.tpad).total <= 160 * 1024;
}
template <int S>
static int launch_finish(const Rows2Args& ra0, int BH, hipStream_t stream) {
  Rows2Args ra = ra0;
  ra.waves = kFinWaves;
  const size_t lds = fin_lds(ra.T, ra.D, ra.kst, ra.nbd, ra.vst, ra.ntb, ra.tpad).total;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_finish_kernel<S>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  // rows per workgroup: whole 16-row tiles; few heads -> split the rows over grid.y
  const int tiles = (ra.N + 15) / 16;
  const int chunks = std::max(1, std::min((tiles + kFinWaves - 1) / kFinWaves, 1024 / std::max(BH, 1)));
  ra.rows_per_wg = 16 * ((tiles + chunks - 1) / chunks);
  const unsigned gy = (unsigned)((ra.N + ra.rows_per_wg - 1) / ra.rows_per_wg);
  hipLaunchKernelGGL((attn_finish_kernel<S>), dim3((unsigned)BH, gy), dim3(64 * kFinWaves), lds, stream, ra);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

// split: the selection kernel, an event, the finishing kernel
template <int S, int MODE, bool TOPK, bool BIG>
static int launch_rows2_b(const Rows2Args& ra, int BH, bool split, hipStream_t stream, hipEvent_t* ev) {
  int rc;
  if (TOPK && split) {
    rc = launch_rows2_p<S, MODE, TOPK, BIG, 1>(ra, BH, stream);
    if (rc) return rc;
    if (ev) (void)hipEventRecord(ev[4], stream);
    rc = finish_mfma_ok(ra) ? launch_finish<S>(ra, BH, stream) : launch_rows2_p<S, MODE, TOPK, BIG, 2>(ra, BH, stream);
  } else {
    rc = launch_rows2_p<S, MODE, TOPK, BIG, 0>(ra, BH, stream);
    if (ev) (void)hipEventRecord(ev[4], stream);
  }
  if (!rc && ev) (void)hipEventRecord(ev[5], stream);
  return rc;
}

// BIG: a sorted prefix longer than 64 is possible (k > 65)
template <int S, int MODE, bool TOPK>
static int launch_rows2_s(const Rows2Args& ra, int BH, bool split, hipStream_t stream, hipEvent_t* ev) {
  if (TOPK && ra.k_top > 65) return launch_rows2_b<S, MODE, TOPK, true>(ra, BH, split, stream, ev);
  return launch_rows2_b<S, MODE, TOPK, false>(ra, BH, split, stream, ev);
}

template <int S>
static int launch_rows2_mode(const Rows2Args& ra, int mode, bool topk, int BH, bool split, hipStream_t stream,
                             hipEvent_t* ev) {
  if (!topk) return launch_rows2_s<S, kModeTrue, false>(ra, BH, false, stream, ev);
  switch (mode) {
    case kModeOpExp: return launch_rows2_s<S, kModeOpExp, true>(ra, BH, split, stream, ev);
    case kModeOpMul: return launch_rows2_s<S, kModeOpMul, true>(ra, BH, split, stream, ev);
    case kModeExSign: return launch_rows2_s<S, kModeExSign, true>(ra, BH, split, stream, ev);
    default: return launch_rows2_s<S, kModeTrue, true>(ra, BH, split, stream, ev);
  }
}

static int launch_rows2(const Rows2Args& ra, int mode, bool topk, int S, int BH, bool split, hipStream_t stream,
                        hipEvent_t* ev) {
  switch (S) {
    case 1: return launch_rows2_mode<1>(ra, mode, topk, BH, split, stream, ev);
    case 2: return launch_rows2_mode<2>(ra, mode, topk, BH, split, stream, ev);
    case 4: return launch_rows2_mode<4>(ra, mode, topk, BH, split, stream, ev);
    default: return launch_rows2_mode<8>(ra, mode, topk, BH, split, stream, ev);
  }
}

// plan != nullptr: only report the kernel path (MXA_PATH_*), launch nothing
static int attention_impl(const mxa_attn_params* p, hipStream_t stream, hipEvent_t* ev, int* plan = nullptr) {
  if (!p || !p->q || !p->k || !p->v || !p->out) return MXA_ERR_ARG;
  if (p->B <= 0 || p->H <= 0 || p->N <= 0 || p->T <= 0 || p->D <= 0) return MXA_ERR_ARG;
  if (p->T > 512) return MXA_ERR_UNSUPPORTED;
  if (p->top_k && (p->k_top <= 0 || p->k_top > p->T)) return MXA_ERR_ARG;
  if (p->pred_mode < MXA_PRED_EX_PRED || p->pred_mode > MXA_PRED_EXION) return MXA_ERR_ARG;
  if (p->bfloat != 0 && p->bfloat != 32 && (p->bfloat < 10 || p->bfloat > 31)) return MXA_ERR_ARG;
  const AttnLayout L = attn_layout(p);
  const int64_t BH = (int64_t)p->B * p->H;

  int opq = MXA_OP_SIGN, opk = MXA_OP_SIGN;
  switch (p->pred_mode) {
    case MXA_PRED_PARTIAL_Q: opq = MXA_OP_MXINT8; break;  // Q = MXINT8, K = exp-sign
    case MXA_PRED_PARTIAL_K: opk = MXA_OP_MXINT8; break;  // Q = exp-sign, K = MXINT8
    case MXA_PRED_MXINT4: opq = opk = MXA_OP_MXINT4; break;
    case MXA_PRED_EXION: opq = opk = MXA_OP_EXION; break;
    default: break;
  }
  const bool need_pred = p->top_k && p->approx;
  // row-oriented fused kernel when the head's K tables fit LDS (attn_rows_kernel)
  const int S = (p->T + 63) / 64;
  const int rows_S = S <= 1 ? 1 : (S <= 2 ? 2 : (S <= 4 ? 4 : 8));
  const int kst = L.dpad + 16;
  const int rows_mode = !need_pred ? kModeTrue
                        : p->pred_mode == MXA_PRED_EX_PRED ? kModeExSign
                        : p->pred_mode == MXA_PRED_EXION   ? kModeOpMul
                                                           : kModeOpExp;
  const char* path_env = getenv("MXA_ATTN_PATH");
  const std::string path = path_env ? path_env : "";
  Rows2Args r2{};
  r2.T = p->T; r2.D = p->D; r2.nbd = L.nbd; r2.ntb = L.ntb; r2.tpad = L.tpad; r2.k_top = p->k_top;
  r2.kst = kst; r2.vst = L.tpad + 16;
  const bool rows2_path = L.nbd <= kMaxNB && path != "tiles" && path != "rows1" &&
                          rows2_waves(rows_mode, p->top_k != 0, r2, rows_S, 0) > 0;
  // split (default for top-k): selection kernel + finishing kernel; "fused": one kernel
  const bool split = p->top_k && path != "fused" && rows2_waves(rows_mode, true, r2, rows_S, 1) > 0 &&
                     rows2_waves(rows_mode, true, r2, rows_S, 2) > 0;
  const bool rows_path = rows2_path ||
                         (L.nbd <= kMaxNB &&
                          rows_lds(rows_mode, p->T, kst, L.nbd, rows_S, L.tpad, p->top_k != 0).total <= 160 * 1024 &&
                          path != "tiles");
  if (plan) {
    *plan = rows2_path ? (split ? MXA_PATH_ROWS_SPLIT : MXA_PATH_ROWS_FUSED) : rows_path ? MXA_PATH_ROWS_V1 : MXA_PATH_TILES;
    return MXA_OK;
  }
  if (!p->workspace || p->workspace_bytes < L.total) return MXA_ERR_WORKSPACE;
  unsigned char* ws = static_cast<unsigned char*>(p->workspace);
  if (!aligned16(ws)) return MXA_ERR_ARG;
  // the ex_pred rows kernel derives the sign operand from the MX codes
  const bool need_op = need_pred && !(rows_path && rows_mode == kModeExSign);

  RowsPrepArgs rq{};
  rq.x = p->q; rq.s0 = p->q_strides[0]; rq.s1 = p->q_strides[1]; rq.s2 = p->q_strides[2];
  rq.H = p->H; rq.R = p->N; rq.rows = BH * p->N; rq.D = p->D; rq.nb = L.nbd; rq.dpad = L.dpad;
  rq.vec4 = aligned16(p->q) && (p->q_strides[0] % 4 == 0) && (p->q_strides[1] % 4 == 0) && (p->q_strides[2] % 4 == 0);
  rq.op_kind = opq; rq.flush = p->flush_subnormals; rq.bfloat = p->bfloat;
  rq.codes = reinterpret_cast<int8_t*>(ws + L.qc);
  rq.sT = reinterpret_cast<int16_t*>(ws + L.qsT);
  rq.op = need_op ? reinterpret_cast<int8_t*>(ws + L.qop) : nullptr;
  rq.signs = rows_path && rows_mode == kModeExSign ? reinterpret_cast<uint32_t*>(ws + L.qsg) : nullptr;
  rq.sA = need_pred ? reinterpret_cast<int16_t*>(ws + L.qsA) : nullptr;
  if (ev) (void)hipEventRecord(ev[0], stream);
  int rc = launch_rows_prep(rq, stream);
  if (rc) return rc;
  if (ev) (void)hipEventRecord(ev[1], stream);

  RowsPrepArgs rk = rq;
  rk.x = p->k; rk.s0 = p->k_strides[0]; rk.s1 = p->k_strides[1]; rk.s2 = p->k_strides[2];
  rk.R = p->T; rk.rows = BH * p->T;
  rk.vec4 = aligned16(p->k) && (p->k_strides[0] % 4 == 0) && (p->k_strides[1] % 4 == 0) && (p->k_strides[2] % 4 == 0);
  rk.op_kind = opk;
  rk.codes = reinterpret_cast<int8_t*>(ws + L.kc);
  rk.sT = reinterpret_cast<int16_t*>(ws + L.ksT);
  rk.op = need_op ? reinterpret_cast<int8_t*>(ws + L.kop) : nullptr;
  rk.signs = rows_path && rows_mode == kModeExSign ? reinterpret_cast<uint32_t*>(ws + L.ksg) : nullptr;
  rk.sA = need_pred ? reinterpret_cast<int16_t*>(ws + L.ksA) : nullptr;
  rc = launch_rows_prep(rk, stream);
  if (rc) return rc;
  if (ev) (void)hipEventRecord(ev[2], stream);

  ColsPrepArgs cv{};
  cv.x = p->v; cv.s0 = p->v_strides[0]; cv.s1 = p->v_strides[1]; cv.s2 = p->v_strides[2];
  cv.H = p->H; cv.mats = BH; cv.R = p->T; cv.C = p->D; cv.nb = L.ntb; cv.rpad = L.tpad;
  cv.mbits = 8; cv.flush = p->flush_subnormals; cv.bfloat = p->bfloat;
  cv.codes_t = reinterpret_cast<int8_t*>(ws + L.vt);
  cv.scale = reinterpret_cast<int16_t*>(ws + L.vs);
  rc = launch_cols_prep(cv, stream);
  if (rc) return rc;
  if (ev) (void)hipEventRecord(ev[3], stream);

  ScoresArgs sa{};
  sa.qc = reinterpret_cast<const int8_t*>(ws + L.qc);
  sa.qop = reinterpret_cast<const int8_t*>(ws + L.qop);
  sa.kc = reinterpret_cast<const int8_t*>(ws + L.kc);
  sa.kop = reinterpret_cast<const int8_t*>(ws + L.kop);
  sa.qsT = reinterpret_cast<const int16_t*>(ws + L.qsT);
  sa.qsA = reinterpret_cast<const int16_t*>(ws + L.qsA);
  sa.ksT = reinterpret_cast<const int16_t*>(ws + L.ksT);
  sa.ksA = reinterpret_cast<const int16_t*>(ws + L.ksA);
  sa.B = p->B; sa.H = p->H; sa.N = p->N; sa.T = p->T;
  sa.nbd = L.nbd; sa.dpad = L.dpad; sa.ntb = L.ntb; sa.tpad = L.tpad;
  sa.k_top = p->k_top; sa.top_k = p->top_k; sa.approx = p->approx;
  sa.mul_combine = p->pred_mode == MXA_PRED_EXION;
  sa.bfloat = p->bfloat; sa.flush_p = p->flush_subnormals;
  sa.scale = p->scale;
  sa.bias = p->bias;
  sa.bs0 = p->bias_strides[0]; sa.bs1 = p->bias_strides[1]; sa.bs2 = p->bias_strides[2]; sa.bs3 = p->bias_strides[3];
  sa.idx_out = p->idx_out; sa.true_out = p->true_out; sa.pred_out = p->pred_out;
  sa.pc = reinterpret_cast<int8_t*>(ws + L.pc);
  sa.ps = reinterpret_cast<int16_t*>(ws + L.ps);
  if (rows2_path) {
    r2.qc = sa.qc; r2.qop = sa.qop; r2.qsT = sa.qsT; r2.qsA = sa.qsA;
    r2.qsg = reinterpret_cast<const uint32_t*>(ws + L.qsg);
    r2.kc = sa.kc; r2.kop = sa.kop; r2.ksT = sa.ksT; r2.ksA = sa.ksA;
    r2.ksg = reinterpret_cast<const uint32_t*>(ws + L.ksg);
    r2.vt = reinterpret_cast<const int8_t*>(ws + L.vt);
    r2.vs = reinterpret_cast<const int16_t*>(ws + L.vs);
    r2.B = p->B; r2.H = p->H; r2.N = p->N; r2.dpad = L.dpad;
    r2.bfloat = p->bfloat; r2.flush_p = p->flush_subnormals; r2.scale = p->scale;
    r2.bias = p->bias;
    r2.bs0 = p->bias_strides[0]; r2.bs1 = p->bias_strides[1]; r2.bs2 = p->bias_strides[2]; r2.bs3 = p->bias_strides[3];
    r2.out = p->out; r2.os0 = p->out_strides[0]; r2.os1 = p->out_strides[1]; r2.os2 = p->out_strides[2];
    r2.idx_out = p->idx_out; r2.true_out = p->true_out; r2.pred_out = p->pred_out;
#ifdef MXA_PHASE_PROF
    r2.dbg = getenv("MXA_DBG_SKIP") ? atoi(getenv("MXA_DBG_SKIP")) : 0;
#endif
    r2.idx32 = reinterpret_cast<int32_t*>(ws + L.idx32);
    return launch_rows2(r2, rows_mode, p->top_k != 0, rows_S, (int)BH, split, stream, ev);
  } else if (rows_path) {
    RowsArgs ra{};
    ra.s = sa;
    ra.qsg = reinterpret_cast<const uint32_t*>(ws + L.qsg);
    ra.ksg = reinterpret_cast<const uint32_t*>(ws + L.ksg);
    ra.D = p->D;
    ra.kst = kst;
    ra.rows_per_wg = p->N;
#ifdef MXA_PHASE_PROF
    ra.dbg = getenv("MXA_DBG_SKIP") ? atoi(getenv("MXA_DBG_SKIP")) : 0;
#endif
    rc = launch_rows(ra, rows_mode, rows_S, (int)BH, stream);
  } else if (S <= 1) rc = launch_scores<1>(sa, (int)BH, p->N, stream);
  else if (S <= 2) rc = launch_scores<2>(sa, (int)BH, p->N, stream);
  else if (S <= 4) rc = launch_scores<4>(sa, (int)BH, p->N, stream);
  else rc = launch_scores<8>(sa, (int)BH, p->N, stream);
  if (rc) return rc;
  if (ev) (void)hipEventRecord(ev[4], stream);

  PVArgs pa{};
  pa.pc = sa.pc; pa.ps = sa.ps;
  pa.vt = reinterpret_cast<const int8_t*>(ws + L.vt);
  pa.vs = reinterpret_cast<const int16_t*>(ws + L.vs);
  pa.B = p->B; pa.H = p->H; pa.N = p->N; pa.D = p->D; pa.ntb = L.ntb; pa.tpad = L.tpad; pa.bfloat = p->bfloat;
  pa.out = p->out; pa.os0 = p->out_strides[0]; pa.os1 = p->out_strides[1]; pa.os2 = p->out_strides[2];
  dim3 grid((unsigned)((p->N + kRowsPerWG - 1) / kRowsPerWG), (unsigned)BH);
  hipLaunchKernelGGL(pv_kernel, grid, dim3(256), 0, stream, pa);
  if (hipGetLastError() != hipSuccess) return MXA_ERR_LAUNCH;
  if (ev) (void)hipEventRecord(ev[5], stream);
  return MXA_OK;
}

extern "C" int mxa_attention(const mxa_attn_params* p, hipStream_t stream) {
  return attention_impl(p, stream, nullptr);
}

extern "C" int mxa_attention_path(const mxa_attn_params* p) {
  int plan = -1;
  const int rc = attention_impl(p, nullptr, nullptr, &plan);
  return rc ? rc : plan;
}

extern "C" int mxa_attention_timed(const mxa_attn_params* p, hipStream_t stream, int32_t iters, float* stage_ms) {
  if (iters <= 0 || !stage_ms) return MXA_ERR_ARG;
  std::vector<hipEvent_t> ev((size_t)iters * MXA_ATTN_STAGES_PLUS1);
  for (auto& e : ev)
    if (hipEventCreate(&e) != hipSuccess) return MXA_ERR_LAUNCH;
  int rc = MXA_OK;
  for (int i = 0; i < iters && rc == MXA_OK; ++i) rc = attention_impl(p, stream, &ev[(size_t)i * MXA_ATTN_STAGES_PLUS1]);
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

template <int S>
static int launch_topk(const TopkArgs& ta, hipStream_t stream) {
  const dim3 grid((unsigned)((ta.rows + 3) / 4));
  const char* env = getenv("MXA_TOPK_IMPL");
  const std::string impl = env ? env : "";
  if (impl == "v1")
    hipLaunchKernelGGL(topk_rows_v1_kernel<S>, grid, dim3(256), (size_t)4 * (2 * 64 * S + kTopkStack / 2) * 8, stream, ta);
  else if (impl == "lds")
    hipLaunchKernelGGL(topk_rows_kernel<S>, grid, dim3(256), (size_t)4 * topk_scratch_bytes(S), stream, ta);
  else if (impl != "reg" && ta.k <= 64) {  // lane-per-row tail
    return ta.k <= 32 ? launch_topk_lane_cfg<S, 32>(ta, stream) : launch_topk_lane_cfg<S, 64>(ta, stream);
  } else
    hipLaunchKernelGGL(topk_reg_kernel<S>, grid, dim3(256), (size_t)4 * topk_scratch_bytes(S), stream, ta);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

extern "C" int mxa_topk(const float* vals, int64_t rows, int32_t n, int64_t ld, int32_t k, int64_t* out_idx,
                        float* out_vals, hipStream_t stream) {
  if (!vals || !out_idx || rows < 0 || n <= 0 || ld < n || k < 0 || k > n) return MXA_ERR_ARG;
  if (n > 512) return MXA_ERR_UNSUPPORTED;
  if (rows == 0 || k == 0) return MXA_OK;
  const char* dbg = getenv("MXA_TOPK_DBG");
  TopkArgs ta{vals, rows, ld, n, k, out_idx, out_vals, dbg ? atoi(dbg) : 0};
  const int S = (n + 63) / 64;
  if (S <= 1) return launch_topk<1>(ta, stream);
  if (S <= 2) return launch_topk<2>(ta, stream);
  if (S <= 4) return launch_topk<4>(ta, stream);
  return launch_topk<8>(ta, stream);
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

extern "C" int mxa_selftest_mfma(const int8_t* a, const int8_t* b, int32_t* c, hipStream_t stream) {
  if (!a || !b || !c) return MXA_ERR_ARG;
  hipLaunchKernelGGL(selftest_mfma_kernel, dim3(1), dim3(64), 0, stream, a, b, c);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
