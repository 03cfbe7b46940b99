// Selection kernel: approximate scores + exact-order top-k, FOUR query rows per wave.
//
// Per workgroup (one head, a chunk of its query rows): the head's score tables are
// staged in LDS once (sel_lds):
//   ex_pred        sign words + block exponents
//   MXINT4 / EXION / partial_*   approximator codes + block scales
//   true_ex        power-of-two codes + zero indicators + block exponents
//   ELSA           hash words + the (D+1)-entry cosine table
//   approx off     MXINT8 codes + exponents (the true scores are ranked)
// Per wave, four rows at a time, one 16-lane DPP row each:
//   1. lane gl computes the scores of keys gl, gl + 16, ... into the row's LDS mirror
//      (exact fp64 block epilogue: the scores are exact sums of integer * 2^e,
//      SURVEY.md F6), bias added in fp32 as the caller does;
//   2. grp_topk (mxa_topk_grp.hpp) reproduces torch's CPU topk index order;
//   3. the k kept indices go out as int64 (the op's idx) and int32 (the finishing
//      kernel's input), four consecutive rows per wave, and the prune-mask words
//      when asked for.
// k_top == 0: scores only (mxa_approx_scores).
// Callers replaced: the approximator + torch.topk of
//   workloads/deit/scripts/main.py:101-123, workloads/DiT/models.py:168-194,
//   workloads/PixArt/models/MX_transformer_block.py:656-678, :805-825.
#pragma once
#include <type_traits>
#include "mxa_rows2.hpp"
#include "mxa_topk_grp.hpp"
#include "mxa_topk_wave.hpp"

namespace mxa {

#ifndef MXA_SEL_ROWS  // tools builds vary these (build_native defines)
#define MXA_SEL_ROWS 32
#endif
#ifndef MXA_SEL_OCC
#define MXA_SEL_OCC 4
#endif
#ifndef MXA_SELW_OCC
#define MXA_SELW_OCC 8
#endif
// 1: the selection kernel with one wave per query row (select_wave_kernel) -- a tools
// A/B build; measured slower than four rows per wave (DeiT-base 1.15 vs 0.80 ms: its
// per-row scalar bookkeeping costs as much issue time as the vector work it saves)
#ifndef MXA_SEL_WAVE
#define MXA_SEL_WAVE 0
#endif
#ifndef MXA_SEL_SHORT_T
#define MXA_SEL_SHORT_T 224
#endif
constexpr int kSelRows = MXA_SEL_ROWS;  // query rows per workgroup (a multiple of 4 * waves)
// waves per workgroup: 2 for rows of <= 224 keys on a large grid (DeiT-base: 0.97 ->
// 0.93 ms), else 4 (DiT: 1.44 vs 1.56 ms with 2; PixArt's 128 heads: 0.069 vs 0.10 ms)
// -- measured, tools/bench_cmp.sh
inline int sel_waves_for(int T, int64_t BH, int N) {
  return T <= MXA_SEL_SHORT_T && BH * ((N + kSelRows - 1) / kSelRows) >= 8192 ? 2 : 4;
}

// LDS layout of the score tables (then the per-row top-k areas)
struct SelLds {
  size_t cd, ex, sg, z, cs, rows;
};
__host__ __device__ inline SelLds sel_lds(int mode, int T, int D, int kst, int nbd) {
  SelLds L;
  size_t o = 0;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const bool codes = mode == kModeTrue || mode == kModeOpExp || mode == kModeOpMul || mode == kModeTrueEx;
  L.cd = o;
  if (codes) o += al((size_t)T * kst);
  L.ex = o;
  if (mode != kModeElsa) o += al((size_t)T * nbd * 2);
  L.sg = o;
  if (mode == kModeExSign || mode == kModeElsa) o += al((size_t)T * nbd * 4);
  L.z = o;
  if (mode == kModeTrueEx) o += al((size_t)T * kst);
  L.cs = o;
  if (mode == kModeElsa) o += al((size_t)(D + 1) * 4);
  L.rows = o;
  return L;
}

__device__ __forceinline__ int dot32(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
  int I = 0;
  I = __builtin_amdgcn_sdot4((int)a0.x, (int)b0.x, I, false);
  I = __builtin_amdgcn_sdot4((int)a0.y, (int)b0.y, I, false);
  I = __builtin_amdgcn_sdot4((int)a0.z, (int)b0.z, I, false);
  I = __builtin_amdgcn_sdot4((int)a0.w, (int)b0.w, I, false);
  I = __builtin_amdgcn_sdot4((int)a1.x, (int)b1.x, I, false);
  I = __builtin_amdgcn_sdot4((int)a1.y, (int)b1.y, I, false);
  I = __builtin_amdgcn_sdot4((int)a1.z, (int)b1.z, I, false);
  I = __builtin_amdgcn_sdot4((int)a1.w, (int)b1.w, I, false);
  return I;
}

// ex_pred score of one key: sum_b m_b 2^(eq_b + ek_b), m_b = n_b - 2 popc(sq_b ^ sk_b)
// (|m_b| <= 32).  When the block exponents span <= 23 bits and the smallest is >= -100,
// the sum shifted to the smallest exponent is an exact int32, so one conversion (round
// to nearest even) and an exact scaling give the correctly rounded float; otherwise
// (and for NaN blocks) the exact fp64 sum.  Both equal fl32 of the exact sum.
template <int NBD>
__device__ __forceinline__ float expred_score(const uint32_t* sq, const int* eq, const int16_t* kex, const uint32_t* ksg,
                                              int D) {
  int m[NBD], e[NBD];
  bool nan = false;
  int emin = 1 << 20, emax = -(1 << 20);
#pragma unroll
  for (int b = 0; b < NBD; ++b) {
    const int ek = exp_from16(kex[b]);
    nan = nan || ek == kExpNaN || eq[b] == kExpNaN;
    e[b] = eq[b] + ek;
    m[b] = min(32, D - 32 * b) - 2 * (int)__popc(sq[b] ^ ksg[b]);
    emin = min(emin, e[b]);
    emax = max(emax, e[b]);
  }
  if (nan) return __uint_as_float(0x7FC00000u);
  if (emax - emin <= 23 && emin >= -100) {
    int sum = 0;
#pragma unroll
    for (int b = 0; b < NBD; ++b) sum += m[b] << (e[b] - emin);
    return ldexpf((float)sum, emin);
  }
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < NBD; ++b) acc += (double)m[b] * pow2d(e[b]);
  return (float)acc;
}

// MX dot product of a query row (codes in registers, two uint4 per 32-block, block
// exponents qe) with key row krow of the LDS code table: exact block sums by v_dot4,
// block scale 2^(qe+ke) (MUL = 0) or qe*ke/4096 (EXION, MUL = 1), fp64 accumulation
template <int MUL, int NBMAX = kMaxNB>
__device__ __forceinline__ double g_dot(const uint4* qv, const int* qe, int nbd, const int8_t* krow,
                                        const int16_t* kexp, bool& nan) {
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < NBMAX; ++b) {
    if (b < nbd) {
      const uint4 x0 = *reinterpret_cast<const uint4*>(krow + 32 * b);
      const uint4 x1 = *reinterpret_cast<const uint4*>(krow + 32 * b + 16);
      const int I = dot32(qv[2 * b], qv[2 * b + 1], x0, x1);
      const int e = exp_from16(kexp[b]);
      if (e == kExpNaN || qe[b] == kExpNaN) nan = true;
      else if (MUL) acc += (double)I * (double)(qe[b] * e) * (1.0 / 4096.0);
      else acc += (double)I * pow2d(qe[b] + e);
    }
  }
  return acc;
}

// The true score fl32(sum_b I_b 2^(qe_b + ke_b)) of a query row (codes in registers)
// and a key row of the LDS code table (MXINT8, exponents in code units): block sums by
// v_dot4; when the block exponents span <= 10 bits (NB x 2^19 x 2^10 < 2^31) and the
// smallest is >= -100, the sum shifted to the smallest exponent is an exact int32 and
// one conversion + exact scaling gives the correctly rounded float (no fp64); otherwise
// the exact fp64 sum (g_dot).  NaN for a NaN block.
template <int NB>
__device__ __forceinline__ float true_dot(const uint4* qv, const int* qe, const int8_t* krow, const int16_t* kexp) {
  int I[NB], e[NB];
  int emin = 1 << 20, emax = -(1 << 20);
  bool nan = false;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint4 x0 = *reinterpret_cast<const uint4*>(krow + 32 * b);
    const uint4 x1 = *reinterpret_cast<const uint4*>(krow + 32 * b + 16);
    I[b] = dot32(qv[2 * b], qv[2 * b + 1], x0, x1);
    const int ke = exp_from16(kexp[b]);
    nan = nan || ke == kExpNaN || qe[b] == kExpNaN;
    e[b] = qe[b] + ke;
    emin = min(emin, e[b]);
    emax = max(emax, e[b]);
  }
  if (nan) return __uint_as_float(0x7FC00000u);
  if (emax - emin <= 10 && emin >= -100) {
    int sum = 0;
#pragma unroll
    for (int b = 0; b < NB; ++b) sum += I[b] << (e[b] - emin);
    return ldexpf((float)sum, emin);
  }
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < NB; ++b) acc += (double)I[b] * pow2d(e[b]);
  return (float)acc;
}

// true_ex: a = c * 2^e + z per element (c the power-of-two code, 0 for a zero MX
// element; z = 1 for a zero element), so per block
//   sum aQ aK = 2^(eq+ek) <cq,ck> + 2^eq <cq,zk> + 2^ek <zq,ck> + <zq,zk>   (exact in fp64)
__device__ __forceinline__ double g_dot_trueex(const uint4* qv, const uint4* qz, const int* qe, int nbd,
                                               const int8_t* krow, const int8_t* kzrow, const int16_t* kexp,
                                               bool& nan) {
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < kMaxNB; ++b) {
    if (b < nbd) {
      const uint4 k0 = *reinterpret_cast<const uint4*>(krow + 32 * b);
      const uint4 k1 = *reinterpret_cast<const uint4*>(krow + 32 * b + 16);
      const uint4 z0 = *reinterpret_cast<const uint4*>(kzrow + 32 * b);
      const uint4 z1 = *reinterpret_cast<const uint4*>(kzrow + 32 * b + 16);
      const int I1 = dot32(qv[2 * b], qv[2 * b + 1], k0, k1);
      const int I2 = dot32(qv[2 * b], qv[2 * b + 1], z0, z1);
      const int I3 = dot32(qz[2 * b], qz[2 * b + 1], k0, k1);
      const int I4 = dot32(qz[2 * b], qz[2 * b + 1], z0, z1);
      const int e = exp_from16(kexp[b]);
      if (e == kExpNaN || qe[b] == kExpNaN) {
        nan = true;
      } else {
        acc += (double)I1 * pow2d(qe[b] + e);
        acc += (double)I2 * pow2d(qe[b]);
        acc += (double)I3 * pow2d(e);
        acc += (double)I4;
      }
    }
  }
  return acc;
}

// ELSA cosine table entry h: cos(clamp(fl32(fl32(pi/D) * h) - 0.127f, 0)) correctly
// rounded (funcs/elsa_approximation.py:138-143; the caller may pass torch's values)
__device__ __forceinline__ float elsa_cos_entry(int D, int h) {
  const float est = (float)(3.141592653589793 / (double)D) * (float)h;
  const float cor = fmaxf(est - 0.127f, 0.0f);
  return (float)cos((double)cor);
}

template <int NP, int MODE, int kSelWaves>
__global__ __launch_bounds__(64 * kSelWaves) __attribute__((amdgpu_waves_per_eu(NP <= 256 ? MXA_SEL_OCC : 2, 8))) void select_kernel(Rows2Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool kOp = MODE == kModeOpExp || MODE == kModeOpMul;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gi = lane >> 4, gl = lane & 15;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst, k = a.k_top;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const SelLds L = sel_lds(MODE, T, D, kst, nbd);
  int8_t* tcd = reinterpret_cast<int8_t*>(smem + L.cd);    // key codes
  int16_t* tex = reinterpret_cast<int16_t*>(smem + L.ex);  // key exponents
  uint32_t* tsg = reinterpret_cast<uint32_t*>(smem + L.sg);  // sign / hash words
  int8_t* tz = reinterpret_cast<int8_t*>(smem + L.z);      // true_ex zero indicators
  float* tcs = reinterpret_cast<float*>(smem + L.cs);      // ELSA cosine table

  // ---- stage the head's score tables ----------------------------------------
  const int64_t kb = (int64_t)bh * T;
  if constexpr (MODE == kModeTrue || kOp || MODE == kModeTrueEx) {
    const int8_t* src = MODE == kModeTrue ? a.kc : a.kop;
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(tcd + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(src + (kb + j) * a.dpad + 16 * c);
      if (MODE == kModeTrueEx)
        *reinterpret_cast<uint4*>(tz + (size_t)j * kst + 16 * c) =
            *reinterpret_cast<const uint4*>(a.kz + (kb + j) * a.dpad + 16 * c);
    }
  }
  {
    const int16_t* esrc = MODE == kModeTrue ? a.ksT : a.ksA;
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) {
      if (MODE != kModeElsa) tex[i] = esrc[kb * nbd + i];
      if (MODE == kModeExSign || MODE == kModeElsa) tsg[i] = a.ksg[kb * nbd + i];
    }
    if (MODE == kModeElsa)
      for (int h = threadIdx.x; h <= D; h += blockDim.x) tcs[h] = a.elsa_cos ? a.elsa_cos[h] : elsa_cos_entry(D, h);
  }
  __syncthreads();

  const int npa = grp_alloc(T);
  const size_t rowb = grp_row_bytes(npa, NP);
  const GrpRow g = carve_grp(smem + L.rows + (size_t)(4 * wave + gi) * rowb, npa, NP);
  const int ntw = (T + 31) / 32;  // prune-mask words per row
  const int r_end = min(a.N, (int)(blockIdx.y + 1) * a.rows_per_wg);
  for (int rq = (int)blockIdx.y * a.rows_per_wg + 4 * wave; rq < r_end; rq += 4 * kSelWaves) {
    const int r = rq + gi;
    const bool valid = r < r_end;
    const int64_t grow = (int64_t)bh * a.N + (valid ? r : rq);
    const int64_t brow = a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)(valid ? r : rq) * a.bs2 : -1;

    // ---- the row's scores into its mirror ------------------------------------
#ifdef MXA_SEL_SKIP
    if (valid && !((MXA_SEL_SKIP) & 2)) {
#else
    if (valid) {
#endif
      // scores in the score dtype: the approximator GEMM's (or the true matmul's) output
      // rounded to it, then + bias (MX_transformer_block.py:821-822), rounded again
      auto emit = [&](int j, float v) {
        v = round_dt(v, a.s_dt);
        if (brow >= 0) v = round_dt(v + load_dt(a.bias, brow + (int64_t)j * a.bs3, a.in_dt), a.s_dt);
        if (MODE == kModeTrue) {
          if (a.true_out) a.true_out[grow * T + j] = v;
        } else if (a.pred_out) {
          a.pred_out[grow * T + j] = v;
        }
        g.A[j] = pack_ki(order_key(v), (uint32_t)j);
      };
      if constexpr (MODE == kModeExSign) {
        // pred = sum_b 2^(eq_b + ek_b) (n_b - 2 popc(sq_b ^ sk_b))   (exact)
        uint32_t sq[kMaxNB];
        int eq[kMaxNB];
#pragma unroll
        for (int b = 0; b < kMaxNB; ++b) {
          sq[b] = b < nbd ? a.qsg[grow * nbd + b] : 0u;
          eq[b] = b < nbd ? exp_from16(a.qsA[grow * nbd + b]) : 0;
        }
        auto keys = [&](auto nbd_c) {  // the key loop for a compile-time block count
          constexpr int NBD = decltype(nbd_c)::value;
          if (brow >= 0 || a.s_dt != kF32) {
            for (int j = gl; j < T; j += 16) emit(j, expred_score<NBD>(sq, eq, tex + j * NBD, tsg + j * NBD, D));
            return;
          }
          // no bias: the raw int16 exponents (NaN = INT16_MIN) go straight into the
          // fast-path test -- a NaN block drives the smallest exponent below -100 --
          // and a fast-path value (finite, never -0) takes the three-instruction key
          int eqr[NBD], nbk[NBD];
#pragma unroll
          for (int b = 0; b < NBD; ++b) {
            eqr[b] = eq[b] == kExpNaN ? (int)kExpNaN16 : eq[b];
            nbk[b] = min(32, D - 32 * b);
          }
          float* prow = a.pred_out ? a.pred_out + grow * T : nullptr;
          for (int j = gl; j < T; j += 16) {
            const int16_t* kex = tex + j * NBD;
            const uint32_t* ksg = tsg + j * NBD;
            int e[NBD], m[NBD];
#pragma unroll
            for (int b = 0; b < NBD; ++b) {
              e[b] = eqr[b] + (int)kex[b];
              m[b] = nbk[b] - 2 * (int)__popc(sq[b] ^ ksg[b]);
            }
            int emin = e[0], emax = e[0];
#pragma unroll
            for (int b = 1; b < NBD; ++b) {
              emin = min(emin, e[b]);
              emax = max(emax, e[b]);
            }
            float v;
            uint32_t key;
            if (emax - emin <= 23 && emin >= -100) {
              int sum = 0;
#pragma unroll
              for (int b = 0; b < NBD; ++b) sum += m[b] << (e[b] - emin);
              v = ldexpf((float)sum, emin);
              const uint32_t u = __float_as_uint(v);
              key = u ^ ((uint32_t)((int)u >> 31) | 0x80000000u);
            } else {
              v = expred_score<NBD>(sq, eq, kex, ksg, D);
              key = order_key(v);
            }
            if (prow) prow[j] = v;
            g.A[j] = pack_ki(key, (uint32_t)j);
          }
        };
        switch (nbd) {
          case 1: keys(std::integral_constant<int, 1>{}); break;
          case 2: keys(std::integral_constant<int, 2>{}); break;
          case 3: keys(std::integral_constant<int, 3>{}); break;
          default: keys(std::integral_constant<int, 4>{}); break;
        }
      } else if constexpr (MODE == kModeElsa) {
        // approx = ||MX_K[row r]|| * cos(clamp(pi/D * hamming - 0.127, 0))
        // (elsa_approximation.py:124-143; the key norm of row r, the reference's broadcast)
        uint32_t hq[kMaxNB];
#pragma unroll
        for (int b = 0; b < kMaxNB; ++b) hq[b] = b < nbd ? a.qsg[grow * nbd + b] : 0u;
        const float nrm = a.knorm[kb + r];
        for (int j = gl; j < T; j += 16) {
          int h = 0;
#pragma unroll
          for (int b = 0; b < kMaxNB; ++b)
            if (b < nbd) h += (int)__popc(hq[b] ^ tsg[j * nbd + b]);
          emit(j, nrm * tcs[h]);
        }
      } else {
        const int8_t* qsrc = (MODE == kModeTrue ? a.qc : a.qop) + grow * a.dpad;
        const int16_t* qesrc = (MODE == kModeTrue ? a.qsT : a.qsA) + grow * nbd;
        uint4 qv[2 * kMaxNB];
        uint4 qz[MODE == kModeTrueEx ? 2 * kMaxNB : 1];
        int qe[kMaxNB];
#pragma unroll
        for (int b = 0; b < kMaxNB; ++b) {
          qv[2 * b] = b < nbd ? *reinterpret_cast<const uint4*>(qsrc + 32 * b) : make_uint4(0, 0, 0, 0);
          qv[2 * b + 1] = b < nbd ? *reinterpret_cast<const uint4*>(qsrc + 32 * b + 16) : make_uint4(0, 0, 0, 0);
          if constexpr (MODE == kModeTrueEx) {
            const int8_t* zsrc = a.qz + grow * a.dpad;
            qz[2 * b] = b < nbd ? *reinterpret_cast<const uint4*>(zsrc + 32 * b) : make_uint4(0, 0, 0, 0);
            qz[2 * b + 1] = b < nbd ? *reinterpret_cast<const uint4*>(zsrc + 32 * b + 16) : make_uint4(0, 0, 0, 0);
          }
          qe[b] = b < nbd ? exp_from16(qesrc[b]) : 0;
        }
        for (int j = gl; j < T; j += 16) {
          bool nan = false;
          double acc;
          if constexpr (MODE == kModeTrueEx)
            acc = g_dot_trueex(qv, qz, qe, nbd, tcd + (size_t)j * kst, tz + (size_t)j * kst, tex + j * nbd, nan);
          else
            acc = g_dot<MODE == kModeOpMul>(qv, qe, nbd, tcd + (size_t)j * kst, tex + j * nbd, nan);
          float v = nan ? __uint_as_float(0x7FC00000u) : (float)acc;
          // true = quantize_elemwise(fl32(QK^T)) * scale   (matmul.py:88-91, caller)
          if (MODE == kModeTrue) v = round_bfloat(round_dt(v, a.s_dt), a.bfloat, kRoundNearest, 1, a.s_dt) * a.scale;
          emit(j, v);
        }
      }
    }
#ifdef MXA_SEL_SKIP  // tools-only phase timing (build_native defines): 2 = scores replaced by hashed keys
    if ((MXA_SEL_SKIP) & 2)
      for (int j = gl; j < T; j += 16) g.A[j] = pack_ki(0x80000000u | ((uint32_t)(j * 2654435761u + r * 40503u) >> 26), (uint32_t)j);
#endif
    if (k <= 0) continue;  // scores only
    wave_lds_sync();

    // ---- torch CPU top-k order ------------------------------------------------
#ifdef MXA_SEL_SKIP  // 1 = no top-k
    if (!((MXA_SEL_SKIP) & 1))
#endif
    grp_topk<NP>(g, T, k, valid, gl);

    // ---- kept indices: four consecutive rows per wave ----------------------------
    // (measured: per-row stores beat 16-B stores over the four rows' span, whose
    // per-element LDS gathers cost more VALU and whose HBM writes were larger)
    if (valid) {
      for (int p = gl; p < k; p += 16) {
        const uint32_t ix = (uint32_t)g.A[p];
        if (a.idx_out) a.idx_out[grow * k + p] = (int64_t)ix;
        a.idx32[grow * k + p] = (int32_t)ix;
      }
    }
    if (a.mask_out) {  // prune mask: zeros.scatter_(-1, idx, 1) as bits
      lu32* mw = g.stk;  // free after grp_topk
      if (gl < ntw) mw[gl] = 0u;
      wave_lds_sync();
      if (valid)
        for (int p = gl; p < k; p += 16) {
          const uint32_t ix = (uint32_t)g.A[p];
          atomicOr((uint32_t*)(mw + (ix >> 5)), 1u << (ix & 31));
        }
      wave_lds_sync();
      if (valid)
        for (int w = gl; w < ntw; w += 16) a.mask_out[grow * ntw + w] = mw[w];
    }
    wave_lds_sync();
  }
}

// ---- the selection kernel, ONE WAVE PER QUERY ROW (mxa_topk_wave.hpp) ------------
// Per workgroup (one head, a chunk of its query rows, kSelWaveW waves): the score
// tables staged in LDS as above; then each wave takes rows wave, wave + W, ...: lane
// computes the scores of keys lane, lane + 64, ... into the row's mirror, wave_topk
// reproduces torch's CPU index order with the row's bookkeeping in scalar registers,
// and the k kept indices (int64 + int32) and the prune-mask words go out.  The query
// row's operands are wave-uniform (scalar loads).
constexpr int kSelWaveW = 4;
__host__ __device__ inline size_t selw_lds(int mode, int T, int D, int kst, int nbd) {
  return sel_lds(mode, T, D, kst, nbd).rows + (size_t)kSelWaveW * wrow_bytes(T);
}

template <int NP, int MODE>
__global__ __launch_bounds__(64 * kSelWaveW) __attribute__((amdgpu_waves_per_eu(NP <= 256 ? MXA_SELW_OCC : 4, 8))) void select_wave_kernel(Rows2Args a0) {
  const Rows2Args& a = a0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool kOp = MODE == kModeOpExp || MODE == kModeOpMul;
  constexpr int EW = NP / 64;
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t lane0 = threadIdx.x & 63;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const SelLds L = sel_lds(MODE, T, D, kst, nbd);
  int8_t* tcd = reinterpret_cast<int8_t*>(smem + L.cd);
  int16_t* tex = reinterpret_cast<int16_t*>(smem + L.ex);
  uint32_t* tsg = reinterpret_cast<uint32_t*>(smem + L.sg);
  int8_t* tz = reinterpret_cast<int8_t*>(smem + L.z);
  float* tcs = reinterpret_cast<float*>(smem + L.cs);

  // ---- stage the head's score tables ----------------------------------------
  const int64_t kb = (int64_t)bh * T;
  if constexpr (MODE == kModeTrue || kOp || MODE == kModeTrueEx) {
    const int8_t* src = MODE == kModeTrue ? a.kc : a.kop;
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(tcd + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(src + (kb + j) * a.dpad + 16 * c);
      if (MODE == kModeTrueEx)
        *reinterpret_cast<uint4*>(tz + (size_t)j * kst + 16 * c) =
            *reinterpret_cast<const uint4*>(a.kz + (kb + j) * a.dpad + 16 * c);
    }
  }
  {
    const int16_t* esrc = MODE == kModeTrue ? a.ksT : a.ksA;
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) {
      if (MODE != kModeElsa) tex[i] = esrc[kb * nbd + i];
      if (MODE == kModeExSign || MODE == kModeElsa) tsg[i] = a.ksg[kb * nbd + i];
    }
    if (MODE == kModeElsa)
      for (int h = threadIdx.x; h <= D; h += blockDim.x) tcs[h] = a.elsa_cos ? a.elsa_cos[h] : elsa_cos_entry(D, h);
  }
  __syncthreads();

  const WRow g = carve_wrow(smem + L.rows + (size_t)wave * wrow_bytes(T), T);
  const int ntw = (T + 31) / 32;  // prune-mask words per row
  const int r_end = min(a.N, (int)(blockIdx.y + 1) * a.rows_per_wg);
  for (int r = (int)blockIdx.y * a.rows_per_wg + wave; r < r_end; r += kSelWaveW) {
    // the argument block re-read per row (scalar loads, cache hits) rather than held in
    // SGPRs across the top-k: SGPRs bound the resident waves
    typedef __attribute__((address_space(4))) const Rows2Args KArgs;
    KArgs* ap = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ap));
    KArgs& a = *ap;
    uint32_t lane = lane0;  // (re-derived per row as well: its hoisted address arithmetic spilled)
    asm volatile("" : "+v"(lane));
    // (every size re-read too: hoisted, the top-k's conditions on k and T were spilled)
    const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst, k = a.k_top;
    const int64_t kb = (int64_t)bh * T;
    const int64_t grow = (int64_t)bh * a.N + r;
    const int64_t brow = a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)r * a.bs2 : -1;

    // ---- the row's scores into its mirror ------------------------------------
    auto emit = [&](int j, float v) {
      v = round_dt(v, a.s_dt);
      if (brow >= 0) v = round_dt(v + load_dt(a.bias, brow + (int64_t)j * a.bs3, a.in_dt), a.s_dt);
      if (MODE == kModeTrue) {
        if (a.true_out) a.true_out[grow * T + j] = v;
      } else if (a.pred_out) {
        a.pred_out[grow * T + j] = v;
      }
      g.A[j] = pack_ki(order_key(v), (uint32_t)j);
    };
    if constexpr (MODE == kModeExSign) {
      // pred = sum_b 2^(eq_b + ek_b) (n_b - 2 popc(sq_b ^ sk_b))   (exact)
      uint32_t sq[kMaxNB];
      int eq[kMaxNB];
#pragma unroll
      for (int b = 0; b < kMaxNB; ++b) {
        sq[b] = b < nbd ? ((cu32)(a.qsg + grow * nbd))[b] : 0u;
        eq[b] = b < nbd ? s_exp16(a.qsA, grow * nbd + b) : 0;
      }
      auto keys = [&](auto nbd_c) {
        constexpr int NBD = decltype(nbd_c)::value;
        if (brow >= 0 || a.s_dt != kF32) {
          for (int j = (int)lane; j < T; j += 64) emit(j, expred_score<NBD>(sq, eq, tex + j * NBD, tsg + j * NBD, D));
          return;
        }
        int eqr[NBD], nbk[NBD];
#pragma unroll
        for (int b = 0; b < NBD; ++b) {
          eqr[b] = eq[b] == kExpNaN ? (int)kExpNaN16 : eq[b];
          nbk[b] = min(32, D - 32 * b);
        }
        float* prow = a.pred_out ? a.pred_out + grow * T : nullptr;
        // the common case branch-free (exponent spread <= 23, smallest >= -100: the exact
        // int32 sum, one rounding); rows with any other key (NaN blocks, wide spreads)
        // get a second pass over the flagged keys with the exact fp64 sum
        uint64_t anyslow = 0;
        for (int j = (int)lane; j < T; j += 64) {
          const int16_t* kex = tex + j * NBD;
          const uint32_t* ksg = tsg + j * NBD;
          int e[NBD], m[NBD];
#pragma unroll
          for (int b = 0; b < NBD; ++b) {
            e[b] = eqr[b] + (int)kex[b];
            m[b] = nbk[b] - 2 * (int)__popc(sq[b] ^ ksg[b]);
          }
          int emin = e[0], emax = e[0];
#pragma unroll
          for (int b = 1; b < NBD; ++b) {
            emin = min(emin, e[b]);
            emax = max(emax, e[b]);
          }
          int sum = 0;
#pragma unroll
          for (int b = 0; b < NBD; ++b) sum += m[b] << ((e[b] - emin) & 31);
          const float v = ldexpf((float)sum, emin);
          const uint32_t u = __float_as_uint(v);
          anyslow |= w_ballot(!(emax - emin <= 23 && emin >= -100));
          if (prow) prow[j] = v;
          g.A[j] = pack_ki(u ^ ((uint32_t)((int)u >> 31) | 0x80000000u), (uint32_t)j);
        }
        if (anyslow) {
          for (int j = (int)lane; j < T; j += 64) {
            const int16_t* kex = tex + j * NBD;
            int emin = 1 << 20, emax = -(1 << 20);
#pragma unroll
            for (int b = 0; b < NBD; ++b) {
              emin = min(emin, eqr[b] + (int)kex[b]);
              emax = max(emax, eqr[b] + (int)kex[b]);
            }
            if (!(emax - emin <= 23 && emin >= -100)) {
              const float v = expred_score<NBD>(sq, eq, kex, tsg + j * NBD, D);
              if (prow) prow[j] = v;
              g.A[j] = pack_ki(order_key(v), (uint32_t)j);
            }
          }
        }
      };
      switch (nbd) {
        case 1: keys(std::integral_constant<int, 1>{}); break;
        case 2: keys(std::integral_constant<int, 2>{}); break;
        case 3: keys(std::integral_constant<int, 3>{}); break;
        default: keys(std::integral_constant<int, 4>{}); break;
      }
    } else if constexpr (MODE == kModeElsa) {
      uint32_t hq[kMaxNB];
#pragma unroll
      for (int b = 0; b < kMaxNB; ++b) hq[b] = b < nbd ? ((cu32)(a.qsg + grow * nbd))[b] : 0u;
      const float nrm = a.knorm[kb + r];
      for (int j = (int)lane; j < T; j += 64) {
        int h = 0;
#pragma unroll
        for (int b = 0; b < kMaxNB; ++b)
          if (b < nbd) h += (int)__popc(hq[b] ^ tsg[j * nbd + b]);
        emit(j, nrm * tcs[h]);
      }
    } else {
      const int8_t* qsrc = (MODE == kModeTrue ? a.qc : a.qop) + grow * a.dpad;
      const int16_t* qesrc = MODE == kModeTrue ? a.qsT : a.qsA;
      uint4 qv[2 * kMaxNB];
      uint4 qz[MODE == kModeTrueEx ? 2 * kMaxNB : 1];
      int qe[kMaxNB];
#pragma unroll
      for (int b = 0; b < kMaxNB; ++b) {
        const cu32 qw = (cu32)(qsrc + 32 * b);
        qv[2 * b] = b < nbd ? make_uint4(qw[0], qw[1], qw[2], qw[3]) : make_uint4(0, 0, 0, 0);
        qv[2 * b + 1] = b < nbd ? make_uint4(qw[4], qw[5], qw[6], qw[7]) : make_uint4(0, 0, 0, 0);
        if constexpr (MODE == kModeTrueEx) {
          const cu32 zw = (cu32)(a.qz + grow * a.dpad + 32 * b);
          qz[2 * b] = b < nbd ? make_uint4(zw[0], zw[1], zw[2], zw[3]) : make_uint4(0, 0, 0, 0);
          qz[2 * b + 1] = b < nbd ? make_uint4(zw[4], zw[5], zw[6], zw[7]) : make_uint4(0, 0, 0, 0);
        }
        qe[b] = b < nbd ? s_exp16(qesrc, grow * nbd + b) : 0;
      }
      for (int j = (int)lane; j < T; j += 64) {
        bool nan = false;
        double acc;
        if constexpr (MODE == kModeTrueEx)
          acc = g_dot_trueex(qv, qz, qe, nbd, tcd + (size_t)j * kst, tz + (size_t)j * kst, tex + j * nbd, nan);
        else
          acc = g_dot<MODE == kModeOpMul>(qv, qe, nbd, tcd + (size_t)j * kst, tex + j * nbd, nan);
        float v = nan ? __uint_as_float(0x7FC00000u) : (float)acc;
        if (MODE == kModeTrue) v = round_bfloat(round_dt(v, a.s_dt), a.bfloat, kRoundNearest, 1, a.s_dt) * a.scale;
        emit(j, v);
      }
    }
    if (k <= 0) continue;  // scores only
    wave_lds_sync();

    // ---- torch CPU top-k order ------------------------------------------------
    wave_topk<EW>(g, T, k);

    // ---- kept indices, prune mask ----------------------------------------------
    for (int p = (int)lane; p < k; p += 64) {
      const uint32_t ix = (uint32_t)g.A[p];
      if (a.idx_out) a.idx_out[grow * k + p] = (int64_t)ix;
      a.idx32[grow * k + p] = (int32_t)ix;
    }
    if (a.mask_out) {  // prune mask: zeros.scatter_(-1, idx, 1) as bits
      wl32* mw = (wl32*)g.SL;  // free after the top-k
      if ((int)lane < ntw) mw[lane] = 0u;
      wave_lds_sync();
      for (int p = (int)lane; p < k; p += 64) {
        const uint32_t ix = (uint32_t)g.A[p];
        atomicOr((uint32_t*)(mw + (ix >> 5)), 1u << (ix & 31));
      }
      wave_lds_sync();
      if ((int)lane < ntw) a.mask_out[grow * ntw + lane] = mw[lane];
    }
    wave_lds_sync();
  }
}

// ---- standalone top-k over rows of a float matrix (mxa_topk) ------------------
struct GrpTopkArgs {
  const void* vals;  // dtype dt
  int64_t rows, ld;
  int n, k;
  int64_t* out_idx;
  void* out_vals;  // dtype dt
  uint32_t* out_mask;
  int dt;
};

template <int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NP <= 256 ? 4 : 2, 8))) void topk_grp_kernel(GrpTopkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gi = lane >> 4, gl = lane & 15;
  const int64_t row = ((int64_t)blockIdx.x * 4 + wave) * 4 + gi;
  const bool valid = row < a.rows;
  const int npa = grp_alloc(a.n);
  const GrpRow g = carve_grp(smem + (size_t)(4 * wave + gi) * grp_row_bytes(npa, NP), npa, NP);
  const int64_t src = (valid ? row : 0) * a.ld;
  if (valid)
    for (int j = gl; j < a.n; j += 16) g.A[j] = pack_ki(order_key(load_dt(a.vals, src + j, a.dt)), (uint32_t)j);
  wave_lds_sync();
  grp_topk<NP>(g, a.n, a.k, valid, gl);
  if (valid) {
    for (int p = gl; p < a.k; p += 16) {
      const uint32_t ix = (uint32_t)g.A[p];
      a.out_idx[row * a.k + p] = (int64_t)ix;
      if (a.out_vals) store_dt(a.out_vals, row * a.k + p, load_dt(a.vals, src + ix, a.dt), a.dt);
    }
  }
  if (a.out_mask) {
    const int ntw = (a.n + 31) / 32;
    lu32* mw = g.stk;
    if (gl < ntw) mw[gl] = 0u;
    wave_lds_sync();
    if (valid)
      for (int p = gl; p < a.k; p += 16) {
        const uint32_t ix = (uint32_t)g.A[p];
        atomicOr((uint32_t*)(mw + (ix >> 5)), 1u << (ix & 31));
      }
    wave_lds_sync();
    if (valid)
      for (int w = gl; w < ntw; w += 16) a.out_mask[row * ntw + w] = mw[w];
  }
}

// one wave per row (mxa_topk_wave.hpp): waves of a 256-thread workgroup take rows
// 4 blockIdx.x + wave
template <int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NP <= 256 ? MXA_SELW_OCC : NP <= 512 ? 4 : 2, 8))) void topk_wave_kernel(GrpTopkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = (int)(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + wave;
  if (row >= a.rows) return;
  const WRow g = carve_wrow(smem + (size_t)wave * wrow_bytes(a.n), a.n);
  const int64_t src = row * a.ld;
  for (int j = (int)lane; j < a.n; j += 64) g.A[j] = pack_ki(order_key(load_dt(a.vals, src + j, a.dt)), (uint32_t)j);
  wave_lds_sync();
  wave_topk<NP / 64>(g, a.n, a.k);
  for (int p = (int)lane; p < a.k; p += 64) {
    const uint32_t ix = (uint32_t)g.A[p];
    a.out_idx[row * a.k + p] = (int64_t)ix;
    if (a.out_vals) store_dt(a.out_vals, row * a.k + p, load_dt(a.vals, src + ix, a.dt), a.dt);
  }
  if (a.out_mask) {
    const int ntw = (a.n + 31) / 32;
    wl32* mw = (wl32*)g.SL;
    if ((int)lane < ntw) mw[lane] = 0u;
    wave_lds_sync();
    for (int p = (int)lane; p < a.k; p += 64) {
      const uint32_t ix = (uint32_t)g.A[p];
      atomicOr((uint32_t*)(mw + (ix >> 5)), 1u << (ix & 31));
    }
    wave_lds_sync();
    if ((int)lane < ntw) a.out_mask[row * ntw + lane] = mw[lane];
  }
}

}  // namespace mxa
