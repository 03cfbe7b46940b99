// Selection kernels: approximate scores + exact-order top-k.
//
// Per workgroup (one head, a chunk of its query rows): the head's score tables are
// staged in LDS once (sel_lds / sel_stage):
//   ex_pred        sign words + block exponents
//   MXINT4 / EXION / partial_*   approximator codes + block scales
//   true_ex        power-of-two codes + zero indicators + block exponents
//   ELSA           hash words + the (D+1)-entry cosine table
//   approx off     MXINT8 codes + exponents (the true scores are ranked)
// then per row (sel_scores): the scores (exact fp64 block epilogue where needed: the
// scores are exact sums of integer * 2^e), bias added in fp32 as the caller
// does; torch's CPU topk index order; the k kept indices (the op's int64 idx, which the
// finishing kernel reads too, or a 16-bit workspace copy: kept_put), and the prune-mask
// words when asked for.
//   select_kernel<..., uint32_t>  rows of <= 256 keys whose scores pack into 32-bit
//                     elements (mxa_topk_grp.hpp GEl), then
//   select_kernel<..., uint64_t>  the rows that do not (fb_only), and every row of the true
//                     scores, ELSA and rows over 256 keys
// k_top == 0: scores only (mxa_approx_scores).
// Callers replaced: the approximator + torch.topk of
//   workloads/deit/scripts/main.py:101-123, workloads/DiT/models.py:168-194,
//   workloads/PixArt/models/MX_transformer_block.py:656-678, :805-825.
#pragma once
#include <type_traits>
#include "mxa_dot.hpp"
#include "mxa_rows2.hpp"
#include "mxa_topk_grp.hpp"
#include "mxa_tail.hpp"
#include "mxa_topk_wave.hpp"

namespace mxa {

constexpr int kSelRows = 32;   // query rows per workgroup (a multiple of 4 * waves)
// packed-pass workgroup flags per 64-bit-pass workgroup: few, so that a call whose rows mostly
// do not pack still spreads the 64-bit pass over the chip (64 per workgroup ran arbitrary float32
// rows through ops.topk at half the rate of the 64-bit pass alone: 1.60 vs 0.80 ms, round 6)
constexpr int kFbItems = 4;
// waves per SIMD the 64-bit pass is compiled for (rows <= 256 keys; 6 / 8 measured slower at
// PixArt's rows: spills, profiles/r06_ab_tail.txt)
constexpr int kSelOcc = 4;
// ... and the packed pass, with the tail (DeiT: 6 measured slower, spills) and without it
// (k > 33, DiT: 4 removes its spills and measured slower) -- profiles/r06_ab_tail.txt
constexpr int kSelPOcc = 5;
constexpr int kSelPOccNT = 5;
constexpr int kSelShortT = 224;
// waves per workgroup: 2 for rows of <= 224 keys on a large grid (DeiT-base: 0.97 ->
// 0.93 ms), else 4 (DiT: 1.44 vs 1.56 ms with 2; PixArt's 128 heads: 0.069 vs 0.10 ms)
// -- measured, tools/bench_cmp.sh
inline int sel_waves_for(int T, int64_t BH, int N) {
  return T <= kSelShortT && BH * ((N + kSelRows - 1) / kSelRows) >= 8192 ? 2 : 4;
}

// LDS layout of the score tables (then the per-row top-k areas)
struct SelLds {
  size_t cd, ex, sg, z, cs, kf, rows;
};
// ex_pred's key exponents go to LDS as int32 for nbd <= 2 (raw int16 values sign-extended:
// no extraction in the key loop; for nbd >= 3 int16, which keeps DiT's workgroups per CU),
// with 16 flag words kf: bit i of kf[g] = key g + 16 i has a
// block exponent outside [kExpFastLo, kExpFastHi] (or NaN), i.e. its score may need the
// exact slow path (sel_scores)
constexpr int kExpFastLo = -50, kExpFastHi = 61;
__host__ __device__ inline SelLds sel_lds(int mode, int T, int D, int kst, int nbd) {
  SelLds L;
  size_t o = 0;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const bool codes = mode == kModeTrue || mode == kModeOpExp || mode == kModeOpMul || mode == kModeTrueEx;
  L.cd = o;
  if (codes) o += al((size_t)T * kst);
  L.ex = o;
  if (mode != kModeElsa) o += al((size_t)T * nbd * (mode == kModeExSign && nbd <= 2 ? 4 : 2));
  L.sg = o;
  if (mode == kModeExSign || mode == kModeElsa) o += al((size_t)T * nbd * 4);
  L.z = o;
  if (mode == kModeTrueEx) o += al((size_t)T * kst);
  L.cs = o;
  if (mode == kModeElsa) o += al((size_t)(D + 1) * 4);
  L.kf = o;
  if (mode == kModeExSign) o += 16 * 4;
  L.rows = o;
  return L;
}

// ex_pred score of one key: sum_b m_b 2^(eq_b + ek_b), m_b = n_b - 2 popc(sq_b ^ sk_b)
// (|m_b| <= 32).  When the block exponents span <= 23 bits and the smallest is >= -100,
// the sum shifted to the smallest exponent is an exact int32, so one conversion (round
// to nearest even) and an exact scaling give the correctly rounded float; otherwise
// (and for NaN blocks) the exact fp64 sum.  Both equal fl32 of the exact sum.
template <int NBD, typename KE>
__device__ __forceinline__ float expred_score(const uint32_t* sq, const int* eq, const KE* kex, const uint32_t* ksg,
                                              int D) {
  int m[NBD], e[NBD];
  bool nan = false;
  int emin = 1 << 20, emax = -(1 << 20);
#pragma unroll
  for (int b = 0; b < NBD; ++b) {
    const int ek = exp_from16((int16_t)kex[b]);
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

// ---- the head's score tables in LDS (sel_lds) -------------------------------------
struct SelTabs {
  int8_t* tcd;    // key codes
  int16_t* tex;   // key exponents (ex_pred: tex32)
  int* tex32;
  uint32_t* kf;   // ex_pred: the keys outside the fast path's exponent range (SelLds)
  uint32_t* tsg;  // sign / hash words
  int8_t* tz;     // true_ex zero indicators
  float* tcs;     // ELSA cosine table
};
template <int MODE>
__device__ __forceinline__ SelTabs sel_stage(const Rows2Args& a, unsigned char* smem, const SelLds& L, int bh) {
  constexpr bool kOp = MODE == kModeOpExp || MODE == kModeOpMul;
  SelTabs t;
  t.tcd = reinterpret_cast<int8_t*>(smem + L.cd);
  t.tex = reinterpret_cast<int16_t*>(smem + L.ex);
  t.tsg = reinterpret_cast<uint32_t*>(smem + L.sg);
  t.tz = reinterpret_cast<int8_t*>(smem + L.z);
  t.tcs = reinterpret_cast<float*>(smem + L.cs);
  t.tex32 = reinterpret_cast<int*>(smem + L.ex);
  t.kf = reinterpret_cast<uint32_t*>(smem + L.kf);
  const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst;
  if (MODE == kModeExSign && nbd <= 2) {  // (the range flags serve the nbd <= 2 key loop)
    if (threadIdx.x < 16) t.kf[threadIdx.x] = 0u;
    __syncthreads();
  }
  const int64_t kb = (int64_t)bh * T;
  if constexpr (MODE == kModeTrue || kOp || MODE == kModeTrueEx) {
    const int8_t* src = MODE == kModeTrue ? a.kc : a.kop;
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(t.tcd + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(src + (kb + j) * a.dpad + 16 * c);
      if (MODE == kModeTrueEx)
        *reinterpret_cast<uint4*>(t.tz + (size_t)j * kst + 16 * c) =
            *reinterpret_cast<const uint4*>(a.kz + (kb + j) * a.dpad + 16 * c);
    }
  }
  {
    const int16_t* esrc = MODE == kModeTrue ? a.ksT : a.ksA;
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) {
      if (MODE == kModeExSign) {
        const int ek = esrc[kb * nbd + i];  // raw (NaN: INT16_MIN, outside the range)
        if (nbd <= 2) {
          t.tex32[i] = ek;
          if (ek < kExpFastLo || ek > kExpFastHi) {
            const int j = i / nbd;
            atomicOr(t.kf + (j & 15), 1u << (j >> 4));
          }
        } else {
          t.tex[i] = (int16_t)ek;
        }
      } else if (MODE != kModeElsa) {
        t.tex[i] = esrc[kb * nbd + i];
      }
      if (MODE == kModeExSign || MODE == kModeElsa) t.tsg[i] = a.ksg[kb * nbd + i];
    }
    if (MODE == kModeElsa)
      for (int h = threadIdx.x; h <= D; h += blockDim.x) t.tcs[h] = a.elsa_cos ? a.elsa_cos[h] : elsa_cos_entry(D, h);
  }
  __syncthreads();
  return t;
}

// ---- the approximate (or true) scores of query row r: keys j0, j0 + js, ... -------------
// sink(j, v, key, fast): v the score as the caller ranks it (score dtype, + bias), key its order
// key, fast (std::true_type) when v came from the fast ex_pred loop (finite, never -0)
// pred_out / true_out are written here.
template <int MODE, typename Sink>
__device__ __forceinline__ void sel_scores(const Rows2Args& a, const SelTabs& t, int bh, int r, int j0, int js,
                                           Sink&& sink) {
  const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const int64_t kb = (int64_t)bh * T;
  const int64_t grow = (int64_t)bh * a.N + r;
  const int64_t brow = a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)r * a.bs2 : -1;
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
    sink(j, v, order_key(v), std::false_type{});
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
      if (brow >= 0 || a.s_dt != kF32 || js != 16) {
        if constexpr (NBD <= 2)
          for (int j = j0; j < T; j += js) emit(j, expred_score<NBD>(sq, eq, t.tex32 + j * NBD, t.tsg + j * NBD, D));
        else
          for (int j = j0; j < T; j += js) emit(j, expred_score<NBD>(sq, eq, t.tex + j * NBD, t.tsg + j * NBD, D));
        return;
      }
      if constexpr (NBD >= 3) {
        // the bias-free key loop on raw int16 exponents (NaN = INT16_MIN drives the smallest
        // exponent below -100): a fast-path value (finite, never -0) takes the
        // three-instruction key.  (The branch-free loop below measured slower at DiT's three
        // blocks: its extra live values spill.)
        int eqr[NBD], nbk[NBD];
#pragma unroll
        for (int b = 0; b < NBD; ++b) {
          eqr[b] = eq[b] == kExpNaN ? (int)kExpNaN16 : eq[b];
          nbk[b] = min(32, D - 32 * b);
        }
        float* prow = a.pred_out ? a.pred_out + grow * T : nullptr;
        for (int j = j0; j < T; j += js) {
          const int16_t* kex = t.tex + j * NBD;
          const uint32_t* ksg = t.tsg + j * NBD;
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
          sink(j, v, key, std::false_type{});
        }
        return;
      }
      // No bias, float32 scores: every lane runs the same ceil(T / 16) keys (the last trip
      // peeled: keys >= T are dropped), with no branch in the loop.  When every block
      // exponent of the row and of the key lies in [kExpFastLo, kExpFastHi], the block
      // terms m_b 2^(eq_b + ek_b) are exact floats (|m_b| <= 32, 2^-100 <= 2^e <= 2^122):
      // v = x0 + x1, one IEEE addition of two exact terms = fl32(exact sum) (NBD <= 2).
      // Keys outside (range flags kf, a NaN block) are redone afterwards by
      // the exact expred_score, under a wave-uniform branch.  A fast value is finite and
      // never -0, so its order key takes two instructions and its packing test is the low
      // byte of its bits.
      int nbk[NBD];
      bool row_fast = true;
#pragma unroll
      for (int b = 0; b < NBD; ++b) {
        nbk[b] = min(32, D - 32 * b);
        row_fast = row_fast && eq[b] >= kExpFastLo && eq[b] <= kExpFastHi;  // (NaN: kExpNaN)
      }
      float* prow = a.pred_out ? a.pred_out + grow * T : nullptr;
      const int nt = (T + 15) >> 4;
      uint32_t redo = row_fast ? t.kf[j0 & 15] : lowbits(nt);  // per trip i: key j0 + 16 i
      auto one = [&](int i, auto last_c) {
        constexpr bool LAST = decltype(last_c)::value;
        const int j = j0 + 16 * i;
        const int* kex = t.tex32 + j * NBD;
        const uint32_t* ksg = t.tsg + j * NBD;
        float v = ldexpf((float)(nbk[0] - 2 * (int)__popc(sq[0] ^ ksg[0])), eq[0] + kex[0]);
        if constexpr (NBD == 2) v += ldexpf((float)(nbk[1] - 2 * (int)__popc(sq[1] ^ ksg[1])), eq[1] + kex[1]);
        const uint32_t u = __float_as_uint(v);
        const uint32_t key = u ^ ((uint32_t)((int)u >> 31) | 0x80000000u);
        if (!LAST || j < T) {
          if (prow) prow[j] = v;
          sink(j, v, key, std::true_type{});
        }
      };
#pragma unroll 1  // (unrolled by 2 / 4: the same within the spread, profiles/r06_ab_tail.txt)
      for (int i = 0; i < nt - 1; ++i) one(i, std::false_type{});
      one(nt - 1, std::true_type{});
      if (__builtin_amdgcn_ballot_w64(redo != 0u) != 0) {  // rare: the exact path for those keys
        while (redo) {
          const int i = __ffs((int)redo) - 1;
          redo &= redo - 1u;
          const int j = j0 + 16 * i;
          if (j < T) {
            const float v = expred_score<NBD>(sq, eq, t.tex32 + j * NBD, t.tsg + j * NBD, D);
            if (prow) prow[j] = v;
            sink(j, v, order_key(v), std::false_type{});
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
    // approx = ||MX_K[row r]|| * cos(clamp(pi/D * hamming - 0.127, 0))
    // (elsa_approximation.py:124-143; the key norm of row r, the reference's broadcast)
    uint32_t hq[kMaxNB];
#pragma unroll
    for (int b = 0; b < kMaxNB; ++b) hq[b] = b < nbd ? a.qsg[grow * nbd + b] : 0u;
    const float nrm = a.knorm[kb + r];
    for (int j = j0; j < T; j += js) {
      int h = 0;
#pragma unroll
      for (int b = 0; b < kMaxNB; ++b)
        if (b < nbd) h += (int)__popc(hq[b] ^ t.tsg[j * nbd + b]);
      emit(j, nrm * t.tcs[h]);
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
    for (int j = j0; j < T; j += js) {
      bool nan = false;
      double acc;
      if constexpr (MODE == kModeTrueEx)
        acc = g_dot_trueex(qv, qz, qe, nbd, t.tcd + (size_t)j * kst, t.tz + (size_t)j * kst, t.tex + j * nbd, nan);
      else
        acc = g_dot<MODE == kModeOpMul>(qv, qe, nbd, t.tcd + (size_t)j * kst, t.tex + j * nbd, nan);
      float v = nan ? __uint_as_float(0x7FC00000u) : (float)acc;
      // true = quantize_elemwise(fl32(QK^T)) * scale   (matmul.py:88-91, caller)
      if (MODE == kModeTrue) v = round_bfloat(round_dt(v, a.s_dt), a.bfloat, kRoundNearest, 1, a.s_dt) * a.scale;
      emit(j, v);
    }
  }
}

// prune mask words of one row from its kept indices (zeros.scatter_(-1, idx, 1) as bits):
// idx_at(p) for p = p0, p0 + ps, ... < k; mw is a per-row LDS scratch of ntw words
template <typename IdxAt>
__device__ __forceinline__ void sel_mask_words(const Rows2Args& a, __attribute__((address_space(3))) uint32_t* mw,
                                               int64_t grow, bool valid, int p0, int ps, int k, IdxAt&& idx_at) {
  const int ntw = (a.T + 31) / 32;
  for (int w = p0; w < ntw; w += ps) mw[w] = 0u;
  wave_lds_sync();
  if (valid)
    for (int p = p0; p < k; p += ps) {
      const uint32_t ix = idx_at(p);
      atomicOr((uint32_t*)(mw + (ix >> 5)), 1u << (ix & 31));
    }
  wave_lds_sync();
  if (valid)
    for (int w = p0; w < ntw; w += ps) a.mask_out[grow * ntw + w] = mw[w];
}

// ---- four query rows per wave (mxa_topk_grp.hpp) ---------------------------------
// rows rq + (lane >> 4) of head bh; g0 = the wave's per-row areas (grp_row_bytes each).
// El = uint64_t: any row (a.fb_only: only the rows the packed pass left, kept_get(row * k) < 0).
// El = uint32_t (packed): a row whose scores do not all leave the key's low byte free is
// left for the 64-bit pass: its first kept index is -1 (kept_put).
// TW > 0 (packed): rows whose remaining work fits a TW-position prefix go to the one-lane
// tail kernel (mxa_tail.hpp): their state and prefix are written to a.tail_rec (and the
// first kept index set to 0, so the 64-bit pass leaves them alone); it writes their
// indices and mask words.
// Returns (per lane) whether this lane's row was left for the 64-bit pass.
template <int NP, int MODE, typename El, int QM, int TW = 0>
__device__ __forceinline__ bool sel_rows4(const Rows2Args& a, const SelTabs& t, unsigned char* g0, int bh, int rq,
                                          int r_end, int lane) {
  constexpr bool kPacked = sizeof(El) == 4;
  const int gi = lane >> 4, gl = lane & 15;
  const int T = a.T, k = a.k_top;
  const int npa = grp_alloc(T);
  const GrpRow<El> g = carve_grp<El>(g0 + (size_t)gi * grp_row_bytes(npa, NP, sizeof(El)), npa, NP);
  const int r = rq + gi;
  bool valid = r < r_end;
  const int64_t grow = (int64_t)bh * a.N + (valid ? r : rq);
  if (!kPacked && a.fb_only && valid) valid = kept_get(a, grow * k) < 0;
  uint32_t bad = 0u, badf = 0u;
#ifdef MXA_SEL_SKIP
  if (valid && !((MXA_SEL_SKIP) & 2))
#else
  if (valid)
#endif
  {
    if constexpr (kPacked)
      sel_scores<MODE>(a, t, bh, r, gl, 16, [&](int j, float v, uint32_t key, auto fast_c) {
        if constexpr (decltype(fast_c)::value) badf |= __float_as_uint(v);  // finite: the low byte
        else bad |= q_bad_bits(v);
        g.A[j] = qelem(key, (uint32_t)j);
      });
    else
      sel_scores<MODE>(a, t, bh, r, gl, 16, [&](int j, float, uint32_t key, auto) { g.A[j] = pack_ki(key, (uint32_t)j); });
  }
  bad |= badf & 0xFFu;
#ifdef MXA_SEL_SKIP  // tools-only phase timing (build_native defines): 2 = scores replaced by hashed keys
  if ((MXA_SEL_SKIP) & 2)
    for (int j = gl; j < T; j += 16) {
      const uint32_t key = 0x80000000u | ((uint32_t)(j * 2654435761u + r * 40503u) >> 26 << 8);
      if constexpr (kPacked) g.A[j] = qelem(key, (uint32_t)j);
      else g.A[j] = pack_ki(key, (uint32_t)j);
    }
#endif
  if (k <= 0) return false;  // scores only
  bool left = false;
  if constexpr (kPacked) {  // this row's 16 lanes: any score that does not pack
    const uint64_t bw = __builtin_amdgcn_ballot_w64(bad != 0u);
    if (valid && ((bw >> (16 * gi)) & 0xFFFFull) != 0) {
      if (gl == 0) kept_put(a, grow * k, -1);
      valid = false;
      left = true;
    }
  }
  wave_lds_sync();
  GrpHand hand{0u, false};
#ifdef MXA_SEL_SKIP  // 1 = no top-k
  if (!((MXA_SEL_SKIP) & 1))
#endif
    grp_topk<NP, El, QM, TW>(g, T, k, valid, gl, &hand);
  if (TW > 0 && hand.on) {  // the row's state and prefix to the tail kernel
    uint32_t* rec = a.tail_rec + grow * tail_rec_words(TW);
    if (gl == 0) {
      rec[0] = hand.state | kTailPending;
      kept_put(a, grow * k, 0);
    }
    for (int p = gl; p < TW; p += 16) rec[4 + p] = (uint32_t)g.A[p];  // (the tail reads [0, tail_rec_len))
    valid = false;
  } else if (TW > 0 && r < r_end) {  // finished here, or left for the 64-bit pass: not the tail's
    if (gl == 0) a.tail_rec[grow * tail_rec_words(TW)] = 0u;
  }
  // kept indices: four consecutive rows per wave
  if (valid) {
    for (int p = gl; p < k; p += 16) {
      kept_put(a, grow * k + p, (int)GEl<El>::idx(g.A[p]));
    }
  }
  if (a.mask_out) sel_mask_words(a, g.stk, grow, valid, gl, 16, k, [&](int p) { return GEl<El>::idx(g.A[p]); });
  wave_lds_sync();
  return left;
}

// One workgroup's work item: head bh, query-row chunk y (rows y * rows_per_wg ...).
// Returns (on every thread) whether a packed row of the chunk was left for the 64-bit pass.
template <int NP, int MODE, int kSelWaves, typename El, int QM, int TW>
__device__ __forceinline__ bool select_item(const Rows2Args& a, unsigned char* smem, int bh, int y) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = y * a.rows_per_wg, r_end = min(a.N, r0 + a.rows_per_wg);
  const SelLds L = sel_lds(MODE, a.T, a.D, a.kst, a.nbd);
  const SelTabs t = sel_stage<MODE>(a, smem, L, bh);
  unsigned char* g0 = smem + L.rows + (size_t)4 * wave * grp_row_bytes(grp_alloc(a.T), NP, sizeof(El));
  // (packed) whether a row this thread's wave handled was left for the 64-bit pass: tracked
  // per thread, not read back from idx -- other waves' kept_put(-1) need not be visible yet
  bool left = false;
  for (int rq = r0 + 4 * wave; rq < r_end; rq += 4 * kSelWaves) {
    if (sizeof(El) == 8 && a.fb_only) {  // the rows of this group that are left
      const int r = min(rq + (lane >> 4), r_end - 1);
      if (__builtin_amdgcn_ballot_w64(rq + (lane >> 4) < r_end && kept_get(a, ((int64_t)bh * a.N + r) * a.k_top) < 0) == 0)
        continue;
    }
    left |= sel_rows4<NP, MODE, El, QM, TW>(a, t, g0, bh, rq, r_end, lane);
  }
  return __syncthreads_or(left ? 1 : 0) != 0;
}

// Selection kernel, four query rows per wave.  El = uint64_t: rows of up to 512 keys,
// every approximator.  El = uint32_t: the packed pass (rows of <= 256 keys; half the LDS
// per row, so more resident waves); each workgroup flags (a.fb_flags[bh * gy + y]) whether
// it left rows for the 64-bit pass, which then runs with fb_only: one workgroup per kFbItems
// flags, taking the flagged items one after another (a call without such rows costs a
// small grid that exits at once).
template <int NP, int MODE, int kSelWaves, typename El = uint64_t, int QM = 0, int TW = 0>
__global__ __launch_bounds__(64 * kSelWaves) __attribute__((amdgpu_waves_per_eu(sizeof(El) == 4 ? (TW > 0 ? kSelPOcc : kSelPOccNT) : NP <= 256 ? kSelOcc : 2, 8))) void select_kernel(Rows2Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (sizeof(El) == 8 && a.fb_only) {
    __shared__ uint64_t sbits;
    const int gy = a.fb_gy;
    const int64_t items = (int64_t)a.B * a.H * gy, i0 = (int64_t)blockIdx.x * kFbItems;
    if (threadIdx.x < kFbItems) {
      const bool f = i0 + threadIdx.x < items && a.fb_flags[i0 + threadIdx.x] != 0u;
      const uint64_t bits = __builtin_amdgcn_ballot_w64(f);
      if (threadIdx.x == 0) sbits = bits;
    }
    __syncthreads();
    uint64_t bits = sbits;
    while (bits) {
      const int i = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      const int64_t item = i0 + i;
      select_item<NP, MODE, kSelWaves, El, QM, TW>(a, smem, (int)(item / gy), (int)(item % gy));
      __syncthreads();  // the next item re-stages the tables
    }
    return;
  }
  const bool left = select_item<NP, MODE, kSelWaves, El, QM, TW>(a, smem, blockIdx.x, blockIdx.y);
  if (sizeof(El) == 4 && a.fb_flags && threadIdx.x == 0) a.fb_flags[(int64_t)blockIdx.x * gridDim.y + blockIdx.y] = left ? 1u : 0u;
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

// the standalone top-k's workspace path (mxa_topk_ws): the packed pass's tail records and
// per-workgroup flags
struct TopkWs {
  uint32_t* tail_rec;  // [rows][tail_rec_words(TW)] (TW > 0)
  uint32_t* fb_flags;  // per packed workgroup: rows left for the 64-bit pass
  int64_t n_wg;        // packed workgroups (fb pass: flags to read)
  int fb_only;         // 64-bit pass over the flagged workgroups' rows with out_idx[row * k] < 0
};

// sixteen rows (four per wave) from row0: El = uint64_t any row (fb: only rows whose first
// index is -1); El = uint32_t the packed pass (a row whose values do not leave the key's low
// byte free gets first index -1 and is left for the 64-bit pass; TW > 0: rows whose remaining
// work fits the tail's prefix are handed to topk_tail_kernel).  Returns (on every thread)
// whether a row was left.
template <int NP, typename El, int QM, int TW>
__device__ __forceinline__ bool topk_rows16(const GrpTopkArgs& a, const TopkWs& w, unsigned char* smem, int64_t row0,
                                            bool fb) {
  constexpr bool kPacked = sizeof(El) == 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gi = lane >> 4, gl = lane & 15;
  const int64_t row = row0 + 4 * wave + gi;
  bool valid = row < a.rows;
  if (fb && valid) valid = a.out_idx[row * a.k] < 0;
  const int npa = grp_alloc(a.n);
  const GrpRow<El> g = carve_grp<El>(smem + (size_t)(4 * wave + gi) * grp_row_bytes(npa, NP, sizeof(El)), npa, NP);
  const int64_t src = (valid ? row : 0) * a.ld;
  uint32_t bad = 0u;
  // the row's values, 256 (64-bit elements: 128) at a time: every load of a chunk issued before
  // the first is used (one load at a time left each wave waiting out a memory round trip per 16
  // values)
  constexpr int kChunk = NP < (kPacked ? 256 : 128) ? NP : (kPacked ? 256 : 128);
  for (int c0 = 0; c0 < NP; c0 += kChunk) {
    float vv[kChunk / 16];
#pragma unroll
    for (int t = 0; t < kChunk / 16; ++t) {
      const int j = c0 + gl + 16 * t;
      vv[t] = valid && j < a.n ? load_dt(a.vals, src + j, a.dt) : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < kChunk / 16; ++t) {
      const int j = c0 + gl + 16 * t;
      if (!valid || j >= a.n) continue;
      const float v = vv[t];
      if constexpr (kPacked) {
        bad |= q_bad_bits(v);
        if (a.out_vals) bad |= q_val_bad(v);  // the tail rebuilds the values from the elements
        g.A[j] = qelem(order_key(v), (uint32_t)j);
      } else {
        g.A[j] = pack_ki(order_key(v), (uint32_t)j);
      }
    }
  }
  bool left = false;
  if constexpr (kPacked) {
    const uint64_t bw = __builtin_amdgcn_ballot_w64(bad != 0u);
    if (valid && ((bw >> (16 * gi)) & 0xFFFFull) != 0) {
      if (gl == 0) a.out_idx[row * a.k] = -1;
      valid = false;
      left = true;
    }
  }
  wave_lds_sync();
  GrpHand hand{0u, false};
  grp_topk<NP, El, QM, TW>(g, a.n, a.k, valid, gl, &hand);
  if (TW > 0 && hand.on) {  // the row's state and prefix to the tail kernel
    uint32_t* rec = w.tail_rec + row * tail_rec_words(TW);
    if (gl == 0) {
      rec[0] = hand.state | kTailPending;
      a.out_idx[row * a.k] = 0;
    }
    for (int p = gl; p < TW; p += 16) rec[4 + p] = (uint32_t)g.A[p];
    valid = false;
  } else if (TW > 0 && row < a.rows && !fb) {  // not the tail's
    if (gl == 0) w.tail_rec[row * tail_rec_words(TW)] = 0u;
  }
  if (valid) {
    for (int p = gl; p < a.k; p += 16) {
      const uint32_t ix = GEl<El>::idx(g.A[p]);
      a.out_idx[row * a.k + p] = (int64_t)ix;
      if (a.out_vals) store_dt(a.out_vals, row * a.k + p, load_dt(a.vals, src + ix, a.dt), a.dt);
    }
  }
  if (a.out_mask) {
    const int ntw = (a.n + 31) / 32;
    lu32* mw = g.stk;
    for (int i = gl; i < ntw; i += 16) mw[i] = 0u;
    wave_lds_sync();
    if (valid)
      for (int p = gl; p < a.k; p += 16) {
        const uint32_t ix = GEl<El>::idx(g.A[p]);
        atomicOr((uint32_t*)(mw + (ix >> 5)), 1u << (ix & 31));
      }
    wave_lds_sync();
    if (valid)
      for (int i = gl; i < ntw; i += 16) a.out_mask[row * ntw + i] = mw[i];
  }
  wave_lds_sync();
  return __syncthreads_or(left ? 1 : 0) != 0;
}

// El = uint64_t: every row (w.fb_only: one workgroup per kFbItems flags of the packed pass, taking
// the flagged workgroups' left rows); El = uint32_t: the packed pass, flagging per workgroup
template <int NP, typename El = uint64_t, int QM = 0, int TW = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sizeof(El) == 4 ? 5 : NP <= 256 ? 4 : 2, 8))) void topk_grp_kernel(GrpTopkArgs a, TopkWs w) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (sizeof(El) == 8 && w.fb_only) {
    __shared__ uint64_t sbits;
    const int64_t i0 = (int64_t)blockIdx.x * kFbItems;
    if (threadIdx.x < kFbItems) {
      const bool f = i0 + threadIdx.x < w.n_wg && w.fb_flags[i0 + threadIdx.x] != 0u;
      const uint64_t bits = __builtin_amdgcn_ballot_w64(f);
      if (threadIdx.x == 0) sbits = bits;
    }
    __syncthreads();
    uint64_t bits = sbits;
    while (bits) {
      const int i = __ffsll((long long)bits) - 1;
      bits &= bits - 1;
      topk_rows16<NP, El, QM, TW>(a, w, smem, (i0 + i) * 16, true);
    }
    return;
  }
  const bool left = topk_rows16<NP, El, QM, TW>(a, w, smem, (int64_t)blockIdx.x * 16, false);
  if (sizeof(El) == 4 && threadIdx.x == 0) w.fb_flags[blockIdx.x] = left ? 1u : 0u;
}

// one wave per row (mxa_topk_wave.hpp): waves of a 256-thread workgroup take rows
// 4 blockIdx.x + wave
template <int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NP <= 256 ? 8 : NP <= 512 ? 4 : 2, 8))) void topk_wave_kernel(GrpTopkArgs a) {
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
