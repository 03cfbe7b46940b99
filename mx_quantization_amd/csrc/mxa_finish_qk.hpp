// Finishing kernel of the top-k path with the kept-key scores on int8 MFMA (large k: DiT's
// 154 of 256 keys).  Per wave, tiles of 16 query rows; every product is a
// v_mfma_i32_16x16x32_i8 over one 32-element MX block, so each block keeps its exact int32
// sum for the exact epilogue:
//   1. S^T = K . Q^T for every key of the head, one MFMA per (16 keys, block): A = the
//      head's K codes from LDS, B = the tile's query codes straight from memory.  The K
//      rows are staged in "MFMA order" so that the accumulator of key tile (b, t) holds, in
//      lane (q, g) = (lane % 16, lane / 16), the scores of query q against keys
//      32 b + 8 g + 4 t + i (i = 0..3): over the two tiles of a 32-key block the lane has
//      eight consecutive keys of ONE query row -- a whole row per lane group, no transpose.
//      True score fl32(exact sum) * scale (+ bias) (the rule of true_dot);
//      keys outside the prune mask (the selection's mask words) are dropped (-inf).
//   2. softmax over the kept keys of the row: in-register max / sum, then across the four
//      lane groups by v_permlane16/32_swap (no LDS); MX(P) along keys: the 32-key block
//      maxima the same way, P codes packed eight per lane -- exactly the B operand of
//      3. O^T = V^T . P^T, one MFMA per (16 output columns, key block), A = V^T codes from
//      LDS, epilogue acc += C * (sP[q][b] * sV[b][d]) in fp32 (P.V is a tolerance-only
//      product); the output rows go out from the accumulator layout.
// Against the gather kernels (mxa_finish.hpp / mxa_finish16.hpp), which take the kept keys
// one by one (v_dot4 over LDS rows at random kept indices, LDS atomics for the block
// maxima, an LDS P tile): no gather, no per-wave LDS, no kept-index read (the 8-word mask
// per row instead of k indices), at the price of scoring the dropped keys too -- a win
// once k is a large fraction of T.
// The dense branch (top_k=False, Rows2Args::dense) is this kernel with every key < T kept:
// attn = softmax(true scores) over the whole row, then MX(P) . MX(V) (deit main.py:149-152,
// DiT models.py:218-225).
// Reference: microxscaling/mx/matmul.py:68-76, :85-88 (the MX matmuls QK^T and P.V),
// callers workloads/DiT/models.py:168-225 (gather :194-195), workloads/deit/scripts/main.py:
// 124-152, workloads/PixArt/models/MX_transformer_block.py:679-717.
#pragma once
#include "mxa_finish.hpp"

namespace mxa {

constexpr int kFqRows = 16;  // query rows per tile (one wave)

typedef int v4iq_ __attribute__((ext_vector_type(4)));

// LDS (per workgroup, nothing per wave), strides fixed by the template so that every
// operand read is a base register plus an immediate offset (run-time strides make the
// per-tile addresses loop invariants the compiler hoists into registers):
//   K codes in MFMA order [32 ntb][fq_kst(NB)]   (row stride = 4 (2 NB + 1) dwords: the
//                                                  16 rows of an A read hit distinct banks)
//   K exponents [NB][32 NTB] (int16, key order)
//   V^T codes [32 nb][fq_vst(NTB)] (block b of row d at 32 b; the 16-B pad spreads the 16
//                                  rows of an A read over the banks; rows >= D unused)
//   V block scales as floats [ceil(D / 16)][NTB][16]
//   the exact epilogue's key terms [3][32 NTB] (int32: the key's smallest block exponent,
//   its blocks' offsets from it as bytes, its spread) and per 16-key tile [2][2 NTB]
//   (the tile's smallest exponent and largest spread: the fast-path test)
__host__ __device__ constexpr int fq_kst(int nb) { return 32 * nb + 16; }
__host__ __device__ constexpr int fq_vst(int ntb_max) { return 32 * ntb_max + 16; }
struct FqLds {
  size_t kc, ke, vt, vs, kx, tg, total;
};
__host__ __device__ inline FqLds fq_lds(int ntb, int nb, int ntb_max, int D) {
  FqLds L;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t o = 0;
  L.kc = o;
  o += al((size_t)32 * ntb * fq_kst(nb));
  L.ke = o;
  o += al((size_t)nb * 32 * ntb_max * 2);
  L.vt = o;
  o += al((size_t)32 * nb * fq_vst(ntb_max));
  L.vs = o;
  o += al((size_t)((D + 15) / 16) * ntb_max * 16 * 4);
  L.kx = o;
  o += al((size_t)3 * 32 * ntb_max * 4);
  L.tg = o;
  o += al((size_t)2 * 2 * ntb_max * 4);
  L.total = o;
  return L;
}

// the key held by row p of the MFMA-ordered K table: tile p / 16 = 2 b + t, slot m = p % 16
__device__ __forceinline__ int fq_key_of_row(int p) {
  const int tile = p >> 4, m = p & 15;
  return 32 * (tile >> 1) + 8 * (m >> 2) + 4 * (tile & 1) + (m & 3);
}

// max / sum over the four lane groups of a 16-lane column (lanes q, q+16, q+32, q+48)
__device__ __forceinline__ uint32_t fq_umax4(uint32_t x) {
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  x = max(r[0], r[1]);
  auto s = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return max(s[0], s[1]);
}
__device__ __forceinline__ float fq_fmax4(float x) {
  const uint32_t u = __float_as_uint(x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const uint32_t w = __float_as_uint(x);
  auto s = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return fmaxf(__uint_as_float(s[0]), __uint_as_float(s[1]));
}
__device__ __forceinline__ float fq_fsum4(float x) {
  const uint32_t u = __float_as_uint(x);
  auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const uint32_t w = __float_as_uint(x);
  auto s = __builtin_amdgcn_permlane16_swap(w, w, false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// fl32 of sum_b I_b 2^e_b, exactly rounded (true_dot's rule): the int32 sum shifted to the
// smallest exponent when the exponents span <= 10 bits and the smallest is >= -100, else
// the exact fp64 sum; NaN for a NaN block (an exponent near kExpNaN)
template <int NB>
__device__ __forceinline__ float fq_exact(const int* I, const int* e) {
  int emin = e[0], emax = e[0];
#pragma unroll
  for (int b = 1; b < NB; ++b) {
    emin = min(emin, e[b]);
    emax = max(emax, e[b]);
  }
  if (emax - emin <= 10 && emin >= -100) {
    int sum = 0;
#pragma unroll
    for (int b = 0; b < NB; ++b) sum += I[b] << (e[b] - emin);
    return ldexpf((float)sum, emin);
  }
  if (emin < kExpNaN / 2) return __uint_as_float(0x7FC00000u);
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < NB; ++b) acc += (double)I[b] * pow2d(e[b]);
  return (float)acc;
}

// NB: 32-element blocks per head dim; NTB: key blocks the registers hold (T <= 32 NTB);
// XDT: float16 / bfloat16 inputs or scores (the dtype roundings at run time); EXTRA: a bias,
// the debug true-score output or bfloatX rounding (the bias / output addresses per key are
// loop invariants the compiler would otherwise hoist into 64 register pairs)
template <int NB, int NTB, bool XDT, bool EXTRA>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 8))) void finish_qk_kernel(Rows2Args a) {
  const int sdt = XDT ? a.s_dt : (int)kF32, idt = XDT ? a.in_dt : (int)kF32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = lane & 15, g = lane >> 4;
  const int bh = blockIdx.x;
  constexpr int kst = fq_kst(NB), vst = fq_vst(NTB), kes = 32 * NTB;
  const int T = a.T, D = a.D, ntb = a.ntb, ntw = (a.T + 31) / 32;
  const int tpad = 32 * ntb;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const FqLds L = fq_lds(ntb, NB, NTB, D);
  int8_t* tkc = reinterpret_cast<int8_t*>(smem + L.kc);
  int16_t* tke = reinterpret_cast<int16_t*>(smem + L.ke);
  int8_t* tvt = reinterpret_cast<int8_t*>(smem + L.vt);
  float* tvs = reinterpret_cast<float*>(smem + L.vs);
  int* tkx = reinterpret_cast<int*>(smem + L.kx);
  int* ttg = reinterpret_cast<int*>(smem + L.tg);
  constexpr bool kRound = XDT || EXTRA;  // else the scores / P are plain float32 (bfloat 0 or 32)

  // ---- stage the head's tables ------------------------------------------------------
  const int64_t kb = (int64_t)bh * T;
  {
    constexpr int cpr = 2 * NB;
    for (int i = threadIdx.x; i < tpad * cpr; i += blockDim.x) {
      const int p = i / cpr, c = i - p * cpr;
      const int key = fq_key_of_row(p);
      uint4 x = make_uint4(0, 0, 0, 0);
      if (key < T) x = *reinterpret_cast<const uint4*>(a.kc + (kb + key) * (32 * NB) + 16 * c);
      *reinterpret_cast<uint4*>(tkc + (size_t)p * kst + 16 * c) = x;
    }
    for (int key = threadIdx.x; key < tpad; key += blockDim.x) {
      int e[NB], emin = 1 << 20, emax = -(1 << 20);
      bool nan = false;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const int16_t raw = key < T ? a.ksT[(kb + key) * NB + b] : (int16_t)0;
        tke[b * kes + key] = raw;
        e[b] = exp_from16(raw);
        nan = nan || e[b] == kExpNaN;
        emin = min(emin, e[b]);
        emax = max(emax, e[b]);
      }
      tkx[key] = nan ? -100000 : emin;
      uint32_t dkp = 0u;  // offsets as bytes (the fast form needs them <= 10)
#pragma unroll
      for (int b = 0; b < NB; ++b) dkp |= (uint32_t)min(e[b] - emin, 255) << (8 * b);
      tkx[kes + key] = (int)dkp;
      tkx[2 * kes + key] = nan ? 1000 : emax - emin;
    }
    const int8_t* vsrc = a.vt + (int64_t)bh * D * a.tpad;  // [ntb][D][32] in HBM
    for (int i = threadIdx.x; i < ntb * D * 2; i += blockDim.x) {
      const int half = i & 1, row = i >> 1, tb = row / D, dd = row - tb * D;
      *reinterpret_cast<uint4*>(tvt + (size_t)dd * vst + 32 * tb + 16 * half) =
          *reinterpret_cast<const uint4*>(vsrc + (int64_t)row * 32 + 16 * half);
    }
    const int16_t* vssrc = a.vs + (int64_t)bh * ntb * D;
    for (int i = threadIdx.x; i < ntb * D; i += blockDim.x) {
      const int tb = i / D, dd = i - tb * D;
      tvs[((dd >> 4) * NTB + tb) * 16 + (dd & 15)] = scale_f(exp_from16(vssrc[i]));
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * ntb) {  // per key tile: the smallest exponent, the largest spread
    const int tile = threadIdx.x;
    int mn = 1 << 20, sp = 0;
    for (int m = 0; m < 16; ++m) {
      const int key = 32 * (tile >> 1) + 8 * (m >> 2) + 4 * (tile & 1) + (m & 3);
      mn = min(mn, tkx[key]);
      sp = max(sp, tkx[2 * kes + key]);
    }
    ttg[tile] = mn;
    ttg[2 * NTB + tile] = sp;
  }
  __syncthreads();

  const int r_beg = (int)blockIdx.y * a.rows_per_wg, r_end = min(a.N, r_beg + a.rows_per_wg);
  for (int r0 = r_beg + kFqRows * wave; r0 < r_end; r0 += kFqRows * a.waves) {
    const int r = r0 + q;
    const bool valid = r < r_end;
    const int64_t grow = (int64_t)bh * a.N + (valid ? r : r0);
    const int64_t brow = EXTRA && a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)(valid ? r : r0) * a.bs2 : -1;
    // the tile's query codes (B operand: row q, elements 32 b + 8 g ..) and exponents
    int64_t qb[NB];
    int qe[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      qb[b] = *reinterpret_cast<const int64_t*>(a.qc + grow * (32 * NB) + 32 * b + 8 * g);
      qe[b] = exp_from16(a.qsT[grow * NB + b]);
    }
    // exact epilogue, fast form: sum_b I_b 2^(e_b) = 2^(qmin + kmin) sum_b I_b 2^(dq_b + dk_b),
    // an exact int32 while every shift dq_b + dk_b <= 10 -- the wave's largest query spread
    // plus the key tile's largest spread -- and qmin + kmin >= -100 (no subnormal result):
    // the same float as true_dot's rule (fq_exact), which the tiles that fail it take
    int qmin = qe[0], qmax = qe[0];
    bool qnan = false;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      qmin = min(qmin, qe[b]);
      qmax = max(qmax, qe[b]);
      qnan = qnan || qe[b] == kExpNaN;
    }
    uint32_t dqp = 0u;  // the query's offsets as bytes (<= 10 on the fast form: no carries)
#pragma unroll
    for (int b = 0; b < NB; ++b) dqp |= (uint32_t)min(qe[b] - qmin, 255) << (8 * b);
    const int wq_spread = (int)wave_reduce((uint32_t)(qnan ? 1000 : qmax - qmin),
                                           [](uint32_t x, uint32_t y) { return (int)x > (int)y ? x : y; });
    const int wq_min = (int)wave_reduce((uint32_t)(qnan ? -100000 : qmin),
                                        [](uint32_t x, uint32_t y) { return (int)x < (int)y ? x : y; });
    // the row's kept bits of keys 32 blk + 8 g .. + 7: byte blk % 4 of kw[blk / 4]
    uint32_t kw[(NTB + 3) / 4];
#pragma unroll
    for (int w = 0; w < (NTB + 3) / 4; ++w) kw[w] = 0u;
    if (a.dense) {  // the dense branch: every key < T (wave-uniform)
#pragma unroll
      for (int blk = 0; blk < NTB; ++blk) {
        const int n = min(max(T - (32 * blk + 8 * g), 0), 8);
        if (blk < ntb && valid) kw[blk >> 2] |= ((1u << n) - 1u) << (8 * (blk & 3));
      }
    } else {
#pragma unroll
      for (int blk = 0; blk < NTB; ++blk)
        if (blk < ntb && valid) kw[blk >> 2] |= ((a.mask_out[grow * ntw + blk] >> (8 * g)) & 0xFFu) << (8 * (blk & 3));
    }
    auto kept = [&](int blk, int j) { return (kw[blk >> 2] >> (8 * (blk & 3) + j)) & 1u; };

    // ---- 1. scores of every key; the kept ones enter the softmax ------------------------
    float v[NTB][8];
    float mx = -INFINITY;
#pragma unroll
    for (int blk = 0; blk < NTB; ++blk) {
      if (blk < ntb) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int tile = 2 * blk + t;
          v4iq_ c[NB];
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const int64_t ka = *reinterpret_cast<const int64_t*>(tkc + (size_t)(16 * tile + q) * kst + 32 * b + 8 * g);
            const v4iq_ zero = {0, 0, 0, 0};
            c[b] = __builtin_amdgcn_mfma_i32_16x16x32_i8(ka, qb[b], zero, 0, 0, 0);
          }
          const int key0 = 32 * blk + 8 * g + 4 * t;
          float sc[4];
          const int tkm = __builtin_amdgcn_readfirstlane(ttg[tile]);
          const int tsp = __builtin_amdgcn_readfirstlane(ttg[2 * NTB + tile]);
          if (wq_spread + tsp <= 10 && wq_min + tkm >= -100) {
            const int4 km = *reinterpret_cast<const int4*>(tkx + key0);
            const int4 dk = *reinterpret_cast<const int4*>(tkx + kes + key0);
            auto comp = [](const int4& x, int i) { return i == 0 ? x.x : (i == 1 ? x.y : (i == 2 ? x.z : x.w)); };
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint32_t sh = dqp + (uint32_t)comp(dk, i);  // byte b: the shift of block b
              int sum = 0;
#pragma unroll
              for (int b = 0; b < NB; ++b) sum += c[b][i] << ((sh >> (8 * b)) & 31u);
              sc[i] = ldexpf((float)sum, qmin + comp(km, i));
            }
          } else {
            int ke[NB][4];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
              const uint2 w = *reinterpret_cast<const uint2*>(tke + b * kes + key0);
              ke[b][0] = exp_from16((int16_t)(w.x & 0xFFFFu));
              ke[b][1] = exp_from16((int16_t)(w.x >> 16));
              ke[b][2] = exp_from16((int16_t)(w.y & 0xFFFFu));
              ke[b][3] = exp_from16((int16_t)(w.y >> 16));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              int I[NB], e[NB];
#pragma unroll
              for (int b = 0; b < NB; ++b) {
                I[b] = c[b][i];
                e[b] = qe[b] + ke[b][i];
              }
              sc[i] = fq_exact<NB>(I, e);
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float s = sc[i];
            if (kRound) {
              s = round_bfloat(round_dt(s, sdt), a.bfloat, kRoundNearest, 1, sdt);
              s = round_dt(s * a.scale, sdt);
            } else {
              s = s * a.scale;
            }
            const int key = key0 + i;
            if (EXTRA) {
              if (brow >= 0 && key < T) s = round_dt(s + load_dt(a.bias, brow + (int64_t)key * a.bs3, idt), sdt);
              if (a.true_out && valid && key < T) a.true_out[grow * T + key] = s;
            }
            // a dropped key: -inf (the kept bit as an all-ones / zero mask, one bit select)
            const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)kw[blk >> 2], 8 * (blk & 3) + 4 * t + i, 1);
            uint32_t sv;
            asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(sv) : "v"(m), "v"(__float_as_uint(s)), "v"(0xFF800000u));
            v[blk][4 * t + i] = __uint_as_float(sv);
            mx = fmaxf(mx, v[blk][4 * t + i]);
          }
          // one key tile's MFMAs and epilogue at a time: hoisting the later tiles' MFMAs
          // keeps their accumulators live and spills
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    mx = fq_fmax4(mx);

    // ---- 2. softmax over the kept keys, MX(P) along keys --------------------------------
    // a dropped key holds -inf, so exp(v - mx) = 0 and p = 0 / sum = 0 for it -- except in
    // a row whose max is -inf (every kept score -inf: the kept p are NaN) or whose sum is
    // NaN (a NaN kept score): there the dropped keys are put back to 0 from the mask bits
    // (the kept bits are not reused on the common path: 64 live lane masks would spill)
    // exp(v - mx) as 2^((v - mx) log2 e) on v_exp_f32 (P is a tolerance-only product:
    // SURVEY.md F7; the difference first -- folding mx log2 e into an fma loses the
    // argument for scores of 2^40)
    float sum = 0.0f;
#pragma unroll
    for (int blk = 0; blk < NTB; ++blk)
      if (blk < ntb)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[blk][j] = __builtin_amdgcn_exp2f((v[blk][j] - mx) * 1.4426950408889634f);
          sum += v[blk][j];
        }
    if (__builtin_amdgcn_ballot_w64(mx == -INFINITY)) {  // wave-uniform branch: rare rows only
      if (mx == -INFINITY)
#pragma unroll
      for (int blk = 0; blk < NTB; ++blk)
        if (blk < ntb)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (!kept(blk, j)) v[blk][j] = 0.0f;
      sum = 0.0f;
#pragma unroll
      for (int blk = 0; blk < NTB; ++blk)
        if (blk < ntb)
#pragma unroll
          for (int j = 0; j < 8; ++j) sum += v[blk][j];
    }
    sum = fq_fsum4(sum);
    const bool nan_sum = sum != sum;
    const bool any_nan = __builtin_amdgcn_ballot_w64(nan_sum) != 0;  // wave-uniform: rare rows only
    // p = v / sum correctly rounded without a division per element (Markstein: y = RN(1/sum),
    // q = RN(v y), r = v - q sum exact by fma, RN(q + r y) = RN(v / sum); v in [0, 1],
    // sum in [1, T]: no overflow, and subnormal p only where the block is negligible)
    const float rs = 1.0f / sum;
    // ---- 3. per key block: P codes, then P.V: O^T = V^T . P^T, one MFMA per (16 columns,
    // block); A[m][k] = V^T[dt + m][32 blk + 8 g ..]: m = lane % 16; C[m][n]: m = 4 g + i
    // (column dt + 4 g + i), n = lane % 16 = q.  Block-outer: a block's scores die once its
    // codes are in the accumulators (the blocks still add in key order per column)
    constexpr int NDT = 2 * NB;  // 16-column tiles of D <= 32 NB
    float acc[NDT][4];
#pragma unroll
    for (int u = 0; u < NDT; ++u) acc[u][0] = acc[u][1] = acc[u][2] = acc[u][3] = 0.0f;
#pragma unroll
    for (int blk = 0; blk < NTB; ++blk) {
      if (blk < ntb) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float q0 = v[blk][j] * rs;
          const float q1 = __builtin_fmaf(__builtin_fmaf(-q0, sum, v[blk][j]), rs, q0);
          v[blk][j] = kRound ? round_dt(round_bfloat(q1, a.bfloat, kRoundNearest, 1, sdt), sdt) : q1;
        }
        if (any_nan)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (nan_sum && !kept(blk, j)) v[blk][j] = 0.0f;
        uint32_t bm = 0u;
#pragma unroll
        for (int j = 0; j < 8; ++j) bm = max(bm, __float_as_uint(v[blk][j]) & 0x7FFFFFFFu);
        bm = fq_umax4(bm);
        int e_raw;
        const int es = scale_exponent_dt(bm, 127, sdt, &e_raw);
        const bool fl = a.flush_p && !(e_raw != kExpNaN && e_raw > -127);
        const float sP = scale_f(es == kExpNaN ? kExpNaN : es - 6);
        uint32_t lo = 0u, hi = 0u;
        if (es != kExpNaN) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float x = fl ? v[blk][j] * 0.0f : v[blk][j];
            uint32_t code;
            if (XDT) {
              code = (uint32_t)(int)round_code(x, es, 8, kRoundNearest, sdt) & 0xFFu;
            } else {  // round_code for x >= 0, finite (a NaN block has no codes): floor(x 2^-es 64 + 0.5), <= 127
              const float y = (x * pow2f(-es)) * 64.0f;
              code = (uint32_t)fminf(floorf(y + 0.5f), 127.0f);
            }
            if (j < 4) lo |= code << (8 * j);
            else hi |= code << (8 * (j - 4));
          }
        }
        const int64_t pc = (int64_t)(((uint64_t)hi << 32) | lo);
#pragma unroll
        for (int u = 0; u < NDT; ++u) {
          if (16 * u < D) {
            const int64_t va = *reinterpret_cast<const int64_t*>(tvt + (size_t)(16 * u + q) * vst + 32 * blk + 8 * g);
            const v4iq_ zero = {0, 0, 0, 0};
            const v4iq_ c = __builtin_amdgcn_mfma_i32_16x16x32_i8(va, pc, zero, 0, 0, 0);
            const float4 sv = *reinterpret_cast<const float4*>(tvs + (u * NTB + blk) * 16 + 4 * g);
            acc[u][0] = fmaf((float)c[0], sP * sv.x, acc[u][0]);
            acc[u][1] = fmaf((float)c[1], sP * sv.y, acc[u][1]);
            acc[u][2] = fmaf((float)c[2], sP * sv.z, acc[u][2]);
            acc[u][3] = fmaf((float)c[3], sP * sv.w, acc[u][3]);
          }
        }
      }
    }
    // ---- 4. the tile's output rows --------------------------------------------------------
    if (valid) {
      const int64_t ob = b_ * a.os0 + h_ * a.os1 + (int64_t)r * a.os2;
#pragma unroll
      for (int u = 0; u < NDT; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int dd = 16 * u + 4 * g + i;
          if (dd < D) store_dt(a.out, ob + dd, round_bfloat(round_dt(acc[u][i], sdt), a.bfloat, kRoundNearest, 1, sdt), sdt);
        }
    }
  }
}

}  // namespace mxa
