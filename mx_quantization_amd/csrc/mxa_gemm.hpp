// Block-scaled MX GEMM on int8 MFMA: C[b] = MX(A[b], along K) @ MX(B[b], along K)^T,
// each product rounded once from its exact value.
//
// Serves the two plain GEMMs around the attention core that the patched modules run
// through the reference's mx ops:
//   mx.matmul   microxscaling/mx/matmul.py:31-100 (the drop-in's QK^T and P.V,
//               workloads/deit/scripts/main.py:101, :152)
//   mx.Linear   microxscaling/mx/linear.py:20-103 (the proj Linear behind the attention,
//               deit main.py:154, DiT models.py:227; the drop-in's every Linear)
// Operands are what the prep kernels write: codes int8 row-major along K (A: [M][lda],
// B^T: [Nc][ldb]) and a code unit's exponent per 32-element block (value = code * 2^e,
// -32768 = a NaN block).
//
// Workgroup: 64 rows x 128 columns, four waves of 32 rows x 64 columns -- two
// independent 32x32 accumulator chains per wave sharing the A operand.  Operands go
// straight from global memory into the MFMA registers (the lane maps of
// v_mfma_i32_32x32x32_i8 read 16 contiguous bytes of one row: no LDS staging), loaded two
// K-blocks ahead.  K = 32 = one MX block per MFMA, so every block keeps its exact int32
// sum; the block's scale 2^(ea + eb) is applied as a shift of that sum relative to the
// row's and the column's smallest block exponent (exponent offsets staged in LDS), and the
// int32 total converts once: the correctly rounded exact product.  A wave whose rows' and
// columns' exponent spreads could overflow int32 (or whose result could be subnormal)
// sums the blocks in fp64 instead (exact while they span <= 34 bits, within fp32 rounding
// beyond; the reference's own fp32 GEMM order is unpinned).  The MFMA of
// block j + 1 is issued before the epilogue of block j.
#pragma once
#include "mxa_proj_args.hpp"

namespace mxa {

constexpr int kGemmRows = 64, kGemmCols = 128;
// Tile shapes (four waves of 32 rows x 64 columns each):
//   kGemmSquare  64 x 128, waves 2 x 2 (the general case, the Linear)
//   kGemmTall    128 x 64, waves 4 x 1: products of <= 64 columns (the drop-in's P.V: the
//                64 x 128 tile would leave half its waves without columns)
//   kGemmWide    32 x 256, waves 1 x 4: float32 products of 65..256 contiguous columns (the
//                drop-in's QK^T, 197 x 197 per head): a 32-row strip of whole output rows, staged
//                in LDS and written as one contiguous run (rows of 197 floats are not 16-B
//                aligned: per-lane column stores touched two lines per 128-B segment)
constexpr int kGemmSquare = 0, kGemmTall = 1, kGemmWide = 2;
template <int SH>
struct GemmShape {
  static constexpr int RW = SH == kGemmTall ? 128 : SH == kGemmWide ? 32 : kGemmRows;
  static constexpr int CW = SH == kGemmTall ? 64 : SH == kGemmWide ? 256 : kGemmCols;
  static constexpr int RPT = 256 / RW, CPT = 256 / CW;  // prologue threads per row / column
};

struct GemmLds {
  size_t xe, ce, rlo, rn, clo, cn, rhi, chi, part, stage, total;
};
__host__ __device__ inline GemmLds gemm_lds(int nbk, int sh) {
  GemmLds L;
  size_t o = 0;
  // (per-row arrays of 128, per-column arrays of 256: any tile shape)
  L.xe = o;  // row exponent offsets [nbk][RW] int16
  o += (size_t)nbk * 128 * 2;
  L.ce = o;  // column exponent offsets [nbk][CW] int16
  o += (size_t)nbk * 256 * 2;
  o = (o + 15) & ~(size_t)15;
  L.rlo = o;
  o += 128 * 4;
  L.rn = o;
  o += 128 * 4;
  L.clo = o;
  o += 256 * 4;
  L.cn = o;
  o += 256 * 4;
  L.rhi = o;
  o += 128 * 4;
  L.chi = o;
  o += 256 * 4;
  L.part = o;  // prologue partials [3][256]
  o += 3 * 256 * 4;
  L.stage = o;  // kGemmWide: the strip's float32 output rows [32][Nc <= 256]
  if (sh == kGemmWide) o += 32 * 256 * 4;
  L.total = o;
  return L;
}

// The shifted-int32 path; a wave whose spreads fail its test sums its blocks in fp64 itself
// (run_f64: no list, no follow-up kernel).
// PLAIN: float32 output, no bfloat / autocast rounding (the bench and workload settings):
// the epilogue is a store (+ bias), compiled without the general rounding code.
template <bool PLAIN, int SH>
__device__ __forceinline__ void gemm_tile(const GemmArgs& a, int64_t bat, int tm, int tn, unsigned char* smem) {
  using S = GemmShape<SH>;
  constexpr bool kStage = SH == kGemmWide;  // (PLAIN, one column tile, ldc == Nc: the launcher)
  constexpr int RW = S::RW, CW = S::CW, RPT = S::RPT, CPT = S::CPT;
  typedef int v16i_g __attribute__((ext_vector_type(16)));
  typedef int v4i_g __attribute__((ext_vector_type(4)));
  const int nbk = a.nbk;
  const GemmLds L = gemm_lds(nbk, SH);
  int16_t* xe = reinterpret_cast<int16_t*>(smem + L.xe);
  int16_t* ce = reinterpret_cast<int16_t*>(smem + L.ce);
  int* rlo = reinterpret_cast<int*>(smem + L.rlo);
  int* rn = reinterpret_cast<int*>(smem + L.rn);
  int* clo = reinterpret_cast<int*>(smem + L.clo);
  int* cn = reinterpret_cast<int*>(smem + L.cn);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int m0g = tm * RW, n0g = tn * CW;
  const int16_t* aeb = a.ae + bat * a.ae_bat;
  const int16_t* beb = a.be + bat * a.be_bat;

  // ---- per row / column of the tile: smallest finite block exponent, spread, NaN ----
  // (rows / columns beyond the matrix: exponents 0, never NaN -- their results are dropped).
  // An all-zero block (shared exponent -126: code unit 2^-132 for int8, 2^-128 for int4)
  // adds exactly 0 whatever its exponent: it is left out of the spread -- the pruned blocks of P in P.V would otherwise
  // send every wave to the fp64 kernel.
  const int8_t* abase = a.a + bat * a.a_bat;
  const int8_t* bbase = a.b + bat * a.b_bat;
  auto zero_blk = [&](bool isrow, int i, int kb, int e) {
    if (e > -128 || e == kExpNaN) return false;
    const int m = m0g + i;
    const int8_t* p = !isrow   ? bbase + (int64_t)(n0g + i) * a.ldb + 32 * kb
                      : a.a_mfma ? abase + (((int64_t)(m >> 5) * nbk + kb) * 64 + (m & 31)) * 16
                                 : abase + (int64_t)m * a.lda + 32 * kb;
    const int hoff = (isrow && a.a_mfma) ? 512 : 16;  // the block's second 16 elements
    const uint4 u = *reinterpret_cast<const uint4*>(p), v = *reinterpret_cast<const uint4*>(p + hoff);
    return ((u.x | u.y | u.z | u.w) | (v.x | v.y | v.z | v.w)) == 0u;
  };
  // Per row RPT threads and per column CPT threads reduce strided K-block subsets (consecutive
  // threads on consecutive exponents: coalesced, independent loads), partials through LDS.
  int* chi = reinterpret_cast<int*>(smem + L.chi);
  int* rhi_ = reinterpret_cast<int*>(smem + L.rhi);
  int* part = reinterpret_cast<int*>(smem + L.part);  // [3][256]: lo, hi, nan per thread
  const bool bk_major = a.be_k != 1;  // B exponents [kb][n] (cols_prep) vs [n][kb] (a weight)
  auto a_exp = [&](int r, int kb) { return exp_from16(aeb[(int64_t)(m0g + r) * nbk + kb]); };
  auto b_exp = [&](int c, int kb) { return exp_from16(beb[(int64_t)(n0g + c) * a.be_n + kb * a.be_k]); };
  {
    int lo = 1 << 20, hi = -(1 << 20), nan = 0;
    auto take = [&](bool isrow, int i, int kb, int e) {
      if (e == kExpNaN) {
        nan = 1;
      } else if (!zero_blk(isrow, i, kb, e)) {
        lo = min(lo, e);
        hi = max(hi, e);
      }
    };
    // rows: thread (r = tid / RPT, q = tid % RPT) takes K-blocks q, q + RPT, ...
    {
      const int r = tid / RPT, q = tid % RPT;
      if (m0g + r < a.M)
        for (int kb = q; kb < nbk; kb += RPT) take(true, r, kb, a_exp(r, kb));
    }
    part[tid] = lo;
    part[256 + tid] = hi;
    part[512 + tid] = nan;
  }
  __syncthreads();
  if (tid < RW) {
    int lo = 1 << 20, hi = -(1 << 20), nan = 0;
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      lo = min(lo, part[RPT * tid + q]);
      hi = max(hi, part[256 + RPT * tid + q]);
      nan |= part[512 + RPT * tid + q];
    }
    if (lo > hi) lo = hi = 0;
    rlo[tid] = lo;
    rhi_[tid] = hi;
    rn[tid] = nan;
  }
  __syncthreads();
  {
    int lo = 1 << 20, hi = -(1 << 20), nan = 0;
    // columns: [kb][n] exponents -- thread (c = tid % CW, h = tid / CW) takes K-blocks
    // h, h + CPT, ...; [n][kb] -- thread (c = tid / CPT, h = tid % CPT)
    const int c = bk_major ? (tid % CW) : (tid / CPT), h = bk_major ? (tid / CW) : (tid % CPT);
    if (n0g + c < a.Nc)
      for (int kb = h; kb < nbk; kb += CPT) {
        const int e = b_exp(c, kb);
        if (e == kExpNaN) {
          nan = 1;
        } else if (!zero_blk(false, c, kb, e)) {
          lo = min(lo, e);
          hi = max(hi, e);
        }
      }
    part[tid] = lo;
    part[256 + tid] = hi;
    part[512 + tid] = nan;
  }
  __syncthreads();
  if (tid < CW) {
    int lo = 1 << 20, hi = -(1 << 20), nan = 0;
#pragma unroll
    for (int h = 0; h < CPT; ++h) {
      const int t = bk_major ? tid + CW * h : CPT * tid + h;
      lo = min(lo, part[t]);
      hi = max(hi, part[256 + t]);
      nan |= part[512 + t];
    }
    if (lo > hi) lo = hi = 0;
    clo[tid] = lo;
    chi[tid] = hi;
    cn[tid] = nan;
  }
  __syncthreads();
  for (int i = tid; i < nbk * RW; i += 256) {
    const int kb = i / RW, r = i - kb * RW;
    const int e = m0g + r < a.M ? a_exp(r, kb) : 0;
    xe[i] = (int16_t)(e == kExpNaN || zero_blk(true, r, kb, e) ? 0 : e - rlo[r]);
  }
  for (int i = tid; i < nbk * CW; i += 256) {
    const int kb = i / CW, c = i - kb * CW;
    const int e = n0g + c < a.Nc ? b_exp(c, kb) : 0;
    ce[i] = (int16_t)(e == kExpNaN || zero_blk(false, c, kb, e) ? 0 : e - clo[c]);
  }
  __syncthreads();

  // ---- this wave: rows wr0 .. +31, columns wc0 .. +63 of the tile ------------------
  const int wr0 = SH == kGemmTall ? 32 * wave : SH == kGemmWide ? 0 : 32 * (wave & 1);
  const int wc0 = SH == kGemmTall ? 0 : SH == kGemmWide ? 64 * wave : 64 * (wave >> 1);
  float* stage = reinterpret_cast<float*>(smem + L.stage);
  const int ln = lane & 31, kh = 16 * (lane >> 5), m0 = 4 * (lane >> 5);
  // the wave's fast-path test: its rows' largest spread + its columns' largest spread,
  // and the smallest output scale (a subnormal result would round twice)
  auto wmax = [](int v) {
    return (int)wave_reduce((uint32_t)(v + (1 << 20)), [](uint32_t x, uint32_t y) { return x > y ? x : y; }) - (1 << 20);
  };
  auto wmin = [](int v) {
    return (int)wave_reduce((uint32_t)(v + (1 << 20)), [](uint32_t x, uint32_t y) { return x < y ? x : y; }) - (1 << 20);
  };
  const int rr = wr0 + ln, cc = wc0 + lane;
  const bool rv = m0g + rr < a.M, cv = n0g + cc < a.Nc;
  // spreads (row rr: lanes 0..31 and 32..63 alike)
  const int rsp = rhi_[rr] - rlo[rr], csp = chi[cc] - clo[cc];
  const int srow = wmax(rv ? rsp : 0), scol = wmax(cv ? csp : 0);
  const int lrow = wmin(rv ? rlo[rr] : (1 << 19)), lcol = wmin(cv ? clo[cc] : (1 << 19));
  const bool fast = srow + scol <= a.smax && lrow + lcol >= -126;

  const int arow = min(m0g + wr0 + ln, a.M - 1);
  const int bc0 = min(n0g + wc0 + ln, a.Nc - 1), bc1 = min(n0g + wc0 + 32 + ln, a.Nc - 1);
  // A: row-major (lane: 16 B of its row at 32 kb + kh; K-block step 32 B), or the MFMA-ready
  // row-block layout (lane: 16 B at lane * 16 of the wave's 1-KB chunk; step 1 KB)
  // (the row block clamped to the last one that exists: when M % 64 is 1..32 the second
  // wave of the last row tile has no rows, and the layout holds whole 32-row blocks only)
  const int8_t* ap = a.a_mfma ? a.a + bat * a.a_bat + ((int64_t)min((m0g + wr0) >> 5, (a.M - 1) >> 5) * nbk * 64 + lane) * 16
                              : a.a + bat * a.a_bat + (int64_t)arow * a.lda + kh;
  const int astep = a.a_mfma ? 1024 : 32;
  // B: row-major codes (lane: 16 B of its column at 32 kb + kh; K-block step 32 B), or the
  // MFMA-ready pk layout (lane: 16 B at lane * 16 of its column block's 1-KB chunk; step 1 KB)
  const int8_t *bp0, *bp1;
  int bstep;
  if (a.bpk) {
    const int cb0 = min((n0g + wc0) / 32, a.b_nb32 - 1), cb1 = min((n0g + wc0 + 32) / 32, a.b_nb32 - 1);
    bp0 = a.bpk + ((int64_t)cb0 * nbk * 64 + lane) * 16;
    bp1 = a.bpk + ((int64_t)cb1 * nbk * 64 + lane) * 16;
    bstep = 1024;
  } else {
    bp0 = a.b + bat * a.b_bat + (int64_t)bc0 * a.ldb + kh;
    bp1 = a.b + bat * a.b_bat + (int64_t)bc1 * a.ldb + kh;
    bstep = 32;
  }
  auto ld = [astep](const int8_t* p, int kb) { return *reinterpret_cast<const v4i_g*>(p + (int64_t)astep * kb); };
  auto ldb = [bstep](const int8_t* p, int kb) { return *reinterpret_cast<const v4i_g*>(p + (int64_t)bstep * kb); };
  const v16i_g zero = {};
  const int last = nbk - 1;
  const int16_t* xrow = xe + wr0 + m0;
  const int16_t* xcol = ce + wc0 + ln;

  // output of chain j (columns wc0 + 32 j ..): value of element i of the lane
  auto store = [&](int j, int i, float o) {
    const int m = m0g + wr0 + 8 * (i >> 2) + m0 + (i & 3);
    const int n = n0g + wc0 + 32 * j + ln;
    if (m >= a.M || n >= a.Nc) return;
    const int lr = wr0 + 8 * (i >> 2) + m0 + (i & 3), lc = wc0 + 32 * j + ln;
    if (rn[lr] || cn[lc]) o = __uint_as_float(0x7FC00000u);
    const int64_t off = bat * a.c_bat + (int64_t)m * a.ldc + n;
    if constexpr (kStage) {
      stage[lr * a.Nc + n] = a.bias ? o + a.bias[n] : o;
    } else if constexpr (PLAIN) {
      static_cast<float*>(a.c)[off] = a.bias ? o + a.bias[n] : o;
    } else if (a.linear) {
      // autocast: F.linear returns the dtype, then the output rounding (linear.py:88-92),
      // then + fp32 bias promotes back (the same order as the mx.matmul branch below)
      o = round_bfloat(round_dt(o, a.autocast), a.bfloat, kRoundNearest, 1, a.autocast);
      if (a.bias) o = round_bfloat(o + round_bfloat(a.bias[n], a.bfloat, kRoundNearest, 1), a.bfloat, kRoundNearest, 1);
      static_cast<float*>(a.c)[off] = o;
    } else {
      store_dt(a.c, off, round_bfloat(round_dt(o, a.dt), a.bfloat, kRoundNearest, 1, a.dt), a.dt);
    }
  };

  // fp64 block sums, one chain at a time (registers for one double accumulator set): the
  // waves whose spreads could overflow int32 (or whose result could be subnormal)
  auto run_f64 = [&]() {
    for (int j = 0; j < 2; ++j) {
      const int8_t* bp = j ? bp1 : bp0;
      const int lc = clo[wc0 + 32 * j + ln];
      double acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.0;
      for (int kb = 0; kb < nbk; ++kb) {
        const v16i_g c = __builtin_amdgcn_mfma_i32_32x32x32_i8(ld(ap, kb), ldb(bp, kb), zero, 0, 0, 0);
        const int dc = xcol[kb * CW + 32 * j] + lc;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int lr = wr0 + 8 * (i >> 2) + m0 + (i & 3);
          acc[i] += ldexp((double)c[i], xe[kb * RW + lr] + rlo[lr] + dc);
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) store(j, i, (float)acc[i]);
    }
  };
  if (!fast) {
    run_f64();
  } else {
    int acc0[16], acc1[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc0[i] = acc1[i] = 0;
    // block kb's shifted sums: row offset (4 rows per uint2 read) + column offset
    auto epi = [&](const v16i_g& c0, const v16i_g& c1, int kb) {
      const int d0 = xcol[kb * CW], d1 = xcol[kb * CW + 32];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint2 e4 = *reinterpret_cast<const uint2*>(xrow + kb * RW + 8 * q);
        const int dx[4] = {(int)(int16_t)(e4.x & 0xFFFFu), (int)(int16_t)(e4.x >> 16), (int)(int16_t)(e4.y & 0xFFFFu),
                           (int)(int16_t)(e4.y >> 16)};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          acc0[4 * q + r] += (int)((uint32_t)c0[4 * q + r] << (dx[r] + d0));
          acc1[4 * q + r] += (int)((uint32_t)c1[4 * q + r] << (dx[r] + d1));
        }
      }
    };
    // Pairs of K-blocks: the pair's four MFMAs are issued together, then the next pair's
    // operands are loaded together (the A loads of blocks kb, kb + 1 touch the same 128-B
    // line of each row, so it is fetched once), then the two epilogues run while those
    // loads are in flight.  Operands of a pair: E (even block) and O (odd block) slots.
    const int last2 = last;
    v4i_g aE = ld(ap, 0), bE0 = ldb(bp0, 0), bE1 = ldb(bp1, 0);
    v4i_g aO = ld(ap, min(1, last2)), bO0 = ldb(bp0, min(1, last2)), bO1 = ldb(bp1, min(1, last2));
    for (int kb = 0; kb < nbk; kb += 2) {
      const bool h1 = kb + 1 < nbk;
      const v16i_g cA0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(aE, bE0, zero, 0, 0, 0);
      const v16i_g cA1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(aE, bE1, zero, 0, 0, 0);
      v16i_g cB0 = zero, cB1 = zero;
      if (h1) {
        cB0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(aO, bO0, zero, 0, 0, 0);
        cB1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(aO, bO1, zero, 0, 0, 0);
      }
      const int ke = min(kb + 2, last2), ko = min(kb + 3, last2);
      aE = ld(ap, ke); aO = ld(ap, ko);
      bE0 = ldb(bp0, ke); bO0 = ldb(bp0, ko);
      bE1 = ldb(bp1, ke); bO1 = ldb(bp1, ko);
      __builtin_amdgcn_sched_barrier(0);
      epi(cA0, cA1, kb);
      if (h1) epi(cB0, cB1, kb + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int lc0 = clo[wc0 + ln], lc1 = clo[wc0 + 32 + ln];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int lr = rlo[wr0 + 8 * (i >> 2) + m0 + (i & 3)];
      store(0, i, ldexpf((float)acc0[i], lr + lc0));
      store(1, i, ldexpf((float)acc1[i], lr + lc1));
    }
  }
  if constexpr (kStage) {  // the strip's rows, contiguous in the output: 16-B stores
    typedef float f32x4_a4g __attribute__((ext_vector_type(4), aligned(4)));
    __syncthreads();
    const int n = min(RW, a.M - m0g) * a.Nc;
    float* dst = static_cast<float*>(a.c) + bat * a.c_bat + (int64_t)m0g * a.Nc;
    for (int i = 4 * tid; i < n; i += 4 * 256) {
      if (i + 4 <= n) {
        const float4 v = *reinterpret_cast<const float4*>(stage + i);
        *reinterpret_cast<f32x4_a4g*>(dst + i) = f32x4_a4g{v.x, v.y, v.z, v.w};
      } else {
        for (int t = i; t < n; ++t) dst[t] = stage[t];
      }
    }
  }
}

// (3 waves per SIMD: 166 VGPRs without spills; a cap of 4 spills ~640 registers)
template <bool PLAIN, int SH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) void mx_gemm_kernel(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  gemm_tile<PLAIN, SH>(a, blockIdx.z, blockIdx.y, blockIdx.x, smem);
}

// ---- exponent-folded digits (mx.Linear with a prepared weight) ----------------------
// One workgroup per 32-row block of A: the rows' codes times 2^(block exponent - row's
// smallest) are staged in LDS as two signed base-256 digits (MFMA-ready: [kb][digit][lane]
// [16 B]), the weight's digits (mxa_linear_weight_prep's pd) stream from memory, and the
// four digit products accumulate in the MFMA's own int32 accumulators over all K-blocks
// (lo x lo; lo x hi + hi x lo; hi x hi: |sum| <= 2 nbk 32 128^2 < 2^31) -- no VALU per
// block -- so sum = c0 + 2^8 c1 + 2^16 c2 (exact in fp64) rounds once: the same correctly
// rounded exact product as gemm_tile's shifted int32 sums.  A row block whose spreads or
// the weight's column spreads exceed kDigitSpread (or whose result could be subnormal) is
// summed here block by block in fp64 instead (the MFMA-ready weight codes, ascending
// K-blocks: the sums of gemm_tile's run_f64, exact while the scaled blocks span <= 34 bits
// -- so also wherever the shifted int32 sums are exact), so one launch covers every row
// block: no flag, no follow-up kernels.
struct GemmDigLds {
  size_t ad, rlo, rhi, rn, st, total;
};
__host__ __device__ inline GemmDigLds gemm_dig_lds(int nbk) {
  GemmDigLds L;
  L.ad = 0;
  L.rlo = (size_t)nbk * 2048;
  L.rhi = L.rlo + 128;
  L.rn = L.rhi + 128;
  L.st = L.rn + 128;
  L.total = L.st + 16;
  return L;
}
constexpr int kGemmDigNbkMax = 72;  // 2 KB of LDS per K-block: <= 144 KB

template <bool PLAIN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 8))) void mx_gemm_dig_kernel(GemmArgs a) {
  typedef int v16i_g __attribute__((ext_vector_type(16)));
  typedef int v4i_g __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nbk = a.nbk;
  const GemmDigLds L = gemm_dig_lds(nbk);
  int8_t* ad = reinterpret_cast<int8_t*>(smem + L.ad);
  int* rlo = reinterpret_cast<int*>(smem + L.rlo);
  int* rhi = reinterpret_cast<int*>(smem + L.rhi);
  int* rn = reinterpret_cast<int*>(smem + L.rn);
  int* st = reinterpret_cast<int*>(smem + L.st);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int rb = blockIdx.x, m0g = 32 * rb, rows = min(32, a.M - m0g);
  auto code_at = [&](int m, int kb, int h) -> const int8_t* {  // 16 codes of row m, block kb, half h
    return a.a_mfma ? a.a + (((int64_t)rb * nbk + kb) * 64 + m + 32 * h) * 16
                    : a.a + (int64_t)(m0g + m) * a.lda + 32 * kb + 16 * h;
  };
  auto exp_at = [&](int m, int kb) { return exp_from16(a.ae[(int64_t)(m0g + m) * nbk + kb]); };

  // ---- per row: smallest / largest finite block exponent (all-zero blocks left out, as
  // in gemm_tile), NaN flag -------------------------------------------------------------
  if (tid < 32) {
    rlo[tid] = 1 << 20;
    rhi[tid] = -(1 << 20);
    rn[tid] = 0;
  }
  __syncthreads();
  for (int i = tid; i < 32 * nbk; i += 256) {
    const int m = i / nbk, kb = i - m * nbk;
    if (m >= rows) continue;
    const int e = exp_at(m, kb);
    if (e == kExpNaN) {
      rn[m] = 1;
      continue;
    }
    if (e <= -128) {
      const uint4 u = *reinterpret_cast<const uint4*>(code_at(m, kb, 0));
      const uint4 v = *reinterpret_cast<const uint4*>(code_at(m, kb, 1));
      if (((u.x | u.y | u.z | u.w) | (v.x | v.y | v.z | v.w)) == 0u) continue;
    }
    atomicMin(&rlo[m], e);
    atomicMax(&rhi[m], e);
  }
  __syncthreads();
  if (wave == 0) {  // the block's gate: row spreads, the weight's column spreads, subnormal results
    const int m = lane & 31;
    const bool em = rlo[m] > rhi[m];
    const uint32_t smx = wave_reduce(lane < 32 && !em ? (uint32_t)(rhi[m] - rlo[m]) : 0u,
                                     [](uint32_t u, uint32_t w) { return u > w ? u : w; });
    const uint32_t lmn = wave_reduce(lane < 32 && !em ? (uint32_t)(rlo[m] + (1 << 20)) : 0xFFFFFFFFu,
                                     [](uint32_t u, uint32_t w) { return u < w ? u : w; });
    uint32_t gsp = 0, glo = 0xFFFFFFFFu;
    for (int g = lane; g < a.bG; g += 64) {
      gsp = max(gsp, (uint32_t)a.bgs[2 * g + 1]);
      glo = min(glo, (uint32_t)(a.bgs[2 * g] + (1 << 20)));
    }
    gsp = wave_reduce(gsp, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
    glo = wave_reduce(glo, [](uint32_t u, uint32_t w) { return u < w ? u : w; });
    const bool ok = smx <= (uint32_t)kDigitSpread && gsp <= (uint32_t)kDigitSpread &&
                    (lmn == 0xFFFFFFFFu || (int)lmn + (int)glo - (2 << 20) >= -126);
    if (lane == 0) st[0] = ok;
  }
  __syncthreads();
  const int ncb = (a.Nc + 31) / 32, last = nbk - 1;
  const int ln = lane & 31, m0 = 4 * (lane >> 5);
  // out = bf(fl32(sum)); out = bf(out + bf(bias))  (linear.py:88-101) for element i of the
  // lane's 32 x 32 tile of column block cb; value(i, m) the fp32 sum of row m
  auto store_out = [&](int cb, auto&& value) {
    const int n = 32 * cb + ln;
    if (n >= a.Nc) return;
    const bool cnan = a.bpn[n] != 0;
    const float bb = a.bias ? (PLAIN ? a.bias[n] : round_bfloat(a.bias[n], a.bfloat, kRoundNearest, 1)) : 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int m = 8 * (i >> 2) + m0 + (i & 3);
      if (m >= rows) continue;
      float o = (cnan || rn[m]) ? __uint_as_float(0x7FC00000u) : value(i, m);
      if constexpr (PLAIN) {
        o = a.bias ? o + bb : o;
      } else {
        // autocast: F.linear returns the dtype, then the output rounding, then + fp32 bias
        o = round_bfloat(round_dt(o, a.autocast), a.bfloat, kRoundNearest, 1, a.autocast);
        if (a.bias) o = round_bfloat(o + bb, a.bfloat, kRoundNearest, 1);
      }
      static_cast<float*>(a.c)[(int64_t)(m0g + m) * a.ldc + n] = o;
    }
  };
  if (!st[0]) {  // (uniform over the workgroup) the fp64 block sums
    const v16i_g zero = {};
    for (int cb = wave; cb < ncb; cb += 4) {
      const int8_t* bp = a.bpk + ((int64_t)min(cb, a.b_nb32 - 1) * nbk * 64 + lane) * 16;
      const int n = min(32 * cb + ln, a.Nc - 1);
      double acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.0;
      for (int kb = 0; kb < nbk; ++kb) {
        const v4i_g av = *reinterpret_cast<const v4i_g*>(code_at(min(ln, rows - 1), kb, lane >> 5));
        const v4i_g bv = *reinterpret_cast<const v4i_g*>(bp + (int64_t)kb * 1024);
        const v16i_g c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, zero, 0, 0, 0);
        const int eb = exp_from16(a.be[(int64_t)n * a.be_n + (int64_t)kb * a.be_k]);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = min(8 * (i >> 2) + m0 + (i & 3), rows - 1);
          const int ea = exp_at(m, kb);
          // a NaN block: the row / column flag makes the output NaN; its term adds 0 here
          acc[i] += (ea == kExpNaN || eb == kExpNaN) ? 0.0 : ldexp((double)c[i], ea + eb);
        }
      }
      store_out(cb, [&](int i, int) { return (float)acc[i]; });
    }
    return;
  }

  // ---- the rows' digits: chunk (kb, lane) = row lane % 32, half lane / 32 ----------------
  for (int i = tid; i < 64 * nbk; i += 256) {
    const int kb = i >> 6, ln = i & 63, m = ln & 31;
    uint4 v = make_uint4(0, 0, 0, 0);
    int sh = 0;
    if (m < rows) {
      v = *reinterpret_cast<const uint4*>(code_at(m, kb, ln >> 5));
      const int e = exp_at(m, kb), lo = rlo[m] > rhi[m] ? 0 : rlo[m];
      sh = e == kExpNaN ? 0 : min(max(e - lo, 0), kDigitSpread);  // (a left-out zero block: any shift)
    }
    uint4 d0, d1;
    fold_digits16(v, sh, d0, d1);
    *reinterpret_cast<uint4*>(ad + kb * 2048 + ln * 16) = d0;
    *reinterpret_cast<uint4*>(ad + kb * 2048 + 1024 + ln * 16) = d1;
  }
  __syncthreads();

  // ---- per wave: 32-column blocks wave, wave + 4, ... --------------------------------
  const int8_t* adl = ad + lane * 16;
  auto cl = [&](int kb) { return min(kb, last); };
  for (int cb = wave; cb < ncb; cb += 4) {
    const int8_t* bp = a.bpd + (int64_t)cb * nbk * 2048 + lane * 16;
    auto ldd = [&](int kb, int p) { return *reinterpret_cast<const v4i_g*>(bp + (int64_t)kb * 2048 + p * 1024); };
    v16i_g c0 = {}, c1 = {}, c2 = {};
    v4i_g L0 = ldd(0, 0), H0 = ldd(0, 1), L1 = ldd(cl(1), 0), H1 = ldd(cl(1), 1);
    v4i_g L2 = ldd(cl(2), 0), H2 = ldd(cl(2), 1), L3 = ldd(cl(3), 0), H3 = ldd(cl(3), 1);
    auto step = [&](int kb, v4i_g& Ls, v4i_g& Hs) {
      const v4i_g al = *reinterpret_cast<const v4i_g*>(adl + kb * 2048);
      const v4i_g ah = *reinterpret_cast<const v4i_g*>(adl + kb * 2048 + 1024);
      c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(al, Ls, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(al, Hs, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ah, Hs, c2, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(ah, Ls, c1, 0, 0, 0);
      Ls = ldd(cl(kb + 4), 0);
      Hs = ldd(cl(kb + 4), 1);
      __builtin_amdgcn_sched_barrier(0);  // reload each slot right after its use
    };
    int kb = 0;
    for (; kb + 4 <= nbk; kb += 4) {
      step(kb, L0, H0);
      step(kb + 1, L1, H1);
      step(kb + 2, L2, H2);
      step(kb + 3, L3, H3);
    }
    if (kb < nbk) step(kb, L0, H0);
    if (kb + 1 < nbk) step(kb + 1, L1, H1);
    if (kb + 2 < nbk) step(kb + 2, L2, H2);
    const int clo = a.bps[2 * min(32 * cb + ln, a.Nc - 1)];
    store_out(cb, [&](int i, int m) {
      const int lo = rlo[m] > rhi[m] ? 0 : rlo[m];
      const double v = (double)c0[i] + 256.0 * (double)c1[i] + 65536.0 * (double)c2[i];
      return (float)ldexp(v, lo + clo);
    });
  }
}

}  // namespace mxa
