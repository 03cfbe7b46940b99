// Fused MX Linear qkv projection -> the attention path's MX operands.
//
// The patched attention modules compute qkv = mx.Linear(x) and split it into the
// heads' q, k, v (workloads/deit/scripts/main.py:87-88, workloads/DiT/models.py:156-157);
// the Linear forward is microxscaling/mx/linear.py:20-103:
//   out = bf(fl32(MX(bf(x), along C) @ MX(bf(W), along C)^T));  out = bf(out + bf(bias))
// (bf = quantize_elemwise_op, identity at bfloat 0/32).  Here one workgroup takes one
// 32-token MX block of one image: the x code tile (staged in LDS once) times each
// head's q / k / v weight rows (prepared MFMA-ready: one coalesced load per K-block) on v_mfma_i32_32x32x32_i8 -- K = 32 = one
// MX block, so each block's int32 sum is exact -- with the block scale 2^(ex + ew)
// applied exactly -- as int32 sums shifted to the row's and column's smallest block
// exponent (the common case; v_lshl_add_u32), else in fp64 -- so the projection is
// the correctly rounded exact product (the reference's MKL sgemm order is unpinned, SURVEY.md F7:
// tolerance there, bit-exact against the oracle).  The fp32 tile then stays in LDS
// and is quantized in place into exactly what rows_prep / cols_prep would produce
// from q, k, v: q and k rows (codes, block exponents, approximator operands) and V's
// codes along the 32 tokens (transposed) -- the fp32 q / k / v never reach HBM.
#pragma once
#include <type_traits>

#include "mxa_finish.hpp"
#include "mxa_prep.hpp"
#include "mxa_proj_args.hpp"

namespace mxa {



struct ProjLds {
  size_t xt, xe, rlo, rhi, rn, st, ot, total;
  int xst, ost;
};
// x code tile [32][Cpad + 16], x exponents relative to the row's smallest [nbk][32]
// (int16, NaN -> 0), per-row smallest / largest exponent and NaN flag, tile stats, the
// fp32 output tile of one head [32][3D + 1] (odd stride: V's column reads are
// conflict-free)
__host__ __device__ inline ProjLds proj_lds(int Cpad, int nbk, int D) {
  ProjLds L;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t o = 0;
  L.xst = Cpad + 16;
  L.xt = o;
  o += (size_t)32 * L.xst;
  L.xe = o;
  o += al((size_t)nbk * 32 * 2);
  L.rlo = o;
  o += 32 * 4;
  L.rhi = o;
  o += 32 * 4;
  L.rn = o;
  o += 32 * 4;
  L.st = o;
  o += 16;
  L.ost = 3 * D + 1;
  L.ot = o;
  o += al((size_t)32 * L.ost * 4);
  L.total = o;
  return L;
}

// One workgroup per (32-token block, image, head group), looping over the group's heads; 3 * NBD waves,
// wave (s, cb) = sub-matrix s (q, k, v) and its 32-column block cb of the head.
#ifndef MXA_PROJ_WAVES
#define MXA_PROJ_WAVES 4  // waves per SIMD the register budget targets (tools builds vary it)
#endif
#ifndef MXA_PROJ_PF
#define MXA_PROJ_PF 2  // K-blocks of weight codes in flight per wave (measured: 4 and 8 slower, registers)
#endif
template <int NBD>
__global__ __launch_bounds__(64 * 3 * NBD) __attribute__((amdgpu_waves_per_eu(MXA_PROJ_WAVES, 8))) void qkv_proj_kernel(ProjArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int kThreads = 64 * 3 * NBD;
  const int tb = blockIdx.x, b = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int D = a.D, HD = a.H * D, nbk = a.nbk;
  const ProjLds L = proj_lds(a.Cpad, nbk, D);
  int8_t* xt = reinterpret_cast<int8_t*>(smem + L.xt);
  int16_t* xe = reinterpret_cast<int16_t*>(smem + L.xe);
  int* rlo = reinterpret_cast<int*>(smem + L.rlo);
  int* rhi = reinterpret_cast<int*>(smem + L.rhi);
  int* rn = reinterpret_cast<int*>(smem + L.rn);
  int* st = reinterpret_cast<int*>(smem + L.st);
  float* ot = reinterpret_cast<float*>(smem + L.ot);
  const int n0 = 32 * tb, rows = min(32, a.N - n0);
  const int64_t row0 = (int64_t)b * a.N + n0;

  // ---- stage the token block's x codes (zero beyond N) and exponents ----------
  const int cpr = a.Cpad / 16;
  for (int i = threadIdx.x; i < 32 * cpr; i += kThreads) {
    const int m = i / cpr, c = i - m * cpr;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < rows) v = *reinterpret_cast<const uint4*>(a.xc + (row0 + m) * a.Cpad + 16 * c);
    *reinterpret_cast<uint4*>(xt + m * L.xst + 16 * c) = v;
  }
  if (threadIdx.x < 32) {
    rlo[threadIdx.x] = 1 << 20;
    rhi[threadIdx.x] = -(1 << 20);
    rn[threadIdx.x] = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 32 * nbk; i += kThreads) {  // per row: finite min / max, NaN flag
    const int m = i / nbk, kb = i - m * nbk;
    const int e = m < rows ? exp_from16(a.xs[(row0 + m) * nbk + kb]) : 0;
    if (e == kExpNaN) {
      rn[m] = 1;  // a NaN block makes the whole output row NaN
    } else {
      atomicMin(&rlo[m], e);
      atomicMax(&rhi[m], e);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 32 * nbk; i += kThreads) {
    const int m = i / nbk, kb = i - m * nbk;
    const int e = m < rows ? exp_from16(a.xs[(row0 + m) * nbk + kb]) : 0;
    const int lo = rlo[m] > rhi[m] ? 0 : rlo[m];
    xe[kb * 32 + m] = (int16_t)(e == kExpNaN ? 0 : e - lo);
  }
  if (wave == 0) {  // tile stats over the 32 rows (lanes 32..63 neutral)
    const int m = lane & 31;
    const bool em = rlo[m] > rhi[m];
    const int lo = em ? 0 : rlo[m], sp = em ? 0 : rhi[m] - lo;
    const uint32_t smx = wave_reduce(lane < 32 ? (uint32_t)sp : 0u, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
    const uint32_t bmn = wave_reduce(lane < 32 ? (uint32_t)(lo + (1 << 20)) : 0xFFFFFFFFu,
                                     [](uint32_t u, uint32_t w) { return u < w ? u : w; });
    if (lane == 0) {
      st[0] = (int)smx;
      st[1] = (int)bmn - (1 << 20);
    }
  }
  __syncthreads();

  // lane maps of v_mfma_i32_32x32x32_i8 (mxa_selftest_mfma32): A[m][k], m = lane % 32,
  // k = 16 (lane / 32) + 0..15; B[k][n], n = lane % 32; C[m][n] in c[i],
  // m = 8 (i / 4) + 4 (lane / 32) + i % 4
  const int s = wave / NBD, cb = wave - s * NBD;
  const int ln = lane & 31, kh = 16 * (lane >> 5), m0 = 4 * (lane >> 5);
  const int dcol = 32 * cb + ln;
  const bool colv = dcol < D;
  const int8_t* xa = xt + ln * L.xst + kh;
  const int64_t hrow_b = (int64_t)b * a.H;

  const int h_end = min(a.H, ((int)blockIdx.z + 1) * a.hpg);
  for (int h = (int)blockIdx.z * a.hpg; h < h_end; ++h) {
    // ---- this wave's 32 x 32 output block of head h -------------------------------
    const int64_t blkc = (int64_t)(s * a.H + h) * NBD + cb;  // padded 32-column block
    const int64_t pc = 32 * blkc + ln;
    const int8_t* wp = a.pk + (blkc * nbk) * 1024 + lane * 16;
    const int16_t* wep = a.pe + pc * nbk;
    const int wlo = a.ps[2 * pc], wsp = a.ps[2 * pc + 1];
    bool cnan = false;
    // Every block product is c * 2^(ex + ew) with |c| <= 32 * 127^2 < 2^19.  When the
    // row and column exponent spreads sum to <= smax, the block sums shifted by
    // (ex - rowmin) + (ew - colmin) add up exactly in int32, and one conversion gives
    // the correctly rounded result (2 VALU per element and block).  Otherwise (or when
    // the result could be subnormal) each block is added exactly in fp64.
    const int wsp_max = (int)wave_max_u32((uint32_t)wsp);
    const int wlo_min =
        (int)wave_reduce((uint32_t)(wlo + (1 << 20)), [](uint32_t u, uint32_t w) { return u < w ? u : w; }) - (1 << 20);
    const bool fast = st[0] + wsp_max <= a.smax && st[1] + wlo_min >= -126;
    const int64_t jcol = (int64_t)s * HD + (int64_t)h * D + dcol;
    const float bb = (a.bias && colv) ? round_bfloat(a.bias[jcol], a.bfloat, kRoundNearest, 1) : 0.0f;
    // the K loop and the epilogue, specialised on the accumulation (FAST: shifted int32;
    // else exact fp64): separate live ranges, so the two never hold registers together
    auto run = [&](auto fast_c) {
      constexpr bool FAST = decltype(fast_c)::value;
      typename std::conditional<FAST, int, double>::type acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0;
      // the weight codes and the column's block exponents ride kPf K-blocks ahead (a
      // load per block issued right before its use left an L2 round trip on every
      // step), the x operand one block ahead
      constexpr int kPf = MXA_PROJ_PF;
      v4i_ bq[kPf];
      int16_t eq[kPf];
#pragma unroll
      for (int i = 0; i < kPf; ++i) {
        const int kk = i < nbk ? i : 0;
        bq[i] = *reinterpret_cast<const v4i_*>(wp + kk * 1024);
        eq[i] = wep[kk];
      }
      v4i_ an = *reinterpret_cast<const v4i_*>(xa);
      for (int kb = 0; kb < nbk; ++kb) {
        const v4i_ bv = bq[0];
        const int16_t ewr = eq[0];
#pragma unroll
        for (int i = 0; i + 1 < kPf; ++i) {
          bq[i] = bq[i + 1];
          eq[i] = eq[i + 1];
        }
        if (kb + kPf < nbk) {
          bq[kPf - 1] = *reinterpret_cast<const v4i_*>(wp + (kb + kPf) * 1024);
          eq[kPf - 1] = wep[kb + kPf];
        }
        const v4i_ av = an;
        if (kb + 1 < nbk) an = *reinterpret_cast<const v4i_*>(xa + 32 * (kb + 1));
        const v16i zero = {};
        const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, zero, 0, 0, 0);
        int ew = exp_from16(ewr);
        cnan = cnan || ew == kExpNaN;
        ew = ew == kExpNaN ? wlo : ew;
        const int16_t* eb = xe + kb * 32 + m0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint2 e4 = *reinterpret_cast<const uint2*>(eb + 8 * q);  // rows 8q + m0 .. + 3
          const int dx[4] = {(int)(e4.x & 0xFFFFu), (int)(e4.x >> 16), (int)(e4.y & 0xFFFFu), (int)(e4.y >> 16)};
          if constexpr (FAST) {
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[4 * q + r] += (int)((uint32_t)c[4 * q + r] << (dx[r] + ew - wlo));
          } else {
            const int4 lo4 = *reinterpret_cast<const int4*>(rlo + 8 * q + m0);
            const int lo[4] = {lo4.x, lo4.y, lo4.z, lo4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[4 * q + r] += ldexp((double)c[4 * q + r], dx[r] + lo[r] + ew);
          }
        }
      }
      // ---- out = bf(fl32(sum)); out = bf(out + bf(bias))  (linear.py:88-101) -------
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int m = 8 * (i >> 2) + m0 + (i & 3);
        float o;
        if constexpr (FAST) o = ldexpf((float)acc[i], rlo[m] + wlo);
        else o = (float)acc[i];
        if (cnan || rn[m]) o = __uint_as_float(0x7FC00000u);
        o = round_bfloat(o, a.bfloat, kRoundNearest, 1);
        o = round_dt(o, a.autocast);  // autocast: F.linear returns the dtype, + fp32 bias promotes back
        if (a.bias) o = round_bfloat(o + bb, a.bfloat, kRoundNearest, 1);
        if (colv) {
          ot[m * L.ost + s * D + dcol] = o;
          if (a.qkv_out && m < rows) a.qkv_out[(row0 + m) * (3 * HD) + jcol] = o;
        }
      }
    };
    if (fast) run(std::integral_constant<bool, true>{});
    else run(std::integral_constant<bool, false>{});
    __syncthreads();

    // ---- q and k rows (waves 0 .. 2 NBD - 1) beside V's columns (the other NBD waves:
    // 64 NBD >= D lanes, one column each).  Before, the wave that took the first q rows
    // then took V as well while the rest waited at the barrier.
    const int64_t hrow0 = (hrow_b + h) * a.N + n0;  // row of (b, h, n0) in the q / k tables
    constexpr int kPer = 32 * NBD * 2;              // lanes per sub-matrix: a multiple of 64
    static_assert(kThreads - 2 * kPer == 64 * NBD, "V lanes");
    if ((int)threadIdx.x < 2 * kPer) {
      // rows_prep's per-block body on the tile (2 lanes per 32-element block)
      const int t = (int)threadIdx.x;
      const int sk = __builtin_amdgcn_readfirstlane(t / kPer);  // uniform per wave: q or k
      const int rem = t - sk * kPer;
      const int g = rem >> 1, sub = rem & 1;
      const int m = g / NBD, blk = g - m * NBD;
      const int c0 = 32 * blk + 16 * sub;
      float xv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) xv[j] = c0 + j < D ? ot[m * L.ost + sk * D + c0 + j] : 0.0f;
      const RowsPrepArgs& ra = sk ? a.rk : a.rq;
      if (rows_prep_plain(ra)) rows_prep_block_plain<16>(ra, hrow0 + m, blk, sub, c0, xv, m < rows);
      else rows_prep_block<16>(ra, hrow0 + m, blk, sub, c0, xv, m < rows);
    } else if (const int c = (int)threadIdx.x - 2 * kPer; c < D) {
      // V: cols_prep's per-column body over the 32 tokens
      float xv[32];
      uint32_t mx = 0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float v = j < rows ? round_bfloat(ot[j * L.ost + 2 * D + c], a.cv.bfloat, kRoundNearest, 1) : 0.0f;
        xv[j] = v;
        const uint32_t ub = __float_as_uint(v) & 0x7FFFFFFFu;
        mx = ub > mx ? ub : mx;
      }
      cols_prep_column(a.cv, hrow_b + h, tb, c, xv, mx);
    }
    __syncthreads();
  }
}

}  // namespace mxa
