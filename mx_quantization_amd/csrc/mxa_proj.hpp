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
// the correctly rounded exact product whenever the blocks' scaled exponents span <= 34
// bits (fp64 holds such a sum exactly); wider spreads round in the fp64 sum and again
// to fp32, i.e. within fp32 rounding (the reference's MKL sgemm order is unpinned,
// tolerance there, bit-exact against the oracle on the tested spreads).  The fp32 tile then stays in LDS
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
  size_t xt, xh, xe, rlo, rhi, rn, st, ot, total;
  int xst, ost;
};
// x code tile [32][Cpad + 16] (or its exponent-folded low digits; the high digits in a
// second tile), x exponents relative to the row's smallest [nbk][32]
// (int16, NaN -> 0), per-row smallest / largest exponent and NaN flag, tile stats, the
// fp32 output tile of one head [32][96 NBD + 1]: q, k, v at columns 0, 32 NBD, 64 NBD
// (padding columns beyond D take the padded MFMA columns, so every lane stores
// unpredicated; the odd stride keeps V's column reads conflict-free; compile-time, so
// the epilogue's 16 stores take immediate offsets)
__host__ __device__ inline ProjLds proj_lds(int Cpad, int nbk, int D) {
  ProjLds L;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t o = 0;
  L.xst = Cpad + 16;
  L.xt = o;
  o += (size_t)32 * L.xst;
  L.xh = o;
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
  o += 16;  // max row spread, smallest row exponent, the digit-path flag
  L.ost = 96 * ((D + 31) / 32) + 1;
  L.ot = o;
  o += al((size_t)32 * L.ost * 4);
  L.total = o;
  return L;
}

// One workgroup per (32-token block, image, head group), looping over the group's heads; 3 * NBD waves,
// wave (s, cb) = sub-matrix s (q, k, v) and its 32-column block cb of the head.
#ifndef MXA_PROJ_SKIP
#define MXA_PROJ_SKIP 0  // tools-only timing variants (never the product): 1 no K loop, 2 no operand epilogue,
                         // 4 the digit loop re-reads its first block (L1-resident weights)
#endif
// PLAIN (proj_plain): no bfloat rounding, no flush, no autocast, q / k operands of
// rows_prep_block_plain and V's MXINT8 -- the bench path, compiled without the general
// rounding code (a third of the code and registers of the general instantiation).
// Per head: the exponent-folded digits, the shifted int32 block sums, or (wide spreads, a
// subnormal result) fp64 block sums, all in this workgroup.
template <int NBD, bool PLAIN>
__device__ __forceinline__ void proj_block(const ProjArgs& a, int tb, int b, int h_begin, int h_end,
                                           unsigned char* smem) {
  constexpr int kThreads = 64 * 3 * NBD;
  constexpr int kOst = 96 * NBD + 1;  // == proj_lds(...).ost
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

  // ---- the token block's x exponents, then its codes (zero beyond N) ----------------
  // When the tile's exponents and codes are at most four items per thread (DeiT, DiT),
  // both are loaded into registers up front, so the code loads overlap the exponent
  // passes and each exponent is read once; else they are (re)read where used.
  const int cpr = a.Cpad / 16;
  constexpr int kPre = 4;
  const bool pre = 32 * cpr <= kPre * kThreads && 32 * nbk <= kPre * kThreads;  // uniform
  uint4 cpre[kPre];
  int epre[kPre];
  auto code_of = [&](int i) {
    const int m = i / cpr, c = i - m * cpr;
    return m < rows ? *reinterpret_cast<const uint4*>(a.xc + (row0 + m) * a.Cpad + 16 * c) : make_uint4(0, 0, 0, 0);
  };
  auto exp_of = [&](int i) {
    const int m = i / nbk, kb = i - m * nbk;
    return m < rows ? exp_from16(a.xs[(row0 + m) * nbk + kb]) : 0;
  };
  if (pre) {
#pragma unroll
    for (int u = 0; u < kPre; ++u) {
      const int i = (int)threadIdx.x + u * kThreads;
      cpre[u] = i < 32 * cpr ? code_of(i) : make_uint4(0, 0, 0, 0);
      epre[u] = i < 32 * nbk ? exp_of(i) : 0;
    }
  }
  if (threadIdx.x < 32) {
    rlo[threadIdx.x] = 1 << 20;
    rhi[threadIdx.x] = -(1 << 20);
    rn[threadIdx.x] = 0;
  }
  __syncthreads();
  auto take_exp = [&](int i, int e) {  // per row: finite min / max, NaN flag
    const int m = i / nbk;
    if (e == kExpNaN) {
      rn[m] = 1;  // a NaN block makes the whole output row NaN
    } else {
      atomicMin(&rlo[m], e);
      atomicMax(&rhi[m], e);
    }
  };
  auto put_xe = [&](int i, int e) {
    const int m = i / nbk, kb = i - m * nbk;
    const int lo = rlo[m] > rhi[m] ? 0 : rlo[m];
    xe[kb * 32 + m] = (int16_t)(e == kExpNaN ? 0 : e - lo);
  };
  if (pre) {
#pragma unroll
    for (int u = 0; u < kPre; ++u)
      if ((int)threadIdx.x + u * kThreads < 32 * nbk) take_exp((int)threadIdx.x + u * kThreads, epre[u]);
  } else {
    for (int i = threadIdx.x; i < 32 * nbk; i += kThreads) take_exp(i, exp_of(i));
  }
  __syncthreads();
  if (pre) {
#pragma unroll
    for (int u = 0; u < kPre; ++u)
      if ((int)threadIdx.x + u * kThreads < 32 * nbk) put_xe((int)threadIdx.x + u * kThreads, epre[u]);
  } else {
    for (int i = threadIdx.x; i < 32 * nbk; i += kThreads) put_xe(i, exp_of(i));
  }
  if (wave == 0) {  // tile stats over the 32 rows (lanes 32..63 neutral)
    const int m = lane & 31;
    const bool em = rlo[m] > rhi[m];
    const int lo = em ? 0 : rlo[m], sp = em ? 0 : rhi[m] - lo;
    const uint32_t smx = wave_reduce(lane < 32 ? (uint32_t)sp : 0u, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
    const uint32_t bmn = wave_reduce(lane < 32 ? (uint32_t)(lo + (1 << 20)) : 0xFFFFFFFFu,
                                     [](uint32_t u, uint32_t w) { return u < w ? u : w; });
    // the digit path: every row's spread and every column spread of the workgroup's
    // heads within kDigitSpread (the weight's folded digits exist for those columns)
    uint32_t gmx = 0;
    for (int i = lane; i < 3 * (h_end - h_begin); i += 64) {
      const int hh = h_begin + i / 3, s3 = i - 3 * (i / 3);
      gmx = max(gmx, (uint32_t)a.gs[2 * (s3 * a.H + hh) + 1]);
    }
    gmx = wave_reduce(gmx, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
    if (lane == 0) {
      st[0] = (int)smx;
      st[1] = (int)bmn - (1 << 20);
      st[2] = smx <= kDigitSpread && gmx <= kDigitSpread;
    }
  }
  __syncthreads();
  const bool dig = st[2];  // uniform over the workgroup
  int8_t* xh = reinterpret_cast<int8_t*>(smem + L.xh);
  auto put_code = [&](int i, const uint4& v) {
    const int m = i / cpr, c = i - m * cpr;
    if (dig) {
      uint4 d0, d1;
      fold_digits16(v, xe[(c >> 1) * 32 + m], d0, d1);
      *reinterpret_cast<uint4*>(xt + m * L.xst + 16 * c) = d0;
      *reinterpret_cast<uint4*>(xh + m * L.xst + 16 * c) = d1;
    } else {
      *reinterpret_cast<uint4*>(xt + m * L.xst + 16 * c) = v;
    }
  };
  if (pre) {
#pragma unroll
    for (int u = 0; u < kPre; ++u)
      if ((int)threadIdx.x + u * kThreads < 32 * cpr) put_code((int)threadIdx.x + u * kThreads, cpre[u]);
  } else {
    for (int i = threadIdx.x; i < 32 * cpr; i += kThreads) put_code(i, code_of(i));
  }
  __syncthreads();

  // lane maps of v_mfma_i32_32x32x32_i8 (mxa_selftest_mfma32): A[m][k], m = lane % 32,
  // k = 16 (lane / 32) + 0..15; B[k][n], n = lane % 32; C[m][n] in c[i],
  // m = 8 (i / 4) + 4 (lane / 32) + i % 4
  // uniform per wave (readfirstlane: the weight addresses then live in SGPRs, the
  // per-lane part is a loop-invariant VGPR offset)
  const int s = __builtin_amdgcn_readfirstlane(wave / NBD), cb = __builtin_amdgcn_readfirstlane(wave - s * NBD);
  const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.pk), 0, a.pk_bytes, 0x00020000);
  const auto ers = __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(a.pe), 0, a.pe_bytes, 0x00020000);
  const int ln = lane & 31, kh = 16 * (lane >> 5), m0 = 4 * (lane >> 5);
  const int dcol = 32 * cb + ln;
  const bool colv = dcol < D;
  const int8_t* xa = xt + ln * L.xst + kh;
  const int64_t hrow_b = (int64_t)b * a.H;

  for (int h = h_begin; h < h_end; ++h) {
    // ---- this wave's 32 x 32 output block of head h -------------------------------
    const int64_t blkc = (int64_t)(s * a.H + h) * NBD + cb;  // padded 32-column block
    const int64_t pc = 32 * blkc + ln;
    // buffer loads: descriptor and the K-block's offset in SGPRs, the per-lane part a
    // loop-invariant VGPR (no per-load address arithmetic; checked by proj_buffers_fit)
    const int wsoff = __builtin_amdgcn_readfirstlane((int)(blkc * nbk) * 1024);
    const int esoff = __builtin_amdgcn_readfirstlane((int)(32 * blkc * nbk) * 2);
    const int woff = lane * 16, eoff = ln * nbk * 2;
    const int wlo = a.ps[2 * pc];
    bool cnan = false;
    // Every block product is c * 2^(ex + ew) with |c| <= 32 * 127^2 < 2^19.  When the
    // row and column exponent spreads sum to <= smax, the block sums shifted by
    // (ex - rowmin) + (ew - colmin) add up exactly in int32, and one conversion gives
    // the correctly rounded result (2 VALU per element and block).  Otherwise (or when
    // the result could be subnormal) the blocks are summed in fp64 (run_f64, below):
    // exact while their scaled exponents span <= 34 bits, within fp32 rounding beyond.
    // The decision is per head (the largest column spread of its q, k, v weight groups,
    // uniform over the workgroup).  A workgroup whose row spreads and heads' column spreads
    // are all <= kDigitSpread takes the exponent-folded operands instead (run_dig below).
    bool fast_ok;
    {
      int gsp = 0, glo = 1 << 20;
#pragma unroll
      for (int s3 = 0; s3 < 3; ++s3) {
        const int g = s3 * a.H + h;
        glo = min(glo, (int)a.gs[2 * g]);
        gsp = max(gsp, (int)a.gs[2 * g + 1]);
      }
      // (the digit path's sums are exact at any spread it takes: only the subnormal test)
      fast_ok = (dig || st[0] + gsp <= a.smax) && st[1] + glo >= -126;  // uniform over the workgroup
    }
    const int64_t jcol = (int64_t)s * HD + (int64_t)h * D + dcol;
    const float bb = (a.bias && colv) ? (PLAIN ? a.bias[jcol] : round_bfloat(a.bias[jcol], a.bfloat, kRoundNearest, 1)) : 0.0f;
    // ---- out = bf(fl32(sum)); out = bf(out + bf(bias))  (linear.py:88-101) -------
    // value(i, row_lo): element i's fp32 sum; branch-free: NaN by select; bb = 0 without
    // a bias and o + 0 = o here (o is never -0: an integer sum converts to +0)
    auto store_tile = [&](auto&& value, bool cn) {
      float* orow = ot + m0 * kOst + s * 32 * NBD + dcol;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int4 lo4 = *reinterpret_cast<const int4*>(rlo + 8 * q + m0);
        const int4 rn4 = *reinterpret_cast<const int4*>(rn + 8 * q + m0);
        const int lo[4] = {lo4.x, lo4.y, lo4.z, lo4.w}, nf[4] = {rn4.x, rn4.y, rn4.z, rn4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float o = value(4 * q + r, lo[r]);
          o = (cn || nf[r]) ? __uint_as_float(0x7FC00000u) : o;
          if constexpr (PLAIN) {
            o += bb;
          } else {
            // autocast: F.linear returns the autocast dtype, quantize_elemwise_op rounds that
            // (as mx_gemm's epilogue); + fp32 bias promotes back
            o = round_bfloat(round_dt(o, a.autocast), a.bfloat, kRoundNearest, 1, a.autocast);
            if (a.bias) o = round_bfloat(o + bb, a.bfloat, kRoundNearest, 1);
          }
          orow[(8 * q + r) * kOst] = o;
        }
      }
    };
    // the K loop and the epilogue of the shifted int32 sums (FAST; the fp64 form: run_f64)
    auto run = [&](auto fast_c) {
      constexpr bool FAST = decltype(fast_c)::value;
      static_assert(FAST, "the fp64 sums: run_f64");
      int acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0;
      // Software pipeline over the K-blocks, unrolled by four so that every operand is
      // loaded straight into the register it is consumed from (a rotating copy waits for
      // the load it copies) and reloaded right after its use: the MFMA of block j + 1 is
      // issued before the epilogue of block j, so the matrix core works while the VALU
      // shifts and adds; the weight codes (one coalesced 1-KB load per wave) and the
      // column's block exponent are loaded four blocks ahead, the rows' exponent offsets
      // (LDS) one.  sched_barrier keeps this order (the scheduler otherwise sinks the
      // MFMAs next to the loads they wait for).
      auto ldw = [&](int kb) {
        return __builtin_bit_cast(v4i_, __builtin_amdgcn_raw_buffer_load_b128(wrs, woff, wsoff + kb * 1024, 0));
      };
      auto lew = [&](int kb) { return (int16_t)__builtin_amdgcn_raw_buffer_load_b16(ers, eoff, esoff + kb * 2, 0); };
      auto ldx = [&](int kb) { return *reinterpret_cast<const v4i_*>(xa + 32 * kb); };
      auto lde = [&](int kb, uint2 (&e)[4]) {
        const int16_t* eb = xe + kb * 32 + m0;
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] = *reinterpret_cast<const uint2*>(eb + 8 * q);  // rows 8q + m0 .. + 3
      };
      auto epi = [&](const v16i& c, int16_t e16, const uint2 (&xcur)[4]) {
        int ew = exp_from16(e16);
        cnan = cnan || ew == kExpNaN;
        ew = ew == kExpNaN ? wlo : ew;
        const int ewd = ew - wlo;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint2 e4 = xcur[q];
          const int dx[4] = {(int)(e4.x & 0xFFFFu), (int)(e4.x >> 16), (int)(e4.y & 0xFFFFu), (int)(e4.y >> 16)};
          if constexpr (FAST) {
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[4 * q + r] += (int)((uint32_t)c[4 * q + r] << (dx[r] + ewd));
          } else {
            const int4 lo4 = *reinterpret_cast<const int4*>(rlo + 8 * q + m0);
            const int lo[4] = {lo4.x, lo4.y, lo4.z, lo4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[4 * q + r] += ldexp((double)c[4 * q + r], dx[r] + lo[r] + ew);
          }
        }
      };
      const v16i zero = {};
      const int last = nbk - 1;
      auto cl = [&](int kb) { return min(kb, last); };
      auto mfma = [&](int kb, const v4i_& w) { return __builtin_amdgcn_mfma_i32_32x32x32_i8(ldx(kb), w, zero, 0, 0, 0); };
      // slot s = block mod 4 (weights W*, column exponents E*); cA / cB the two products
      // in flight, xA / xB their rows' exponent offsets
      v4i_ W1 = ldw(cl(1)), W2 = ldw(cl(2)), W3 = ldw(cl(3));
      int16_t E0 = lew(0), E1 = lew(cl(1)), E2 = lew(cl(2)), E3 = lew(cl(3));
      v16i cA = mfma(0, ldw(0)), cB;
      v4i_ W0 = ldw(cl(4));
      uint2 xA[4], xB[4];
      lde(0, xA);
      // step: issue block j + 1 into cN (operand slot W, refilled with block j + 5), then
      // the epilogue of block j from cP (exponent slot E, refilled with block j + 4)
#define MXA_PROJ_STEP(cN, xN, W, cP, xP, E, j)              \
  cN = mfma((j) + 1, W);                                   \
  W = ldw(cl((j) + 5));                                    \
  lde((j) + 1, xN);                                        \
  __builtin_amdgcn_sched_barrier(0);                       \
  epi(cP, E, xP);                                          \
  E = lew(cl((j) + 4));                                    \
  __builtin_amdgcn_sched_barrier(0);
      // whole quads (blocks kb .. kb + 4 all real), one exit at the bottom
      const int nquad = last >> 2;
      int kb = 0;
      for (int p = 0; p < nquad; ++p, kb += 4) {
        MXA_PROJ_STEP(cB, xB, W1, cA, xA, E0, kb)
        MXA_PROJ_STEP(cA, xA, W2, cB, xB, E1, kb + 1)
        MXA_PROJ_STEP(cB, xB, W3, cA, xA, E2, kb + 2)
        MXA_PROJ_STEP(cA, xA, W0, cB, xB, E3, kb + 3)
      }
#undef MXA_PROJ_STEP
      // the last 1 .. 4 blocks kb .. last (cA = block kb in flight)
      const int r = nbk - kb;
      if (r > 1) {
        cB = mfma(kb + 1, W1);
        lde(kb + 1, xB);
      }
      epi(cA, E0, xA);
      if (r > 1) {
        if (r > 2) {
          cA = mfma(kb + 2, W2);
          lde(kb + 2, xA);
        }
        epi(cB, E1, xB);
      }
      if (r > 2) {
        if (r > 3) {
          cB = mfma(kb + 3, W3);
          lde(kb + 3, xB);
        }
        epi(cA, E2, xA);
      }
      if (r > 3) epi(cB, E3, xB);
      store_tile(
          [&](int i, int lo) {
            if constexpr (FAST) return ldexpf((float)acc[i], lo + wlo);
            else return (float)acc[i];
          },
          cnan);
    };
    // Exponent-folded operands (dig): the tile's codes times 2^(block exponent - row's
    // smallest) and the weight's times 2^(block exponent - column's smallest), each as two
    // signed base-256 digits, so every block's scale is already in the operands: the four
    // digit products accumulate in the MFMA's own int32 accumulators over all K-blocks
    // (lo x lo; lo x hi + hi x lo; hi x hi: |sum| <= 2 nbk 32 128^2 < 2^31) with no VALU
    // per block, and sum = c0 + 2^8 c1 + 2^16 c2 (exact in fp64) rounds once.
    auto run_dig = [&]() {
      const auto drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(a.pd), 0, a.pd_bytes, 0x00020000);
      const int dsoff = __builtin_amdgcn_readfirstlane((int)(blkc * nbk) * 2048);
      auto ldd = [&](int kb, int p) {
        return __builtin_bit_cast(v4i_, __builtin_amdgcn_raw_buffer_load_b128(drs, woff, dsoff + ((MXA_PROJ_SKIP & 4) ? 0 : kb * 2048) + p * 1024, 0));
      };
      const int8_t* xha = xh + ln * L.xst + kh;
      const int last = nbk - 1;
      auto cl = [&](int kb) { return min(kb, last); };
      v16i c0 = {}, c1 = {}, c2 = {};
      // weight digits four blocks ahead (slot = block mod 4), the tile's from LDS
      v4i_ L0 = ldd(0, 0), H0 = ldd(0, 1), L1 = ldd(cl(1), 0), H1 = ldd(cl(1), 1);
      v4i_ L2 = ldd(cl(2), 0), H2 = ldd(cl(2), 1), L3 = ldd(cl(3), 0), H3 = ldd(cl(3), 1);
      auto step = [&](int kb, v4i_& Ls, v4i_& Hs) {
        const v4i_ al = *reinterpret_cast<const v4i_*>(xa + 32 * kb);
        const v4i_ ah = *reinterpret_cast<const v4i_*>(xha + 32 * kb);
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
      store_tile(
          [&](int i, int lo) {
            const double v = (double)c0[i] + 256.0 * (double)c1[i] + 65536.0 * (double)c2[i];
            return (float)ldexp(v, lo + wlo);
          },
          a.pn[pc] != 0);
    };
    // the fp64 block sums for a head whose spreads allow neither the digits nor the shifted
    // int32 sums (rare): one K-block at a time, ascending (exact while the scaled blocks span
    // <= 34 bits, within fp32 rounding beyond) -- few registers, so the common paths keep theirs
    auto run_f64 = [&]() {
      double acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.0;
      const v16i zero = {};
      // (a digit tile -- its subnormal test failed -- holds code * 2^xe as two base-256 digits:
      // the block's sum c0 + 256 c1 is then the shifted sum, scaled by the row's base exponent)
      const int8_t* xha = reinterpret_cast<int8_t*>(smem + L.xh) + ln * L.xst + kh;
      for (int kb = 0; kb < nbk; ++kb) {
        const v4i_ w = __builtin_bit_cast(v4i_, __builtin_amdgcn_raw_buffer_load_b128(wrs, woff, wsoff + kb * 1024, 0));
        v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(*reinterpret_cast<const v4i_*>(xa + 32 * kb), w, zero, 0, 0, 0);
        if (dig) {
          const v16i ch = __builtin_amdgcn_mfma_i32_32x32x32_i8(*reinterpret_cast<const v4i_*>(xha + 32 * kb), w, zero, 0, 0, 0);
#pragma unroll
          for (int i = 0; i < 16; ++i) c[i] += ch[i] << 8;
        }
        int ew = exp_from16((int16_t)__builtin_amdgcn_raw_buffer_load_b16(ers, eoff, esoff + kb * 2, 0));
        cnan = cnan || ew == kExpNaN;
        ew = ew == kExpNaN ? wlo : ew;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = 8 * (i >> 2) + m0 + (i & 3);
          const int base = dig ? (rlo[m] > rhi[m] ? 0 : rlo[m]) : (int)xe[kb * 32 + m] + rlo[m];
          acc[i] += ldexp((double)c[i], base + ew);
        }
      }
      store_tile([&](int i, int) { return (float)acc[i]; }, cnan);
    };
    if (MXA_PROJ_SKIP & 1) store_tile([](int, int) { return 0.0f; }, false);
    else if (fast_ok && dig) run_dig();
    else if (fast_ok) run(std::true_type{});
    else run_f64();  // wide spreads or a subnormal result: fp64, in this workgroup

    __syncthreads();
    if (a.qkv_out) {  // the fp32 projection (tests): whole rows of the tile, coalesced
      for (int i = threadIdx.x; i < 32 * 3 * D; i += kThreads) {
        const int m = i / (3 * D), col = i - m * (3 * D), sc = col / D;
        if (m < rows)
          a.qkv_out[(row0 + m) * (3 * HD) + (int64_t)sc * HD + (int64_t)h * D + (col - sc * D)] =
              ot[m * kOst + sc * 32 * NBD + col - sc * D];
      }
    }

    // ---- q and k rows (waves 0 .. 2 NBD - 1) beside V's columns (the other NBD waves:
    // 64 NBD >= D lanes, one column each).  Before, the wave that took the first q rows
    // then took V as well while the rest waited at the barrier.
    const int64_t hrow0 = (hrow_b + h) * a.N + n0;  // row of (b, h, n0) in the q / k tables
    constexpr int kPer = 32 * NBD * 2;              // lanes per sub-matrix: a multiple of 64
    static_assert(kThreads - 2 * kPer == 64 * NBD, "V lanes");
    if (MXA_PROJ_SKIP & 2) {
    } else if ((int)threadIdx.x < 2 * kPer) {
      // rows_prep's per-block body on the tile (2 lanes per 32-element block)
      const int t = (int)threadIdx.x;
      const int sk = __builtin_amdgcn_readfirstlane(t / kPer);  // uniform per wave: q or k
      const int rem = t - sk * kPer;
      const int g = rem >> 1, sub = rem & 1;
      const int m = g / NBD, blk = g - m * NBD;
      const int c0 = 32 * blk + 16 * sub;
      float xv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) xv[j] = c0 + j < D ? ot[m * kOst + sk * 32 * NBD + c0 + j] : 0.0f;
      const RowsPrepArgs& ra = sk ? a.rk : a.rq;
      if constexpr (PLAIN) {
        rows_prep_block_plain<16, kF32>(ra, hrow0 + m, blk, sub, c0, xv, m < rows);
      } else {
        if (rows_prep_plain(ra)) rows_prep_block_plain<16>(ra, hrow0 + m, blk, sub, c0, xv, m < rows);
        else rows_prep_block<16>(ra, hrow0 + m, blk, sub, c0, xv, m < rows);
      }
    } else if (const int c = (int)threadIdx.x - 2 * kPer; c < D) {
      // V: cols_prep's per-column body over the 32 tokens
      float xv[32];
      uint32_t mx = 0;
#pragma unroll
      for (int j = 0; j < 32; ++j) {
        const float v = j >= rows ? 0.0f : PLAIN ? ot[j * kOst + 64 * NBD + c]
                                                 : round_bfloat(ot[j * kOst + 64 * NBD + c], a.cv.bfloat, kRoundNearest, 1);
        xv[j] = v;
        const uint32_t ub = __float_as_uint(v) & 0x7FFFFFFFu;
        mx = ub > mx ? ub : mx;
      }
      cols_prep_column<PLAIN, PLAIN ? kF32 : -1>(a.cv, hrow_b + h, tb, c, xv, mx);
    }
    __syncthreads();
  }
}

template <int NBD, bool PLAIN>
__global__ __launch_bounds__(64 * 3 * NBD) __attribute__((amdgpu_waves_per_eu(4, 8))) void qkv_proj_kernel(ProjArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  proj_block<NBD, PLAIN>(a, blockIdx.x, blockIdx.y, (int)blockIdx.z * a.hpg,
                                min(a.H, ((int)blockIdx.z + 1) * a.hpg), smem);
}

}  // namespace mxa
