// Per-block bodies of the attention operand builders, shared by the standalone
// prep kernels (mxa_quant.hip) and the fused qkv projection (mxa_proj.hpp).
#pragma once
#include <type_traits>
#include "mxa_kernels.hpp"

namespace mxa {

// ---------------------------------------------------------------------------
// attention operand builder for rows quantized along the last axis (Q, K)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int exion_m(int raw) {
  // two_step_leading_ones on an integer code (funcs/exponent_based_prediction.py:110-127):
  //   l1 = floor(log2|raw|), t = max(raw - 2^l1, 0) (signed!), l2 = floor(log2 t),
  //   approx = sign(raw) * e * (2^l1 + 2^l2) / 64   (2^-126 terms vanish in fp32)
  if (raw == 0) return 0;
  if (raw < 0) return -(1 << (31 - __clz(-raw)));
  const int p1 = 1 << (31 - __clz(raw));
  const int t = raw - p1;
  return p1 + (t > 0 ? (1 << (31 - __clz(t))) : 0);
}

// reduction over the LPB consecutive lanes that share one 32-element block
template <int LPB, class Op>
__device__ __forceinline__ uint32_t blk_reduce(uint32_t v, Op op) {
  v = op(v, dpp_u32<0xB1>(v));  // quad_perm [1,0,3,2]
  if constexpr (LPB >= 4) v = op(v, dpp_u32<0x4E>(v));   // quad_perm [2,3,0,1]
  if constexpr (LPB >= 8) v = op(v, dpp_u32<0x141>(v));  // row_half_mirror
  return v;
}

// where the EPL codes of lane `sub` of a block go: row-major (row * dpad + c0), or with
// a.mfma_rows (EPL >= 8) the MX GEMM's MFMA-ready A layout -- per 32-row block and
// K-block, 64 lanes x 16 B, lane (row & 31) + 32 h holding elements 16 h .. 16 h + 15
template <int EPL>
__device__ __forceinline__ int64_t mfma_base(const RowsPrepArgs& a, int64_t row, int blk, int sub, int c0) {
  if (EPL >= 8 && a.mfma_rows) {
    const int e0 = EPL * sub;  // first element of the lane within the block
    return (((row >> 5) * a.nb + blk) * 64 + (row & 31) + 32 * (e0 >> 4)) * 16 + (e0 & 15);
  }
  return row * a.dpad + c0;
}

// One 32-element block of a row, 32/EPL lanes x EPL elements (lane sub of its group,
// c0 = 32 blk + EPL sub): MXINT8 codes, block exponent, approximator operand and sign
// word into the RowsPrepArgs outputs (row `row`, block `blk`).  The lanes of a group
// must be consecutive and all call it (DPP reductions).  EPL = 16: the standalone
// prep (two lanes per block: the per-block work is shared by 2 lanes, not 8);
// EPL = 4: the fused projection's tile epilogue.
template <int EPL>
__device__ __forceinline__ void rows_prep_block(const RowsPrepArgs& a, int64_t row, int blk, int sub, int c0,
                                                float xv[EPL], bool valid) {
  constexpr int LPB = 32 / EPL;
  uint32_t mb = 0;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    xv[j] = round_bfloat(xv[j], a.bfloat, kRoundNearest, 1, a.dt);
    const uint32_t ub = __float_as_uint(xv[j]) & 0x7FFFFFFFu;
    mb = ub > mb ? ub : mb;
  }
  mb = blk_reduce<LPB>(mb, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
  int e_raw;
  const int es = scale_exponent_dt(mb, 127, a.dt, &e_raw);
  const bool nanblk = es == kExpNaN;
  if (a.flush && !(e_raw != kExpNaN && e_raw > -127)) {
#pragma unroll
    for (int j = 0; j < EPL; ++j) xv[j] = xv[j] * 0.0f;
  }
  int code[EPL];
  int maxc = 0;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    code[j] = nanblk ? 0 : (int)round_code(xv[j], es, 8, kRoundNearest, a.dt);
    const int ac = code[j] < 0 ? -code[j] : code[j];
    maxc = ac > maxc ? ac : maxc;
  }
  maxc = (int)blk_reduce<LPB>((uint32_t)maxc, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
  // exponent of the MX-quantized block (funcs/exponent_based_prediction.py:35-36):
  // floor(log2(max |MX|)), unclamped, in the dtype; MX max = maxc * 2^(es-6) (a value
  // of the dtype: exact in float32 / bfloat16, and in float16 for es >= -18)
  int eA;
  if (nanblk) eA = kExpNaN;
  else if (maxc == 0) eA = -126;
  else eA = floor_log2_dt(__float_as_uint(round_dt((float)maxc * pow2f(es - 6), a.dt)), a.dt);
  int op[EPL];
  int sA;
  switch (a.op_kind) {
    case MXA_OP_SIGN:
#pragma unroll
      for (int j = 0; j < EPL; ++j) op[j] = (c0 + j < a.D) ? (code[j] < 0 ? -1 : 1) : 0;
      sA = eA;
      break;
    case MXA_OP_MXINT4:
#pragma unroll
      for (int j = 0; j < EPL; ++j) op[j] = nanblk ? 0 : (int)round_code(xv[j], es, 4, kRoundNearest, a.dt);
      sA = nanblk ? kExpNaN : es - 2;
      break;
    case MXA_OP_EXION: {
      const int sh = nanblk ? 0 : es - eA;  // MX / 2^eA * 64 = code * 2^(es-eA), an integer < 128
#pragma unroll
      for (int j = 0; j < EPL; ++j) op[j] = nanblk ? 0 : exion_m(code[j] << sh);
      sA = eA;
      break;
    }
    case MXA_OP_TRUE_EX:
      // exponent_based_sign_leading_ones (examples/deit/exponent_based_prediction.py:163-178):
      // (mx < 0 ? -1 : 1) * 2^floor(log2|mx|), zeros -> +1.  Nonzero elements as the
      // power-of-two code sign * 2^floor(log2|code|) in units of 2^(es-6); zeros in zind
#pragma unroll
      for (int j = 0; j < EPL; ++j) {
        const int ac = code[j] < 0 ? -code[j] : code[j];
        const int p2 = ac ? 1 << (31 - __clz(ac)) : 0;
        op[j] = code[j] < 0 ? -p2 : p2;
      }
      // a NaN block's MX values are NaN, and get_true_exponents maps them like zeros
      // (mask |x| > 0 is false: exponent 0, value +1; examples :98-110): codes 0, zind 1
      sA = nanblk ? 0 : es - 6;
      break;
    default:  // MXA_OP_MXINT8
#pragma unroll
      for (int j = 0; j < EPL; ++j) op[j] = code[j];
      sA = nanblk ? kExpNaN : es - 6;
      break;
  }
  if (valid) {
    const int64_t base = mfma_base<EPL>(a, row, blk, sub, c0);
    uint32_t pc[EPL / 4], po[EPL / 4], pz[EPL / 4];
#pragma unroll
    for (int w = 0; w < EPL / 4; ++w) {
      pc[w] = po[w] = pz[w] = 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pc[w] |= (uint32_t)(code[4 * w + j] & 0xFF) << (8 * j);
        po[w] |= (uint32_t)(op[4 * w + j] & 0xFF) << (8 * j);
        pz[w] |= (c0 + 4 * w + j < a.D && code[4 * w + j] == 0 ? 1u : 0u) << (8 * j);
      }
    }
    if constexpr (EPL == 16) {
      if (a.codes) *reinterpret_cast<uint4*>(a.codes + base) = make_uint4(pc[0], pc[1], pc[2], pc[3]);
      if (a.op) *reinterpret_cast<uint4*>(a.op + base) = make_uint4(po[0], po[1], po[2], po[3]);
      if (a.zind) *reinterpret_cast<uint4*>(a.zind + base) = make_uint4(pz[0], pz[1], pz[2], pz[3]);
    } else if constexpr (EPL == 8) {
      if (a.codes) *reinterpret_cast<uint2*>(a.codes + base) = make_uint2(pc[0], pc[1]);
      if (a.op) *reinterpret_cast<uint2*>(a.op + base) = make_uint2(po[0], po[1]);
      if (a.zind) *reinterpret_cast<uint2*>(a.zind + base) = make_uint2(pz[0], pz[1]);
    } else {
      if (a.codes) *reinterpret_cast<uint32_t*>(a.codes + base) = pc[0];
      if (a.op) *reinterpret_cast<uint32_t*>(a.op + base) = po[0];
      if (a.zind) *reinterpret_cast<uint32_t*>(a.zind + base) = pz[0];
    }
  }
  // packed sign word of the block, bit (EPL*sub + j) = (code < 0): the exp-sign
  // operand of ex_pred (codes beyond D are 0, i.e. positive)
  uint32_t sw = 0u;
#pragma unroll
  for (int j = 0; j < EPL; ++j) sw |= (code[j] < 0 ? 1u : 0u) << (EPL * sub + j);
  sw = blk_reduce<LPB>(sw, [](uint32_t u, uint32_t w) { return u | w; });
  if (valid && sub == 0) {
    if (a.sT) a.sT[row * a.nb + blk] = exp_to16(nanblk ? kExpNaN : es - 6);
    if (a.sA) a.sA[row * a.nb + blk] = exp_to16(sA);
    if (a.signs) a.signs[row * a.nb + blk] = sw;
  }
}

// rows_prep_block for the plain case -- no bfloat rounding, no subnormal flush, no
// true_ex zero indicators, approximator operand the sign (ex_pred) or the MXINT8 code --
// with the int8 code path of q8_code: the same outputs in about a third of the VALU
// (the prep launch is VALU-bound next to its HBM stream otherwise)
__device__ __forceinline__ bool rows_prep_plain(const RowsPrepArgs& a) {
  return (a.bfloat == 0 || a.bfloat == 32) && !a.flush && !a.zind &&
         (a.op_kind == MXA_OP_MXINT8 || (a.op_kind == MXA_OP_SIGN && !a.op));
}
// DT >= 0: the storage dtype known at compile time (the fused projection: float32)
template <int EPL, int DT = -1>
__device__ __forceinline__ void rows_prep_block_plain(const RowsPrepArgs& a, int64_t row, int blk, int sub, int c0,
                                                      const float xv[EPL], bool valid) {
  constexpr int LPB = 32 / EPL;
  const int dt = DT >= 0 ? DT : a.dt;
  uint32_t mb = 0;
#pragma unroll
  for (int j = 0; j < EPL; ++j) mb = max(mb, __float_as_uint(xv[j]) & 0x7FFFFFFFu);
  mb = blk_reduce<LPB>(mb, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
  int e_raw;
  const int es = scale_exponent_dt(mb, 127, dt, &e_raw);
  const bool nanblk = es == kExpNaN;
  int code[EPL];
  auto quant = [&](auto tiny) {
    const float s = q8_scale(es);
#pragma unroll
    for (int j = 0; j < EPL; ++j) code[j] = q8_code<decltype(tiny)::value>(xv[j], s, dt);
  };
  if (nanblk) {
#pragma unroll
    for (int j = 0; j < EPL; ++j) code[j] = 0;
  } else if (es >= -121) {
    quant(std::false_type{});
  } else {
    quant(std::true_type{});
  }
  int maxc = 0;
  uint32_t sw = 0u;
#pragma unroll
  for (int j = 0; j < EPL; ++j) {
    maxc = max(maxc, abs(code[j]));
    sw |= (code[j] < 0 ? 1u : 0u) << (EPL * sub + j);
  }
  maxc = (int)blk_reduce<LPB>((uint32_t)maxc, [](uint32_t u, uint32_t w) { return u > w ? u : w; });
  sw = blk_reduce<LPB>(sw, [](uint32_t u, uint32_t w) { return u | w; });
  if (valid) {
    uint32_t pc[EPL / 4];
#pragma unroll
    for (int w = 0; w < EPL / 4; ++w)
      pc[w] = (uint32_t)(code[4 * w] & 0xFF) | (uint32_t)(code[4 * w + 1] & 0xFF) << 8 |
              (uint32_t)(code[4 * w + 2] & 0xFF) << 16 | (uint32_t)code[4 * w + 3] << 24;
    const int64_t base = mfma_base<EPL>(a, row, blk, sub, c0);
    if constexpr (EPL == 16) {
      const uint4 v = make_uint4(pc[0], pc[1], pc[2], pc[3]);
      if (a.codes) *reinterpret_cast<uint4*>(a.codes + base) = v;
      if (a.op) *reinterpret_cast<uint4*>(a.op + base) = v;  // MXA_OP_MXINT8 (SIGN has none)
    } else if constexpr (EPL == 8) {
      const uint2 v = make_uint2(pc[0], pc[1]);
      if (a.codes) *reinterpret_cast<uint2*>(a.codes + base) = v;
      if (a.op) *reinterpret_cast<uint2*>(a.op + base) = v;
    } else {
      if (a.codes) *reinterpret_cast<uint32_t*>(a.codes + base) = pc[0];
      if (a.op) *reinterpret_cast<uint32_t*>(a.op + base) = pc[0];
    }
    if (sub == 0) {
      // exponent of the MX-quantized block (funcs/exponent_based_prediction.py:35-36):
      // floor(log2(maxc * 2^(es-6))) = floor(log2 maxc) + es - 6 exactly (maxc <= 127)
      int eA = nanblk ? kExpNaN : (maxc == 0 ? -126 : 31 - __clz(maxc) + es - 6);
      if (dt != kF32 && !nanblk && maxc != 0)  // log2 rounded to the dtype
        eA = floor_log2_dt(__float_as_uint(round_dt((float)maxc * pow2f(es - 6), dt)), dt);
      if (a.sT) a.sT[row * a.nb + blk] = exp_to16(nanblk ? kExpNaN : es - 6);
      if (a.sA) a.sA[row * a.nb + blk] = exp_to16(a.op_kind == MXA_OP_SIGN ? eA : (nanblk ? kExpNaN : es - 6));
      if (a.signs) a.signs[row * a.nb + blk] = sw;
    }
  }
}

// ---------------------------------------------------------------------------
// operand builder for matrices quantized along the row axis (V, and in2 of
// mx.matmul): blocks of 32 rows per column; output transposed [col][row] codes.
// ---------------------------------------------------------------------------
// One 32-row block of one column (m = matrix, blk, column c) from its 32 values
// (already bfloat-rounded, zero beyond the matrix): codes into the transposed
// [m][C][rpad] table, the exponent into [m][nb][C].  PLAIN: MXINT8, no flush (the
// caller checked), DT >= 0 the storage dtype known at compile time.
template <bool PLAIN = false, int DT = -1>
__device__ __forceinline__ void cols_prep_column(const ColsPrepArgs& a, int64_t m, int blk, int c, const float xv[32],
                                                 uint32_t mx) {
  const int r0 = blk * 32;
  const int dt = DT >= 0 ? DT : a.dt;
  int e_raw;
  const int es = scale_exponent_dt(mx, 127, dt, &e_raw);
  const bool nanblk = es == kExpNaN;
  const bool flush = !PLAIN && a.flush && !(e_raw != kExpNaN && e_raw > -127);
  const int mbits = PLAIN ? 8 : a.mbits;
  uint32_t w[8];
  if (PLAIN && nanblk) {
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = 0u;
  } else if (!flush && !nanblk && mbits == 8) {  // the plain MXINT8 case: q8_code
    const float s = q8_scale(es);
    auto quant = [&](auto tiny) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        int cd[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) cd[j] = q8_code<decltype(tiny)::value>(xv[q * 4 + j], s, dt);
        w[q] = (uint32_t)(cd[0] & 0xFF) | (uint32_t)(cd[1] & 0xFF) << 8 | (uint32_t)(cd[2] & 0xFF) << 16 |
               (uint32_t)cd[3] << 24;
      }
    };
    if (es >= -121) quant(std::false_type{});
    else quant(std::true_type{});
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint32_t acc = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = xv[q * 4 + j];
        if (flush) v = v * 0.0f;
        const int cd = nanblk ? 0 : (int)round_code(v, es, mbits, kRoundNearest, dt);
        acc |= (uint32_t)(cd & 0xFF) << (8 * j);
      }
      w[q] = acc;
    }
  }
  int8_t* dst = a.tb_major ? a.codes_t + ((m * a.nb + blk) * a.C + c) * 32 : a.codes_t + (m * a.C + c) * a.rpad + r0;
  uint4* d4 = reinterpret_cast<uint4*>(dst);
  d4[0] = make_uint4(w[0], w[1], w[2], w[3]);
  d4[1] = make_uint4(w[4], w[5], w[6], w[7]);
  a.scale[(m * a.nb + blk) * a.C + c] = exp_to16(nanblk ? kExpNaN : es - (mbits - 2));
}


}  // namespace mxa
