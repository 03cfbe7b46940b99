// MX quantization kernels for gfx950 (wave64).
//
//   mxa_quantize_mx        generic quantize_mx_op replacement (mx_ops.py:180-341)
//   mxa_shared_exponents   _shared_exponents replacement      (mx_ops.py:49-99)
//   mxa_quantize_bfloat    quantize_elemwise_op (bfloat)      (elemwise_ops.py:201-277)
//   mxa_approx_values      exponent_approximation operands    (funcs/exponent_based_prediction.py)
//   rows_prep / cols_prep  the attention path's operand builders (int8 codes + block
//                          exponents + approximator operands), used by mxa_attn.hip
//
// All of it is HBM-bound byte work: coalesced fp32 loads, 32-element blocks
// reduced with lane shuffles, int8 codes + int16 block exponents written out.
#include "mxa_kernels.hpp"
#include "mxa_prep.hpp"

#include <algorithm>

namespace mxa {

// ---------------------------------------------------------------------------
// generic MX quantize of a (outer, L, inner) tensor, one thread per block
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void quantize_mx_kernel(QuantArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nblocks = a.outer * a.nb * a.inner;
  if (t >= nblocks) return;
  const int64_t i = t % a.inner;
  const int64_t ob = t / a.inner;
  const int64_t blk = ob % a.nb;
  const int64_t o = ob / a.nb;
  const int64_t l0 = blk * a.bs;
  const int64_t l1 = (l0 + a.bs < a.L) ? l0 + a.bs : a.L;
  const int64_t xp = (o * a.L) * a.inner + i;
  uint32_t mb = 0;
  for (int64_t l = l0; l < l1; ++l) {
    const float xv = round_bfloat(load_dt(a.x, xp + l * a.inner, a.dt), a.bfloat, kRoundNearest, 1, a.dt);
    const uint32_t ub = __float_as_uint(xv) & 0x7FFFFFFFu;
    mb = ub > mb ? ub : mb;
  }
  int e_raw;
  const int es = scale_exponent_dt(mb, a.scale_emax, a.dt, &e_raw);
  const bool flush = a.flush && !(e_raw != kExpNaN && e_raw > -127);
  const int shift = a.mbits - 2;
  for (int64_t l = l0; l < l1; ++l) {
    float xv = round_bfloat(load_dt(a.x, xp + l * a.inner, a.dt), a.bfloat, kRoundNearest, 1, a.dt);
    if (flush) xv = xv * 0.0f;
    float yv, cv = 0.0f;
    if (es == kExpNaN) {
      yv = __uint_as_float(0x7FC00000u);
    } else {
      cv = round_code(xv, es, a.mbits, a.rnd, a.dt);
      yv = (cv * pow2f(-shift)) * pow2f(es);
    }
    const int64_t off = (o * a.L + l) * a.inner + i;
    store_dt(a.y, off, yv, a.dt);  // (code * 2^(es-shift) rounded once to the dtype)
    if (a.codes) a.codes[off] = (int8_t)cv;
  }
  if (a.exps) a.exps[(o * a.nb + blk) * a.inner + i] = exp_to16(es);
}

// ---------------------------------------------------------------------------
// shared exponents (method "max" per block, or "none" per element)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float sexp_value(uint32_t ub, int ebits, int dt) {
  int e = floor_log2_dt(ub & 0x7FFFFFFFu, dt);
  float v;
  if (e == kExpZeroF16) {
    v = -INFINITY;  // float16: 2^-126 underflows, log2(0) = -inf
  } else if (e == kExpNaN) {
    // log2(inf) = inf -> floor = inf; NaN stays NaN
    v = ((ub & 0x7FFFFFFFu) == 0x7F800000u) ? INFINITY : __uint_as_float(0x7FC00000u);
  } else {
    v = (float)e;
  }
  if (ebits > 0) {
    const float emax = (float)((1 << (ebits - 1)) - 1);
    if (v > emax) v = __uint_as_float(0x7FC00000u);
    else if (v < -emax) v = -emax;
  }
  return v;
}

__global__ __launch_bounds__(256) void shared_exp_kernel(SexpArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a.method == 1) {  // none: elementwise
    const int64_t n = a.outer * a.L * a.inner;
    if (t >= n) return;
    store_dt(a.out, t, sexp_value(__float_as_uint(load_dt(a.x, t, a.dt)) & 0x7FFFFFFFu, a.ebits, a.dt), a.dt);
    return;
  }
  const int64_t nblocks = a.outer * a.nb * a.inner;
  if (t >= nblocks) return;
  const int64_t i = t % a.inner;
  const int64_t ob = t / a.inner;
  const int64_t blk = ob % a.nb;
  const int64_t o = ob / a.nb;
  const int64_t l0 = blk * a.bs;
  const int64_t l1 = (l0 + a.bs < a.L) ? l0 + a.bs : a.L;
  uint32_t mb = 0;
  for (int64_t l = l0; l < l1; ++l) {
    const uint32_t ub = __float_as_uint(load_dt(a.x, (o * a.L + l) * a.inner + i, a.dt)) & 0x7FFFFFFFu;
    mb = ub > mb ? ub : mb;  // NaN bits compare above Inf: max propagates NaN like torch.max
  }
  store_dt(a.out, t, sexp_value(mb, a.ebits, a.dt), a.dt);
}

// ---------------------------------------------------------------------------
// elementwise bfloat quantization (vectorized, grid-stride)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bfloat_kernel(const void* __restrict__ x, void* __restrict__ y, int64_t n,
                                                     int bfloat, int rnd, int allow_denorm, int dt) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride)
    store_dt(y, t, round_bfloat(load_dt(x, t, dt), bfloat, rnd, allow_denorm, dt), dt);
}

// ---------------------------------------------------------------------------
// attention operand builder for rows quantized along the last axis (Q, K):
// 8 lanes per 32-element block, 4 floats (16 B) per lane (body: mxa_prep.hpp)
// ---------------------------------------------------------------------------
// 16 consecutive elements of a row (from element c0) of storage dtype DT as floats
// (float32: 16-B loads at any 4-B alignment -- rows of a length that is not a multiple of 4,
// such as the drop-in's 197-key P rows, take global_load_dwordx4 too: gfx950 executes
// dword-aligned 16-B global loads; the vector type states the 4-B alignment)
typedef float f32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
template <int DT>
__device__ __forceinline__ void load_row16(const void* xr, int c0, int D, bool vec, bool valid, float xv[16]) {
  if constexpr (DT == kF32) {
    const float* x = static_cast<const float*>(xr);
    if (valid && c0 + 16 <= D) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4_a4 v = *reinterpret_cast<const f32x4_a4*>(x + c0 + 4 * q);
        xv[4 * q] = v.x; xv[4 * q + 1] = v.y; xv[4 * q + 2] = v.z; xv[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) xv[j] = (valid && c0 + j < D) ? x[c0 + j] : 0.0f;
    }
  } else {
    const uint16_t* x = static_cast<const uint16_t*>(xr);
    auto cvt = [](uint16_t h) { return DT == kF16 ? f16_bits_to_f(h) : bf16_bits_to_f(h); };
    if (valid && vec && c0 + 16 <= D) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const uint4 v = *reinterpret_cast<const uint4*>(x + c0 + 8 * q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          xv[8 * q + 2 * t] = cvt((uint16_t)(w[t] & 0xFFFFu));
          xv[8 * q + 2 * t + 1] = cvt((uint16_t)(w[t] >> 16));
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) xv[j] = (valid && c0 + j < D) ? cvt(x[c0 + j]) : 0.0f;
    }
  }
}

template <int DT>
__device__ __forceinline__ void rows_prep_body(const RowsPrepArgs& a, uint32_t bid) {
  // two lanes per 32-element block, 16 elements per lane; 32-bit index math
  // (the launcher checks rows * nb < 2^31): a 64-bit division is a ~50-instruction
  // software sequence per thread, 32-bit ~10
  const uint32_t gt = bid * 256u + threadIdx.x;
  const int sub = threadIdx.x & 1;
  const uint32_t g = gt >> 1;
  const uint32_t ngroups = (uint32_t)(a.rows * a.nb);
  const bool valid = g < ngroups;
  const uint32_t nb = (uint32_t)a.nb, R = (uint32_t)a.R, H = (uint32_t)a.H;
  const uint32_t row32 = valid ? g / nb : 0u;
  const int64_t row = row32;
  const int blk = valid ? (int)(g - row32 * nb) : 0;
  const uint32_t bh32 = row32 / R;
  const int64_t r = row32 - bh32 * R;
  const uint32_t b32 = bh32 / H;
  const int64_t h = bh32 - b32 * H;
  const int64_t b = b32;
  constexpr int esz = DT == kF32 ? 4 : 2;
  const void* xr = static_cast<const char*>(a.x) + (b * a.s0 + h * a.s1 + r * a.s2) * esz;
  const int c0 = blk * 32 + sub * 16;
  float xv[16];
  load_row16<DT>(xr, c0, a.D, a.vec4, valid, xv);
  if (rows_prep_plain(a)) rows_prep_block_plain<16>(a, row, blk, sub, c0, xv, valid);
  else rows_prep_block<16>(a, row, blk, sub, c0, xv, valid);
}
template <int DT>
__global__ __launch_bounds__(256) void rows_prep_kernel(RowsPrepArgs a) { rows_prep_body<DT>(a, blockIdx.x); }

// ---------------------------------------------------------------------------
// operand builder for matrices quantized along the row axis (V, and in2 of
// mx.matmul): one thread per (matrix, block, column), coalesced along columns
// ---------------------------------------------------------------------------
template <int DT>
__device__ __forceinline__ void cols_prep_body(const ColsPrepArgs& a, uint32_t bid) {
  // 32-bit index math (the launcher checks the thread count fits)
  const uint32_t t = bid * 256u + threadIdx.x;
  const uint32_t total = (uint32_t)(a.mats * a.nb * a.C);
  if (t >= total) return;
  const uint32_t C = (uint32_t)a.C, NB = (uint32_t)a.nb, H = (uint32_t)a.H;
  const uint32_t mb_ = t / C;
  const int c = (int)(t - mb_ * C);
  const uint32_t m32 = mb_ / NB;
  const int blk = (int)(mb_ - m32 * NB);
  const uint32_t b32 = m32 / H;
  const int64_t m = m32;
  const int64_t h = m32 - b32 * H;
  const int64_t b = b32;
  const int64_t base = b * a.s0 + h * a.s1 + c;
  const int r0 = blk * 32;
  float xv[32];
  uint32_t mx = 0;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int rr = r0 + j;
    float v = rr < a.R ? load_dt(a.x, base + (int64_t)rr * a.s2, DT) : 0.0f;
    v = round_bfloat(v, a.bfloat, kRoundNearest, 1, DT);
    xv[j] = v;
    const uint32_t ub = __float_as_uint(v) & 0x7FFFFFFFu;
    mx = ub > mx ? ub : mx;
  }
  cols_prep_column(a, m, blk, c, xv, mx);
}
template <int DT>
__global__ __launch_bounds__(256) void cols_prep_kernel(ColsPrepArgs a) { cols_prep_body<DT>(a, blockIdx.x); }

// The attention path's three operand builders in ONE launch (no launch gaps / tails
// between them): blocks [0, nq) quantize Q rows, [nq, nq + nk) K rows, the rest V
// columns.  The role is uniform per workgroup.
template <int DT>
__global__ __launch_bounds__(256) void attn_prep_kernel(RowsPrepArgs q, RowsPrepArgs k, ColsPrepArgs v, uint32_t nq,
                                                        uint32_t nk) {
  const uint32_t b = blockIdx.x;
  if (b < nq) rows_prep_body<DT>(q, b);
  else if (b < nq + nk) rows_prep_body<DT>(k, b - nq);
  else cols_prep_body<DT>(v, b - nq - nk);
}

// ---------------------------------------------------------------------------
// ELSA hashes / key norms (funcs/elsa_approximation.py:105-112, :126), one wave
// per row: lane j (and j + 64) forms projected_j = sum_i MX_i * P[j][i] with P^T
// staged in LDS (lane-contiguous reads), MX_i = code_i * 2^e exact in fp64, the
// products exact in fp64 (8 x 24 bits); hash bit j = (projected_j >= 0) by ballot.
// norm = sqrt(exact sum of MX_i^2) rounded once (torch.norm's result on these rows).
// ---------------------------------------------------------------------------
constexpr int kElsaWaves = 4;
__global__ __launch_bounds__(64 * kElsaWaves) void elsa_prep_kernel(ElsaPrepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* pt = reinterpret_cast<float*>(smem);  // pt[i * D + j] = P[j][i]
  const int D = a.D;
  for (int t = threadIdx.x; t < D * D; t += blockDim.x) {
    const int j = t / D, i = t - j * D;
    pt[i * D + j] = a.proj[t];
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * kElsaWaves + wave; row < a.rows; row += (int64_t)gridDim.x * kElsaWaves) {
    const int8_t* cr = a.codes + row * a.dpad;
    double acc0 = 0.0, acc1 = 0.0, nrm = 0.0;
    bool nan = false;
    for (int b = 0; b < a.nb; ++b) {
      const int e = exp_from16(a.sT[row * a.nb + b]);
      nan = nan || e == kExpNaN;
      const double s = nan ? 0.0 : pow2d(e);
      const int i1 = min(32, D - 32 * b);
      for (int ii = 0; ii < i1; ++ii) {
        const int i = 32 * b + ii;
        const double x = (double)cr[i] * s;  // uniform
        nrm += x * x;
        acc0 += x * (double)pt[i * D + min(lane, D - 1)];
        if (D > 64) acc1 += x * (double)pt[i * D + min(lane + 64, D - 1)];
      }
    }
    const uint64_t h0 = __builtin_amdgcn_ballot_w64(!nan && lane < D && acc0 >= 0.0);
    const uint64_t h1 = __builtin_amdgcn_ballot_w64(!nan && lane + 64 < D && acc1 >= 0.0);
    if (lane < a.nb) {
      const uint64_t h = lane < 2 ? h0 : h1;
      a.hash[row * a.nb + lane] = (uint32_t)((lane & 1) ? h >> 32 : h);
    }
    if (a.norm && lane == 0) a.norm[row] = nan ? __uint_as_float(0x7FC00000u) : (float)sqrt(nrm);
  }
}

// ---------------------------------------------------------------------------
// approximator operand VALUES (what exponent_approximation's methods return)
// one lane per element, 32 lanes per (row, 32-block): coalesced loads and stores, the
// block's max |x| and max |code| by lane shuffles; exact fp32 op order of the reference.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lanes32_max(uint32_t v) {
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) {
    const uint32_t w = (uint32_t)__shfl_xor((int)v, o);
    v = v > w ? v : w;
  }
  return v;
}

__global__ __launch_bounds__(256) void approx_values_kernel(ApproxArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nb = (a.d + 31) / 32;
  const int64_t bid = t >> 5;
  const int j = (int)(t & 31);
  const bool live = bid < a.rows * nb;  // every lane takes part in the shuffles
  const int64_t row = live ? bid / nb : 0;
  const int blk = live ? (int)(bid % nb) : 0;
  const int c = blk * 32 + j;
  const bool valid = live && c < a.d;
  const int dt = a.dt;
  const float xin = valid ? round_bfloat(load_dt(a.x, row * a.ld_x + c, dt), a.bfloat, kRoundNearest, 1, dt) : 0.0f;
  const uint32_t mb = lanes32_max(__float_as_uint(xin) & 0x7FFFFFFFu);
  int e_raw;
  const int es = scale_exponent_dt(mb, 127, dt, &e_raw);
  const bool nanblk = es == kExpNaN;
  const bool flush = a.flush && !(e_raw != kExpNaN && e_raw > -127);
  const float qnan = __uint_as_float(0x7FC00000u);
  const float xv = flush ? xin * 0.0f : xin;
  const int cd = nanblk ? 0 : (int)round_code(xv, es, 8, kRoundNearest, dt);
  const int maxc = (int)lanes32_max((uint32_t)(cd < 0 ? -cd : cd));
  // exponent of the MX block (in the dtype: the MX max is a value of the dtype)
  const int eA = nanblk ? kExpNaN
                        : (maxc == 0 ? -126 : floor_log2_dt(__float_as_uint(round_dt((float)maxc * pow2f(es - 6), dt)), dt));
  if (!valid) return;
  float out;
  if (nanblk) {
    out = a.op_kind == MXA_OP_TRUE_EX ? 1.0f : qnan;  // true_ex: NaN -> exponent 0 -> +1 (examples :98-110)
  } else if (a.op_kind == MXA_OP_MXINT4) {
    out = (round_code(xv, es, 4, kRoundNearest, dt) * 0.25f) * pow2f(es);
  } else {
    const float mxv = round_dt(((float)cd * pow2f(-6)) * pow2f(es), dt);  // MX int8 value
    switch (a.op_kind) {
      case MXA_OP_SIGN:  // (mx < 0 ? -1 : +1) * 2^eA
        out = (mxv < 0.0f ? -1.0f : 1.0f) * pow2f(eA);
        break;
      case MXA_OP_EXION: {  // sign(mx) * eA * (2^l1 + 2^l2) / 64
        const int m = exion_m(cd << (es - eA));
        const float sg = cd > 0 ? 1.0f : (cd < 0 ? -1.0f : 0.0f);
        out = ((sg * (float)eA) * (float)(m < 0 ? -m : m)) / 64.0f;
        break;
      }
      case MXA_OP_TRUE_EX: {  // (mx < 0 ? -1 : +1) * 2^(floor(log2|mx|)), zeros -> 2^0
        const float am = fabsf(mxv);
        const int te = am > 0.0f ? floor_log2_dt(__float_as_uint(am), dt) : 0;
        out = (mxv < 0.0f ? -1.0f : 1.0f) * pow2f(te);
        break;
      }
      default:
        out = mxv;
    }
  }
  store_dt(a.out, row * a.ld_out + c, round_dt(out, dt), dt);
}

// approx_values_kernel for float32 rows of whole 32-element blocks at 16-B aligned
// strides: eight lanes per block, four elements per lane (one float4 load and store),
// the block maxima over the eight lanes by DPP, 32-bit index math -- the same values
// (it is HBM-bound: 8 bytes per element)
template <int OPK>
__global__ __launch_bounds__(256) void approx_values_v4_kernel(ApproxArgs a) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  const uint32_t gid = t >> 3, nb = (uint32_t)(a.d >> 5);
  const int sub = (int)(t & 7u);
  const bool live = gid < (uint32_t)a.rows * nb;  // every lane takes part in the DPP steps
  const uint32_t row = live ? gid / nb : 0u, blk = live ? gid - row * nb : 0u;
  const int c = (int)blk * 32 + 4 * sub;
  float xin[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (live) {
    const float4 x4 = *reinterpret_cast<const float4*>(static_cast<const float*>(a.x) + (int64_t)row * a.ld_x + c);
    xin[0] = x4.x; xin[1] = x4.y; xin[2] = x4.z; xin[3] = x4.w;
    if (a.bfloat != 0 && a.bfloat != 32)
#pragma unroll
      for (int i = 0; i < 4; ++i) xin[i] = round_bfloat(xin[i], a.bfloat, kRoundNearest, 1);
  }
  auto umax = [](uint32_t p, uint32_t q) { return p > q ? p : q; };
  uint32_t mb = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) mb = umax(mb, __float_as_uint(xin[i]) & 0x7FFFFFFFu);
  mb = oct_reduce(mb, umax);
  int e_raw;
  const int es = scale_exponent(mb, 127, &e_raw);
  const bool nanblk = es == kExpNaN;
  const bool flush = a.flush && !(e_raw != kExpNaN && e_raw > -127);
  int cd[4];
  uint32_t mc = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float xv = flush ? xin[i] * 0.0f : xin[i];
    cd[i] = nanblk ? 0 : (int)round_code(xv, es, 8, kRoundNearest);
    mc = umax(mc, (uint32_t)(cd[i] < 0 ? -cd[i] : cd[i]));
  }
  const int maxc = (int)oct_reduce(mc, umax);
  const int eA = nanblk ? kExpNaN : (maxc == 0 ? -126 : floor_log2_pos((float)maxc * pow2f(es - 6)));
  if (!live) return;
  float out[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (nanblk) {
      out[i] = OPK == MXA_OP_TRUE_EX ? 1.0f : __uint_as_float(0x7FC00000u);
    } else if (OPK == MXA_OP_MXINT4) {
      const float xv = flush ? xin[i] * 0.0f : xin[i];
      out[i] = (round_code(xv, es, 4, kRoundNearest) * 0.25f) * pow2f(es);
    } else {
      const float mxv = ((float)cd[i] * pow2f(-6)) * pow2f(es);
      if (OPK == MXA_OP_SIGN) {
        out[i] = (mxv < 0.0f ? -1.0f : 1.0f) * pow2f(eA);
      } else if (OPK == MXA_OP_EXION) {
        const int m = exion_m(cd[i] << (es - eA));
        const float sg = cd[i] > 0 ? 1.0f : (cd[i] < 0 ? -1.0f : 0.0f);
        out[i] = ((sg * (float)eA) * (float)(m < 0 ? -m : m)) / 64.0f;
      } else if (OPK == MXA_OP_TRUE_EX) {
        const float am = fabsf(mxv);
        const int te = am > 0.0f ? floor_log2_pos(am) : 0;
        out[i] = (mxv < 0.0f ? -1.0f : 1.0f) * pow2f(te);
      } else {
        out[i] = mxv;
      }
    }
  }
  *reinterpret_cast<float4*>(static_cast<float*>(a.out) + (int64_t)row * a.ld_out + c) =
      make_float4(out[0], out[1], out[2], out[3]);
}

// quantize_mx along a contiguous axis in 32-element blocks (the mx ops' axes=[-1] case):
// one lane per element, the block max by lane shuffles -- quantize_mx_kernel's result
__global__ __launch_bounds__(256) void quantize_mx_row32_kernel(QuantArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t bid = t >> 5;
  const int j = (int)(t & 31);
  const bool live = bid < a.outer * a.nb;
  const int64_t o = live ? bid / a.nb : 0, blk = live ? bid % a.nb : 0;
  const int64_t l = blk * 32 + j;
  const bool valid = live && l < a.L;
  const int64_t off = o * a.L + l;
  float xv = valid ? round_bfloat(load_dt(a.x, off, a.dt), a.bfloat, kRoundNearest, 1, a.dt) : 0.0f;
  const uint32_t mb = lanes32_max(__float_as_uint(xv) & 0x7FFFFFFFu);
  int e_raw;
  const int es = scale_exponent_dt(mb, a.scale_emax, a.dt, &e_raw);
  if (!valid) return;
  if (a.flush && !(e_raw != kExpNaN && e_raw > -127)) xv = xv * 0.0f;
  const int shift = a.mbits - 2;
  float yv, cv = 0.0f;
  if (es == kExpNaN) {
    yv = __uint_as_float(0x7FC00000u);
  } else {
    cv = round_code(xv, es, a.mbits, a.rnd, a.dt);
    yv = (cv * pow2f(-shift)) * pow2f(es);
  }
  store_dt(a.y, off, yv, a.dt);  // (code * 2^(es-shift) rounded once to the dtype)
  if (a.codes) a.codes[off] = (int8_t)cv;
  if (a.exps && j == 0) a.exps[o * a.nb + blk] = exp_to16(es);
}

}  // namespace mxa

using namespace mxa;

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static bool dtype_ok(int dt) { return dt == kF32 || dt == kF16 || dt == kBF16; }

extern "C" int mxa_quantize_mx(const void* x, void* y, int8_t* codes, int16_t* exps, int64_t outer,
                               int64_t axis_len, int64_t inner, int32_t block_size, int32_t elem_mbits,
                               int32_t scale_bits, int32_t round_mode, int32_t flush_subnormals, int32_t bfloat,
                               int32_t dtype, hipStream_t stream) {
  if (!x || !y || outer < 0 || axis_len < 0 || inner < 0 || block_size < 0 || !dtype_ok(dtype)) return MXA_ERR_ARG;
  if (elem_mbits != 8 && elem_mbits != 4 && elem_mbits != 2) return MXA_ERR_UNSUPPORTED;
  if (scale_bits < 2 || scale_bits > 8 || round_mode < 0 || round_mode > 2) return MXA_ERR_ARG;
  if (bfloat != 0 && bfloat != 32 && (bfloat < 10 || bfloat > 31)) return MXA_ERR_ARG;
  if (outer == 0 || axis_len == 0 || inner == 0) return MXA_OK;
  QuantArgs a{};
  a.x = x; a.y = y; a.codes = codes; a.exps = exps;
  a.outer = outer; a.L = axis_len; a.inner = inner;
  a.bs = block_size == 0 ? axis_len : block_size;
  a.nb = (axis_len + a.bs - 1) / a.bs;
  a.mbits = elem_mbits; a.scale_emax = (1 << (scale_bits - 1)) - 1; a.rnd = round_mode;
  a.flush = flush_subnormals; a.bfloat = bfloat; a.dt = dtype;
  const int64_t nblocks = outer * a.nb * inner;
  if (inner == 1 && a.bs == 32) {  // contiguous 32-blocks: one lane per element
    hipLaunchKernelGGL(quantize_mx_row32_kernel, dim3((unsigned)((nblocks * 32 + 255) / 256)), dim3(256), 0, stream, a);
    return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
  }
  hipLaunchKernelGGL(quantize_mx_kernel, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

extern "C" int mxa_shared_exponents(const void* x, void* out, int64_t outer, int64_t axis_len, int64_t inner,
                                    int32_t block_size, int32_t method, int32_t ebits, int32_t dtype,
                                    hipStream_t stream) {
  if (!x || !out || outer < 0 || axis_len < 0 || inner < 0 || block_size < 0 || !dtype_ok(dtype)) return MXA_ERR_ARG;
  if (method != 0 && method != 1) return MXA_ERR_ARG;
  if (outer == 0 || axis_len == 0 || inner == 0) return MXA_OK;
  SexpArgs a{};
  a.x = x; a.out = out; a.outer = outer; a.L = axis_len; a.inner = inner;
  a.bs = block_size == 0 ? axis_len : block_size;
  a.nb = (axis_len + a.bs - 1) / a.bs;
  a.method = method; a.ebits = ebits; a.dt = dtype;
  const int64_t n = method == 1 ? outer * axis_len * inner : outer * a.nb * inner;
  hipLaunchKernelGGL(shared_exp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

extern "C" int mxa_quantize_bfloat(const void* x, void* y, int64_t n, int32_t bfloat, int32_t round_mode,
                                   int32_t allow_denorm, int32_t dtype, hipStream_t stream) {
  if (!x || !y || n < 0 || !dtype_ok(dtype)) return MXA_ERR_ARG;
  if (bfloat != 0 && bfloat != 32 && (bfloat < 10 || bfloat > 31)) return MXA_ERR_ARG;
  if (round_mode < 0 || round_mode > 2) return MXA_ERR_ARG;
  if (n == 0) return MXA_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 256 * 16) blocks = 256 * 16;
  hipLaunchKernelGGL(bfloat_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, y, n, bfloat, round_mode,
                     allow_denorm, dtype);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

extern "C" int mxa_approx_values(const void* x, void* out, int64_t rows, int32_t d, int64_t ld_x, int64_t ld_out,
                                 int32_t op_kind, int32_t flush_subnormals, int32_t bfloat, int32_t dtype,
                                 hipStream_t stream) {
  if (!x || !out || rows < 0 || d <= 0 || ld_x < d || ld_out < d || !dtype_ok(dtype)) return MXA_ERR_ARG;
  if (op_kind < MXA_OP_SIGN || op_kind > MXA_OP_TRUE_EX) return MXA_ERR_ARG;
  if (rows == 0) return MXA_OK;
  ApproxArgs a{};
  a.x = x; a.out = out; a.rows = rows; a.d = d; a.ld_x = ld_x; a.ld_out = ld_out;
  a.op_kind = op_kind; a.flush = flush_subnormals; a.bfloat = bfloat; a.dt = dtype;
  const int64_t nbk = rows * ((d + 31) / 32);
  if (dtype == MXA_DT_F32 && d % 32 == 0 && ld_x % 4 == 0 && ld_out % 4 == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) & 15u) == 0 &&
      nbk * 8 < ((int64_t)1 << 31)) {  // eight lanes per block, float4 in and out
    const dim3 grid((unsigned)((nbk * 8 + 255) / 256));
    switch (op_kind) {
      case MXA_OP_SIGN: hipLaunchKernelGGL(approx_values_v4_kernel<MXA_OP_SIGN>, grid, dim3(256), 0, stream, a); break;
      case MXA_OP_EXION: hipLaunchKernelGGL(approx_values_v4_kernel<MXA_OP_EXION>, grid, dim3(256), 0, stream, a); break;
      case MXA_OP_MXINT4: hipLaunchKernelGGL(approx_values_v4_kernel<MXA_OP_MXINT4>, grid, dim3(256), 0, stream, a); break;
      case MXA_OP_TRUE_EX: hipLaunchKernelGGL(approx_values_v4_kernel<MXA_OP_TRUE_EX>, grid, dim3(256), 0, stream, a); break;
      default: hipLaunchKernelGGL(approx_values_v4_kernel<MXA_OP_MXINT8>, grid, dim3(256), 0, stream, a); break;
    }
    return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
  }
  const int64_t n = nbk * 32;  // one lane per element of the padded blocks
  if (n / 256 >= ((int64_t)1 << 31)) return MXA_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(approx_values_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}

namespace mxa {
int launch_rows_prep(const RowsPrepArgs& a, hipStream_t stream) {
  const int64_t threads = a.rows * a.nb * 2;
  if (threads == 0) return MXA_OK;
  if (a.rows * a.nb >= ((int64_t)1 << 30)) return MXA_ERR_UNSUPPORTED;  // 32-bit thread indices (x2 lanes)
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (a.dt == kF16) hipLaunchKernelGGL(rows_prep_kernel<kF16>, grid, dim3(256), 0, stream, a);
  else if (a.dt == kBF16) hipLaunchKernelGGL(rows_prep_kernel<kBF16>, grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL(rows_prep_kernel<kF32>, grid, dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
int launch_elsa_prep(const ElsaPrepArgs& a, hipStream_t stream) {
  if (a.rows == 0) return MXA_OK;
  if (a.D > 128 || a.nb > 4) return MXA_ERR_UNSUPPORTED;
  const size_t lds = (size_t)a.D * a.D * 4;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&elsa_prep_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  const int64_t blocks = std::min<int64_t>((a.rows + kElsaWaves - 1) / kElsaWaves, 2048);
  hipLaunchKernelGGL(elsa_prep_kernel, dim3((unsigned)blocks), dim3(64 * kElsaWaves), lds, stream, a);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
int launch_attn_prep(const RowsPrepArgs& q, const RowsPrepArgs& k, const ColsPrepArgs& v, hipStream_t stream) {
  if (q.rows * q.nb >= ((int64_t)1 << 30) || k.rows * k.nb >= ((int64_t)1 << 30) ||
      v.mats * v.nb * v.C >= ((int64_t)1 << 31))
    return MXA_ERR_UNSUPPORTED;  // 32-bit thread indices
  if (q.dt != k.dt || q.dt != v.dt) return MXA_ERR_ARG;
  const int64_t nq = (q.rows * q.nb * 2 + 255) / 256, nk = (k.rows * k.nb * 2 + 255) / 256;
  const int64_t nv = (v.mats * v.nb * v.C + 255) / 256;
  if (nq + nk + nv == 0) return MXA_OK;
  const dim3 grid((unsigned)(nq + nk + nv));
  if (q.dt == kF16) hipLaunchKernelGGL(attn_prep_kernel<kF16>, grid, dim3(256), 0, stream, q, k, v, (uint32_t)nq, (uint32_t)nk);
  else if (q.dt == kBF16) hipLaunchKernelGGL(attn_prep_kernel<kBF16>, grid, dim3(256), 0, stream, q, k, v, (uint32_t)nq, (uint32_t)nk);
  else hipLaunchKernelGGL(attn_prep_kernel<kF32>, grid, dim3(256), 0, stream, q, k, v, (uint32_t)nq, (uint32_t)nk);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
int launch_cols_prep(const ColsPrepArgs& a, hipStream_t stream) {
  const int64_t threads = a.mats * a.nb * a.C;
  if (threads == 0) return MXA_OK;
  if (threads >= ((int64_t)1 << 31)) return MXA_ERR_UNSUPPORTED;  // 32-bit thread indices
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (a.dt == kF16) hipLaunchKernelGGL(cols_prep_kernel<kF16>, grid, dim3(256), 0, stream, a);
  else if (a.dt == kBF16) hipLaunchKernelGGL(cols_prep_kernel<kBF16>, grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL(cols_prep_kernel<kF32>, grid, dim3(256), 0, stream, a);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}
}  // namespace mxa
