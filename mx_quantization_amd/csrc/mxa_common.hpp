// Device helpers shared by every MX kernel (gfx950 / CDNA4, wave64).
//
// Numerics follow the reference's *Python* path bit for bit (the workloads
// run it with custom_cuda=False), not the reference's CUDA
// kernels, which use exponent bits and therefore disagree:
//   shared exponent   microxscaling/mx/mx_ops.py:49-99
//   scale clamp       microxscaling/mx/mx_ops.py:276-300
//   element rounding  microxscaling/mx/elemwise_ops.py:45-86, :92-180
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>


namespace mxa {

// int sentinel for a NaN shared exponent (NaN/Inf in the block, or scale overflow)
constexpr int kExpNaN = -1000000;
// int16 storage of the same sentinel
constexpr int16_t kExpNaN16 = INT16_MIN;

enum Round : int { kRoundNearest = 0, kRoundFloor = 1, kRoundEven = 2 };  // formats.py:12-16

// floor(torch.log2(m + 2^-126 * (m == 0))) for m = |x| given as float bits with
// the sign cleared (mx_ops.py:83-87).  Exact for every float32.
// fl32(log2 m) rounds up to the next integer for mantissas within `gap` ulps
// below 2^23; gap depends only on the octave of the exponent.  The closed form
// below reproduces the per-binade thresholds that tools/gen_exp_lut.py bisects
// out of torch.log2 (tests/golden/exp_lut.npz; tests/test_oracle_golden.py checks
// the two agree), and needs no memory access.
__device__ __forceinline__ int floor_log2_abs_bits(uint32_t ub) {
  if (ub >= 0x7F800000u) return kExpNaN;  // Inf / NaN -> NaN exponent (log2(inf)=inf > emax)
  if (ub == 0u) return -126;
  const uint32_t E = ub >> 23, M = ub & 0x7FFFFFu;
  if (E) {
    const int e = (int)E - 127;
    const uint32_t u = (uint32_t)(e >= 0 ? e : -e - 1);
    const int o = u >= 2u ? 31 - __clz((int)u) : 0;  // octave, 0..6
    const uint32_t gap = (uint32_t)(0x2C160B05020100ull >> (8 * o)) & 0xFFu;  // 0,1,2,5,11,22,44
    return e + (M + gap >= (1u << 23) ? 1 : 0);
  }
  const int j = 31 - __clz((int)M);  // subnormal: leading mantissa bit
  const uint32_t gap = j < 17 ? 0u : (uint32_t)(0x160B0B050201ull >> (8 * (j - 17))) & 0xFFu;  // 1,2,5,11,11,22
  return -149 + j + (j >= 17 && M + gap >= (2u << j) ? 1 : 0);
}

// Same rule without the zero trick: floor(log2(m)) of a strictly positive finite m.
__device__ __forceinline__ int floor_log2_pos(float m) { return floor_log2_abs_bits(__float_as_uint(m)); }

// exact 2^e as float for e in [-149, 127]
__device__ __forceinline__ float pow2f(int e) {
  return e >= -126 ? __uint_as_float((uint32_t)(e + 127) << 23) : __uint_as_float(1u << (e + 149));
}
// exact 2^e as double for e in [-1022, 1023]
__device__ __forceinline__ double pow2d(int e) {
  return __longlong_as_double((long long)(e + 1023) << 52);
}

__device__ __forceinline__ int16_t exp_to16(int e) { return e == kExpNaN ? kExpNaN16 : (int16_t)e; }
__device__ __forceinline__ int exp_from16(int16_t e) { return e == kExpNaN16 ? kExpNaN : (int)e; }

// Shared exponent of a block from the bits of its max |x|, after the optional
// subnormal flush test and the scale clamp (mx_ops.py:276-291).  Returns the
// raw exponent through *e_raw for the flush decision.
__device__ __forceinline__ int scale_exponent(uint32_t maxbits, int scale_emax, int* e_raw) {
  const int e = floor_log2_abs_bits(maxbits);
  *e_raw = e;
  if (e == kExpNaN || e > scale_emax) return kExpNaN;  // shared_exp > scale_emax -> NaN
  return e < -scale_emax ? -scale_emax : e;
}

// ---- storage dtypes (include/mxa.h MXA_DT_*) ---------------------------------
// The reference's mx ops follow their input's dtype (microxscaling/mx/mx_ops.py:85,
// :283; elemwise_ops.py:146): on a float16 / bfloat16 tensor every step runs in that
// dtype.  Element values convert exactly to float; what differs is (i) the shared
// exponent, floor(log2(max)) with log2 rounded to the dtype, (ii) for float16 the
// zero block: 2^-126 underflows to 0, log2(0) = -inf, the scale 2^-127 is 0 in
// float16 and 0/0 makes the whole block NaN, and (iii) the rounding's |y| + 0.5 is
// rounded to the dtype (round_code).  Probes in DESIGN.md §2.
enum DType : int { kF32 = 0, kF16 = 1, kBF16 = 2 };

__device__ __forceinline__ float bf16_bits_to_f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ float f16_bits_to_f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
// round-to-nearest-even to the dtype, returned as float (NaN stays NaN, overflow -> inf)
__device__ __forceinline__ float round_dt(float x, int dt) {
  if (dt == kF16) return __half2float(__float2half_rn(x));
  if (dt == kBF16) {
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7FFFFFFFu) > 0x7F800000u) return __uint_as_float(u | 0x00400000u);
    return __uint_as_float(((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16) << 16);
  }
  return x;
}
__device__ __forceinline__ uint16_t f_to_dt_bits(float x, int dt) {
  if (dt == kF16) return __half_as_ushort(__float2half_rn(x));
  return (uint16_t)(__float_as_uint(round_dt(x, kBF16)) >> 16);
}
__device__ __forceinline__ float load_dt(const void* p, int64_t i, int dt) {
  if (dt == kF16) return f16_bits_to_f(static_cast<const uint16_t*>(p)[i]);
  if (dt == kBF16) return bf16_bits_to_f(static_cast<const uint16_t*>(p)[i]);
  return static_cast<const float*>(p)[i];
}
__device__ __forceinline__ void store_dt(void* p, int64_t i, float v, int dt) {
  if (dt == kF32) static_cast<float*>(p)[i] = v;
  else static_cast<uint16_t*>(p)[i] = f_to_dt_bits(v, dt);
}

// floor(log2(m)) computed in the dtype, for m = |x| exactly representable in it, given
// as float bits: log2 rounds up to the next integer for the top `gap` mantissa codes of
// a binade, gap depending only on the octave of the exponent (float16: 0, 1, 2, 5;
// bfloat16: 0, 1, 2, 5, 10, 21, 40), and for dtype subnormals above a per-leading-bit
// threshold.  Restated by oracle/mx_oracle.py floor_log2_dtype and pinned against torch
// on every value (tests/test_oracle_golden.py, tests/test_gpu_dtype.py).  Zero: float16
// -> kExpZeroF16 (log2(0) = -inf), bfloat16 -> -126 (2^-126 is a bfloat16).
constexpr int kExpZeroF16 = -100000;
__device__ __forceinline__ int floor_log2_dt(uint32_t ub, int dt) {
  if (dt == kF32) return floor_log2_abs_bits(ub);
  if (ub >= 0x7F800000u) return kExpNaN;
  if (ub == 0u) return dt == kF16 ? kExpZeroF16 : -126;
  const int mb = dt == kF16 ? 10 : 7;
  const int emin = dt == kF16 ? -14 : -126;
  int e;        // floor(log2 m) exactly
  uint32_t fm;  // float mantissa bits below the leading one (23 bits)
  if (ub >= 0x00800000u) {
    e = (int)(ub >> 23) - 127;
    fm = ub & 0x7FFFFFu;
  } else {  // float subnormal (bfloat16 subnormals only)
    const int j = 31 - __clz((int)ub);
    e = -149 + j;
    fm = (ub << (23 - j)) & 0x7FFFFFu;
  }
  if (e >= emin) {  // normal in the dtype: mb mantissa bits
    const uint32_t M = fm >> (23 - mb);
    const uint32_t u = (uint32_t)(e >= 0 ? e : -e - 1);
    const int o = u >= 2u ? 31 - __clz((int)u) : 0;  // octave of |e|
    const uint32_t gap = dt == kF16 ? (uint32_t)(0x05020100u >> (8 * o)) & 0xFFu
                                    : (uint32_t)(0x28150A05020100ull >> (8 * o)) & 0xFFu;
    return e + (M + gap >= (1u << mb) ? 1 : 0);
  }
  // subnormal in the dtype: M = m / 2^(emin - mb), leading bit j
  const int j = e - (emin - mb);
  const uint32_t M = (1u << j) | (fm >> (23 - j));
  uint32_t thr;  // smallest M of the sub-binade whose log2 rounds up (2^(j+1): none)
  if (dt == kF16) thr = j == 9 ? 1022u : (j == 8 ? 511u : (j == 7 ? 255u : (2u << j)));
  else thr = (uint32_t)(j == 0 ? 2 : (j == 1 ? 3 : (j == 2 ? 6 : (j == 3 ? 12 : (j == 4 ? 23 : (j == 5 ? 54 : 108))))));
  return e + (M >= thr ? 1 : 0);
}

// scale_exponent for a block of a dtype tensor: the float16 zero block is NaN
__device__ __forceinline__ int scale_exponent_dt(uint32_t maxbits, int scale_emax, int dt, int* e_raw) {
  if (dt == kF32) return scale_exponent(maxbits, scale_emax, e_raw);
  const int e = floor_log2_dt(maxbits, dt);
  *e_raw = e == kExpZeroF16 ? -1000 : e;
  if (e == kExpNaN || e == kExpZeroF16 || e > scale_emax) return kExpNaN;
  return e < -scale_emax ? -scale_emax : e;
}

// Element rounding of x / 2^es * 2^(mbits-2) (elemwise_ops.py:45-65, :150-164);
// returns the integer code as float, clamped to +-(2^(mbits-1)-1).
// es is finite and in [-127, 127], so 2^-es is an exact float and x * 2^-es is
// the correctly rounded x / 2^es.  Compiled with -ffp-contract=off.
// On a float16 / bfloat16 tensor (dt) the reference adds the 0.5 in that dtype: |y| + 0.5
// rounds to it (bfloat16 0.498046875 + 0.5 -> 1.0), so the sum is rounded to dt before the
// floor (y itself is exact in dt: a power-of-two scaling of a dt value).
__device__ __forceinline__ float round_code(float x, int es, int mbits, int rnd, int dt = 0) {
  float y = x * pow2f(-es);
  y = y * (float)(1 << (mbits - 2));
  const float a = fabsf(y);
  float r;
  if (rnd == kRoundFloor) {
    r = floorf(a);
  } else {
    r = floorf(round_dt(a + 0.5f, dt));
    if (rnd == kRoundEven) {
      const float d = round_dt(a - 0.5f, dt);  // ((|A| - 0.5) % 2 == 0) -> step back to even
      if (floorf(d * 0.5f) * 2.0f == d) r -= 1.0f;
    }
  }
  const float lim = (float)((1 << (mbits - 1)) - 1);
  r = r > lim ? lim : r;
  return y < 0.0f ? -r : r;
}

// The MXINT8 nearest-rounding case of round_code as an int: x * 2^(6-es) is exact and
// equals (x * 2^-es) * 64, so one multiply by q8_scale(es) does, except for es < -121
// where 2^(6-es) is no float (then q8_scale = 2^-es and TINY multiplies by 64 after);
// the sign goes back on with a bit copy (-0 converts to 0 like +0).
__device__ __forceinline__ float q8_scale(int es) { return pow2f(es >= -121 ? 6 - es : -es); }
template <bool TINY>
__device__ __forceinline__ int q8_code(float x, float s, int dt = 0) {
  float y = x * s;
  if (TINY) y = y * 64.0f;
  const float r = fminf(floorf(round_dt(fabsf(y) + 0.5f, dt)), 127.0f);
  return (int)__builtin_copysignf(r, y);
}

// bfloatX element quantization, exp_bits = 8, mbits = bfloat-7 (elemwise_ops.py:201-216
// -> _quantize_elemwise_core :92-180 with saturate_normals=False).  bfloat in {0,32} = identity.
// On a float16 / bfloat16 tensor (dt) the private exponent is floor(log2) computed in the
// dtype (floor_log2_dt) and the result is a value of the dtype.
__device__ __forceinline__ float round_bfloat(float x, int bfloat, int rnd, int allow_denorm, int dt = 0) {
  if (bfloat == 0 || bfloat == 32) return x;
  const uint32_t ub = __float_as_uint(x) & 0x7FFFFFFFu;
  if (ub >= 0x7F800000u) return x;  // +-Inf restored, NaN stays NaN
  const int bits = bfloat - 7;
  float xin = x;
  if (!allow_denorm && ub < 0x00800000u) xin = 0.0f * x;  // |A| < min_norm -> 0 (sign kept)
  int pe = ub == 0u ? 0 : floor_log2_dt(ub, dt);  // log2(|A| + (A==0))
  pe = pe < -126 ? -126 : pe;
  float y = xin * pow2f(-pe);
  y = y * (float)(1 << (bits - 2));
  const float a = fabsf(y);
  float r;
  if (rnd == kRoundFloor) {
    r = floorf(a);
  } else {
    r = floorf(round_dt(a + 0.5f, dt));
    if (rnd == kRoundEven) {
      const float d = round_dt(a - 0.5f, dt);
      if (floorf(d * 0.5f) * 2.0f == d) r -= 1.0f;
    }
  }
  float o = (y < 0.0f ? -r : r) * (1.0f / (float)(1 << (bits - 2)));
  o = o * pow2f(pe > 127 ? 127 : pe);
  const float max_norm = 1.7014118346046923e38f * ((float)((1 << (bits - 1)) - 1) / (float)(1 << (bits - 2)));
  if (fabsf(o) > max_norm) o = o < 0.0f ? -INFINITY : INFINITY;
  return round_dt(o, dt);
}

// ---- wave64 helpers -------------------------------------------------------
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
// wave-wide ballot straight from the compare mask (HIP's __ballot materialises the
// predicate in a VGPR and compares it again)
__device__ __forceinline__ uint64_t ballot64(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// bits [lo, hi) of a 64-bit lane mask, 0 <= lo <= hi <= 64 (uniform)
__device__ __forceinline__ uint64_t range_mask64(int lo, int hi) {
  const uint64_t h = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  return lo >= 64 ? 0ull : h & ~((1ull << lo) - 1ull);
}
// set bits of m at or below this lane
__device__ __forceinline__ int mbcnt_incl(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, (uint32_t)__builtin_amdgcn_inverse_ballot_w64(m)));
}
__device__ __forceinline__ int mbcnt(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Cross-lane reductions on DPP (no LDS traffic): reduce within each row of 16
// lanes (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror),
// then combine the four rows through readlane.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xF, 0xF, false);
}
// reduction over each group of 8 consecutive lanes
template <class Op>
__device__ __forceinline__ uint32_t oct_reduce(uint32_t v, Op op) {
  v = op(v, dpp_u32<0xB1>(v));
  v = op(v, dpp_u32<0x4E>(v));
  return op(v, dpp_u32<0x141>(v));
}
template <class Op>
__device__ __forceinline__ uint32_t row16_reduce(uint32_t v, Op op) {
  v = op(v, dpp_u32<0xB1>(v));
  v = op(v, dpp_u32<0x4E>(v));
  v = op(v, dpp_u32<0x141>(v));
  v = op(v, dpp_u32<0x140>(v));
  return v;
}
template <class Op>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v, Op op) {
  v = row16_reduce(v, op);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return op(op(r0, r1), op(r2, r3));
}
// reduction over each half-wave of 32 lanes (an MX block of 32 positions per slot)
template <class Op>
__device__ __forceinline__ uint32_t half_reduce(uint32_t v, Op op) {
  v = row16_reduce(v, op);
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
  const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
  return lane_id() < 32 ? op(r0, r1) : op(r2, r3);
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  return wave_reduce(v, [](uint32_t x, uint32_t y) { return x > y ? x : y; });
}

__device__ __forceinline__ float wave_max_f32(float v) {
  return __uint_as_float(wave_reduce(__float_as_uint(v), [](uint32_t x, uint32_t y) {
    return __float_as_uint(fmaxf(__uint_as_float(x), __uint_as_float(y)));
  }));
}

__device__ __forceinline__ float wave_sum_f32(float v) {
  return __uint_as_float(wave_reduce(__float_as_uint(v), [](uint32_t x, uint32_t y) {
    return __float_as_uint(__uint_as_float(x) + __uint_as_float(y));
  }));
}

// LDS ordering between the lanes of one wave (no workgroup barrier needed).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace mxa
