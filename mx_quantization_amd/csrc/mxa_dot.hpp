// MX dot products shared by the selection kernels (mxa_select.hpp) and the finishing
// kernels (mxa_finish*.hpp): a 32-element int8 block on v_dot4, and the true score of a
// query row against a key row with the exact rounding rule of SURVEY.md F6.  (A header of
// its own so that the finishing units do not include the selection kernels.)
#pragma once
#include "mxa_rows2.hpp"

namespace mxa {

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

}  // namespace mxa
