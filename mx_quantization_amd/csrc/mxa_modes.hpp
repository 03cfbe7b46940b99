// Shared constants of the attention kernels: head-dim block limit, score modes, and
// the scalar-load helper of a wave's query row.
#pragma once
#include "mxa_kernels.hpp"
#include "mxa_order.hpp"

namespace mxa {

constexpr int kMaxNB = 4;  // head dim <= 128

enum RowsMode : int {
  kModeTrue = 0,   // row values are the true scores (approx off, or dense)
  kModeOpExp = 1,  // approximator codes, block scale 2^(sa + sb)
  kModeOpMul = 2,  // approximator codes, block scale sa * sb / 4096 (EXION)
  kModeExSign = 3,  // ex_pred: sign words + block exponents
  kModeTrueEx = 4,  // true_ex: power-of-two codes + zero indicators + block exponents
  kModeElsa = 5     // ELSA: hash words, key norms, cosine table
};

// scalar (uniform-address) loads of a wave's query row
typedef __attribute__((address_space(4))) const uint32_t* cu32;
__device__ __forceinline__ int s_exp16(const int16_t* base, int64_t i) {
  const uint32_t d = ((cu32)(base + (i & ~(int64_t)1)))[0];
  return exp_from16((int16_t)(i & 1 ? d >> 16 : d & 0xFFFFu));
}

}  // namespace mxa
