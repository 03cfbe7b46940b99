// Kernel argument blocks and the block-scaled int8 MFMA tile shared by the
// attention, P.V and mx.matmul kernels.
#pragma once
#include "../../include/mxa.h"
#include "mxa_common.hpp"

namespace mxa {

struct QuantArgs {
  const void* x;  // dtype dt
  void* y;        // dtype dt
  int8_t* codes;
  int16_t* exps;
  int64_t outer, L, inner, bs, nb;
  int mbits, scale_emax, rnd, flush, bfloat, dt;
};

struct SexpArgs {
  const void* x;  // dtype dt
  void* out;      // dtype dt
  int64_t outer, L, inner, bs, nb;
  int method, ebits, dt;
};

struct ApproxArgs {
  const void* x;  // dtype dt
  void* out;      // dtype dt
  int64_t rows;
  int d;
  int64_t ld_x, ld_out;
  int op_kind, flush, bfloat, dt;
};

// rows of D elements at x + b*s0 + h*s1 + r*s2 (r < R, h < H), quantized along D
struct RowsPrepArgs {
  const void* x;  // dtype dt
  int64_t s0, s1, s2;
  int64_t H, R, rows;  // rows = B*H*R
  int D, nb, dpad;
  int vec4;  // 16-B aligned rows -> float4 loads
  int op_kind, flush, bfloat;
  int dt;         // storage dtype of x (MXA_DT_*): loads and the shared-exponent rule
  int8_t* codes;  // [rows][dpad] MXINT8 codes (nullable)
  int16_t* sT;    // [rows][nb] exponent of a code unit: es - 6 (nullable)
  int8_t* op;     // [rows][dpad] approximator operand (nullable)
  int16_t* sA;    // [rows][nb] approximator scale (nullable)
  uint32_t* signs;  // [rows][nb] bit i = (MX code i < 0) (nullable)
  int8_t* zind;     // [rows][dpad] 1 where the MX code is 0 (column < D), else 0 (true_ex; nullable)
  int mfma_rows;    // codes layout: 0 row-major [rows][dpad]; 1 MFMA-ready for the MX GEMM's A operand,
                    // [rows / 32][nb][lane][16 B] with lane = row % 32 + 32 * (16-element half)
                    // (one coalesced 1-KB load per wave and K-block; rows padded to 32)
};

// ELSA sign hashes (and key norms) of rows already quantized by rows_prep:
// hash bit j of a row = (sum_i MX_i * P[j][i] >= 0), norm = ||MX row||_2
// (funcs/elsa_approximation.py:105-112, :126)
struct ElsaPrepArgs {
  const int8_t* codes;  // [rows][dpad]
  const int16_t* sT;    // [rows][nb] exponent of a code unit
  const float* proj;    // [D][D] row-major P
  int64_t rows;
  int D, nb, dpad;
  uint32_t* hash;  // [rows][nb] hash words
  float* norm;     // [rows] (nullable)
};

// matrices (R x C) at x + b*s0 + h*s1 + r*s2 + c quantized along R in 32-blocks
struct ColsPrepArgs {
  const void* x;  // dtype dt
  int64_t s0, s1, s2;
  int64_t H, mats;  // mats = B*H
  int R, C, nb, rpad;
  int mbits, flush, bfloat;
  int dt;  // storage dtype of x
  int tb_major;     // codes layout: 0 = [mats][C][rpad]; 1 = [mats][nb][C][32] (the attention's V^T:
                    // a 32-token block of a head is one contiguous C x 32-byte run, whole lines)
  int8_t* codes_t;  // transposed codes
  int16_t* scale;   // [mats][nb][C] exponent of a code unit: es - (mbits-2)
};

int launch_rows_prep(const RowsPrepArgs& a, hipStream_t stream);
int launch_cols_prep(const ColsPrepArgs& a, hipStream_t stream);
// Q rows, K rows and V columns of the attention path in one launch
int launch_attn_prep(const RowsPrepArgs& q, const RowsPrepArgs& k, const ColsPrepArgs& v, hipStream_t stream);
int launch_elsa_prep(const ElsaPrepArgs& a, hipStream_t stream);

typedef int v4i __attribute__((ext_vector_type(4)));

// One wave computes a 16x16 tile  C[i][j] = sum_b I_b[i][j] * scale(i,b) (x) scale(j,b)
// with I_b = A[i][32b:32b+32] . Bt[j][32b:32b+32] from one v_mfma_i32_16x16x32_i8 per
// 32-element MX block (K = 32 = one block, so every block keeps its own exact int32 sum).
//   combine EXP: scale = 2^(sa + sb)        MUL: scale = sa * sb / 4096  (EXION quirk)
// The block products are exact in double and summed in double (exact while the
// block exponents span < 34 bits), then rounded once by the caller: the reference's
// fp32 matmul of these operands gives the same float.
//
// Lane maps of v_mfma_i32_16x16x32_i8 (checked on hardware by mxa_selftest_mfma):
//   A: lane l holds A[l & 15][8*(l >> 4) + j], j = 0..7  (one int64)
//   B: lane l holds B[8*(l >> 4) + j][l & 15]            (= Bt[l & 15][8*(l >> 4) + j])
//   C: acc[i] = C[4*(l >> 4) + i][l & 15]
// Rows/cols beyond the valid count are clamped on load and must be ignored by the caller.
template <bool MUL>
__device__ __forceinline__ void scaled_tile(const int8_t* __restrict__ A, int64_t lda, int a_valid,
                                            const int16_t* __restrict__ SA, int64_t sa_row, int64_t sa_blk,
                                            const int8_t* __restrict__ Bt, int64_t ldb, int b_valid,
                                            const int16_t* __restrict__ SB, int64_t sb_row, int64_t sb_blk,
                                            int nblk, double acc[4]) {
  const int lane = lane_id();
  const int r = lane & 15, kg = lane >> 4;
  const int ar = r < a_valid ? r : a_valid - 1;
  const int bc = r < b_valid ? r : b_valid - 1;
  const int8_t* ap = A + ar * lda + kg * 8;
  const int8_t* bp = Bt + bc * ldb + kg * 8;
  int crow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = 4 * kg + i;
    crow[i] = rr < a_valid ? rr : a_valid - 1;
  }
  const v4i zero = {0, 0, 0, 0};
  for (int b = 0; b < nblk; ++b) {
    const long av = *reinterpret_cast<const long*>(ap + b * 32);
    const long bv = *reinterpret_cast<const long*>(bp + b * 32);
    const v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, zero, 0, 0, 0);
    const int sb = exp_from16(SB[bc * sb_row + b * sb_blk]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int sa = exp_from16(SA[crow[i] * sa_row + b * sa_blk]);
      if (sa == kExpNaN || sb == kExpNaN) {
        acc[i] = __longlong_as_double(0x7FF8000000000000LL);
      } else if (MUL) {
        acc[i] += (double)c[i] * (double)(sa * sb) * (1.0 / 4096.0);
      } else {
        acc[i] += (double)c[i] * pow2d(sa + sb);
      }
    }
  }
}

}  // namespace mxa
