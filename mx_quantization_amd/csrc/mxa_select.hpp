// Selection kernel: approximate scores + exact-order top-k, FOUR query rows per wave.
//
// Per workgroup (one head, a chunk of its query rows): the head's score tables
// (ex_pred: sign words + block exponents; MXINT4 / EXION / partial: approximator
// codes + block scales; true scores: MXINT8 codes + exponents) are staged in LDS
// once.  Per wave, four rows at a time, one 16-lane DPP row each:
//   1. lane gl computes the scores of keys gl, gl + 16, ... into the row's LDS mirror
//      (exact fp64 block epilogue: the scores are exact sums of integer * 2^e,
//      SURVEY.md F6), bias added in fp32 as the caller does;
//   2. grp_topk (mxa_topk_grp.hpp) reproduces torch's CPU topk index order;
//   3. the k kept indices go out as int64 (the op's idx) and int32 (the finishing
//      kernel's input), four consecutive rows per wave: contiguous stores.
// Callers replaced: the approximator + torch.topk of
//   workloads/deit/scripts/main.py:101-123, workloads/DiT/models.py:168-194,
//   workloads/PixArt/models/MX_transformer_block.py:660-678, :805-825.
#pragma once
#include "mxa_topk_grp.hpp"

namespace mxa {

constexpr int kSelWaves = 4;  // waves per workgroup
constexpr int kSelRows = 32;  // query rows per workgroup (a multiple of 4 * kSelWaves)

// MX dot product of a query row (codes in registers, two uint4 per 32-block, block
// exponents qe) with key row krow of the LDS code table: exact block sums by v_dot4,
// block scale 2^(qe+ke) (MUL = 0) or qe*ke/4096 (EXION, MUL = 1), fp64 accumulation
template <int MUL, int NBMAX = kMaxNB>
__device__ __forceinline__ double g_dot(const uint4* qv, const int* qe, int nbd, const int8_t* krow,
                                        const int16_t* kexp, bool& nan) {
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < NBMAX; ++b) {
    if (b < nbd) {
      const uint4 x0 = *reinterpret_cast<const uint4*>(krow + 32 * b);
      const uint4 x1 = *reinterpret_cast<const uint4*>(krow + 32 * b + 16);
      const uint4 q0 = qv[2 * b], q1 = qv[2 * b + 1];
      int I = 0;
      I = __builtin_amdgcn_sdot4((int)q0.x, (int)x0.x, I, false);
      I = __builtin_amdgcn_sdot4((int)q0.y, (int)x0.y, I, false);
      I = __builtin_amdgcn_sdot4((int)q0.z, (int)x0.z, I, false);
      I = __builtin_amdgcn_sdot4((int)q0.w, (int)x0.w, I, false);
      I = __builtin_amdgcn_sdot4((int)q1.x, (int)x1.x, I, false);
      I = __builtin_amdgcn_sdot4((int)q1.y, (int)x1.y, I, false);
      I = __builtin_amdgcn_sdot4((int)q1.z, (int)x1.z, I, false);
      I = __builtin_amdgcn_sdot4((int)q1.w, (int)x1.w, I, false);
      const int e = exp_from16(kexp[b]);
      if (e == kExpNaN || qe[b] == kExpNaN) nan = true;
      else if (MUL) acc += (double)I * (double)(qe[b] * e) * (1.0 / 4096.0);
      else acc += (double)I * pow2d(qe[b] + e);
    }
  }
  return acc;
}

template <int NP, int MODE>
__global__ __launch_bounds__(64 * kSelWaves) __attribute__((amdgpu_waves_per_eu(NP <= 256 ? 4 : 2, 8))) void select_kernel(Rows2Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr bool kOp = MODE == kModeOpExp || MODE == kModeOpMul;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gi = lane >> 4, gl = lane & 15;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const Rows2Lds L = rows2_lds(MODE, T, D, kst, nbd, a.vst, a.ntb, 1, a.tpad, 0, 0, 1);
  int8_t* tcd = reinterpret_cast<int8_t*>(smem + (MODE == kModeTrue ? L.mx : L.op));  // key codes
  int16_t* tex = reinterpret_cast<int16_t*>(smem + (MODE == kModeTrue ? L.sT : L.sA));  // key exponents
  uint32_t* tsg = reinterpret_cast<uint32_t*>(smem + L.sg);

  // ---- stage the head's score tables ----------------------------------------
  const int64_t kb = (int64_t)bh * T;
  if constexpr (MODE == kModeTrue || kOp) {
    const int8_t* src = MODE == kModeTrue ? a.kc : a.kop;
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(tcd + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(src + (kb + j) * a.dpad + 16 * c);
    }
  }
  {
    const int16_t* esrc = MODE == kModeTrue ? a.ksT : a.ksA;
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) {
      tex[i] = esrc[kb * nbd + i];
      if (MODE == kModeExSign) tsg[i] = a.ksg[kb * nbd + i];
    }
  }
  __syncthreads();

  const int npa = grp_alloc(T);
  const GrpRow g = carve_grp(smem + L.waves + (size_t)(4 * wave + gi) * grp_row_bytes(npa, NP), npa, NP);
  const int r_end = min(a.N, (int)(blockIdx.y + 1) * a.rows_per_wg);
  for (int rq = (int)blockIdx.y * a.rows_per_wg + 4 * wave; rq < r_end; rq += 4 * kSelWaves) {
    const int r = rq + gi;
    const bool valid = r < r_end;
    const int64_t grow = (int64_t)bh * a.N + (valid ? r : rq);
    const float* brow = a.bias ? a.bias + b_ * a.bs0 + h_ * a.bs1 + (int64_t)(valid ? r : rq) * a.bs2 : nullptr;

    // ---- the row's scores into its mirror ------------------------------------
    if (valid) {
      if constexpr (MODE == kModeExSign) {
        // pred = sum_b 2^(eq_b + ek_b) (n_b - 2 popc(sq_b ^ sk_b))   (exact)
        uint32_t sq[kMaxNB];
        int eq[kMaxNB];
#pragma unroll
        for (int b = 0; b < kMaxNB; ++b) {
          sq[b] = b < nbd ? a.qsg[grow * nbd + b] : 0u;
          eq[b] = b < nbd ? exp_from16(a.qsA[grow * nbd + b]) : 0;
        }
        for (int j = gl; j < T; j += 16) {
          double acc = 0.0;
          bool nan = false;
#pragma unroll
          for (int b = 0; b < kMaxNB; ++b) {
            if (b < nbd) {
              const int e = exp_from16(tex[j * nbd + b]);
              nan = nan || e == kExpNaN || eq[b] == kExpNaN;
              const int m = min(32, D - 32 * b) - 2 * (int)__popc(sq[b] ^ tsg[j * nbd + b]);
              acc += (double)m * pow2d(nan ? 0 : eq[b] + e);
            }
          }
          float v = nan ? __uint_as_float(0x7FC00000u) : (float)acc;
          if (brow) v = v + brow[(int64_t)j * a.bs3];
          if (a.pred_out) a.pred_out[grow * T + j] = v;
          g.A[j] = pack_ki(order_key(v), (uint32_t)j);
        }
      } else {
        const int8_t* qsrc = (MODE == kModeTrue ? a.qc : a.qop) + grow * a.dpad;
        const int16_t* qesrc = (MODE == kModeTrue ? a.qsT : a.qsA) + grow * nbd;
        uint4 qv[2 * kMaxNB];
        int qe[kMaxNB];
#pragma unroll
        for (int b = 0; b < kMaxNB; ++b) {
          qv[2 * b] = b < nbd ? *reinterpret_cast<const uint4*>(qsrc + 32 * b) : make_uint4(0, 0, 0, 0);
          qv[2 * b + 1] = b < nbd ? *reinterpret_cast<const uint4*>(qsrc + 32 * b + 16) : make_uint4(0, 0, 0, 0);
          qe[b] = b < nbd ? exp_from16(qesrc[b]) : 0;
        }
        for (int j = gl; j < T; j += 16) {
          bool nan = false;
          const double acc = g_dot<MODE == kModeOpMul>(qv, qe, nbd, tcd + (size_t)j * kst, tex + j * nbd, nan);
          float v = nan ? __uint_as_float(0x7FC00000u) : (float)acc;
          // true = quantize_elemwise(fl32(QK^T)) * scale   (matmul.py:88-91, caller)
          if (MODE == kModeTrue) v = round_bfloat(v, a.bfloat, kRoundNearest, 1) * a.scale;
          if (brow) v = v + brow[(int64_t)j * a.bs3];
          if (MODE == kModeTrue) {
            if (a.true_out) a.true_out[grow * T + j] = v;
          } else if (a.pred_out) {
            a.pred_out[grow * T + j] = v;
          }
          g.A[j] = pack_ki(order_key(v), (uint32_t)j);
        }
      }
    }
    wave_lds_sync();

    // ---- torch CPU top-k order ------------------------------------------------
    grp_topk<NP>(g, T, a.k_top, valid, gl);

    // ---- kept indices: four consecutive rows per wave ----------------------------
    if (valid) {
      for (int p = gl; p < a.k_top; p += 16) {
        const uint32_t ix = (uint32_t)g.A[p];
        if (a.idx_out) a.idx_out[grow * a.k_top + p] = (int64_t)ix;
        a.idx32[grow * a.k_top + p] = (int32_t)ix;
      }
    }
    wave_lds_sync();
  }
}

// ---- standalone top-k over rows of a float matrix (mxa_topk) ------------------
struct GrpTopkArgs {
  const float* vals;
  int64_t rows, ld;
  int n, k;
  int64_t* out_idx;
  float* out_vals;
};

template <int NP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NP <= 256 ? 4 : 2, 8))) void topk_grp_kernel(GrpTopkArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gi = lane >> 4, gl = lane & 15;
  const int64_t row = ((int64_t)blockIdx.x * 4 + wave) * 4 + gi;
  const bool valid = row < a.rows;
  const int npa = grp_alloc(a.n);
  const GrpRow g = carve_grp(smem + (size_t)(4 * wave + gi) * grp_row_bytes(npa, NP), npa, NP);
  const float* src = a.vals + (valid ? row : 0) * a.ld;
  if (valid)
    for (int j = gl; j < a.n; j += 16) g.A[j] = pack_ki(order_key(src[j]), (uint32_t)j);
  wave_lds_sync();
  grp_topk<NP>(g, a.n, a.k, valid, gl);
  if (valid) {
    for (int p = gl; p < a.k; p += 16) {
      const uint32_t ix = (uint32_t)g.A[p];
      a.out_idx[row * a.k + p] = (int64_t)ix;
      if (a.out_vals) a.out_vals[row * a.k + p] = src[ix];
    }
  }
}

}  // namespace mxa
