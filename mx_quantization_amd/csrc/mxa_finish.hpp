// Finishing kernel of the split path, P.V on int8 MFMA.
//
// Input: the kept key indices of every query row (idx32, written by the selection
// kernel).  One head per workgroup; the head's K MXINT8 codes (+ exponents) and
// V^T codes (+ exponents) are staged in LDS once.  A wave takes 16 consecutive
// query rows (one MFMA tile):
//   per row   the k true scores  fl32(sum_b 2^(eq+ek) I_b) * scale (+ bias)
//             (v_dot4, exact fp64 block epilogue), softmax over them
//             (DPP reductions), zeros.scatter_(idx, softmax), then P -> MXINT8
//             along keys (block maxima by LDS atomic max): the row's codes land in
//             the wave's 16-row P tile in LDS, its block exponents beside it;
//   per tile  out[16][D] = sum_b 2^(eP_rb + eV_bd) * (P_b[16x32] . V_b[32x16])
//             with v_mfma_i32_16x16x32_i8, one MFMA per 32-key MX block and 16
//             output columns: the block's int32 dot is exact, the fp64 epilogue
//             adds the scaled block sums exactly (the MX matmul of P.V,
//             microxscaling/mx/matmul.py:68-76; F7: the reference's fp32 GEMM order
//             is not pinned, the output is compared normwise).
// Callers: workloads/deit/scripts/main.py:124-152, workloads/DiT/models.py:195-225,
// workloads/PixArt/models/MX_transformer_block.py:679-717, :829-859.
#pragma once
#include "mxa_rows2.hpp"

namespace mxa {

constexpr int kFinWaves = 4;  // waves per workgroup

struct FinLds {
  size_t mx, sT, vt, vs, waves, per_wave, tst, total;
};
// per wave: the 16-row P tile (row stride tst = tpad + 8: spreads the banks of the
// MFMA A-operand reads), 16 x 8 block exponents, 16 block maxima
__host__ __device__ inline FinLds fin_lds(int T, int D, int kst, int nbd, int vst, int ntb, int tpad) {
  FinLds L;
  size_t o = 0;
  L.mx = o;
  o += r2_al16((size_t)T * kst);
  L.sT = o;
  o += r2_al16((size_t)T * nbd * 2);
  L.vt = o;
  o += r2_al16((size_t)D * vst);
  L.vs = o;
  o += r2_al16((size_t)ntb * D * 2);
  L.waves = o;
  L.tst = (size_t)tpad + 8;
  L.per_wave = r2_al16(16 * L.tst) + 16 * 8 * 4 + 64;
  L.total = o + (size_t)kFinWaves * L.per_wave;
  (void)ntb;
  return L;
}

template <int S>
__global__ __launch_bounds__(64 * kFinWaves) void attn_finish_kernel(Rows2Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst, vst = a.vst, ntb = a.ntb;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const FinLds L = fin_lds(T, D, kst, nbd, vst, ntb, a.tpad);
  int8_t* tmx = reinterpret_cast<int8_t*>(smem + L.mx);
  int16_t* tsT = reinterpret_cast<int16_t*>(smem + L.sT);
  int8_t* tvt = reinterpret_cast<int8_t*>(smem + L.vt);
  int16_t* tvs = reinterpret_cast<int16_t*>(smem + L.vs);
  unsigned char* wbase = smem + L.waves + (size_t)wave * L.per_wave;
  const int tst = (int)L.tst;
  int8_t* ptile = reinterpret_cast<int8_t*>(wbase);                     // [16][tst] P codes
  int* pe16 = reinterpret_cast<int*>(wbase + r2_al16(16 * L.tst));      // [16][8] P block exponents
  uint32_t* bm = reinterpret_cast<uint32_t*>(pe16 + 16 * 8);            // [16] block maxima

  // ---- stage the head's K codes and V^T tables; clear the P tile ----------
  const int64_t kb = (int64_t)bh * T;
  {
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(tmx + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(a.kc + (kb + j) * a.dpad + 16 * c);
    }
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) tsT[i] = a.ksT[kb * nbd + i];
    const int vpr = a.tpad / 16;
    const int8_t* vsrc = a.vt + (int64_t)bh * D * a.tpad;
    for (int i = threadIdx.x; i < D * vpr; i += blockDim.x) {
      const int d = i / vpr, c = i - d * vpr;
      *reinterpret_cast<uint4*>(tvt + (size_t)d * vst + 16 * c) =
          *reinterpret_cast<const uint4*>(vsrc + (int64_t)d * a.tpad + 16 * c);
    }
    const int16_t* vssrc = a.vs + (int64_t)bh * ntb * D;
    for (int i = threadIdx.x; i < ntb * D; i += blockDim.x) tvs[i] = vssrc[i];
    for (int c = lane; c < 16 * tst / 4; c += 64) reinterpret_cast<uint32_t*>(ptile)[c] = 0u;
    if (lane < 16) bm[lane] = 0u;
  }
  __syncthreads();

  const int r_end = min(a.N, (int)(blockIdx.y + 1) * a.rows_per_wg);
  for (int t0 = (int)blockIdx.y * a.rows_per_wg + 16 * __builtin_amdgcn_readfirstlane(wave); t0 < r_end;
       t0 += 16 * kFinWaves) {
    const int nt = min(16, r_end - t0);
    for (int rr = 0; rr < nt; ++rr) {
      const int r = t0 + rr;
      const int64_t grow = (int64_t)bh * a.N + r;
      const float* brow = a.bias ? a.bias + b_ * a.bs0 + h_ * a.bs1 + (int64_t)r * a.bs2 : nullptr;
      const int8_t* qmx = a.qc + grow * a.dpad;
      // the true score of key j for this row (bias included)
      auto true_of = [&](int j, bool& nan) -> float {
        const double acc = r2_dot<0>(qmx, a.qsT, grow * nbd, nbd, tmx + (size_t)j * kst, tsT + j * nbd, nan);
        float t = round_bfloat(nan ? __uint_as_float(0x7FC00000u) : (float)acc, a.bfloat, kRoundNearest, 1) * a.scale;
        if (brow) t = t + brow[(int64_t)j * a.bs3];
        return t;
      };
      if (a.true_out) {  // debug output: every key's true score
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int j = 64 * s + lane;
          bool nan = false;
          const float t = true_of(min(j, T - 1), nan);
          if (j < T) a.true_out[grow * T + j] = t;
        }
      }
      // ---- vals = true.gather(idx); softmax ------------------------------------
      int ix[S];
      bool kept[S];
      float v[S];
      float mx = -INFINITY;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int pos = 64 * s + lane;
        kept[s] = pos < a.k_top;
        ix[s] = 0;
        v[s] = -INFINITY;
        if (64 * s < a.k_top) {
          ix[s] = kept[s] ? a.idx32[grow * a.k_top + pos] : 0;
          if (kept[s]) {
            bool nan = false;
            v[s] = true_of(ix[s], nan);
            mx = fmaxf(mx, v[s]);
          }
        }
      }
      mx = wave_max_f32(mx);
      float sum = 0.0f;
#pragma unroll
      for (int s = 0; s < S; ++s) {
        v[s] = kept[s] ? expf(v[s] - mx) : 0.0f;
        sum += v[s];
      }
      sum = wave_sum_f32(sum);
      // ---- zeros.scatter_(idx, softmax) -> MXINT8 along keys (row rr of the tile)
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (kept[s]) {
          v[s] = round_bfloat(v[s] / sum, a.bfloat, kRoundNearest, 1);
          atomicMax(&bm[ix[s] >> 5], __float_as_uint(v[s]) & 0x7FFFFFFFu);
        }
      }
      wave_lds_sync();
      if (lane < ntb) {
        int e_raw;
        const int es = scale_exponent(bm[lane], 127, &e_raw);
        const bool fl = a.flush_p && !(e_raw != kExpNaN && e_raw > -127);
        pe16[rr * 8 + lane] = es == kExpNaN ? kExpNaN : es - 6;
        bm[lane] = (es == kExpNaN ? 0u : (uint32_t)(es + 1024)) | (fl ? 0x10000u : 0u);  // 0: NaN block
      }
      wave_lds_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (kept[s]) {
          const uint32_t e = bm[ix[s] >> 5];
          int code = 0;
          if (e & 0xFFFFu) {
            const int es = (int)(e & 0xFFFFu) - 1024;
            const float x = (e & 0x10000u) ? v[s] * 0.0f : v[s];
            code = (int)round_code(x, es, 8, kRoundNearest);
          }
          ptile[rr * tst + ix[s]] = (int8_t)code;
        }
      }
      wave_lds_sync();
      if (lane < 16) bm[lane] = 0u;
    }
    // (rows >= nt of a partial last tile hold zero codes and are not stored)
    wave_lds_sync();

    // ---- out[16][D] = MX(P) @ MX(V): int8 MFMA per 32-key block, fp64 epilogue --
    {
      const int r16 = lane & 15, kg = lane >> 4;
      const int8_t* ap = ptile + r16 * tst + kg * 8;
      for (int c0 = 0; c0 < D; c0 += 16) {
        const int col = min(c0 + r16, D - 1);
        const int8_t* bp = tvt + (size_t)col * vst + kg * 8;
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
        bool nan[4] = {false, false, false, false};
        const v4i zero = {0, 0, 0, 0};
        for (int b = 0; b < ntb; ++b) {
          const long av = *reinterpret_cast<const long*>(ap + 32 * b);
          const long bv = *reinterpret_cast<const long*>(bp + 32 * b);
          const v4i c = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv, zero, 0, 0, 0);
          const int eV = exp_from16(tvs[b * D + col]);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int eP = pe16[(4 * kg + i) * 8 + b];
            if (eP == kExpNaN || eV == kExpNaN) nan[i] = true;
            else acc[i] += (double)c[i] * pow2d(eP + eV);
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = 4 * kg + i;
          if (rr < nt && c0 + r16 < D) {
            const float o = nan[i] ? __uint_as_float(0x7FC00000u) : (float)acc[i];
            a.out[b_ * a.os0 + h_ * a.os1 + (int64_t)(t0 + rr) * a.os2 + c0 + r16] =
                round_bfloat(o, a.bfloat, kRoundNearest, 1);
          }
        }
      }
    }
    // ---- clear the tile for the next 16 rows -------------------------------------
    wave_lds_sync();
    for (int c = lane; c < 16 * tst / 4; c += 64) reinterpret_cast<uint32_t*>(ptile)[c] = 0u;
    wave_lds_sync();
  }
}

}  // namespace mxa
