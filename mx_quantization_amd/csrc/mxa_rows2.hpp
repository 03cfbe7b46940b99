// The dense branch (top_k=False: DeiT block 11, DiT / PixArt excluded timesteps,
// SURVEY.md §8a a13), one wave per query row: all T true scores (v_dot4 over the LDS
// codes, exact fp64 block epilogue), softmax over every key (DPP
// reductions), P MX-quantized along keys into an LDS code row, and
//   out[d] = sum_b 2^(eP_b + eV_bd) * sum_{t in b} P_t V_td
// (v_dot4 of the P row against lane d's V^T row, fp64 block epilogue).  The head's K
// codes + exponents and V^T codes + exponents are staged in LDS once per workgroup.
// Also home of Rows2Args, the argument block of the selection / finishing kernels.
// Callers: workloads/deit/scripts/main.py:100-152, workloads/DiT/models.py:168-225,
// workloads/PixArt/models/MX_transformer_block.py:648-717, :792-859; the MX matmul
// of P.V: microxscaling/mx/matmul.py:68-76.
#pragma once
#include "mxa_modes.hpp"

namespace mxa {

struct Rows2Args {
  // query side (rows_prep outputs)
  const int8_t *qc, *qop, *qz;
  const int16_t *qsT, *qsA;
  const uint32_t* qsg;  // ex_pred sign words / ELSA hash words
  // key side
  const int8_t *kc, *kop, *kz;
  const int16_t *ksT, *ksA;
  const uint32_t* ksg;
  const float* knorm;     // ELSA: key row norms
  const float* elsa_cos;  // ELSA: (D+1) cosine table (nullable)
  // value side (cols_prep outputs: V^T codes [BH][D][tpad], exps [BH][ntb][D])
  const int8_t* vt;
  const int16_t* vs;
  int B, H, N, T, D, nbd, dpad, ntb, tpad;
  int kst, vst;  // LDS row strides of the K code tables and the V^T table
  int k_top, bfloat, flush_p;
  int in_dt;  // dtype of q, k, v and the bias (MXA_DT_*)
  int s_dt;   // dtype of the scores, P and the output (the GEMM outputs: include/mxa.h score_dtype)
  float scale;
  const void* bias;  // dtype in_dt
  int64_t bs0, bs1, bs2, bs3;
  void* out;  // dtype s_dt
  int64_t os0, os1, os2;
  int64_t* idx_out;
  float* true_out;
  float* pred_out;
  uint32_t* mask_out;
  int waves;        // waves per workgroup
  int rows_per_wg;  // query rows per workgroup (grid.y splits a head when there are few heads)
  uint16_t* idx16;  // split path: the kept indices [B*H*N][k_top] between the two kernels when
                    // the caller takes no idx_out (else the finishing kernel reads idx_out)
  int fb_only;      // selection kernel: only the rows the packed pass left (kept_get(row * k) < 0)
  uint32_t* tail_rec;  // the one-lane tail's staging records (mxa_tail.hpp), when it runs
  uint32_t* fb_flags;  // packed selection pass: per workgroup (bh * gy + y), rows left for the 64-bit pass
  int fb_gy;           // the packed pass's gy (fb_only launches)
  // finishing kernel with the proj Linear behind it (D % 32 == 0): the output rows
  // (B, N, H*D) MX-quantized along C straight from the P.V tile -- rows_prep's layout,
  // codes [B*N][H*D], code-unit exponents [B*N][H*D/32] -- instead of fp32 in `out`
  int8_t* xo_codes;
  int16_t* xo_exps;
  // the dense branch (top_k=False) on the MFMA finishing kernel (mxa_finish_qk.hpp): every
  // key < T kept, no prune-mask words read
  int dense;
};

// words of a one-lane top-k tail staging record (mxa_tail.hpp): state, pad, TW elements
__host__ __device__ constexpr int tail_rec_words(int TW) { return TW + 4; }

// the kept indices between the selection and the finishing kernel: the caller's int64
// idx_out when it takes one (no second copy), else a 16-bit copy in the workspace; -1
// (0xFFFF) marks a row the packed selection pass left for the 64-bit one
__device__ __forceinline__ int kept_get(const Rows2Args& a, int64_t i) {
  if (a.idx_out) return (int)a.idx_out[i];
  const uint32_t v = a.idx16[i];
  return v == 0xFFFFu ? -1 : (int)v;
}
__device__ __forceinline__ void kept_put(const Rows2Args& a, int64_t i, int ix) {
  if (a.idx_out) a.idx_out[i] = (int64_t)ix;
  else a.idx16[i] = (uint16_t)ix;
}


struct Rows2Lds {
  size_t mx, sT, vt, vs, waves, per_wave, total;
};

__host__ __device__ inline size_t r2_al16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS of the dense kernel: K codes + exponents, V^T codes + exponents, then per wave
// the P code row, P block exponents and block maxima (16 each)
__host__ __device__ inline Rows2Lds rows2_lds(int T, int D, int kst, int nbd, int vst, int ntb, int tpad, int waves) {
  Rows2Lds L;
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
  L.per_wave = r2_al16((size_t)tpad) + 64 + 64;
  L.total = o + (size_t)waves * L.per_wave;
  return L;
}

// the true score of key row krow (MXINT8 codes in LDS, exponents kexp) against the
// uniform query codes qw / exponents qe: fl32(exact sum) * scale, bfloat-rounded
template <int MUL>
__device__ __forceinline__ double r2_dot(const int8_t* qrow, const int16_t* qs, int64_t qs0, int nbd,
                                         const int8_t* krow, const int16_t* kexp, bool& nan) {
  double acc = 0.0;
#pragma unroll
  for (int b = 0; b < kMaxNB; ++b) {
    if (b < nbd) {
      const cu32 src = (cu32)(qrow + 32 * b);  // scalar loads: 8 SGPRs live per block
      uint32_t qw[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) qw[c] = src[c];
      const int qe = s_exp16(qs, qs0 + b);
      const uint4 x0 = *reinterpret_cast<const uint4*>(krow + 32 * b);
      const uint4 x1 = *reinterpret_cast<const uint4*>(krow + 32 * b + 16);
      int I = 0;
      I = __builtin_amdgcn_sdot4((int)qw[0], (int)x0.x, I, false);
      I = __builtin_amdgcn_sdot4((int)qw[1], (int)x0.y, I, false);
      I = __builtin_amdgcn_sdot4((int)qw[2], (int)x0.z, I, false);
      I = __builtin_amdgcn_sdot4((int)qw[3], (int)x0.w, I, false);
      I = __builtin_amdgcn_sdot4((int)qw[4], (int)x1.x, I, false);
      I = __builtin_amdgcn_sdot4((int)qw[5], (int)x1.y, I, false);
      I = __builtin_amdgcn_sdot4((int)qw[6], (int)x1.z, I, false);
      I = __builtin_amdgcn_sdot4((int)qw[7], (int)x1.w, I, false);
      const int e = exp_from16(kexp[b]);
      if (e == kExpNaN || qe == kExpNaN) nan = true;
      else if (MUL) acc += (double)I * (double)(qe * e) * (1.0 / 4096.0);
      else acc += (double)I * pow2d(qe + e);
    }
  }
  return acc;
}

template <int S>
__global__ __launch_bounds__(1024, 1) void dense_rows_kernel(Rows2Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, nbd = a.nbd, kst = a.kst, vst = a.vst, ntb = a.ntb;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const Rows2Lds L = rows2_lds(T, D, kst, nbd, vst, ntb, a.tpad, a.waves);
  int8_t* tmx = reinterpret_cast<int8_t*>(smem + L.mx);
  int16_t* tsT = reinterpret_cast<int16_t*>(smem + L.sT);
  int8_t* tvt = reinterpret_cast<int8_t*>(smem + L.vt);
  int16_t* tvs = reinterpret_cast<int16_t*>(smem + L.vs);
  unsigned char* wbase = smem + L.waves + (size_t)wave * L.per_wave;
  int8_t* prow = reinterpret_cast<int8_t*>(wbase);
  int* pe = reinterpret_cast<int*>(wbase + r2_al16(a.tpad));

  // ---- stage the head's K and V tables ---------------------------------------
  const int64_t kb = (int64_t)bh * T;
  {
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(tmx + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(a.kc + (kb + j) * a.dpad + 16 * c);
    }
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) tsT[i] = a.ksT[kb * nbd + i];
    // V^T codes, token-block-major in HBM ([ntb][D][32] per head: contiguous 2-KB runs)
    const int8_t* vsrc = a.vt + (int64_t)bh * D * a.tpad;
    for (int i = threadIdx.x; i < a.ntb * D * 2; i += blockDim.x) {
      const int half = i & 1, dd = (i >> 1) % D, tb = (i >> 1) / D;
      *reinterpret_cast<uint4*>(tvt + (size_t)dd * vst + 32 * tb + 16 * half) =
          *reinterpret_cast<const uint4*>(vsrc + ((int64_t)tb * D + dd) * 32 + 16 * half);
    }
    const int16_t* vssrc = a.vs + (int64_t)bh * ntb * D;
    for (int i = threadIdx.x; i < ntb * D; i += blockDim.x) tvs[i] = vssrc[i];
  }
  __syncthreads();

  const int r_end = min(a.N, (int)(blockIdx.y + 1) * a.rows_per_wg);
  for (int r = (int)blockIdx.y * a.rows_per_wg + __builtin_amdgcn_readfirstlane(wave); r < r_end; r += a.waves) {
    const int64_t grow = (int64_t)bh * a.N + r;
    const int64_t brow = a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)r * a.bs2 : -1;
    const int8_t* qmx = a.qc + grow * a.dpad;

    // ---- the row's T true scores in position order ----------------------------
    float vals[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = min(64 * s + lane, T - 1);  // clamped: no exec branch
      bool nan = false;
      const double acc = r2_dot<0>(qmx, a.qsT, grow * nbd, nbd, tmx + (size_t)j * kst, tsT + j * nbd, nan);
      // true = quantize_elemwise(fl32(QK^T)) * scale   (matmul.py:88-91, caller)
      vals[s] = round_dt(round_bfloat(round_dt(nan ? __uint_as_float(0x7FC00000u) : (float)acc, a.s_dt), a.bfloat,
                                      kRoundNearest, 1, a.s_dt) * a.scale, a.s_dt);
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int j = 64 * s + lane;
      if (j < T) {
        if (brow >= 0) vals[s] = round_dt(vals[s] + load_dt(a.bias, brow + (int64_t)j * a.bs3, a.in_dt), a.s_dt);
        if (a.true_out) a.true_out[grow * T + j] = vals[s];
      }
    }

    // ---- attn = softmax(true) over every key ------------------------------------
    float mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      if (pos >= T) vals[s] = -INFINITY;
      mx = fmaxf(mx, vals[s]);
    }
    mx = wave_max_f32(mx);
    float sum = 0.0f;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      vals[s] = pos < T ? expf(vals[s] - mx) : 0.0f;
      sum += vals[s];
    }
    sum = wave_sum_f32(sum);
    // ---- MX(P) along keys: one 32-block per half-wave ----------------------------
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      if (s * 64 >= a.tpad) break;
      const float x = round_dt(round_bfloat(vals[s] / sum, a.bfloat, kRoundNearest, 1, a.s_dt), a.s_dt);
      const uint32_t mb = half_reduce(__float_as_uint(x) & 0x7FFFFFFFu,
                                      [](uint32_t u, uint32_t w) { return u > w ? u : w; });
      int e_raw;
      const int es = scale_exponent_dt(mb, 127, a.s_dt, &e_raw);
      float xv = x;
      if (a.flush_p && !(e_raw != kExpNaN && e_raw > -127)) xv = xv * 0.0f;
      const int code = es == kExpNaN ? 0 : (int)round_code(xv, es, 8, kRoundNearest, a.s_dt);
      if (pos < a.tpad) {
        prow[pos] = (int8_t)code;
        if ((lane & 31) == 0) pe[pos >> 5] = es == kExpNaN ? kExpNaN : es - 6;
      }
    }
    wave_lds_sync();

    // ---- out = MX(P) @ MX(V): v_dot4 over 16 keys per read, fp64 block epilogue
    {
      double acc[2] = {0.0, 0.0};
      bool nan[2] = {false, false};
      const int dsl = D > 64 ? 2 : 1;
      for (int blk = 0; blk < ntb; ++blk) {
        const uint4 p0 = *reinterpret_cast<const uint4*>(prow + 32 * blk);
        const uint4 p1 = *reinterpret_cast<const uint4*>(prow + 32 * blk + 16);
        const int ep = pe[blk];
#pragma unroll
        for (int ds = 0; ds < 2; ++ds) {
          if (ds < dsl) {
            const int d = min(64 * ds + lane, D - 1);
            const int8_t* vr = tvt + (size_t)d * vst + 32 * blk;
            const uint4 x0 = *reinterpret_cast<const uint4*>(vr);
            const uint4 x1 = *reinterpret_cast<const uint4*>(vr + 16);
            int I = 0;
            I = __builtin_amdgcn_sdot4((int)p0.x, (int)x0.x, I, false);
            I = __builtin_amdgcn_sdot4((int)p0.y, (int)x0.y, I, false);
            I = __builtin_amdgcn_sdot4((int)p0.z, (int)x0.z, I, false);
            I = __builtin_amdgcn_sdot4((int)p0.w, (int)x0.w, I, false);
            I = __builtin_amdgcn_sdot4((int)p1.x, (int)x1.x, I, false);
            I = __builtin_amdgcn_sdot4((int)p1.y, (int)x1.y, I, false);
            I = __builtin_amdgcn_sdot4((int)p1.z, (int)x1.z, I, false);
            I = __builtin_amdgcn_sdot4((int)p1.w, (int)x1.w, I, false);
            const int ev = exp_from16(tvs[blk * D + d]);
            if (ep == kExpNaN || ev == kExpNaN) nan[ds] = true;
            else acc[ds] += (double)I * pow2d(ep + ev);
          }
        }
      }
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const int d = 64 * ds + lane;
        if (ds < dsl && d < D) {
          const float o = nan[ds] ? __uint_as_float(0x7FC00000u) : (float)acc[ds];
          store_dt(a.out, b_ * a.os0 + h_ * a.os1 + (int64_t)r * a.os2 + d,
                   round_bfloat(round_dt(o, a.s_dt), a.bfloat, kRoundNearest, 1, a.s_dt), a.s_dt);
        }
      }
    }
    wave_lds_sync();
  }
}

}  // namespace mxa
