// Finishing kernel of the top-k path, 16-ROW TILES: for every query row and its k
// kept keys (the selection kernel's indices) the true scores, softmax, MX(P) along
// keys and P.V, with P.V on v_mfma_i32_16x16x32_i8.
//
// Why 16-row tiles (against the 32-row tiles of mxa_finish.hpp): the per-wave LDS is the
// P code tile of the wave's rows, so halving the tile halves it, and the V^T operand is
// read straight from HBM / L2 -- token-block-major V^T codes give each 16 x 32 MFMA B
// operand as one contiguous 512-B run, so the loads coalesce -- instead of being staged
// in LDS; only the head's K table (the gathered keys of the true scores) stays in LDS.
// That lets twice the waves stay resident to hide the gather / softmax latency, which is
// what bounds this kernel (SQ_WAIT_ANY, not the VALU or the MFMA, in the PMC passes).
//
// Per workgroup (one head, or a chunk of its query rows): the head's K codes + exponents
// and the V block exponents staged in LDS once.  Per wave, tiles of 16 query rows:
//   1. LPR = 4: the 16 rows in one pass, four lanes per row (k <= 4 KS; DeiT's k = 20);
//      LPR = 16: four passes of four rows, one 16-lane DPP row per query row (DiT's
//      k = 154).  Lane slots s, s + LPR, ...: the kept key's true score fl32(exact sum)
//      * scale (+ bias) by v_dot4 over the LDS codes (exact block epilogue);
//      softmax over the kept scores (DPP reductions); P MX-quantized along keys (block
//      maxima by LDS atomic max) into the tile's dense code rows (zero elsewhere).
//   2. P.V for the tile: per 16 output columns and per 32-key MX block ONE
//      v_mfma_i32_16x16x32_i8 (K = 32 = one block: each block keeps its exact int32 sum),
//      epilogue acc += C * (sP[row][b] * sV[b][d]) in fp32 (P.V is a tolerance-only
//      product).
//   3. the tile's output rows go out.  (The proj Linear's MX input codes stay on the
//      32-row kernel, whose 32 x 32 output blocks are whole MX blocks of the rows.)
// Reference: microxscaling/mx/matmul.py:68-76 (MX P.V), callers
// workloads/deit/scripts/main.py:124-152, workloads/DiT/models.py:195-225,
// workloads/PixArt/models/MX_transformer_block.py:679-717, :826-859.
#pragma once
#include "mxa_finish.hpp"

namespace mxa {

constexpr int kFin16 = 16;  // query rows per MFMA tile (one wave)
constexpr int kFin16Occ = 4;  // waves per SIMD the register allocation aims at
// (the MFMA B operands, V^T codes, come straight from memory: staged in LDS with the K
// table they measured 0.214 ms at 3 waves per SIMD against 0.200 ms at 4, DeiT-base)

typedef int v4i16_ __attribute__((ext_vector_type(4)));

// LDS: tables (K codes, K exponents, V block exponents), then per wave the P code tile
// [16][vst], the P block scales sP [ntb][16] (float), the block maxima bm [16][ntb] (u32)
struct Fin16Lds {
  size_t kc, ke, vt, ve, waves, per_wave, sp, bm, total;
};
__host__ __device__ inline Fin16Lds fin16_lds(int T, int D, int kst, int nbd, int vst, int ntb, int waves) {
  Fin16Lds L;
  size_t o = 0;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  L.kc = o;
  o += al((size_t)T * kst);
  L.ke = o;
  o += al((size_t)T * nbd * 2);
  L.vt = o;
  L.ve = o;
  o += al((size_t)ntb * D * 2);
  L.waves = o;
  L.sp = al((size_t)kFin16 * vst);
  L.bm = L.sp + al((size_t)ntb * kFin16 * 4);
  L.per_wave = L.bm + al((size_t)kFin16 * ntb * 4);
  L.total = o + (size_t)waves * L.per_wave;
  return L;
}

template <int NB, int KS, int LPR, bool XDT>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(NB <= 2 && KS <= 12 ? kFin16Occ : (NB * KS <= 64 ? 3 : 2), 8))) void finish16_kernel(Rows2Args a) {
  static_assert(LPR == 4 || LPR == 16, "four or sixteen lanes per query row");
  const int sdt = XDT ? a.s_dt : (int)kF32, idt = XDT ? a.in_dt : (int)kF32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, kst = a.kst, vst = a.vst, ntb = a.ntb, k = a.k_top;
  constexpr int nbd = NB;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const Fin16Lds L = fin16_lds(T, D, kst, nbd, vst, ntb, a.waves);
  int8_t* tkc = reinterpret_cast<int8_t*>(smem + L.kc);
  int16_t* tke = reinterpret_cast<int16_t*>(smem + L.ke);
  int16_t* tve = reinterpret_cast<int16_t*>(smem + L.ve);
  unsigned char* wb = smem + L.waves + (size_t)wave * L.per_wave;
  int8_t* ptile = reinterpret_cast<int8_t*>(wb);
  float* sP = reinterpret_cast<float*>(wb + L.sp);
  // the lane's query row within its pass (LPR 4: the tile row; LPR 16: the pass row)
  // and its slot phase
  const int pr = LPR == 4 ? lane >> 2 : lane >> 4, ph = LPR == 4 ? lane & 3 : lane & 15;
  uint32_t* bmw = reinterpret_cast<uint32_t*>(wb + L.bm);  // [16][ntb]

  // ---- stage the head's K table and V block exponents; clear the code tile ---------
  const int64_t kb = (int64_t)bh * T;
  {
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(tkc + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(a.kc + (kb + j) * a.dpad + 16 * c);
    }
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) tke[i] = a.ksT[kb * nbd + i];
    const int16_t* vssrc = a.vs + (int64_t)bh * ntb * D;
    for (int i = threadIdx.x; i < ntb * D; i += blockDim.x) tve[i] = vssrc[i];
    for (int i = lane; i < kFin16 * vst / 16; i += 64) reinterpret_cast<uint4*>(ptile)[i] = make_uint4(0, 0, 0, 0);
    for (int i = lane; i < kFin16 * ntb; i += 64) bmw[i] = 0u;
  }
  __syncthreads();

  const int r_beg = (int)blockIdx.y * a.rows_per_wg, r_end = min(a.N, r_beg + a.rows_per_wg);
  constexpr int kPasses = LPR == 4 ? 1 : kFin16 / 4;
  // a pass's global inputs (the row's query codes / exponents and kept indices); loaded
  // at the start of the pass -- the resident waves hide their latency (a copy loaded one
  // pass ahead costs the registers of a resident wave)
  struct PassIn {
    uint4 qv[2 * NB];
    int qe[NB];
    int ix[KS];
  };
  auto load_pass = [&](int r0, int pass, PassIn& in) {
    const int r = r0 + (LPR == 4 ? pr : 4 * pass + pr);
    const bool valid = r < r_end;
    const int64_t grow = (int64_t)bh * a.N + (valid ? r : r_beg);
    const int8_t* qsrc = a.qc + grow * a.dpad;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      in.qv[2 * b] = *reinterpret_cast<const uint4*>(qsrc + 32 * b);
      in.qv[2 * b + 1] = *reinterpret_cast<const uint4*>(qsrc + 32 * b + 16);
      in.qe[b] = exp_from16(a.qsT[grow * nbd + b]);
    }
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const int s = ph + LPR * t;
      in.ix[t] = valid && s < k ? kept_get(a, grow * k + s) : -1;
    }
  };

  for (int r0 = r_beg + kFin16 * wave; r0 < r_end; r0 += kFin16 * a.waves) {
    // ---- 1. kept scores, softmax, MX(P) into the code tile ------------------------------
    for (int pass = 0; pass < kPasses; ++pass) {
      PassIn cur;
      load_pass(r0, pass, cur);
      const int tr = LPR == 4 ? pr : 4 * pass + pr;  // row within the tile
      const int r = r0 + tr;
      const bool valid = r < r_end;
      const int64_t grow = (int64_t)bh * a.N + (valid ? r : r0);
      const int64_t brow = a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)(valid ? r : r0) * a.bs2 : -1;
      auto true_of = [&](int j) -> float {  // true = quantize_elemwise(fl32(QK^T)) * scale (+ bias)
        const float acc = true_dot<NB>(cur.qv, cur.qe, tkc + (size_t)j * kst, tke + j * nbd);
        float t = round_bfloat(round_dt(acc, sdt), a.bfloat, kRoundNearest, 1, sdt);
        t = round_dt(t * a.scale, sdt);
        if (brow >= 0) t = round_dt(t + load_dt(a.bias, brow + (int64_t)j * a.bs3, idt), sdt);
        return t;
      };
      if (a.true_out && valid)  // debug output: every key's true score
        for (int j = ph; j < T; j += LPR) a.true_out[grow * T + j] = true_of(j);
      auto rmax = [](float x) {
        uint32_t u = __float_as_uint(x);
        auto op = [](uint32_t p, uint32_t q) { return __float_as_uint(fmaxf(__uint_as_float(p), __uint_as_float(q))); };
        u = op(u, dpp_u32<0xB1>(u));
        u = op(u, dpp_u32<0x4E>(u));
        if (LPR == 16) {
          u = op(u, dpp_u32<0x141>(u));
          u = op(u, dpp_u32<0x140>(u));
        }
        return __uint_as_float(u);
      };
      auto rsum = [](float x) {
        uint32_t u = __float_as_uint(x);
        auto op = [](uint32_t p, uint32_t q) { return __float_as_uint(__uint_as_float(p) + __uint_as_float(q)); };
        u = op(u, dpp_u32<0xB1>(u));
        u = op(u, dpp_u32<0x4E>(u));
        if (LPR == 16) {
          u = op(u, dpp_u32<0x141>(u));
          u = op(u, dpp_u32<0x140>(u));
        }
        return __uint_as_float(u);
      };
      float v[KS];
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        v[t] = cur.ix[t] >= 0 ? true_of(cur.ix[t]) : -INFINITY;
        mx = fmaxf(mx, v[t]);
      }
      mx = rmax(mx);
      float sum = 0.0f;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        v[t] = cur.ix[t] >= 0 ? expf(v[t] - mx) : 0.0f;
        sum += v[t];
      }
      sum = rsum(sum);
      // zeros.scatter_(idx, softmax) -> MXINT8 along keys (block maxima by atomic max)
      uint32_t* bm = bmw + tr * ntb;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        if (cur.ix[t] >= 0) {
          v[t] = round_dt(round_bfloat(v[t] / sum, a.bfloat, kRoundNearest, 1, sdt), sdt);
          atomicMax(&bm[cur.ix[t] >> 5], __float_as_uint(v[t]) & 0x7FFFFFFFu);
        }
      }
      wave_lds_sync();
      for (int bk = ph; bk < ntb; bk += LPR) {  // block bk: scale exponent (+1024; 0 = NaN block), flush flag
        int e_raw;
        const int es = scale_exponent_dt(bm[bk], 127, sdt, &e_raw);
        const bool fl = a.flush_p && !(e_raw != kExpNaN && e_raw > -127);
        sP[bk * kFin16 + tr] = scale_f(es == kExpNaN ? kExpNaN : es - 6);
        bm[bk] = (es == kExpNaN ? 0u : (uint32_t)(es + 1024)) | (fl ? 0x10000u : 0u);
      }
      wave_lds_sync();
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        if (cur.ix[t] >= 0) {
          const uint32_t e = bm[cur.ix[t] >> 5];
          int code = 0;
          if (e & 0xFFFFu) {
            const int es = (int)(e & 0xFFFFu) - 1024;
            const float x = (e & 0x10000u) ? v[t] * 0.0f : v[t];
            code = (int)round_code(x, es, 8, kRoundNearest, sdt);
          }
          ptile[tr * vst + cur.ix[t]] = (int8_t)code;
        }
      }
      wave_lds_sync();
      for (int bk = ph; bk < ntb; bk += LPR) bm[bk] = 0u;
    }
    wave_lds_sync();

    // ---- 2. P.V on int8 MFMA: one v_mfma_i32_16x16x32_i8 per (16 columns, key block) ----
    // lane maps (checked on hardware by mxa_selftest_mfma): A[m][k], m = lane % 16,
    // k = 8 (lane / 16) + 0..7; B[k][n], n = lane % 16, the same k; C[m][n] in c[i],
    // m = 4 (lane / 16) + i, n = lane % 16.  B (V^T) straight from memory: the head's
    // codes are [ntb][D][32], so the operand of (block b, columns dt..dt+15) is one
    // contiguous 512-B run.
    const int ln = lane & 15, kg = lane >> 4;
    const int8_t* vbase = a.vt + (int64_t)bh * D * a.tpad + 8 * kg;
    for (int dt = 0; dt < D; dt += 16) {
      const int d = min(dt + ln, D - 1);
      float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      for (int b0 = 0; b0 < ntb; b0 += 4) {  // the B operands of up to 4 blocks in flight
        int64_t bv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (b0 + u < ntb) bv[u] = *reinterpret_cast<const int64_t*>(vbase + ((int64_t)(b0 + u) * D + d) * 32);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int b = b0 + u;
          if (b < ntb) {
            const int64_t av = *reinterpret_cast<const int64_t*>(ptile + ln * vst + 32 * b + 8 * kg);
            const v4i16_ zero = {0, 0, 0, 0};
            const v4i16_ c = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv[u], zero, 0, 0, 0);
            const float sv = scale_f(exp_from16(tve[b * D + d]));
            const float4 s4 = *reinterpret_cast<const float4*>(sP + b * kFin16 + 4 * kg);
            acc[0] = fmaf((float)c[0], s4.x * sv, acc[0]);
            acc[1] = fmaf((float)c[1], s4.y * sv, acc[1]);
            acc[2] = fmaf((float)c[2], s4.z * sv, acc[2]);
            acc[3] = fmaf((float)c[3], s4.w * sv, acc[3]);
          }
        }
      }
      // ---- 3. output rows (64-B segments per row) ------------------------------------
      if (dt + ln < D) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = r0 + 4 * kg + i;
          if (r < r_end)
            store_dt(a.out, b_ * a.os0 + h_ * a.os1 + (int64_t)r * a.os2 + dt + ln,
                     round_bfloat(round_dt(acc[i], sdt), a.bfloat, kRoundNearest, 1, sdt), sdt);
        }
      }
    }
    wave_lds_sync();
    for (int i = lane; i < kFin16 * vst / 16; i += 64) reinterpret_cast<uint4*>(ptile)[i] = make_uint4(0, 0, 0, 0);
    wave_lds_sync();
  }
}

}  // namespace mxa
