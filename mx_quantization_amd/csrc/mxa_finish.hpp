// Finishing kernel of the top-k path: for every query row and its k kept keys
// (select_kernel's indices), the true scores, softmax, MX(P) along keys and P.V,
// with P.V on int8 MFMA.
//
// Per workgroup (one head, or a chunk of its query rows when there are few heads):
// the head's K codes + exponents and V^T codes + exponents are staged in LDS once.
// Per wave, tiles of 32 query rows:
//   1. eight passes of four rows, one 16-lane DPP row per query row (the layout of
//      select_kernel): lane gl takes kept slots gl, gl+16, ...; the kept key's true
//      score fl32(exact sum) * scale (+ bias) by v_dot4 over the LDS codes with an
//      exact fp64 block epilogue; softmax over the kept scores (DPP
//      row reductions); P MX-quantized along keys (block maxima by LDS atomic max)
//      into the tile's dense code rows in LDS (zero elsewhere), block scales as
//      floats (NaN for a NaN block);
//   2. P.V for the tile: per 32 output columns and per 32-key MX block ONE
//      v_mfma_i32_32x32x32_i8 (K = 32 = one block, so each block keeps its exact
//      int32 sum), epilogue acc += C * (sP[row][b] * sV[b][d]) in fp32 (P.V is a
//      tolerance-only product);
//   3. the tile's output rows are written as 128-B row segments and its code rows
//      are cleared for the next tile.
// Reference: microxscaling/mx/matmul.py:68-76 (MX P.V), callers
// workloads/deit/scripts/main.py:124-152, workloads/DiT/models.py:195-225,
// workloads/PixArt/models/MX_transformer_block.py:679-717, :826-859.
#pragma once
#include "mxa_prep.hpp"
#include "mxa_dot.hpp"

namespace mxa {

constexpr int kFinTile = 32;  // query rows per MFMA tile (one wave)

typedef int v16i __attribute__((ext_vector_type(16)));
typedef int v4i_ __attribute__((ext_vector_type(4)));

// LDS layout: tables, then per wave the P code tile [32][vst], the P block scales
// sP [ntb][32] (float), the block maxima bm [4][16] (u32, one DPP row each)
struct FinLds {
  size_t kc, ke, vt, ve, waves, per_wave, sp, bm, ot, total;
};
// xo: + the 32 x 32 fp32 output block being MX-quantized for the proj Linear
__host__ __device__ inline FinLds fin_lds(int T, int D, int kst, int nbd, int vst, int ntb, int waves, bool pair,
                                          bool xo = false) {
  FinLds L;
  size_t o = 0;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  L.kc = o;
  o += al((size_t)T * kst);
  L.ke = o;
  o += al((size_t)T * nbd * 2);
  L.vt = o;
  o += al((size_t)D * vst);
  L.ve = o;
  o += al((size_t)ntb * D * 2);
  L.waves = o;
  L.sp = al((size_t)kFinTile * vst);
  L.bm = L.sp + al((size_t)ntb * kFinTile * 4);
  L.ot = L.bm + (pair ? 32 : 4) * 16 * 4;  // block maxima: 16 per row of a pass
  L.per_wave = L.ot + (xo ? kFinTile * 33 * 4 : 0);
  L.total = o + (size_t)waves * L.per_wave;
  return L;
}

// exact 2^e as float (subnormal below -126, 0 below -149); NaN for the NaN exponent
__device__ __forceinline__ float scale_f(int e) {
  return e == kExpNaN ? __uint_as_float(0x7FC00000u) : (e < -149 ? 0.0f : pow2f(e));
}

// NB: 32-blocks per head dim (nbd); KS: kept slots per lane.
// PAIR = false: eight passes of four rows per tile, one 16-lane DPP row per query row
//   (k <= 16 KS; DiT's k = 154);
// PAIR = true: the tile's 32 rows in ONE pass, two lanes per query row (k <= 2 KS <= 32,
//   DeiT's k = 20): every lane busy, one round of softmax / MX(P) synchronisation per
//   tile instead of eight.
// XDT: float16 / bfloat16 inputs or scores (include/mxa.h dtype / score_dtype): the
// dtype roundings at run time; XDT = false compiles them away (the float32 path).
// XO: the output goes to the proj Linear as MX codes along C (Rows2Args::xo_codes;
// float32, D % 32 == 0: every 32-column P.V tile is one MX block of the output row)
template <int NB, int KS, bool PAIR, bool XDT, bool XO = false>
__global__ __launch_bounds__(512) void finish_kernel(Rows2Args a) {
  const int sdt = XDT ? a.s_dt : (int)kF32, idt = XDT ? a.in_dt : (int)kF32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, gi = lane >> 4, gl = lane & 15;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, kst = a.kst, vst = a.vst, ntb = a.ntb, k = a.k_top;
  constexpr int nbd = NB;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const FinLds L = fin_lds(T, D, kst, nbd, vst, ntb, a.waves, PAIR, XO);
  int8_t* tkc = reinterpret_cast<int8_t*>(smem + L.kc);
  int16_t* tke = reinterpret_cast<int16_t*>(smem + L.ke);
  int8_t* tvt = reinterpret_cast<int8_t*>(smem + L.vt);
  int16_t* tve = reinterpret_cast<int16_t*>(smem + L.ve);
  unsigned char* wb = smem + L.waves + (size_t)wave * L.per_wave;
  int8_t* ptile = reinterpret_cast<int8_t*>(wb);
  float* sP = reinterpret_cast<float*>(wb + L.sp);
  // block maxima of the P row being quantized: 16 words per row (T <= 512)
  uint32_t* bm = reinterpret_cast<uint32_t*>(wb + L.bm) + 16 * (PAIR ? (lane >> 1) : gi);

  // ---- stage the head's K and V tables; clear the code tile -----------------------
  const int64_t kb = (int64_t)bh * T;
  {
    const int cpr = a.dpad / 16;
    for (int i = threadIdx.x; i < T * cpr; i += blockDim.x) {
      const int j = i / cpr, c = i - j * cpr;
      *reinterpret_cast<uint4*>(tkc + (size_t)j * kst + 16 * c) =
          *reinterpret_cast<const uint4*>(a.kc + (kb + j) * a.dpad + 16 * c);
    }
    for (int i = threadIdx.x; i < T * nbd; i += blockDim.x) tke[i] = a.ksT[kb * nbd + i];
    // V^T codes, token-block-major in HBM ([ntb][D][32] per head: contiguous 2-KB runs)
    const int8_t* vsrc = a.vt + (int64_t)bh * D * a.tpad;
    for (int i = threadIdx.x; i < a.ntb * D * 2; i += blockDim.x) {
      const int half = i & 1, dd = (i >> 1) % D, tb = (i >> 1) / D;
      *reinterpret_cast<uint4*>(tvt + (size_t)dd * vst + 32 * tb + 16 * half) =
          *reinterpret_cast<const uint4*>(vsrc + ((int64_t)tb * D + dd) * 32 + 16 * half);
    }
    const int16_t* vssrc = a.vs + (int64_t)bh * ntb * D;
    for (int i = threadIdx.x; i < ntb * D; i += blockDim.x) tve[i] = vssrc[i];
    for (int i = lane; i < kFinTile * vst / 16; i += 64) reinterpret_cast<uint4*>(ptile)[i] = make_uint4(0, 0, 0, 0);
    if (PAIR) {
      for (int i = lane & 1; i < 16; i += 2) bm[i] = 0u;
    } else {
      bm[gl] = 0u;
    }
  }
  __syncthreads();

  const int r_beg = (int)blockIdx.y * a.rows_per_wg, r_end = min(a.N, r_beg + a.rows_per_wg);

    // a pass's global inputs (the row's query codes / exponents and kept indices),
    // loaded one pass ahead so that their latency hides behind the previous pass
    struct PassIn {
      uint4 qv[2 * NB];
      int qe[NB];
      int ix[KS];
    };
    auto load_pass = [&](int r0, int pass, PassIn& in) {
      const int r = r0 + 4 * pass + gi;
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
        const int s = gl + 16 * t;
        in.ix[t] = valid && s < k ? kept_get(a, grow * k + s) : -1;
      }
    };
    PassIn nxt;
    if (!PAIR && r_beg + kFinTile * wave < r_end) load_pass(r_beg + kFinTile * wave, 0, nxt);
  // PAIR: the tile's inputs, loaded one tile ahead
  struct TileIn {
    uint4 qv[2 * NB];
    int qe[NB];
    int ix[KS];
  };
  const int pr = lane >> 1, ph = lane & 1;  // PAIR: the lane's row within the tile, its half
  auto load_tile = [&](int r0, TileIn& in) {
    const int r = r0 + pr;
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
      const int sl = ph + 2 * t;
      in.ix[t] = valid && sl < k ? kept_get(a, grow * k + sl) : -1;
    }
  };
  TileIn tnxt;
  if (PAIR && r_beg + kFinTile * wave < r_end) load_tile(r_beg + kFinTile * wave, tnxt);
  for (int r0 = r_beg + kFinTile * wave; r0 < r_end; r0 += kFinTile * a.waves) {
    if constexpr (PAIR) {
      // ---- 1. kept scores, softmax, MX(P) of the tile's 32 rows: two lanes per row ----
      const TileIn cur = tnxt;
      if (r0 + kFinTile * a.waves < r_end) load_tile(r0 + kFinTile * a.waves, tnxt);
      const int r = r0 + pr;
      const bool valid = r < r_end;
      const int64_t grow = (int64_t)bh * a.N + (valid ? r : r0);
      const int64_t brow = a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)(valid ? r : r0) * a.bs2 : -1;
      auto true_of = [&](int j) -> float {  // true = quantize_elemwise(fl32(QK^T)) * scale (+ bias)
        const float acc = true_dot<NB>(cur.qv, cur.qe, tkc + (size_t)j * kst, tke + j * nbd);
        // (true scores in the score dtype: the matmul's output, then * scale, + bias)
        float t = round_bfloat(round_dt(acc, sdt), a.bfloat, kRoundNearest,
                              1, sdt);
        t = round_dt(t * a.scale, sdt);
        if (brow >= 0) t = round_dt(t + load_dt(a.bias, brow + (int64_t)j * a.bs3, idt), sdt);
        return t;
      };
      if (a.true_out && valid)  // debug output: every key's true score
        for (int j = ph; j < T; j += 2) a.true_out[grow * T + j] = true_of(j);
      float v[KS];
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        v[t] = cur.ix[t] >= 0 ? true_of(cur.ix[t]) : -INFINITY;
        mx = fmaxf(mx, v[t]);
      }
      mx = fmaxf(mx, __uint_as_float(dpp_u32<0xB1>(__float_as_uint(mx))));
      float sum = 0.0f;
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        v[t] = cur.ix[t] >= 0 ? expf(v[t] - mx) : 0.0f;
        sum += v[t];
      }
      sum = sum + __uint_as_float(dpp_u32<0xB1>(__float_as_uint(sum)));
      // zeros.scatter_(idx, softmax) -> MXINT8 along keys (block maxima by atomic max)
#pragma unroll
      for (int t = 0; t < KS; ++t) {
        if (cur.ix[t] >= 0) {
          v[t] = round_dt(round_bfloat(v[t] / sum, a.bfloat, kRoundNearest, 1, sdt), sdt);
          atomicMax(&bm[cur.ix[t] >> 5], __float_as_uint(v[t]) & 0x7FFFFFFFu);
        }
      }
      wave_lds_sync();
      for (int bk = ph; bk < ntb; bk += 2) {  // block bk: scale exponent (+1024; 0 = NaN block), flush flag
        int e_raw;
        const int es = scale_exponent_dt(bm[bk], 127, sdt, &e_raw);
        const bool fl = a.flush_p && !(e_raw != kExpNaN && e_raw > -127);
        sP[bk * kFinTile + pr] = scale_f(es == kExpNaN ? kExpNaN : es - 6);
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
          ptile[pr * vst + cur.ix[t]] = (int8_t)code;
        }
      }
      wave_lds_sync();
      for (int bk = ph; bk < ntb; bk += 2) bm[bk] = 0u;
      wave_lds_sync();
    } else {
    // ---- 1. kept scores, softmax, MX(P) into the code tile: four rows per pass ----
      for (int pass = 0; pass < kFinTile / 4; ++pass) {
        const PassIn cur = nxt;
        if (pass + 1 < kFinTile / 4) load_pass(r0, pass + 1, nxt);
        else if (r0 + kFinTile * a.waves < r_end) load_pass(r0 + kFinTile * a.waves, 0, nxt);
        const int tr = 4 * pass + gi;  // row within the tile
        const int r = r0 + tr;
        const bool valid = r < r_end;
        const int64_t grow = (int64_t)bh * a.N + (valid ? r : r0);
        const int64_t brow = a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)(valid ? r : r0) * a.bs2 : -1;
        auto true_of = [&](int j) -> float {  // true = quantize_elemwise(fl32(QK^T)) * scale (+ bias)
          const float acc = true_dot<NB>(cur.qv, cur.qe, tkc + (size_t)j * kst, tke + j * nbd);
          // (true scores in the score dtype: the matmul's output, then * scale, + bias)
          float t = round_bfloat(round_dt(acc, sdt), a.bfloat, kRoundNearest,
                                1, sdt);
          t = round_dt(t * a.scale, sdt);
          if (brow >= 0) t = round_dt(t + load_dt(a.bias, brow + (int64_t)j * a.bs3, idt), sdt);
          return t;
        };
        if (a.true_out && valid)  // debug output: every key's true score
          for (int j = gl; j < T; j += 16) a.true_out[grow * T + j] = true_of(j);
  
        int ix[KS];
        float v[KS];
        float mx = -INFINITY;
  #pragma unroll
        for (int t = 0; t < KS; ++t) {
          ix[t] = cur.ix[t];
          v[t] = ix[t] >= 0 ? true_of(ix[t]) : -INFINITY;
          mx = fmaxf(mx, v[t]);
        }
        mx = __uint_as_float(row16_reduce(__float_as_uint(mx), [](uint32_t x, uint32_t y) {
          return __float_as_uint(fmaxf(__uint_as_float(x), __uint_as_float(y)));
        }));
        float sum = 0.0f;
  #pragma unroll
        for (int t = 0; t < KS; ++t) {
          v[t] = ix[t] >= 0 ? expf(v[t] - mx) : 0.0f;
          sum += v[t];
        }
        sum = __uint_as_float(row16_reduce(__float_as_uint(sum), [](uint32_t x, uint32_t y) {
          return __float_as_uint(__uint_as_float(x) + __uint_as_float(y));
        }));
      // zeros.scatter_(idx, softmax) -> MXINT8 along keys (block maxima by atomic max)
  #pragma unroll
        for (int t = 0; t < KS; ++t) {
          if (ix[t] >= 0) {
            v[t] = round_dt(round_bfloat(v[t] / sum, a.bfloat, kRoundNearest, 1, sdt), sdt);
            atomicMax(&bm[ix[t] >> 5], __float_as_uint(v[t]) & 0x7FFFFFFFu);
          }
        }
        wave_lds_sync();
        if (gl < ntb) {  // block gl: scale exponent (+1024; 0 = NaN block) and flush flag
          int e_raw;
          const int es = scale_exponent_dt(bm[gl], 127, sdt, &e_raw);
          const bool fl = a.flush_p && !(e_raw != kExpNaN && e_raw > -127);
          sP[gl * kFinTile + tr] = scale_f(es == kExpNaN ? kExpNaN : es - 6);
          bm[gl] = (es == kExpNaN ? 0u : (uint32_t)(es + 1024)) | (fl ? 0x10000u : 0u);
        }
        wave_lds_sync();
  #pragma unroll
        for (int t = 0; t < KS; ++t) {
          if (ix[t] >= 0) {
            const uint32_t e = bm[ix[t] >> 5];
            int code = 0;
            if (e & 0xFFFFu) {
              const int es = (int)(e & 0xFFFFu) - 1024;
              const float x = (e & 0x10000u) ? v[t] * 0.0f : v[t];
              code = (int)round_code(x, es, 8, kRoundNearest, sdt);
            }
            ptile[tr * vst + ix[t]] = (int8_t)code;
          }
        }
        wave_lds_sync();
        bm[gl] = 0u;
      }
      wave_lds_sync();
  
    }
    // ---- 2. P.V on int8 MFMA: one v_mfma_i32_32x32x32_i8 per (32 columns, key block) ----
    // lane maps (checked on hardware by mxa_selftest_mfma32): A[m][k], m = lane % 32,
    // k = 16 (lane / 32) + 0..15; B[k][n], n = lane % 32, the same k; C[m][n] in c[i],
    // m = 8 (i / 4) + 4 (lane / 32) + i % 4, n = lane % 32
    const int m0 = 4 * (lane >> 5), ln = lane & 31, kh = 16 * (lane >> 5);
    for (int dt = 0; dt < D; dt += 32) {
      const int d = min(dt + ln, D - 1);
      float acc[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
      for (int b = 0; b < ntb; ++b) {
        const v4i_ av = *reinterpret_cast<const v4i_*>(ptile + ln * vst + 32 * b + kh);
        const v4i_ bv = *reinterpret_cast<const v4i_*>(tvt + (size_t)d * vst + 32 * b + kh);
        const v16i zero = {};
        const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, zero, 0, 0, 0);
        const float sv = scale_f(exp_from16(tve[b * D + d]));
        const float* sp = sP + b * kFinTile;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 s4 = *reinterpret_cast<const float4*>(sp + 8 * q + m0);
          acc[4 * q + 0] = fmaf((float)c[4 * q + 0], s4.x * sv, acc[4 * q + 0]);
          acc[4 * q + 1] = fmaf((float)c[4 * q + 1], s4.y * sv, acc[4 * q + 1]);
          acc[4 * q + 2] = fmaf((float)c[4 * q + 2], s4.z * sv, acc[4 * q + 2]);
          acc[4 * q + 3] = fmaf((float)c[4 * q + 3], s4.w * sv, acc[4 * q + 3]);
        }
      }
      if constexpr (XO) {
        // ---- 3'. the 32 x 32 block -> MX codes of block (h D + dt) / 32 of each output
        // row (what rows_prep makes of the (B, N, C) output for the proj Linear) -------
        float* ot = reinterpret_cast<float*>(wb + L.ot);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          ot[(8 * (i >> 2) + m0 + (i & 3)) * 33 + ln] = round_bfloat(acc[i], a.bfloat, kRoundNearest, 1);
        wave_lds_sync();
        const int row = lane >> 1, sub = lane & 1, r = r0 + row;
        float xv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) xv[j] = ot[row * 33 + 16 * sub + j];
        RowsPrepArgs ro{};
        ro.codes = a.xo_codes; ro.sT = a.xo_exps;
        ro.dpad = a.H * D; ro.nb = a.H * nbd; ro.D = a.H * D;
        ro.op_kind = MXA_OP_MXINT8; ro.flush = a.flush_p; ro.bfloat = a.bfloat; ro.dt = kF32;
        ro.mfma_rows = 1;  // the MX GEMM's A layout
        const int64_t orow = (int64_t)b_ * a.N + (r < r_end ? r : r0);
        const int blk = h_ * nbd + dt / 32, c0 = h_ * D + dt + 16 * sub;
        if (rows_prep_plain(ro)) rows_prep_block_plain<16, kF32>(ro, orow, blk, sub, c0, xv, r < r_end);
        else rows_prep_block<16>(ro, orow, blk, sub, c0, xv, r < r_end);
        wave_lds_sync();
        continue;
      }
      // ---- 3. output rows (128-B segments per row) --------------------------------
      if (dt + ln < D) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = r0 + 8 * (i >> 2) + m0 + (i & 3);
          if (r < r_end)
            store_dt(a.out, b_ * a.os0 + h_ * a.os1 + (int64_t)r * a.os2 + dt + ln,
                     round_bfloat(round_dt(acc[i], sdt), a.bfloat, kRoundNearest, 1, sdt), sdt);
        }
      }
    }
    wave_lds_sync();
    for (int i = lane; i < kFinTile * vst / 16; i += 64) reinterpret_cast<uint4*>(ptile)[i] = make_uint4(0, 0, 0, 0);
    wave_lds_sync();
  }
}

}  // namespace mxa
