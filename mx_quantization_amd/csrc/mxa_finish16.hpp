// Finishing kernel of the top-k path for small k (k <= 64: DeiT's 20 / 30, PixArt's 20),
// 16-ROW TILES: for every query row and its k kept keys (the selection kernel's indices) the
// true scores, softmax, MX(P) along keys and P.V, with P.V on v_mfma_i32_16x16x32_i8.
//
// Per workgroup (one head, or a chunk of its query rows): the head's K codes + exponents and
// the V block scales (as floats) staged in LDS once.  Per wave, tiles of 16 query rows, four
// lanes per row, lane slots ph, ph + 4, ... (KS of them: k <= 4 KS):
//   1. the kept key's true score fl32(exact sum) * scale (+ bias) by v_dot4 over the LDS codes
//      (exact block epilogue); softmax over the kept scores (quad DPP); P
//      MX-quantized along keys: block maxima by LDS atomic max, the block's code multiplier
//      2^-es, the codes into the tile's dense code rows (zero elsewhere);
//   2. P.V for the tile, key block outer: per 32-key MX block the P operand and row scales
//      once, then per 16 output columns ONE v_mfma_i32_16x16x32_i8 (K = 32 = one block: each
//      block keeps its exact int32 sum), epilogue acc += C * (sP[row][b] * sV[b][d]) in fp32
//      (P.V is a tolerance-only product); the V^T operands (token-block-major
//      codes: one contiguous 512-B run per MFMA) straight from HBM / L2, two blocks ahead
//      of their MFMAs (the first two issued at the tile's start, in flight through step 1);
//      the next tile's kept indices loaded during this tile's P.V;
//   3. the tile's output rows go out; the written code positions are cleared.
// Every slot runs the same instructions (an unused slot -- k < 4 KS, or a row past the end --
// scores key 0 and writes its code to a pad column), so the per-slot work has no branches.
// exp / divide: the softmax on v_exp_f32 (2^((v - mx) log2 e)) and a corrected reciprocal
// (P is a tolerance-only operand, as in mxa_finish_qk.hpp).
// (The proj Linear's MX input codes stay on the 32-row kernel, whose 32 x 32 output blocks
// are whole MX blocks of the rows.)
// Reference: microxscaling/mx/matmul.py:68-76 (MX P.V), callers
// workloads/deit/scripts/main.py:124-152, workloads/DiT/models.py:195-225,
// workloads/PixArt/models/MX_transformer_block.py:679-717, :826-859.
#pragma once
#include "mxa_finish.hpp"

namespace mxa {

constexpr int kFin16 = 16;  // query rows per MFMA tile (one wave)
constexpr int kFin16Occ = 4;  // waves per SIMD the register allocation aims at
// Measured (DeiT-base, same box): the V^T codes staged in LDS per workgroup instead of read
// from L2: 0.172 vs 0.166 ms (3 workgroups per CU instead of 4; PixArt 0.019 vs 0.021); the
// next tile's query codes loaded one tile ahead: 0.193 ms (registers).  Phase timing (tools
// builds): without the V^T loads 0.125 ms, without the score gathers 0.138, neither 0.104.

typedef int v4i16_ __attribute__((ext_vector_type(4)));

// LDS: tables (K codes, K exponents, V block scales as floats [ntb][D]), then per wave the P
// code tile [16][vst] (columns >= tpad: the unused slots' pad), the P block scales sP
// [ntb][16] (float), the block maxima / code multipliers bm [16][ntb] (u32)
struct Fin16Lds {
  size_t kc, ke, vt, ve, waves, per_wave, sp, bm, total;
};
// xo: the per-wave area also holds the 16 x (D + 1) fp32 output tile being MX-quantized for
// the proj Linear (over the code tile, sP and bm, which are rewritten afterwards)
__host__ __device__ inline Fin16Lds fin16_lds(int T, int D, int kst, int nbd, int vst, int ntb, int waves,
                                              bool xo = false) {
  Fin16Lds L;
  size_t o = 0;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  L.kc = o;
  o += al((size_t)T * kst);
  L.ke = o;
  o += al((size_t)T * nbd * 2);
  L.ve = o;
  o += al((size_t)ntb * D * 4);
  L.vt = o;
  L.waves = o;
  L.sp = al((size_t)kFin16 * vst);
  L.bm = L.sp + al((size_t)ntb * kFin16 * 4);
  L.per_wave = L.bm + al((size_t)kFin16 * ntb * 4);
  if (xo && L.per_wave < al((size_t)kFin16 * (D + 1) * 4)) L.per_wave = al((size_t)kFin16 * (D + 1) * 4);
  L.total = o + (size_t)waves * L.per_wave;
  return L;
}

// NB: 32-blocks per head dim; KS: kept slots per lane (k <= 4 KS); XDT: float16 / bfloat16
// inputs or scores (the dtype roundings at run time); EXTRA: a bias, the debug true-score
// output or bfloatX rounding (else the scores and P are plain float32); XO: the output rows
// go to the proj Linear as MX codes along C (Rows2Args::xo_codes; float32, D % 32 == 0):
// the tile's 16 x D block is transposed through LDS and every 32-column block of every row
// quantized by rows_prep's per-block body (two lanes per block, all 64 lanes for D = 64)
template <int NB, int KS, bool XDT, bool EXTRA, bool XO = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(NB <= 2 && KS <= 12 ? kFin16Occ : (NB * KS <= 64 ? 3 : 2), 8))) void finish16_kernel(Rows2Args a) {
  constexpr bool kRound = XDT || EXTRA;
  const int sdt = XDT ? a.s_dt : (int)kF32, idt = XDT ? a.in_dt : (int)kF32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bh = blockIdx.x;
  const int T = a.T, D = a.D, kst = a.kst, vst = a.vst, ntb = a.ntb, k = a.k_top;
  constexpr int nbd = NB;
  const int b_ = bh / a.H, h_ = bh % a.H;
  const Fin16Lds L = fin16_lds(T, D, kst, nbd, vst, ntb, a.waves, XO);
  int8_t* tkc = reinterpret_cast<int8_t*>(smem + L.kc);
  int16_t* tke = reinterpret_cast<int16_t*>(smem + L.ke);
  float* tvs = reinterpret_cast<float*>(smem + L.ve);
  unsigned char* wb = smem + L.waves + (size_t)wave * L.per_wave;
  int8_t* ptile = reinterpret_cast<int8_t*>(wb);
  float* sP = reinterpret_cast<float*>(wb + L.sp);
  uint32_t* bmw = reinterpret_cast<uint32_t*>(wb + L.bm);  // [16][ntb]
  const int pr = lane >> 2, ph = lane & 3;  // the lane's tile row and slot phase

  const int r_beg = (int)blockIdx.y * a.rows_per_wg, r_end = min(a.N, r_beg + a.rows_per_wg);
  uint32_t* bm = bmw + pr * ntb;
  const int pad = a.tpad + ph;  // an unused slot's code column (never read by the MFMA)
  const int ln = lane & 15, kg = lane >> 4;
  const int8_t* vbase = a.vt + (int64_t)bh * D * a.tpad + 8 * kg;
  constexpr int NDT = 2 * NB;  // 16-column tiles of D <= 32 NB
  int64_t bv[NDT], bw[NDT];  // V^T operands of key blocks b, b + 1 (in flight ahead of use)
  auto load_v = [&](int b, int64_t* dst) {
#pragma unroll
    for (int u = 0; u < NDT; ++u)
      if (16 * u < D) dst[u] = *reinterpret_cast<const int64_t*>(vbase + ((int64_t)b * D + min(16 * u + ln, D - 1)) * 32);
  };
  // the next tile's kept indices, loaded while the current tile finishes (the query codes are
  // loaded at the tile's start: one tile ahead they cost more registers than they save)
  int ixn[KS];
  auto load_ix = [&](int r0n) {
    const int rn = r0n + pr;
    const int64_t gn = (int64_t)bh * a.N + (rn < r_end ? rn : r_beg);
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const int s = ph + 4 * t;
      ixn[t] = rn < r_end && s < k ? kept_get(a, gn * k + s) : 0;
    }
  };
  load_ix(r_beg + kFin16 * wave);  // (in flight through the staging)

  // ---- stage the head's K table and V block scales; clear the code tile ---------------
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
    for (int i = threadIdx.x; i < ntb * D; i += blockDim.x) tvs[i] = scale_f(exp_from16(vssrc[i]));
    for (int i = lane; i < kFin16 * vst / 16; i += 64) reinterpret_cast<uint4*>(ptile)[i] = make_uint4(0, 0, 0, 0);
    for (int i = lane; i < kFin16 * ntb; i += 64) bmw[i] = 0u;
  }
  __syncthreads();

  for (int r0 = r_beg + kFin16 * wave; r0 < r_end; r0 += kFin16 * a.waves) {
    const int r = r0 + pr;
    const bool valid = r < r_end;
    const int64_t grow = (int64_t)bh * a.N + (valid ? r : r0);
    const int64_t brow = EXTRA && a.bias ? b_ * a.bs0 + h_ * a.bs1 + (int64_t)(valid ? r : r0) * a.bs2 : -1;
    // the first two key blocks' V^T operands, in flight through the scores and softmax
    load_v(0, bv);
    if (ntb > 1) load_v(1, bw);
    // the row's query codes / exponents and its kept indices
    uint4 qv[2 * NB];
    int qe[NB];
    {
      const int8_t* qsrc = a.qc + grow * a.dpad;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        qv[2 * b] = *reinterpret_cast<const uint4*>(qsrc + 32 * b);
        qv[2 * b + 1] = *reinterpret_cast<const uint4*>(qsrc + 32 * b + 16);
        qe[b] = exp_from16(a.qsT[grow * nbd + b]);
      }
    }
    int ix[KS];
    bool on[KS];
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      on[t] = valid && ph + 4 * t < k;
      ix[t] = ixn[t];
    }
    auto true_of = [&](int j) -> float {  // true = quantize_elemwise(fl32(QK^T)) * scale (+ bias)
      const float acc = true_dot<NB>(qv, qe, tkc + (size_t)j * kst, tke + j * nbd);
      if (!kRound) return acc * a.scale;
      float t = round_bfloat(round_dt(acc, sdt), a.bfloat, kRoundNearest, 1, sdt);
      t = round_dt(t * a.scale, sdt);
      if (brow >= 0) t = round_dt(t + load_dt(a.bias, brow + (int64_t)j * a.bs3, idt), sdt);
      return t;
    };
    if (EXTRA && a.true_out && valid)  // debug output: every key's true score
      for (int j = ph; j < T; j += 4) a.true_out[grow * T + j] = true_of(j);

    // ---- 1. kept scores, softmax, MX(P) into the code tile ------------------------------
    float v[KS];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const float s = true_of(ix[t]);
      v[t] = on[t] ? s : -INFINITY;
      mx = fmaxf(mx, v[t]);
    }
    auto qmax = [](float x) {
      uint32_t u = __float_as_uint(x);
      auto op = [](uint32_t p, uint32_t q) { return __float_as_uint(fmaxf(__uint_as_float(p), __uint_as_float(q))); };
      u = op(u, dpp_u32<0xB1>(u));
      return __uint_as_float(op(u, dpp_u32<0x4E>(u)));
    };
    auto qsum = [](float x) {
      uint32_t u = __float_as_uint(x);
      auto op = [](uint32_t p, uint32_t q) { return __float_as_uint(__uint_as_float(p) + __uint_as_float(q)); };
      u = op(u, dpp_u32<0xB1>(u));
      return __uint_as_float(op(u, dpp_u32<0x4E>(u)));
    };
    mx = qmax(mx);
    // exp(v - mx) as 2^((v - mx) log2 e) (the difference first: folding mx log2 e into an
    // fma loses the argument for large scores); an unused slot adds 0 (also where mx = -inf)
    float sum = 0.0f;
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      v[t] = on[t] ? __builtin_amdgcn_exp2f((v[t] - mx) * 1.4426950408889634f) : 0.0f;
      sum += v[t];
    }
    sum = qsum(sum);
    // p = v / sum from y = RN(1 / sum): q = RN(v y), r = v - q sum exact by fma, RN(q + r y)
    const float rs = 1.0f / sum;
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const float q0 = v[t] * rs;
      float p = __builtin_fmaf(__builtin_fmaf(-q0, sum, v[t]), rs, q0);
      if (kRound) p = round_dt(round_bfloat(p, a.bfloat, kRoundNearest, 1, sdt), sdt);
      v[t] = p;
      // zeros.scatter_(idx, softmax) -> MXINT8 along keys: the block maxima (an unused slot
      // adds max(., 0) to block 0: no change)
      atomicMax(&bm[ix[t] >> 5], __float_as_uint(p) & 0x7FFFFFFFu);
    }
    wave_lds_sync();
    // per block: the scale sP (NaN for a NaN block) and the code multiplier 2^-es (0 for a NaN
    // or flushed block: its codes 0; XDT: es + 1024 and the flush flag, round_code at run time)
    for (int bk = ph; bk < ntb; bk += 4) {
      int e_raw;
      const int es = scale_exponent_dt(bm[bk], 127, sdt, &e_raw);
      const bool fl = a.flush_p && !(e_raw != kExpNaN && e_raw > -127);
      sP[bk * kFin16 + pr] = scale_f(es == kExpNaN ? kExpNaN : es - 6);
      if (XDT) bm[bk] = (es == kExpNaN ? 0u : (uint32_t)(es + 1024)) | (fl ? 0x10000u : 0u);
      else bm[bk] = __float_as_uint(es == kExpNaN || fl ? 0.0f : pow2f(-es));
    }
    wave_lds_sync();
#pragma unroll
    for (int t = 0; t < KS; ++t) {
      const uint32_t e = bm[ix[t] >> 5];
      int code;
      if (XDT) {
        code = 0;
        if (e & 0xFFFFu) {
          const int es = (int)(e & 0xFFFFu) - 1024;
          const float x = (e & 0x10000u) ? v[t] * 0.0f : v[t];
          code = (int)round_code(x, es, 8, kRoundNearest, sdt);
        }
      } else {  // round_code for p >= 0: floor(p 2^-es 64 + 0.5), <= 127 (a NaN block: sP is NaN)
        const float y = (v[t] * __uint_as_float(e)) * 64.0f;
        code = (int)fminf(floorf(y + 0.5f), 127.0f);
      }
      ptile[pr * vst + (on[t] ? ix[t] : pad)] = (int8_t)code;
    }
    wave_lds_sync();

    // ---- 2. P.V on int8 MFMA, key block outer -----------------------------------------------
    // lane maps (checked on hardware by mxa_selftest_mfma): A[m][k], m = lane % 16,
    // k = 8 (lane / 16) + 0..7; B[k][n], n = lane % 16, the same k; C[m][n] in c[i],
    // m = 4 (lane / 16) + i, n = lane % 16.  A = the P code rows, B = V^T: the head's codes
    // are [ntb][D][32], so the operand of (block b, columns 16 u ..) is one contiguous 512-B run
    float acc[NDT][4];
#pragma unroll
    for (int u = 0; u < NDT; ++u) acc[u][0] = acc[u][1] = acc[u][2] = acc[u][3] = 0.0f;
    if (r0 + kFin16 * a.waves < r_end) load_ix(r0 + kFin16 * a.waves);
    for (int b = 0; b < ntb; ++b) {
      int64_t bn[NDT];
      if (b + 2 < ntb) load_v(b + 2, bn);  // two blocks ahead
      const int64_t av = *reinterpret_cast<const int64_t*>(ptile + ln * vst + 32 * b + 8 * kg);
      const float4 s4 = *reinterpret_cast<const float4*>(sP + b * kFin16 + 4 * kg);
#pragma unroll
      for (int u = 0; u < NDT; ++u) {
        if (16 * u < D) {
          const v4i16_ zero = {0, 0, 0, 0};
          const v4i16_ c = __builtin_amdgcn_mfma_i32_16x16x32_i8(av, bv[u], zero, 0, 0, 0);
          const float sv = tvs[b * D + min(16 * u + ln, D - 1)];
          acc[u][0] = fmaf((float)c[0], s4.x * sv, acc[u][0]);
          acc[u][1] = fmaf((float)c[1], s4.y * sv, acc[u][1]);
          acc[u][2] = fmaf((float)c[2], s4.z * sv, acc[u][2]);
          acc[u][3] = fmaf((float)c[3], s4.w * sv, acc[u][3]);
        }
      }
#pragma unroll
      for (int u = 0; u < NDT; ++u) {
        bv[u] = bw[u];
        bw[u] = bn[u];
      }
    }
    if constexpr (XO) {
      // ---- 3'. the 16 x D block -> MX codes of blocks h NB .. of each output row (what
      // rows_prep makes of the (B, N, C) output for the proj Linear: finish_kernel's XO) ------
      wave_lds_sync();  // every lane's MFMA reads of the code tile are done
      float* ot = reinterpret_cast<float*>(wb);
      const int ost = D + 1;
#pragma unroll
      for (int u = 0; u < NDT; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (16 * u + ln < D) ot[(4 * kg + i) * ost + 16 * u + ln] = round_bfloat(acc[u][i], a.bfloat, kRoundNearest, 1);
      wave_lds_sync();
      RowsPrepArgs ro{};
      ro.codes = a.xo_codes; ro.sT = a.xo_exps;
      ro.dpad = a.H * D; ro.nb = a.H * nbd; ro.D = a.H * D;
      ro.op_kind = MXA_OP_MXINT8; ro.flush = a.flush_p; ro.bfloat = a.bfloat; ro.dt = kF32;
      ro.mfma_rows = 1;  // the MX GEMM's A layout
      const int row = (lane & 31) >> 1, sub = lane & 1, rr = r0 + row;
      const int64_t orow = (int64_t)b_ * a.N + (rr < r_end ? rr : r0);
#pragma unroll
      for (int bp = 0; bp < NB; bp += 2) {
        const int bl = bp + (lane >> 5), blc = min(bl, NB - 1);
        float xv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) xv[j] = ot[row * ost + 32 * blc + 16 * sub + j];
        const int blk = h_ * nbd + blc, c0 = h_ * D + 32 * blc + 16 * sub;
        if (rows_prep_plain(ro)) rows_prep_block_plain<16, kF32>(ro, orow, blk, sub, c0, xv, rr < r_end && bl < NB);
        else rows_prep_block<16>(ro, orow, blk, sub, c0, xv, rr < r_end && bl < NB);
      }
      wave_lds_sync();
      // the area back to a clear code tile and zero block maxima (sP is rewritten per tile)
      for (int i = lane; i < (int)(L.per_wave / 16); i += 64) reinterpret_cast<uint4*>(wb)[i] = make_uint4(0, 0, 0, 0);
      wave_lds_sync();
      continue;
    }
    // ---- 3. output rows (64-B segments per row); clear the written code positions ---------
#pragma unroll
    for (int u = 0; u < NDT; ++u) {
      if (16 * u + ln < D) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rr = r0 + 4 * kg + i;
          if (rr < r_end)
            store_dt(a.out, b_ * a.os0 + h_ * a.os1 + (int64_t)rr * a.os2 + 16 * u + ln,
                     kRound ? round_bfloat(round_dt(acc[u][i], sdt), a.bfloat, kRoundNearest, 1, sdt) : acc[u][i], sdt);
        }
      }
    }
    wave_lds_sync();  // every lane's MFMA reads of the tile are done
#pragma unroll
    for (int t = 0; t < KS; ++t) ptile[pr * vst + (on[t] ? ix[t] : pad)] = 0;
    for (int bk = ph; bk < ntb; bk += 4) bm[bk] = 0u;
    wave_lds_sync();
  }
}

}  // namespace mxa
