// Argument block and prepared-weight layout of the fused qkv projection (mxa_proj.hpp).
#pragma once
#include "mxa_kernels.hpp"

namespace mxa {

// Prepared Linear weight (mxa_linear_weight_prep): output columns in groups of gw (a
// head's q, k or v: gw = D), each group padded to NB32 = ceil(gw/32) 32-column blocks.
//   hdr the geometry and settings it was prepared with (LinearWeightHeader, 256 B at
//       offset 0, so a buffer of any size holds it): mxa_qkv_attention refuses a buffer
//       whose header does not match the call instead of reading past its end
//   raw row-major codes [out][Cpad] + exponents [out][nbk] (rows_prep output, packed from;
//       first, so their offsets do not depend on gw: mxa_linear reads them for any gw)
//   pk  MFMA-ready codes [group][cb][kb][lane 0..63][16 B]: lane = n + 32 h holds
//       W[col n][32 kb + 16 h .. + 16] -- one coalesced 1-KB load per wave and K-block
//   pe  block exponents [padded column][nbk] (int16, NaN = -32768)
//   ps  per padded column: smallest finite block exponent, spread (int16 pair)
//   gs  per group (of gw real columns): the smallest ps exponent, the largest spread
//   pn  per padded column: 1 when a block exponent is NaN (int16)
//   pd  exponent-folded codes [group][cb][kb][digit 0, 1][lane][16 B]: the code times
//       2^(block exponent - column's smallest) as two signed base-256 digits (column
//       spread <= kDigitSpread; else zeros, and the column's group never takes them)
struct LinearLayout {
  int G, NB32, nbk, Cpad;
  int64_t hdr, rawc, rawe, pk, pe, ps, gs, pn, pd, total;
};
constexpr int kDigitSpread = 8;  // 127 * 2^8 < 2^15: two signed int8 digits
constexpr uint32_t kLinearWeightMagic = 0x5741584du;  // "MXAW"
struct LinearWeightHeader {
  uint32_t magic;
  int32_t version, out_f, in_f, gw, flush, bfloat, reserved;
  bool operator==(const LinearWeightHeader& o) const {
    return magic == o.magic && version == o.version && out_f == o.out_f && in_f == o.in_f && gw == o.gw &&
           flush == o.flush && bfloat == o.bfloat;
  }
};
__host__ __device__ inline LinearLayout linear_layout(int out_f, int in_f, int gw) {
  LinearLayout L;
  auto al = [](int64_t x) { return (x + 255) / 256 * 256; };
  L.G = out_f / gw;
  L.NB32 = (gw + 31) / 32;
  L.nbk = (in_f + 31) / 32;
  L.Cpad = 32 * L.nbk;
  const int64_t pcols = (int64_t)L.G * L.NB32 * 32;
  int64_t o = 0;
  L.hdr = o;
  o += 256;
  L.rawc = o;
  o += al((int64_t)out_f * L.Cpad);
  L.rawe = o;
  o += al((int64_t)out_f * L.nbk * 2);
  L.pk = o;
  o += al(pcols * L.Cpad);
  L.pe = o;
  o += al(pcols * L.nbk * 2);
  L.ps = o;
  o += al(pcols * 4);
  L.gs = o;
  o += al((int64_t)L.G * 4);
  L.pn = o;
  o += al(pcols * 2);
  L.pd = o;
  o += al(2 * pcols * L.Cpad);
  L.total = o;
  return L;
}

// 16 codes times 2^s (0 <= s <= kDigitSpread) as two signed base-256 digits:
// c * 2^s = d0 + 256 d1, d0 in [-128, 127], |d1| <= 127
__device__ __forceinline__ void fold_digits16(const uint4& v, int s, uint4& d0, uint4& d1) {
  const uint32_t in[4] = {v.x, v.y, v.z, v.w};
  uint32_t o0[4], o1[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    uint32_t p0 = 0, p1 = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int c = (int)(int8_t)(in[w] >> (8 * b));
      const int f = c << s;
      const int lo = (int)(int8_t)f;
      p0 |= ((uint32_t)lo & 0xFFu) << (8 * b);
      p1 |= ((uint32_t)((f - lo) >> 8) & 0xFFu) << (8 * b);
    }
    o0[w] = p0;
    o1[w] = p1;
  }
  d0 = make_uint4(o0[0], o0[1], o0[2], o0[3]);
  d1 = make_uint4(o1[0], o1[1], o1[2], o1[3]);
}

struct ProjArgs {
  const int8_t* xc;   // x codes [B*N][Cpad]
  const int16_t* xs;  // x code-unit exponents [B*N][nbk]
  const int8_t* pk;   // prepared weight (LinearLayout with gw = D)
  const int16_t* pe;
  const int16_t* ps;
  const int16_t* gs;  // per weight group: smallest exponent, largest spread (the head's fast-path test)
  const int16_t* pn;  // per padded column: NaN block flag
  const int8_t* pd;   // exponent-folded digit codes
  const float* bias;  // [3*H*D] or null
  float* qkv_out;     // optional [B*N][3*H*D] projection (tests)
  int B, N, H, D, nbk, Cpad, bfloat, ntb;
  int pk_bytes, pe_bytes, pd_bytes;  // buffer-descriptor extents of pk / pe / pd (< 2 GiB: launch_proj checks)
  int smax;  // largest exponent spread whose shifted int32 block sums cannot overflow
  int hpg;   // heads per workgroup (grid z = head groups: fills the last round of workgroups)
  int autocast;  // 0, or the dtype torch.autocast rounds the product to before the fp32 bias add
  RowsPrepArgs rq, rk;  // q / k row outputs (rows_prep layout)
  ColsPrepArgs cv;      // V outputs (cols_prep layout)
};

// block-scaled MX GEMM (mxa_gemm.hpp): mx.matmul and mx.Linear
struct GemmArgs {
  const int8_t* a;   // A codes: (bat, m, k) at bat * a_bat + m * lda + k
  const int16_t* ae; // A exponents: (bat, m, kb) at bat * ae_bat + m * nbk + kb
  const int8_t* b;   // B^T codes: (bat, n, k) at bat * b_bat + n * ldb + k
  const int16_t* be; // B exponents: (bat, n, kb) at bat * be_bat + n * be_n + kb * be_k
  int64_t a_bat, ae_bat, b_bat, be_bat, be_n, be_k, lda, ldb;
  int M, Nc, nbk;
  int smax;           // largest row + column spread whose shifted int32 sums cannot overflow
  int linear;         // epilogue: 0 mx.matmul (store in dt), 1 mx.Linear (fp32, bias)
  int dt, bfloat, autocast;
  const float* bias;  // linear: [Nc] or null
  void* c;            // (bat, m, n) at bat * c_bat + m * ldc + n
  int64_t c_bat, ldc;
  // optional MFMA-ready B (a prepared Linear weight's pk, one group: columns in 32-column
  // blocks, [cb][kb][lane][16 B]): one coalesced 1-KB load per wave, chain and K-block
  const int8_t* bpk;
  int b_nb32;  // 32-column blocks in bpk
  int a_mfma;  // A codes in rows_prep's MFMA-ready layout ([M / 32][nbk][lane][16 B] per batch; lda unused)
  // the prepared weight's exponent-folded digits (mx_gemm_dig_kernel; mx.Linear only): pd,
  // per padded column (= output column here) smallest exponent (ps) and NaN flag (pn), the
  // group stats gs of its bG groups
  const int8_t* bpd;
  const int16_t *bps, *bpn, *bgs;
  int bG;
};

}  // namespace mxa
