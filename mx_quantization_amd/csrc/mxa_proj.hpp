// Fused MX Linear qkv projection -> the attention path's MX operands.
//
// The patched attention modules compute qkv = mx.Linear(x) and split it into the
// heads' q, k, v (workloads/deit/scripts/main.py:87-88, workloads/DiT/models.py:156-157);
// the Linear forward is microxscaling/mx/linear.py:20-103:
//   out = bf(fl32(MX(bf(x), along C) @ MX(bf(W), along C)^T));  out = bf(out + bf(bias))
// (bf = quantize_elemwise_op, identity at bfloat 0/32).  Here one workgroup takes one
// 32-token MX block of one image and one head: the x code tile (staged in LDS once)
// times the head's q / k / v weight rows on v_mfma_i32_32x32x32_i8 -- K = 32 = one
// MX block, so each block's int32 sum is exact -- with the block scale 2^(ex + ew)
// applied in fp64 (ldexp) and summed exactly, so the projection is the correctly
// rounded exact product (the reference's MKL sgemm order is unpinned, SURVEY.md F7:
// tolerance there, bit-exact against the oracle).  The fp32 tile then stays in LDS
// and is quantized in place into exactly what rows_prep / cols_prep would produce
// from q, k, v: q and k rows (codes, block exponents, approximator operands) and V's
// codes along the 32 tokens (transposed) -- the fp32 q / k / v never reach HBM.
#pragma once
#include "mxa_finish.hpp"
#include "mxa_prep.hpp"

namespace mxa {

struct ProjArgs {
  const int8_t* xc;   // x codes [B*N][Cpad]
  const int16_t* xs;  // x code-unit exponents [B*N][nbk]
  const int8_t* wc;   // W codes [3*H*D][Cpad]
  const int16_t* ws;  // W code-unit exponents [3*H*D][nbk]
  const float* bias;  // [3*H*D] or null
  float* qkv_out;     // optional [B*N][3*H*D] projection (tests)
  int B, N, H, D, nbk, Cpad, bfloat;
  RowsPrepArgs rq, rk;  // q / k row outputs (rows_prep layout)
  ColsPrepArgs cv;      // V outputs (cols_prep layout)
};

struct ProjLds {
  size_t xt, xe, rn, ot, total;
  int xst, ost;
};
// x code tile [32][Cpad + 16], x exponents [nbk][32] (int16, NaN -> 0), row NaN flags,
// the fp32 output tile [32][3D + 1] (odd stride: V's column reads are conflict-free)
__host__ __device__ inline ProjLds proj_lds(int Cpad, int nbk, int D) {
  ProjLds L;
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  size_t o = 0;
  L.xst = Cpad + 16;
  L.xt = o;
  o += (size_t)32 * L.xst;
  L.xe = o;
  o += al((size_t)nbk * 32 * 2);
  L.rn = o;
  o += 32 * 4;
  L.ost = 3 * D + 1;
  L.ot = o;
  o += al((size_t)32 * L.ost * 4);
  L.total = o;
  return L;
}

// NBD: 32-blocks per head dim; 3 * NBD waves, wave (s, cb) = sub-matrix s (q, k, v)
// and its 32-column block cb
template <int NBD>
__global__ __launch_bounds__(64 * 3 * NBD) void qkv_proj_kernel(ProjArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int kThreads = 64 * 3 * NBD;
  const int h = blockIdx.x, tb = blockIdx.y, b = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int D = a.D, HD = a.H * D;
  const ProjLds L = proj_lds(a.Cpad, a.nbk, D);
  int8_t* xt = reinterpret_cast<int8_t*>(smem + L.xt);
  int16_t* xe = reinterpret_cast<int16_t*>(smem + L.xe);
  int* rn = reinterpret_cast<int*>(smem + L.rn);
  float* ot = reinterpret_cast<float*>(smem + L.ot);
  const int n0 = 32 * tb, rows = min(32, a.N - n0);
  const int64_t row0 = (int64_t)b * a.N + n0;

  // ---- stage the token block's x codes (zero beyond N) and exponents ----------
  const int cpr = a.Cpad / 16;
  for (int i = threadIdx.x; i < 32 * cpr; i += kThreads) {
    const int m = i / cpr, c = i - m * cpr;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < rows) v = *reinterpret_cast<const uint4*>(a.xc + (row0 + m) * a.Cpad + 16 * c);
    *reinterpret_cast<uint4*>(xt + m * L.xst + 16 * c) = v;
  }
  if (threadIdx.x < 32) rn[threadIdx.x] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < 32 * a.nbk; i += kThreads) {
    const int m = i / a.nbk, kb = i - m * a.nbk;
    int e = m < rows ? exp_from16(a.xs[(row0 + m) * a.nbk + kb]) : 0;
    if (e == kExpNaN) {  // a NaN block makes the whole output row NaN
      rn[m] = 1;
      e = 0;
    }
    xe[kb * 32 + m] = (int16_t)e;
  }
  __syncthreads();

  // ---- the 32 x 32 output block of this wave on int8 MFMA ----------------------
  // lane maps of v_mfma_i32_32x32x32_i8 (mxa_selftest_mfma32): A[m][k], m = lane % 32,
  // k = 16 (lane / 32) + 0..15; B[k][n], n = lane % 32; C[m][n] in c[i],
  // m = 8 (i / 4) + 4 (lane / 32) + i % 4
  const int s = wave / NBD, cb = wave - s * NBD;
  const int ln = lane & 31, kh = 16 * (lane >> 5), m0 = 4 * (lane >> 5);
  const int dcol = 32 * cb + ln;
  const bool colv = dcol < D;
  const int64_t wrow = (int64_t)s * HD + (int64_t)h * D + min(dcol, D - 1);
  const int8_t* wp = a.wc + wrow * a.Cpad + kh;
  const int16_t* wsp = a.ws + wrow * a.nbk;
  double acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0;
  bool cnan = false;
  v4i_ bnext = *reinterpret_cast<const v4i_*>(wp);
  for (int kb = 0; kb < a.nbk; ++kb) {
    const v4i_ bv = bnext;
    if (kb + 1 < a.nbk) bnext = *reinterpret_cast<const v4i_*>(wp + 32 * (kb + 1));
    const v4i_ av = *reinterpret_cast<const v4i_*>(xt + ln * L.xst + 32 * kb + kh);
    const v16i zero = {};
    const v16i c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, zero, 0, 0, 0);
    int ew = exp_from16(wsp[kb]);
    cnan = cnan || ew == kExpNaN;
    ew = ew == kExpNaN ? 0 : ew;
    const int16_t* eb = xe + kb * 32 + m0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint2 e4 = *reinterpret_cast<const uint2*>(eb + 8 * q);  // rows 8q + m0 .. + 3
      const int ex[4] = {(int)(int16_t)(e4.x & 0xFFFFu), (int)(int16_t)(e4.x >> 16), (int)(int16_t)(e4.y & 0xFFFFu),
                         (int)(int16_t)(e4.y >> 16)};
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[4 * q + r] += ldexp((double)c[4 * q + r], ex[r] + ew);
    }
  }
  // ---- out = bf(fl32(sum)); out = bf(out + bf(bias))  (linear.py:88-101) -----------
  const int64_t jcol = (int64_t)s * HD + (int64_t)h * D + dcol;
  const float bb = (a.bias && colv) ? round_bfloat(a.bias[jcol], a.bfloat, kRoundNearest, 1) : 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int m = 8 * (i >> 2) + m0 + (i & 3);
    float o = (cnan || rn[m]) ? __uint_as_float(0x7FC00000u) : (float)acc[i];
    o = round_bfloat(o, a.bfloat, kRoundNearest, 1);
    if (a.bias) o = round_bfloat(o + bb, a.bfloat, kRoundNearest, 1);
    if (colv) {
      ot[m * L.ost + s * D + dcol] = o;
      if (a.qkv_out && m < rows) a.qkv_out[(row0 + m) * (3 * HD) + jcol] = o;
    }
  }
  __syncthreads();

  // ---- q and k rows: rows_prep's per-block body on the tile (8 lanes per block) ----
  const int64_t hrow0 = ((int64_t)b * a.H + h) * a.N + n0;  // row of (b, h, n0) in the q / k tables
  constexpr int kTasks = 2 * 32 * NBD * 8;
  for (int t0 = 0; t0 < kTasks; t0 += kThreads) {
    const int t = t0 + (int)threadIdx.x;
    const bool tv = t < kTasks;  // uniform per 8-lane group
    const int g = t >> 3, sub = t & 7;
    const int sk = tv ? g / (32 * NBD) : 0;
    const int rem = tv ? g - sk * 32 * NBD : 0;
    const int m = rem / NBD, blk = rem - m * NBD;
    const int c0 = 32 * blk + 4 * sub;
    float xv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = (tv && c0 + j < D) ? ot[m * L.ost + sk * D + c0 + j] : 0.0f;
    rows_prep_block(sk ? a.rk : a.rq, hrow0 + m, blk, sub, c0, xv, tv && m < rows);
  }
  // ---- V: cols_prep's per-column body over the 32 tokens -------------------------
  for (int c = threadIdx.x; c < D; c += kThreads) {
    float xv[32];
    uint32_t mx = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const float v = j < rows ? round_bfloat(ot[j * L.ost + 2 * D + c], a.cv.bfloat, kRoundNearest, 1) : 0.0f;
      xv[j] = v;
      const uint32_t ub = __float_as_uint(v) & 0x7FFFFFFFu;
      mx = ub > mx ? ub : mx;
    }
    cols_prep_column(a.cv, (int64_t)b * a.H + h, tb, c, xv, mx);
  }
}

}  // namespace mxa
