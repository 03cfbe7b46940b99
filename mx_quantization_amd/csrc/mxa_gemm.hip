// Launches of the block-scaled MX GEMM (mxa_gemm.hpp) and the mx.Linear entry point of
// include/mxa.h (mxa_linear: x -> MX codes along in_features -> GEMM with a prepared weight).
#include <algorithm>

#include "mxa_gemm.hpp"
#include "mxa_launch.hpp"

namespace mxa {

// shifted int32 block sums stay exact while nbk * 32 * 127^2 * 2^smax < 2^31
int gemm_smax(int nbk) {
  int s = -1;
  while ((int64_t)nbk * 516128 * ((int64_t)1 << (s + 1)) < ((int64_t)1 << 31)) ++s;
  return s;
}

template <bool PLAIN>
static int launch_gemm_p(const GemmArgs& ga0, int64_t batch, hipStream_t stream) {
  GemmArgs ga = ga0;
  ga.smax = gemm_smax(ga.nbk);
  // the tile shape (mxa_gemm.hpp GemmShape): products of <= 64 columns on 128 x 64 tiles;
  // float32 products of 65..256 contiguous columns on 32-row strips of whole rows; else 64 x 128
  const int sh = ga.Nc <= GemmShape<kGemmTall>::CW                           ? kGemmTall
                 : PLAIN && ga.Nc <= GemmShape<kGemmWide>::CW && ga.ldc == ga.Nc ? kGemmWide
                                                                              : kGemmSquare;
  const int RW = sh == kGemmTall ? GemmShape<kGemmTall>::RW : sh == kGemmWide ? GemmShape<kGemmWide>::RW : GemmShape<kGemmSquare>::RW;
  const int CW = sh == kGemmTall ? GemmShape<kGemmTall>::CW : sh == kGemmWide ? GemmShape<kGemmWide>::CW : GemmShape<kGemmSquare>::CW;
  const size_t lds = gemm_lds(ga.nbk, sh).total;
  const int64_t gx = (ga.Nc + CW - 1) / CW, gy = (ga.M + RW - 1) / RW;
  if (lds > 160 * 1024 || gy > 65535) return MXA_ERR_UNSUPPORTED;
  if (ga.bpd && batch == 1 && ga.nbk <= kGemmDigNbkMax) {
    // a prepared weight: the exponent-folded digits, every row block in the one launch (a
    // block the digits cannot take sums its K-blocks in fp64 in the same workgroup)
    const size_t dl = gemm_dig_lds(ga.nbk).total;
    const void* dk = reinterpret_cast<const void*>(&mx_gemm_dig_kernel<PLAIN>);
    if (hipFuncSetAttribute(dk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dl) != hipSuccess) return MXA_ERR_LAUNCH;
    hipLaunchKernelGGL(mx_gemm_dig_kernel<PLAIN>, dim3((unsigned)((ga.M + 31) / 32)), dim3(256), dl, stream, ga);
    return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
  }
  // (the wide strip stages float32 rows: only the PLAIN instantiation has it)
  constexpr int kWide = PLAIN ? kGemmWide : kGemmSquare;
  const void* gk = sh == kGemmTall   ? reinterpret_cast<const void*>(&mx_gemm_kernel<PLAIN, kGemmTall>)
                   : sh == kGemmWide ? reinterpret_cast<const void*>(&mx_gemm_kernel<PLAIN, kWide>)
                                     : reinterpret_cast<const void*>(&mx_gemm_kernel<PLAIN, kGemmSquare>);
  if (hipFuncSetAttribute(gk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return MXA_ERR_LAUNCH;
  // grid.z <= 65535: larger batches in slices; a wave whose spreads the int32 sums cannot
  // take sums its blocks in fp64 itself (gemm_tile's run_f64): one launch per slice
  const int64_t esz = (ga.linear || ga.dt == kF32) ? 4 : 2;
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    GemmArgs gs = ga;
    gs.a += b0 * ga.a_bat; gs.ae += b0 * ga.ae_bat; gs.b += b0 * ga.b_bat; gs.be += b0 * ga.be_bat;
    gs.c = static_cast<unsigned char*>(ga.c) + b0 * ga.c_bat * esz;
    const int64_t nb = std::min<int64_t>(65535, batch - b0);
    const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)nb);
    if (sh == kGemmTall) hipLaunchKernelGGL((mx_gemm_kernel<PLAIN, kGemmTall>), grid, dim3(256), lds, stream, gs);
    else if (sh == kGemmWide) hipLaunchKernelGGL((mx_gemm_kernel<PLAIN, kWide>), grid, dim3(256), lds, stream, gs);
    else hipLaunchKernelGGL((mx_gemm_kernel<PLAIN, kGemmSquare>), grid, dim3(256), lds, stream, gs);
    if (hipGetLastError() != hipSuccess) return MXA_ERR_LAUNCH;
  }
  return MXA_OK;
}

int launch_gemm(const GemmArgs& ga, int64_t batch, hipStream_t stream) {
  if (ga.M <= 0 || ga.Nc <= 0 || ga.nbk <= 0 || batch <= 0) return MXA_ERR_ARG;
  const bool plain = (ga.bfloat == 0 || ga.bfloat == 32) && (ga.linear ? ga.autocast == 0 : ga.dt == kF32);
  return plain ? launch_gemm_p<true>(ga, batch, stream) : launch_gemm_p<false>(ga, batch, stream);
}

// GEMM of MX rows (rows_prep layout: codes [rows][Cpad], exponents [rows][nbk]) with a
// prepared Linear weight (its row-major codes / exponents): out = mx.Linear epilogue
int launch_linear_codes(const int8_t* xc, const int16_t* xs, int64_t rows, int in_f, const void* wq, int out_f,
                        const float* bias, float* out, int64_t out_row_stride, int bfloat, int autocast,
                        hipStream_t stream, bool x_mfma) {
  const LinearLayout W = linear_layout(out_f, in_f, out_f);  // raw regions do not depend on gw
  const unsigned char* wb = static_cast<const unsigned char*>(wq);
  GemmArgs g{};
  g.a = xc; g.ae = xs; g.lda = W.Cpad; g.a_mfma = x_mfma ? 1 : 0;
  g.b = reinterpret_cast<const int8_t*>(wb + W.rawc); g.ldb = W.Cpad;
  g.be = reinterpret_cast<const int16_t*>(wb + W.rawe); g.be_n = W.nbk; g.be_k = 1;
  g.M = (int)rows; g.Nc = out_f; g.nbk = W.nbk;
  // the MFMA-ready codes when the buffer's column blocks are the output columns (one group,
  // or groups of a multiple of 32 columns): its header's group width decides
  LinearWeightHeader h{};
  if (linear_weight_known_header(wq, &h) && (h.gw == out_f || h.gw % 32 == 0)) {
    const LinearLayout P = linear_layout(out_f, in_f, h.gw);
    g.bpk = reinterpret_cast<const int8_t*>(wb + P.pk);
    g.b_nb32 = P.G * P.NB32;
    g.bpd = reinterpret_cast<const int8_t*>(wb + P.pd);
    g.bps = reinterpret_cast<const int16_t*>(wb + P.ps);
    g.bpn = reinterpret_cast<const int16_t*>(wb + P.pn);
    g.bgs = reinterpret_cast<const int16_t*>(wb + P.gs);
    g.bG = P.G;
  }
  g.linear = 1; g.dt = kF32; g.bfloat = bfloat; g.autocast = autocast; g.bias = bias;
  g.c = out; g.ldc = out_row_stride;
  if (rows > ((int64_t)1 << 31) - 1) return MXA_ERR_UNSUPPORTED;
  return launch_gemm(g, 1, stream);
}

}  // namespace mxa

using namespace mxa;

extern "C" int64_t mxa_linear_workspace_bytes(int64_t rows, int32_t in_features, int32_t out_features) {
  if (rows <= 0 || in_features <= 0 || out_features <= 0 || rows > INT32_MAX) return -1;
  const int64_t nbk = (in_features + 31) / 32;
  const int64_t rows32 = (rows + 31) / 32 * 32;  // the MFMA-ready codes hold whole 32-row blocks
  return (rows32 * nbk * 32 + 255) / 256 * 256 + (rows * nbk * 2 + 255) / 256 * 256;
}

extern "C" int mxa_linear(const float* x, int64_t rows, int32_t in_features, int64_t x_row_stride, const void* wq,
                          int32_t out_features, const float* bias, float* out, int64_t out_row_stride,
                          int32_t flush_subnormals, int32_t bfloat, int32_t autocast_dtype, void* workspace,
                          int64_t workspace_bytes, hipStream_t stream) {
  if (!x || !wq || !out || rows <= 0 || in_features <= 0 || out_features <= 0 || x_row_stride < in_features ||
      out_row_stride < out_features)
    return MXA_ERR_ARG;
  if (bfloat != 0 && bfloat != 32 && (bfloat < 10 || bfloat > 31)) return MXA_ERR_ARG;
  if (autocast_dtype != 0 && autocast_dtype != MXA_DT_F16 && autocast_dtype != MXA_DT_BF16) return MXA_ERR_ARG;
  if (!linear_weight_verify_any_group(wq, out_features, in_features, flush_subnormals, bfloat, stream))
    return MXA_ERR_ARG;
  const int64_t need = mxa_linear_workspace_bytes(rows, in_features, out_features);
  if (!workspace || workspace_bytes < need || !aligned16(workspace)) return MXA_ERR_WORKSPACE;
  const int nbk = (in_features + 31) / 32, Cpad = 32 * nbk;
  unsigned char* ws = static_cast<unsigned char*>(workspace);
  RowsPrepArgs rx{};
  rx.x = x; rx.s0 = 0; rx.s1 = 0; rx.s2 = x_row_stride;
  rx.H = 1; rx.R = rows; rx.rows = rows; rx.D = in_features; rx.nb = nbk; rx.dpad = Cpad;
  rx.vec4 = aligned16(x) && x_row_stride % 4 == 0;
  rx.op_kind = MXA_OP_MXINT8; rx.flush = flush_subnormals; rx.bfloat = bfloat; rx.dt = MXA_DT_F32;
  const int64_t rows32 = (rows + 31) / 32 * 32;
  rx.codes = reinterpret_cast<int8_t*>(ws);
  rx.mfma_rows = 1;
  rx.sT = reinterpret_cast<int16_t*>(ws + (rows32 * Cpad + 255) / 256 * 256);
  int rc = launch_rows_prep(rx, stream);
  if (rc) return rc;
  return launch_linear_codes(rx.codes, rx.sT, rows, in_features, wq, out_features, bias, out, out_row_stride, bfloat,
                             autocast_dtype, stream, true);
}
