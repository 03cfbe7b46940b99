// The fused qkv projection's launches (mxa_proj.hpp) and the Linear weight preparation
// entry points of include/mxa.h.
#include <algorithm>
#include <map>
#include <mutex>
#include <unordered_map>
#include <utility>

#include "mxa_launch.hpp"
#include "mxa_proj.hpp"

namespace mxa {

// one thread per (padded column, K-block): the MFMA-ready codes and the exponents
__global__ __launch_bounds__(256) void linear_pack_kernel(const int8_t* rawc, const int16_t* rawe, int out_f, int gw,
                                                          int NB32, int nbk, int Cpad, int64_t pcols, int8_t* pk,
                                                          int16_t* pe) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= pcols * nbk) return;
  const int64_t pc = t / nbk;
  const int kb = (int)(t - pc * nbk);
  const int64_t blkc = pc / 32;  // group * NB32 + cb
  const int n = (int)(pc - blkc * 32);
  const int64_t g = blkc / NB32;
  const int cb = (int)(blkc - g * NB32);
  const int gc = 32 * cb + n;
  const bool real = gc < gw;
  const int64_t col = g * gw + gc;
  uint4 lo = make_uint4(0, 0, 0, 0), hi = make_uint4(0, 0, 0, 0);
  int16_t e = 0;
  if (real) {
    lo = *reinterpret_cast<const uint4*>(rawc + col * Cpad + 32 * kb);
    hi = *reinterpret_cast<const uint4*>(rawc + col * Cpad + 32 * kb + 16);
    e = rawe[col * nbk + kb];
  }
  int8_t* dst = pk + ((blkc * nbk + kb) * 64) * 16;
  *reinterpret_cast<uint4*>(dst + n * 16) = lo;
  *reinterpret_cast<uint4*>(dst + (n + 32) * 16) = hi;
  pe[pc * nbk + kb] = e;
}

// per padded column: smallest finite block exponent and the spread, the NaN flag
__global__ __launch_bounds__(256) void linear_stats_kernel(const int16_t* pe, int64_t pcols, int nbk, int16_t* ps,
                                                           int16_t* pn) {
  const int64_t pc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pc >= pcols) return;
  int lo = 1 << 20, hi = -(1 << 20), nan = 0;
  for (int kb = 0; kb < nbk; ++kb) {
    const int e = exp_from16(pe[pc * nbk + kb]);
    if (e != kExpNaN) {
      lo = min(lo, e);
      hi = max(hi, e);
    } else {
      nan = 1;
    }
  }
  if (lo > hi) lo = hi = 0;
  ps[2 * pc] = (int16_t)lo;
  ps[2 * pc + 1] = (int16_t)(hi - lo);
  pn[pc] = (int16_t)nan;
}

// one thread per (padded column, K-block): the exponent-folded digits of the MFMA-ready
// codes (the column's two 16-B halves sit at lanes n and n + 32 of the block's 1-KB chunk)
__global__ __launch_bounds__(256) void linear_digits_kernel(const int8_t* pk, const int16_t* pe, const int16_t* ps,
                                                            int nbk, int64_t pcols, int8_t* pd) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= pcols * nbk) return;
  const int64_t pc = t / nbk;
  const int kb = (int)(t - pc * nbk);
  const int64_t blkc = pc / 32;
  const int n = (int)(pc - blkc * 32);
  const int e = exp_from16(pe[pc * nbk + kb]);
  const int sp = ps[2 * pc + 1];
  const int s = e == kExpNaN ? 0 : e - ps[2 * pc];
  const bool ok = sp <= kDigitSpread;
  const int8_t* src = pk + ((blkc * nbk + kb) * 64) * 16;
  int8_t* dst = pd + ((blkc * nbk + kb) * 128) * 16;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint4 d0 = make_uint4(0, 0, 0, 0), d1 = d0;
    if (ok) fold_digits16(*reinterpret_cast<const uint4*>(src + (n + 32 * h) * 16), s, d0, d1);
    *reinterpret_cast<uint4*>(dst + (n + 32 * h) * 16) = d0;
    *reinterpret_cast<uint4*>(dst + (64 + n + 32 * h) * 16) = d1;
  }
}

// per group of gw real columns: smallest column exponent, largest column spread
__global__ __launch_bounds__(64) void linear_group_stats_kernel(const int16_t* ps, int G, int NB32, int gw, int16_t* gs) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  int lo = 1 << 20, sp = 0;
  for (int gc = 0; gc < gw; ++gc) {
    const int64_t pc = ((int64_t)g * NB32 + gc / 32) * 32 + gc % 32;
    lo = min(lo, (int)ps[2 * pc]);
    sp = max(sp, (int)ps[2 * pc + 1]);
  }
  gs[2 * g] = (int16_t)lo;
  gs[2 * g + 1] = (int16_t)sp;
}

// ---- fused qkv projection (mxa_proj.hpp) ------------------------------------------
// the operands' settings leave only the plain rounding (qkv_proj_kernel<NBD, true>)
static bool proj_plain(const ProjArgs& pa) {
  auto plain_bf = [](int bf) { return bf == 0 || bf == 32; };
  auto plain_rows = [&](const RowsPrepArgs& r) {
    return plain_bf(r.bfloat) && !r.flush && !r.zind && r.dt == kF32 &&
           (r.op_kind == MXA_OP_MXINT8 || (r.op_kind == MXA_OP_SIGN && !r.op));
  };
  return plain_bf(pa.bfloat) && pa.autocast == 0 && plain_rows(pa.rq) && plain_rows(pa.rk) && pa.cv.mbits == 8 &&
         !pa.cv.flush && plain_bf(pa.cv.bfloat) && pa.cv.dt == kF32;
}

template <int NBD, bool PLAIN>
static int launch_proj_nbd(const ProjArgs& pa, hipStream_t stream) {
  const size_t lds = proj_lds(pa.Cpad, pa.nbk, pa.D).total;
  if (lds > 160 * 1024) return MXA_ERR_UNSUPPORTED;
  const void* kern = reinterpret_cast<const void*>(&qkv_proj_kernel<NBD, PLAIN>);
  if (hipFuncSetAttribute(kern,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return MXA_ERR_LAUNCH;
  // head groups: a workgroup loops over hpg heads after staging its x tile once; the
  // group count minimises (rounds of resident workgroups) x (heads + ~1/4 head of x
  // staging) -- with all heads per workgroup DeiT-base's 1,792 workgroups ran 3.5
  // rounds of 512 resident ones, the last half empty
  // resident workgroups per CU and the CU count, per (device, LDS size), queried once
  int dev = 0;
  (void)hipGetDevice(&dev);
  int per_cu = 1, cus = 256;
  {
    static std::mutex mu;
    static std::map<std::pair<int, size_t>, std::pair<int, int>> cache;  // per instantiation
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({dev, lds});
    if (it == cache.end()) {
      int n = 0, c = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, 64 * 3 * NBD, lds) != hipSuccess || n < 1) n = 1;
      if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c < 1) c = 256;
      it = cache.emplace(std::make_pair(dev, lds), std::make_pair(n, c)).first;
    }
    per_cu = it->second.first;
    cus = it->second.second;
  }
  ProjArgs p = pa;
  const int64_t wg0 = (int64_t)((pa.N + 31) / 32) * pa.B, slots = (int64_t)per_cu * cus;
  int best_g = 1;
  double best = 1e300;
  for (int g = 1; g <= pa.H; ++g) {
    const int hpg = (pa.H + g - 1) / g;
    if (g > 1 && (pa.H + hpg - 1) / hpg != g) continue;  // same hpg as a smaller g
    const double cost = (double)((wg0 * g + slots - 1) / slots) * (hpg + 0.25);
    if (cost < best - 1e-9) {
      best = cost;
      best_g = g;
    }
  }
  p.hpg = (pa.H + best_g - 1) / best_g;
  const int ng = (pa.H + p.hpg - 1) / p.hpg;
  hipLaunchKernelGGL((qkv_proj_kernel<NBD, PLAIN>), dim3((unsigned)((pa.N + 31) / 32), (unsigned)pa.B, (unsigned)ng),
                     dim3(64 * 3 * NBD), lds, stream, p);
  return hipGetLastError() == hipSuccess ? MXA_OK : MXA_ERR_LAUNCH;
}


template <bool PLAIN>
static int launch_proj_p(const ProjArgs& pa, hipStream_t stream) {
  switch ((pa.D + 31) / 32) {
    case 1: return launch_proj_nbd<1, PLAIN>(pa, stream);
    case 2: return launch_proj_nbd<2, PLAIN>(pa, stream);
    case 3: return launch_proj_nbd<3, PLAIN>(pa, stream);
    default: return launch_proj_nbd<4, PLAIN>(pa, stream);
  }
}

int launch_proj(const ProjArgs& pa, hipStream_t stream) {
  return proj_plain(pa) ? launch_proj_p<true>(pa, stream) : launch_proj_p<false>(pa, stream);
}

__global__ void linear_header_kernel(LinearWeightHeader* h, LinearWeightHeader v) {
  if (threadIdx.x == 0) *h = v;
}

LinearWeightHeader linear_weight_header(int out_f, int in_f, int gw, int flush, int bfloat);

// prepared buffers whose header is known to the host (pointer -> header)
static std::mutex g_wmu;
static std::unordered_map<const void*, LinearWeightHeader> g_weights;

static void linear_weight_note(const void* wq, const LinearWeightHeader& h) {
  std::lock_guard<std::mutex> g(g_wmu);
  g_weights[wq] = h;
}

bool linear_weight_verify(const void* wq, const LinearWeightHeader& want, hipStream_t stream) {
  {
    std::lock_guard<std::mutex> g(g_wmu);
    auto it = g_weights.find(wq);
    if (it != g_weights.end()) return it->second == want;
  }
  // a buffer prepared elsewhere (another process, or copied): read its header once
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
  LinearWeightHeader h{};
  if (hipMemcpyAsync(&h, wq, sizeof(h), hipMemcpyDeviceToHost, stream) != hipSuccess) return false;
  if (hipStreamSynchronize(stream) != hipSuccess) return false;
  if (!(h == want)) return false;
  linear_weight_note(wq, h);
  return true;
}

bool linear_weight_known_header(const void* wq, LinearWeightHeader* h) {
  std::lock_guard<std::mutex> g(g_wmu);
  auto it = g_weights.find(wq);
  if (it == g_weights.end()) return false;
  *h = it->second;
  return true;
}

bool linear_weight_verify_any_group(const void* wq, int out_f, int in_f, int flush, int bfloat, hipStream_t stream) {
  LinearWeightHeader h{};
  bool known = false;
  {
    std::lock_guard<std::mutex> g(g_wmu);
    auto it = g_weights.find(wq);
    if (it != g_weights.end()) h = it->second, known = true;
  }
  if (!known) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    if (hipMemcpyAsync(&h, wq, sizeof(h), hipMemcpyDeviceToHost, stream) != hipSuccess) return false;
    if (hipStreamSynchronize(stream) != hipSuccess) return false;
    if (h.magic != kLinearWeightMagic || h.gw <= 0 || h.out_f % h.gw) return false;
    linear_weight_note(wq, h);
  }
  LinearWeightHeader want = linear_weight_header(out_f, in_f, h.gw, flush, bfloat);
  return h == want;
}

LinearWeightHeader linear_weight_header(int out_f, int in_f, int gw, int flush, int bfloat) {
  LinearWeightHeader h{};
  h.magic = kLinearWeightMagic; h.version = 3;
  h.out_f = out_f; h.in_f = in_f; h.gw = gw; h.flush = flush ? 1 : 0; h.bfloat = bfloat;
  return h;
}

}  // namespace mxa

using namespace mxa;

extern "C" int64_t mxa_linear_weight_bytes(int32_t out_features, int32_t in_features, int32_t group_width) {
  if (out_features <= 0 || in_features <= 0 || group_width <= 0 || out_features % group_width) return -1;
  return linear_layout(out_features, in_features, group_width).total;
}

extern "C" int mxa_linear_weight_prep(const float* w, int32_t out_features, int32_t in_features, int32_t group_width,
                                      int32_t flush_subnormals, int32_t bfloat, void* wq, hipStream_t stream) {
  if (!w || !wq || out_features <= 0 || in_features <= 0 || group_width <= 0 || out_features % group_width)
    return MXA_ERR_ARG;
  if (bfloat != 0 && bfloat != 32 && (bfloat < 10 || bfloat > 31)) return MXA_ERR_ARG;
  if (!aligned16(wq)) return MXA_ERR_ARG;
  const LinearLayout W = linear_layout(out_features, in_features, group_width);
  unsigned char* wb = static_cast<unsigned char*>(wq);
  RowsPrepArgs rw{};
  rw.x = w; rw.s0 = 0; rw.s1 = 0; rw.s2 = in_features;
  rw.H = 1; rw.R = out_features; rw.rows = out_features; rw.D = in_features; rw.nb = W.nbk; rw.dpad = W.Cpad;
  rw.vec4 = aligned16(w) && in_features % 4 == 0;
  rw.op_kind = MXA_OP_MXINT8; rw.flush = flush_subnormals; rw.bfloat = bfloat;
  rw.codes = reinterpret_cast<int8_t*>(wb + W.rawc);
  rw.sT = reinterpret_cast<int16_t*>(wb + W.rawe);
  int rc = launch_rows_prep(rw, stream);
  if (rc) return rc;
  const int64_t pcols = (int64_t)W.G * W.NB32 * 32;
  hipLaunchKernelGGL(linear_pack_kernel, dim3((unsigned)((pcols * W.nbk + 255) / 256)), dim3(256), 0, stream,
                     rw.codes, rw.sT, out_features, group_width, W.NB32, W.nbk, W.Cpad, pcols,
                     reinterpret_cast<int8_t*>(wb + W.pk), reinterpret_cast<int16_t*>(wb + W.pe));
  if (hipGetLastError() != hipSuccess) return MXA_ERR_LAUNCH;
  hipLaunchKernelGGL(linear_stats_kernel, dim3((unsigned)((pcols + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const int16_t*>(wb + W.pe), pcols, W.nbk, reinterpret_cast<int16_t*>(wb + W.ps),
                     reinterpret_cast<int16_t*>(wb + W.pn));
  hipLaunchKernelGGL(linear_digits_kernel, dim3((unsigned)((pcols * W.nbk + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const int8_t*>(wb + W.pk), reinterpret_cast<const int16_t*>(wb + W.pe),
                     reinterpret_cast<const int16_t*>(wb + W.ps), W.nbk, pcols, reinterpret_cast<int8_t*>(wb + W.pd));
  hipLaunchKernelGGL(linear_group_stats_kernel, dim3((unsigned)((W.G + 63) / 64)), dim3(64), 0, stream,
                     reinterpret_cast<const int16_t*>(wb + W.ps), W.G, W.NB32, group_width,
                     reinterpret_cast<int16_t*>(wb + W.gs));
  const LinearWeightHeader h = linear_weight_header(out_features, in_features, group_width, flush_subnormals, bfloat);
  hipLaunchKernelGGL(linear_header_kernel, dim3(1), dim3(64), 0, stream, reinterpret_cast<LinearWeightHeader*>(wb + W.hdr),
                     h);
  if (hipGetLastError() != hipSuccess) return MXA_ERR_LAUNCH;
  linear_weight_note(wq, h);
  return MXA_OK;
}

