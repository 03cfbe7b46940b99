// Exact-order top-k with ONE WAVE PER ROW: the row's bookkeeping is scalar.
//
// torch's CPU topk(k, largest, sorted) runs, per row of pair<double,int64>
// (aten/src/ATen/native/TopKImpl.h:45-86, libstdc++ 11):
//     k*64 <= n : std::partial_sort(begin, begin+k, end, cmp)
//     else      : std::nth_element(begin, begin+k-1, end, cmp); std::sort(begin, begin+k-1, cmp)
// and ties are the norm for the approximate scores, so the element
// MOVEMENTS of __introselect / __introsort_loop / __unguarded_partition are
// reproduced, not just the selected set.
//
// One Hoare partition step in rank form (derived in tools/topk_model.py, checked
// against libstdc++ by tests/test_topk_model.py).  For pivot p at `first` (cmp =
// greater on order keys):
//   left stop  x in (first, last): a[x] <= p      right stop y in (first, last): a[y] >= p
//   T(z) = left stops <= z + right stops <= z  (non-decreasing)
//   cut  = first + 1 + #{z in (first,last) : T(z) <= totR}   ({T <= totR} is a prefix)
//   swaps: the left stops below the cut (nsw of them) trade places, in order, with the
//   nsw highest right stops taken from the top.
//
// Why one wave per row: every per-row quantity of a step (first, last, the median, the
// pivot, the stop counts, the cut, the swap count, the introsort stack) is wave-uniform,
// so it lives in SGPRs and the scalar unit does the bookkeeping while the vector unit
// only touches positions.  The stop flags of 64 positions are one compare each, landing
// as a 64-bit lane mask; the in-row prefix counts are v_mbcnt of those masks on top of a
// scalar base (no DPP scans); the window is strided (position f + 64 e + lane), so a
// row of n keys takes ceil(range / 64) vector registers per step.  Rows never wait for
// each other (no lockstep between the rows of a wave), and the few registers per lane
// leave room for 8 waves per SIMD to hide the LDS round trips.
//
// std::sort's final insertion sort is a stable sort of the arrangement the introsort
// loop leaves; because the final segments are mutually ordered it is a stable sort of
// each segment (<= 16 elements, or a heap-sorted segment, already in order), computed
// as a stable rank within the segment.  Depth-limit heap fallbacks, partial_sort and
// the <= 3-element insertion sort run serially on lane 0 (mxa_order.hpp, stl_heap.h
// semantics).
#pragma once
#include "mxa_order.hpp"

namespace mxa {

typedef __attribute__((address_space(3))) uint32_t wl32;
typedef __attribute__((address_space(3))) uint16_t wl16;

// per-row LDS: mirror A[n + 64] (order key << 32 | index; the window of a step may read
// up to 63 positions past the row), slot tables SL[n], SR[n] (u16 positions), 16-B aligned
__host__ __device__ constexpr int wrow_mirror(int n) { return n + 64; }
constexpr int kWMaxN = 1024;  // longest row (positions < 1024: 10-bit fields, 32 boundary words)
__host__ __device__ constexpr size_t wrow_bytes(int n) {
  return (size_t)8 * wrow_mirror(n) + (((size_t)4 * n + 15) & ~(size_t)15) + 128 + 512;
}

struct WRow {
  lu64* A;
  wl16* SL;
  wl16* SR;
  wl32* BW;  // final-segment boundaries of the sort phase, one bit per position (32 words)
  lu64* TR;  // trash: one 8-B slot per lane for the stores of lanes with nothing to store
};
__device__ __forceinline__ WRow carve_wrow(unsigned char* base, int n) {
  WRow g;
  g.A = (lu64*)(wl32*)base;
  g.SL = (wl16*)(base + (size_t)8 * wrow_mirror(n));
  g.SR = g.SL + n;
  g.BW = (wl32*)(base + (size_t)8 * wrow_mirror(n) + (((size_t)4 * n + 15) & ~(size_t)15));
  g.TR = (lu64*)(g.BW + 32);
  return g;
}

__device__ __forceinline__ uint32_t w_lane() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// lanes below this one whose bit is set in m, plus base
__device__ __forceinline__ uint32_t w_mbcnt(uint64_t m, uint32_t base) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, base));
}
__device__ __forceinline__ uint64_t w_ballot(bool c) { return __builtin_amdgcn_ballot_w64(c); }
__device__ __forceinline__ int w_uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t w_readlane(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }

__device__ __forceinline__ bool w_lanebit(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
// positions [lo, hi) of a 64-position window as a lane mask (0 <= lo <= hi)
__device__ __forceinline__ uint64_t w_rng(int lo, int hi) {
  const uint64_t h = hi >= 64 ? ~0ull : ((1ull << (hi < 0 ? 0 : hi)) - 1);
  return h & ~((1ull << (lo > 63 ? 63 : lo)) - 1);
}

// ---- one partition step ------------------------------------------------------
// libstdc++ __unguarded_partition_pivot(first = f, last = l), l - f >= 4: median of
// (f+1, mid, l-1) moved to f, then __unguarded_partition of (f, l).  Window: lane
// holds positions f + 64 e + lane, e < E = ceil((l - f) / 64).  Returns the cut.
// Branch-free: the stop masks are compares straight into SGPR pairs, ANDed with scalar
// range masks; the per-lane stop flags are those masks again (inverse ballot); lanes
// with nothing to store write their own trash slot.
template <int E>
__device__ __forceinline__ int w_part_e(const WRow& g, int f, int l, uint32_t lane) {
  const int mid = f + ((l - f) >> 1);
  // the median candidates (lanes 0..3: f, f+1, mid, l-1) and the window keys in one
  // LDS round trip; the iter_swap(f, median) is applied to the masks in scalar code
  // (selects with a 0 arm: the compiler keeps them as v_cndmask, not exec branches)
  const int cpos = f + (lane == 1 ? 1 : 0) + (lane == 2 ? mid - f : 0) + (lane >= 3 ? l - 1 - f : 0);
  const uint64_t cv = g.A[cpos];
  const wl32* wk = (const wl32*)(g.A + f + lane) + 1;
  uint32_t K[E];
#pragma unroll
  for (int e = 0; e < E; ++e) K[e] = wk[128 * e];
  const uint32_t ch = (uint32_t)(cv >> 32), cl = (uint32_t)cv;
  const uint32_t kf = w_readlane(ch, 0), ka = w_readlane(ch, 1), kb = w_readlane(ch, 2), kc = w_readlane(ch, 3);
  // __move_median_to_first(f, f+1, mid, l-1) with cmp = greater (stl_algo.h:79-99)
  int ms;
  if (ka > kb) ms = kb > kc ? 2 : (ka > kc ? 3 : 1);
  else ms = ka > kc ? 1 : (kb > kc ? 3 : 2);
  const int m = ms == 1 ? f + 1 : ms == 2 ? mid : l - 1;
  const uint32_t p = ms == 1 ? ka : ms == 2 ? kb : kc;
  {  // iter_swap(f, m): lane 0 writes A[f] = old m, lane 1 writes A[m] = old f
    const uint32_t xml = w_readlane(cl, ms), xfl = w_readlane(cl, 0);
    lu64* dst = lane == 0 ? g.A + f : lane == 1 ? g.A + m : g.TR + lane;
    *dst = lane == 0 ? pack_ki(p, xml) : pack_ki(kf, xfl);
  }
  // position m holds old f (key kf) now: its bit of window word em is fixed in the masks
  const int em = (m - f) >> 6;
  const uint64_t mb = 1ull << ((m - f) & 63);
  const bool mL = kf <= p, mR = kf >= p;
  // pass 1: the right stops' count (position f is never a stop)
  auto rmask = [&](int e) {
    const uint64_t sel = e == em ? mb : 0ull;  // scalar selects, no branch
    return ((w_ballot(K[e] >= p) & w_rng(e == 0 ? 1 : 0, l - f - 64 * e)) & ~sel) | (mR ? sel : 0ull);
  };
  constexpr bool kKeepR = E <= 4;  // wider windows recompute the masks (SGPRs are the budget)
  uint64_t Rm[kKeepR ? E : 1];
  int totR = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint64_t r = rmask(e);
    if (kKeepR) Rm[e] = r;
    totR += __popcll(r);
  }
  // pass 2: inclusive prefix counts, the slot tables, the cut and the swap count.
  // Every left stop writes its position at SL[its rank from the bottom], every right stop
  // at SR[its rank from the top]; the first nsw of each then trade places.
  wl16* const slb = g.SL - 1;
  wl16* const srb = g.SR + totR;
  wl16* const trash = (wl16*)(g.TR + lane);
  int baseL = 0, baseR = 0, ncut = 0, nsw = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const uint64_t rng = w_rng(e == 0 ? 1 : 0, l - f - 64 * e);
    const uint64_t sel = e == em ? mb : 0ull;
    const uint64_t Lm = ((w_ballot(K[e] <= p) & rng) & ~sel) | (mL ? sel : 0ull);
    const uint64_t R = kKeepR ? Rm[kKeepR ? e : 0] : rmask(e);
    const uint32_t PLi = w_mbcnt(Lm >> 1, (uint32_t)baseL + (uint32_t)(Lm & 1));
    const uint32_t PRi = w_mbcnt(R >> 1, (uint32_t)baseR + (uint32_t)(R & 1));
    const uint16_t z = (uint16_t)(f + 64 * e + (int)lane);
    *(w_lanebit(Lm) ? slb + PLi : trash) = z;
    *(w_lanebit(R) ? srb - PRi : trash) = z;
    const uint64_t ok = w_ballot(PLi + PRi <= (uint32_t)totR) & rng;
    ncut += __popcll(ok);
    nsw += __popcll(ok & Lm);
    baseL += __popcll(Lm);
    baseR += __popcll(R);
  }
  wave_lds_sync();
  for (int t = (int)lane; t < nsw; t += 64) {
    const int x = g.SL[t], y = g.SR[t];
    const uint64_t ax = g.A[x], ay = g.A[y];
    g.A[x] = ay;
    g.A[y] = ax;
  }
  wave_lds_sync();
  return f + 1 + ncut;
}
template <int EW>
__device__ __forceinline__ int w_partition(const WRow& g, int f, int l, uint32_t lane) {
  const int E = (l - f + 63) >> 6;
  if (E <= 1) return w_part_e<1>(g, f, l, lane);
  if (EW <= 1 || E == 2) return w_part_e<EW < 2 ? 1 : 2>(g, f, l, lane);
  if (EW <= 2 || E == 3) return w_part_e<EW < 3 ? 1 : 3>(g, f, l, lane);
  if (EW <= 3 || E == 4) return w_part_e<EW < 4 ? 1 : 4>(g, f, l, lane);
  if (EW <= 4 || E <= 6) return w_part_e<EW < 6 ? 1 : 6>(g, f, l, lane);
  if (EW <= 6 || E <= 8) return w_part_e<EW < 8 ? 1 : 8>(g, f, l, lane);
  if (EW <= 8 || E <= 12) return w_part_e<EW < 12 ? 1 : 12>(g, f, l, lane);
  return w_part_e<EW < 16 ? 1 : 16>(g, f, l, lane);
}

// boundary bit at position c (ds_or: no return value waited on)
__device__ __forceinline__ void w_mark(const WRow& g, int c) {
  __hip_atomic_fetch_or((uint32_t*)(g.BW + (c >> 5)), 1u << (c & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// ---- the whole top-k ----------------------------------------------------------
// std::nth_element(begin, begin + k - 1, end) then std::sort(begin, begin + k - 1)
// (or std::partial_sort when k*64 <= n) on the wave's row; afterwards A[p], p < k,
// holds torch's p-th index in its low word.  n, k wave-uniform; n <= 64 EW.
template <int EW>
__device__ __forceinline__ void wave_topk(const WRow& g, int n, int k) {
  const uint32_t lane = w_lane();
  if (k <= 0) return;
  if (k * 64 <= n) {  // std::partial_sort(begin, begin + k, end)
    if (lane == 0) {
      ln_heap_select(g.A, 0, k, n);
      ln_sort_heap(g.A, 0, k);
    }
    wave_lds_sync();
    return;
  }
  const int nth = k - 1, m = k - 1;
  {  // std::__introselect(0, nth, n, 2 lg n)
    int f = 0, l = n, d = 2 * ilog2(n);
    bool heap = false;
    while (l - f > 3) {
      if (d == 0) {
        heap = true;
        break;
      }
      --d;
      const int cut = w_partition<EW>(g, f, l, lane);
      if (cut <= nth) f = cut;
      else l = cut;
    }
    if (heap) {  // __heap_select(f, nth + 1, l); iter_swap(f, nth)
      if (lane == 0) {
        ln_heap_select(g.A, f, nth + 1, l);
        const uint64_t t = g.A[f];
        g.A[f] = g.A[nth];
        g.A[nth] = t;
      }
    } else if (l - f > 1 && lane == 0) {
      ln_insertion_sort(g.A, f, l);
    }
    wave_lds_sync();
  }
  if (m < 2) return;
  // std::sort(0, m): __introsort_loop(0, m, 2 lg m), threshold 16.  The partitions of
  // disjoint ranges are independent, so the pending ranges go on a stack (one per lane
  // of a VGPR) in any order; every cut starts a final segment (boundary bits BW, plus 0
  // and m).
  if ((int)lane < 32) g.BW[lane] = lane == 0 ? 1u : 0u;
  wave_lds_sync();
  if (lane == 0) w_mark(g, m);
  int maxlen = 0;  // longest final segment that is not heap-sorted
  {
    uint32_t stk = 0;  // lane s: pending range s (f | l << 11 | d << 22)
    int sp = 0;
    int f = 0, l = m, d = 2 * ilog2(m);
    while (true) {
      while (l - f > 16 && d > 0) {
        --d;
        const int cut = w_partition<EW>(g, f, l, lane);
        if (lane == 0) w_mark(g, cut);
        stk = lane == (uint32_t)sp ? (uint32_t)cut | ((uint32_t)l << 11) | ((uint32_t)d << 22) : stk;
        ++sp;
        l = cut;
      }
      if (l - f > 16) {  // depth limit: std::__partial_sort(f, l, l) -- final as it stands
        if (lane == 0) {
          ln_heap_select(g.A, f, l, l);
          ln_sort_heap(g.A, f, l);
        }
        for (int c = f + 1 + (int)lane; c < l; c += 64) w_mark(g, c);  // singletons: rank = identity
        wave_lds_sync();
      } else {
        maxlen = max(maxlen, l - f);
      }
      if (sp == 0) break;
      --sp;
      const uint32_t s = w_readlane(stk, sp);
      f = (int)(s & 2047u);
      l = (int)((s >> 11) & 2047u);
      d = (int)(s >> 22);
    }
  }
  if (maxlen < 2) return;  // every segment a singleton or heap-sorted
  wave_lds_sync();
  // stable rank of each position z < m within its segment [s, t): the composite
  // (key << 32 | 0xFFFF - position) is unique and larger for the earlier of two equal
  // keys, so the rank is s + the number of larger composites in the segment.  A segment
  // that is not heap-sorted has <= 16 elements, so s >= z - 15 and t <= z + 16: both lie
  // in the 96-bit window of boundary words w - 1 .. w + 1 around z's word w.
  constexpr int EM = EW;  // m < 64 EW
  uint64_t X[EM];
  uint32_t R[EM];
  const wl32* A32 = (const wl32*)g.A;
#pragma unroll
  for (int e = 0; e < EM; ++e) {
    if (64 * e < m) {
      const int z = 64 * e + (int)lane;
      const int zc = min(z, m - 1);
      const uint64_t x = g.A[zc];
      X[e] = x;
      const int w = zc >> 5, o = zc & 31;
      const uint32_t b0 = w > 0 ? g.BW[w - 1] : 0u, b1 = g.BW[w], b2 = w < 31 ? g.BW[w + 1] : 0u;
      // s: highest set bit at or below z (bit 32 + o of b0:b1:b2 is z)
      const uint64_t lowin = ((uint64_t)b1 << 32 | b0) & (~0ull >> (31 - o));  // bits <= 32 + o
      const int s = zc - (32 + o - (63 - (int)__clzll(lowin)));
      // t: lowest set bit above z
      const uint64_t hiwin = ((uint64_t)b2 << 32 | b1) >> o >> 1;  // bit 0 <-> position z + 1
      const int t = zc + 1 + (int)__ffsll((long long)hiwin) - 1;
      const uint64_t cz = (x & 0xFFFFFFFF00000000ull) | (uint32_t)(0xFFFF - zc);
      uint32_t r = (uint32_t)s;
      for (int j = 0; j < maxlen; ++j) {
        const int wp = min(s + j, m - 1);
        const uint32_t kw = A32[2 * wp + 1];
        const uint64_t cw = ((uint64_t)kw << 32) | (uint32_t)(0xFFFF - wp);
        r += (s + j < t && cw > cz) ? 1u : 0u;
      }
      R[e] = r;
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int e = 0; e < EM; ++e)
    if (64 * e < m && 64 * e + (int)lane < m) g.A[R[e]] = X[e];
  wave_lds_sync();
}

}  // namespace mxa
