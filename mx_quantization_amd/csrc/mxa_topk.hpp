// Wave-per-row top-k with torch's CPU index order.
//
// torch.topk(x, k, largest=True, sorted=True) on CPU (aten TopKImpl.h:45-86)
// runs, per row of pair<double,int64>:
//     k*64 <= n : std::partial_sort(begin, begin+k, end, cmp)
//     else      : std::nth_element(begin, begin+k-1, end, cmp); std::sort(begin, begin+k-1, cmp)
// with cmp(x, y) = (isnan(x) && !isnan(y)) || x > y (libstdc++ 11).  Ties are
// the norm for the approximate scores, so reproducing the index
// order means reproducing those algorithms' element movements.
//
// Each Hoare partition step (libstdc++ __unguarded_partition) is computed from
// per-position flags, ballots and prefix counts instead of two serial cursors
// (derivation and an executable model: tools/topk_model.py, checked against
// libstdc++ by tests/test_topk_model.py):
//   left stop  x in [first+1, last): !(a[x] > p)      rank A(x)   = #left stops below x
//   right stop y in [first, last):   !(p > a[y])      rank Bgt(y) = #right stops above y
//   left stop swaps iff Bgt > A, right stop swaps iff A > Bgt; equal ranks pair up;
//   cut = min(first non-swapping left stop, lowest swapping right stop | last).
// The final insertion sorts are stable sorts of segments (<=16 elements in
// std::sort, <=3 in nth_element).  Depth-limit heap fallbacks and the
// partial_sort branch run serially on lane 0 (stl_heap.h semantics).
//
// Row layout: position p lives in lane (p & 63), slot (p >> 6); S slots -> n <= 64*S.
#pragma once
#include "mxa_common.hpp"

namespace mxa {

// Order-preserving key for cmp: NaN largest (all NaNs tie), -0 == +0.
__device__ __forceinline__ uint32_t order_key(float f) {
  uint32_t b = __float_as_uint(f);
  const uint32_t a = b & 0x7FFFFFFFu;
  if (a > 0x7F800000u) return 0xFFFFFFFFu;
  if (a == 0u) b = 0u;
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ uint64_t pack_ki(uint32_t key, uint32_t idx) {
  return ((uint64_t)key << 32) | idx;
}

// per-wave LDS scratch
struct TopkLds {
  uint64_t* a;  // nmax entries
  uint64_t* b;  // nmax entries
  int* stk;     // kTopkStack entries (introsort's pending segments)
};
constexpr int kTopkStack = 24;  // >= 2*lg(511) + 1 pending segments

__device__ __forceinline__ int ilog2(int n) { return 31 - __clz(n); }

// bits [lo, hi) of a 64-bit mask, lo/hi clamped to [0, 64]
__device__ __forceinline__ uint64_t range_mask(int lo, int hi) {
  lo = lo < 0 ? 0 : (lo > 64 ? 64 : lo);
  hi = hi < 0 ? 0 : (hi > 64 ? 64 : hi);
  if (hi <= lo) return 0ull;
  const uint64_t up = hi == 64 ? ~0ull : ((1ull << hi) - 1ull);
  const uint64_t dn = (1ull << lo) - 1ull;
  return up & ~dn;
}

template <int S>
struct WaveRow {
  uint32_t key[S];
  uint32_t idx[S];
  int lane;

  // value at uniform position p: one readlane per slot, selected without branches
  __device__ __forceinline__ uint32_t get_key(int p) const {
    const int sl = p >> 6, ln = p & 63;
    uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)key[0], ln);
#pragma unroll
    for (int s = 1; s < S; ++s) {
      const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)key[s], ln);
      v = sl == s ? w : v;
    }
    return v;
  }
  __device__ __forceinline__ uint32_t get_idx(int p) const {
    const int sl = p >> 6, ln = p & 63;
    uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)idx[0], ln);
#pragma unroll
    for (int s = 1; s < S; ++s) {
      const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)idx[s], ln);
      v = sl == s ? w : v;
    }
    return v;
  }
  __device__ __forceinline__ void set(int p, uint32_t k, uint32_t i) {
    const int sl = p >> 6, ln = p & 63;
    const bool me = lane == ln;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const bool hit = me && s == sl;
      key[s] = hit ? k : key[s];
      idx[s] = hit ? i : idx[s];
    }
  }

  // libstdc++ __unguarded_partition_pivot(first, last) with cmp = greater.
  __device__ int partition_pivot(int first, int last, const TopkLds& sc) {
    const int mid = first + (last - first) / 2;
    const uint32_t ka = get_key(first + 1), kb = get_key(mid), kc = get_key(last - 1);
    int m;  // __move_median_to_first(first, first+1, mid, last-1)
    if (ka > kb) {
      if (kb > kc) m = mid;
      else if (ka > kc) m = last - 1;
      else m = first + 1;
    } else if (ka > kc) m = first + 1;
    else if (kb > kc) m = last - 1;
    else m = mid;
    const uint32_t p = m == first + 1 ? ka : (m == mid ? kb : kc);
    {  // iter_swap(first, m)
      const uint32_t kf = get_key(first), jf = get_idx(first), jm = get_idx(m);
      set(first, p, jm);
      set(m, kf, jf);
    }
    const int s0 = first >> 6, s1 = (last - 1) >> 6;
    uint64_t L[S], R[S];
    int cl[S], cr[S];
    int totL = 0, totR = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      L[s] = R[s] = 0ull;
      cl[s] = totL;
      cr[s] = totR;
      if (s < s0 || s > s1) continue;  // uniform: slot outside the segment
      const uint64_t rr = range_mask(first - 64 * s, last - 64 * s);
      const uint64_t rl = range_mask(first + 1 - 64 * s, last - 64 * s);
      L[s] = ballot64(key[s] <= p) & rl;  // left stop:  !(a > p)
      R[s] = ballot64(key[s] >= p) & rr;  // right stop: !(p > a)
      totL += __popcll(L[s]);
      totR += __popcll(R[s]);
    }
    bool swl[S], swr[S];
    int rank[S];
    int msw = 0;
    uint64_t SWL[S], SWR[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      swl[s] = swr[s] = false;
      rank[s] = 0;
      SWL[s] = SWR[s] = 0ull;
      if (s < s0 || s > s1) continue;
      const bool isl = (L[s] >> lane) & 1ull, isr = (R[s] >> lane) & 1ull;
      const int A = cl[s] + mbcnt(L[s]);
      const int Bgt = totR - cr[s] - mbcnt(R[s]) - (isr ? 1 : 0);
      swl[s] = isl && Bgt > A;
      swr[s] = isr && A > Bgt;
      rank[s] = swl[s] ? A : Bgt;
      SWL[s] = ballot64(swl[s]);
      SWR[s] = ballot64(swr[s]);
      msw += __popcll(SWL[s]);
    }
    if (msw > 0) {  // exchange the t-th swapping left stop with the t-th swapping right stop
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s < s0 || s > s1) continue;
        if (swl[s]) sc.a[rank[s]] = pack_ki(key[s], idx[s]);
        if (swr[s]) sc.b[rank[s]] = pack_ki(key[s], idx[s]);
      }
      wave_lds_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (s < s0 || s > s1) continue;
        if (swl[s] || swr[s]) {
          const uint64_t v = swl[s] ? sc.b[rank[s]] : sc.a[rank[s]];
          key[s] = (uint32_t)(v >> 32);
          idx[s] = (uint32_t)v;
        }
      }
      wave_lds_sync();
    }
    // cut = min(first non-swapping left stop, lowest swapping right stop | last)
    int c1 = 1 << 30, c2 = last;
    bool f1 = false, f2 = msw == 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (s < s0 || s > s1) continue;
      const uint64_t nsl = L[s] & ~SWL[s];
      if (!f1 && nsl) {
        c1 = 64 * s + __ffsll((unsigned long long)nsl) - 1;
        f1 = true;
      }
      if (!f2 && SWR[s]) {
        c2 = 64 * s + __ffsll((unsigned long long)SWR[s]) - 1;
        f2 = true;
      }
    }
    return c1 < c2 ? c1 : c2;
  }

  // Stable sort (key descending) of the segment [lo[s], hi[s]) each position belongs
  // to (segments of at most `maxlen` elements, disjoint; lo == hi: not in a segment).
  __device__ void stable_sort_segments(const int (&lo)[S], const int (&hi)[S], int n, int maxlen,
                                       const TopkLds& sc) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      if (pos < n) sc.a[pos] = pack_ki(key[s], idx[s]);
    }
    wave_lds_sync();
    int r[S];
#pragma unroll
    for (int s = 0; s < S; ++s) r[s] = 0;
    for (int j = 0; j < maxlen; ++j) {  // all slots' loads in flight together
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int q = lo[s] + j;
        if (q < hi[s]) {
          const int pos = s * 64 + lane;
          const uint32_t kj = (uint32_t)(sc.a[q] >> 32);
          r[s] += (kj > key[s] || (kj == key[s] && q < pos)) ? 1 : 0;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (lo[s] < hi[s]) sc.b[lo[s] + r[s]] = pack_ki(key[s], idx[s]);
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (lo[s] < hi[s]) {
        const uint64_t v = sc.b[s * 64 + lane];
        key[s] = (uint32_t)(v >> 32);
        idx[s] = (uint32_t)v;
      }
    }
    wave_lds_sync();
  }

  __device__ void to_lds(uint64_t* arr, int n) const {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      if (pos < n) arr[pos] = pack_ki(key[s], idx[s]);
    }
  }
  __device__ void from_lds(const uint64_t* arr, int n) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      if (pos < n) {
        const uint64_t v = arr[pos];
        key[s] = (uint32_t)(v >> 32);
        idx[s] = (uint32_t)v;
      }
    }
  }
};

// ---- serial heap algorithms on an LDS array (lane 0 only), stl_heap.h ------
__device__ __forceinline__ bool hgt(uint64_t x, uint64_t y) { return (uint32_t)(x >> 32) > (uint32_t)(y >> 32); }

__device__ inline void s_push_heap(uint64_t* f, int hole, int top, uint64_t v) {
  int parent = (hole - 1) / 2;
  while (hole > top && hgt(f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
__device__ inline void s_adjust_heap(uint64_t* f, int hole, int len, uint64_t v) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (hgt(f[second], f[second - 1])) second--;
    f[hole] = f[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    f[hole] = f[second - 1];
    hole = second - 1;
  }
  s_push_heap(f, hole, top, v);
}
__device__ inline void s_make_heap(uint64_t* f, int len) {
  if (len < 2) return;
  int parent = (len - 2) / 2;
  while (true) {
    s_adjust_heap(f, parent, len, f[parent]);
    if (parent == 0) return;
    parent--;
  }
}
__device__ inline void s_pop_heap(uint64_t* first, int len, uint64_t* result) {
  const uint64_t v = *result;
  *result = *first;
  s_adjust_heap(first, 0, len, v);
}
// heap_select(first, middle, last) on arr[first..last)
__device__ inline void s_heap_select(uint64_t* arr, int first, int middle, int last) {
  uint64_t* f = arr + first;
  const int len = middle - first;
  s_make_heap(f, len);
  for (int i = middle; i < last; ++i)
    if (hgt(arr[i], f[0])) s_pop_heap(f, len, arr + i);
}
__device__ inline void s_sort_heap(uint64_t* arr, int first, int last) {
  while (last - first > 1) {
    --last;
    s_pop_heap(arr + first, last - first, arr + last);
  }
}

// Full top-k on a wave's row.  On return positions [0, k) hold torch's order.
template <int S>
__device__ void wave_topk(WaveRow<S>& w, int n, int k, const TopkLds& sc) {
  if (k <= 0) return;
  if (k * 64 <= n) {  // std::partial_sort(begin, begin+k, end)
    w.to_lds(sc.a, n);
    wave_lds_sync();
    if (w.lane == 0) {
      s_heap_select(sc.a, 0, k, n);
      s_sort_heap(sc.a, 0, k);
    }
    wave_lds_sync();
    w.from_lds(sc.a, n);
    wave_lds_sync();
    return;
  }
  // ---- std::nth_element(begin, begin+k-1, end): __introselect ----------------
  {
    int first = 0, last = n;
    const int nth = k - 1;
    int depth = 2 * ilog2(n);
    bool fell_back = false;
    while (last - first > 3) {
      if (depth == 0) {
        w.to_lds(sc.a, n);
        wave_lds_sync();
        if (w.lane == 0) {
          s_heap_select(sc.a, first, nth + 1, last);
          const uint64_t t = sc.a[first];
          sc.a[first] = sc.a[nth];
          sc.a[nth] = t;
        }
        wave_lds_sync();
        w.from_lds(sc.a, n);
        wave_lds_sync();
        fell_back = true;
        break;
      }
      --depth;
      const int cut = w.partition_pivot(first, last, sc);
      if (cut <= nth) first = cut;
      else last = cut;
    }
    if (!fell_back && last - first > 1) {  // __insertion_sort(first, last): <= 3 elements
      int lo[S], hi[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int pos = s * 64 + w.lane;
        const bool in = pos >= first && pos < last;
        lo[s] = in ? first : 0;
        hi[s] = in ? last : 0;
      }
      w.stable_sort_segments(lo, hi, n, last - first, sc);
    }
  }
  // ---- std::sort(begin, begin+k-1): __introsort_loop + final insertion sort --
  const int m = k - 1;
  if (m <= 1) return;
  int lo[S], hi[S];
#pragma unroll
  for (int s = 0; s < S; ++s) lo[s] = hi[s] = 0;
  // pending segments (cut, last, depth) packed 10|10|6 bits; segments are disjoint,
  // so the order they are processed in does not matter
  int sp = 0;
  auto push = [&](int f, int l, int d) {
    if (sp < kTopkStack) sc.stk[sp] = f | (l << 10) | (d << 20);
    ++sp;
  };
  push(0, m, 2 * ilog2(m));
  while (sp > 0) {
    wave_lds_sync();
    --sp;
    const int e = sc.stk[sp];
    const int f = e & 1023;
    int l = (e >> 10) & 1023;
    int d = e >> 20;
    bool heaped = false;
    while (l - f > 16) {
      if (d == 0) {  // std::__partial_sort(f, l, l): heapsort, leaves [f, l) in final order
        w.to_lds(sc.a, n);
        wave_lds_sync();
        if (w.lane == 0) {
          s_heap_select(sc.a, f, l, l);
          s_sort_heap(sc.a, f, l);
        }
        wave_lds_sync();
        w.from_lds(sc.a, n);
        wave_lds_sync();
        heaped = true;
        break;
      }
      --d;
      const int cut = w.partition_pivot(f, l, sc);
      push(cut, l, d);
      l = cut;
    }
    if (!heaped && l - f > 1) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int pos = s * 64 + w.lane;
        const bool in = pos >= f && pos < l;
        lo[s] = in ? f : lo[s];
        hi[s] = in ? l : hi[s];
      }
    }
  }
  w.stable_sort_segments(lo, hi, n, 16, sc);
}

}  // namespace mxa
