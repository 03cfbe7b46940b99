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

// per-wave LDS scratch, 2*nmax uint64 entries
struct TopkLds {
  uint64_t* a;  // nmax entries
  uint64_t* b;  // nmax entries
};

__device__ __forceinline__ int ilog2(int n) { return 31 - __clz(n); }

template <int S>
struct WaveRow {
  uint32_t key[S];
  uint32_t idx[S];
  int lane;

  __device__ __forceinline__ uint32_t get_key(int p) const {
    const int sl = p >> 6, ln = p & 63;
    uint32_t v = 0;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (s == sl) v = (uint32_t)__builtin_amdgcn_readlane((int)key[s], ln);
    return v;
  }
  __device__ __forceinline__ uint32_t get_idx(int p) const {
    const int sl = p >> 6, ln = p & 63;
    uint32_t v = 0;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (s == sl) v = (uint32_t)__builtin_amdgcn_readlane((int)idx[s], ln);
    return v;
  }
  __device__ __forceinline__ void set(int p, uint32_t k, uint32_t i) {
    const int sl = p >> 6, ln = p & 63;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (s == sl && lane == ln) {
        key[s] = k;
        idx[s] = i;
      }
  }
  __device__ __forceinline__ void swap_pos(int p, int q) {
    if (p == q) return;
    const uint32_t kp = get_key(p), ip = get_idx(p), kq = get_key(q), iq = get_idx(q);
    set(p, kq, iq);
    set(q, kp, ip);
  }

  // libstdc++ __unguarded_partition_pivot(first, last) with cmp = greater.
  __device__ int partition_pivot(int first, int last, const TopkLds& sc) {
    const int mid = first + (last - first) / 2;
    const int a = first + 1, b = mid, c = last - 1;
    const uint32_t ka = get_key(a), kb = get_key(b), kc = get_key(c);
    int m;  // __move_median_to_first(first, a, b, c)
    if (ka > kb) {
      if (kb > kc) m = b;
      else if (ka > kc) m = c;
      else m = a;
    } else if (ka > kc) m = a;
    else if (kb > kc) m = c;
    else m = b;
    swap_pos(first, m);
    const uint32_t p = get_key(first);
    const int s0 = first >> 6, s1 = (last - 1) >> 6;
    uint64_t L[S], R[S];
    bool lst[S], rst[S];
    int cl_before[S], cr_before[S];
    int totL = 0, totR = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      const bool in_r = (s >= s0 && s <= s1) && pos >= first && pos < last;
      lst[s] = in_r && pos > first && !(key[s] > p);
      rst[s] = in_r && !(p > key[s]);
      L[s] = __ballot(lst[s]);
      R[s] = __ballot(rst[s]);
      cl_before[s] = totL;
      cr_before[s] = totR;
      totL += __popcll(L[s]);
      totR += __popcll(R[s]);
    }
    bool swl[S], swr[S];
    int rank[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int A = cl_before[s] + mbcnt(L[s]);
      const int Bgt = totR - cr_before[s] - mbcnt(R[s]) - (rst[s] ? 1 : 0);
      swl[s] = lst[s] && Bgt > A;
      swr[s] = rst[s] && A > Bgt;
      rank[s] = swl[s] ? A : Bgt;
      if (swl[s]) sc.a[rank[s]] = pack_ki(key[s], idx[s]);
      if (swr[s]) sc.b[rank[s]] = pack_ki(key[s], idx[s]);
    }
    wave_lds_sync();
    int c1 = 1 << 30, c2 = -1, msw = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (swl[s] || swr[s]) {
        const uint64_t v = swl[s] ? sc.b[rank[s]] : sc.a[rank[s]];
        key[s] = (uint32_t)(v >> 32);
        idx[s] = (uint32_t)v;
      }
      const uint64_t nsl = __ballot(lst[s] && !swl[s]);
      const uint64_t swrb = __ballot(swr[s]);
      msw += __popcll(swrb);
      if (nsl && c1 == (1 << 30)) c1 = s * 64 + __ffsll((unsigned long long)nsl) - 1;
      if (swrb && c2 < 0) c2 = s * 64 + __ffsll((unsigned long long)swrb) - 1;
    }
    wave_lds_sync();
    if (msw == 0) c2 = last;
    return c1 < c2 ? c1 : c2;
  }

  // Stable sort (by key, descending) of the segment each lane's position belongs to:
  // lanes with seg_lo[s] < seg_hi[s] participate.  Segments must be disjoint.
  __device__ void stable_sort_segments(const int (&seg_lo)[S], const int (&seg_hi)[S], int n,
                                       const TopkLds& sc) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      if (pos < n) sc.a[pos] = pack_ki(key[s], idx[s]);
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = s * 64 + lane;
      if (seg_lo[s] < seg_hi[s]) {
        int r = 0;
        const uint32_t mk = key[s];
        for (int j = seg_lo[s]; j < seg_hi[s]; ++j) {
          const uint32_t kj = (uint32_t)(sc.a[j] >> 32);
          r += (kj > mk || (kj == mk && j < pos)) ? 1 : 0;
        }
        sc.b[seg_lo[s] + r] = pack_ki(key[s], idx[s]);
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (seg_lo[s] < seg_hi[s]) {
        const int pos = s * 64 + lane;
        const uint64_t v = sc.b[pos];
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
    if (!fell_back && last - first > 1) {
      int lo[S], hi[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int pos = s * 64 + w.lane;
        const bool in = pos >= first && pos < last;
        lo[s] = in ? first : 0;
        hi[s] = in ? last : 0;
      }
      w.stable_sort_segments(lo, hi, n, sc);
    }
  }
  // ---- std::sort(begin, begin+k-1): __introsort_loop + final insertion sort --
  const int m = k - 1;
  if (m <= 1) return;
  int lo[S], hi[S];
#pragma unroll
  for (int s = 0; s < S; ++s) lo[s] = hi[s] = 0;
  // explicit stack of pending segments (cut, last, depth); order is irrelevant
  // because segments are disjoint.  Depth of the stack <= 2*lg(m) + 1 < 20.
  int st_f[20], st_l[20], st_d[20];
  int sp = 0;
  st_f[0] = 0;
  st_l[0] = m;
  st_d[0] = 2 * ilog2(m);
  sp = 1;
  while (sp > 0) {
    --sp;
    const int f = st_f[sp];
    int l = st_l[sp];
    int d = st_d[sp];
    bool heaped = false;
    while (l - f > 16) {
      if (d == 0) {  // std::__partial_sort(f, l, l): heapsort, already in final order
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
      if (sp < 20) {  // bound: <= 2*lg(m)+1 pending segments
        st_f[sp] = cut;
        st_l[sp] = l;
        st_d[sp] = d;
        ++sp;
      }
      l = cut;
    }
    if (!heaped && l - f > 1) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int pos = s * 64 + w.lane;
        if (pos >= f && pos < l) {
          lo[s] = f;
          hi[s] = l;
        }
      }
    }
  }
  w.stable_sort_segments(lo, hi, n, sc);
}

}  // namespace mxa
