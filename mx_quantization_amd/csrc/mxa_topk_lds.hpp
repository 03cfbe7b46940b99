// Wave-per-row top-k in torch's CPU index order, row held in LDS.
//
// Same algorithm restatement as mxa_topk.hpp (libstdc++ 11 __introselect +
// __introsort_loop + __final_insertion_sort, TopKImpl.h:45-86; ballot/rank form of
// __unguarded_partition, tools/topk_model.py), organised for short ranges:
//   * the row lives in LDS as u64 (order key << 32 | index), positions 0..n-1;
//   * a partition step loads ONLY its range [first, last), relative to lane 0
//     (slot s, lane i <-> position first + 64 s + i), so the step costs
//     ceil((last - first) / 64) slots -- after the first one or two steps every
//     range of introselect / introsort fits one slot -- and every range mask is
//     a plain "lane < len" predicate;
//   * swapped elements are written back; nothing else moves.
// Heap fallbacks (depth limit) and the partial_sort branch run serially on lane 0
// over the same LDS array (stl_heap.h semantics, shared with mxa_topk.hpp).
#pragma once
#include "mxa_topk.hpp"

namespace mxa {

struct TopkLdsV2 {
  uint64_t* A;    // [n] the row
  uint64_t* xa;   // [64 * S] swap exchange, left stops by rank
  uint64_t* xb;   // [64 * S] swap exchange, right stops by rank
  uint32_t* seg;  // [n] final-insertion-sort segment of each position: lo | hi << 16
  int* stk;       // [kTopkStack] introsort pending segments
};

// LDS bytes of one wave's scratch for rows of <= 64*S values (16-B multiple)
__host__ __device__ constexpr size_t topk_scratch_bytes(int S) {
  return (size_t)64 * S * 8 + (size_t)2 * 32 * S * 8 + (size_t)64 * S * 4 + (size_t)kTopkStack * 4 + 0;
}
__device__ __forceinline__ TopkLdsV2 carve_topk(unsigned char* base, int S) {
  TopkLdsV2 sc;
  sc.A = reinterpret_cast<uint64_t*>(base);
  sc.xa = sc.A + 64 * S;
  sc.xb = sc.xa + 32 * S;
  sc.seg = reinterpret_cast<uint32_t*>(sc.xb + 32 * S);
  sc.stk = reinterpret_cast<int*>(sc.seg + 64 * S);
  return sc;
}

__device__ __forceinline__ uint32_t key_of(uint64_t v) { return (uint32_t)(v >> 32); }

// __unguarded_partition_pivot(first, last) with cmp = greater; returns the cut.
template <int S>
__device__ int lds_partition(const TopkLdsV2& sc, int first, int last, int lane) {
  uint64_t* A = sc.A;
  const int len = last - first;
  const int mid = first + len / 2;
  // __move_median_to_first(first, first+1, mid, last-1): uniform LDS reads (broadcast)
  const uint32_t ka = key_of(A[first + 1]), kb = key_of(A[mid]), kc = key_of(A[last - 1]);
  int m;
  if (ka > kb) {
    if (kb > kc) m = mid;
    else if (ka > kc) m = last - 1;
    else m = first + 1;
  } else if (ka > kc) m = first + 1;
  else if (kb > kc) m = last - 1;
  else m = mid;
  const uint32_t p = m == first + 1 ? ka : (m == mid ? kb : kc);
  // load the range; iter_swap(first, m) applied on the loaded values
  const uint64_t vf = A[first], vm = A[m];
  uint64_t v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int rel = 64 * s + lane;
    v[s] = 0ull;
    if (rel < len) {
      const int pos = first + rel;
      v[s] = pos == first ? vm : (pos == m ? vf : A[pos]);
    }
  }
  // stops: left in [first+1, last): !(a > p); right in [first, last): !(p > a)
  uint64_t Lb[S], Rb[S];
  int cl[S], cr[S];
  int totL = 0, totR = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int rel = 64 * s + lane;
    const bool in = rel < len;
    const uint32_t k = key_of(v[s]);
    Lb[s] = __ballot(in && rel > 0 && !(k > p));
    Rb[s] = __ballot(in && !(p > k));
    cl[s] = totL;
    cr[s] = totR;
    totL += __popcll(Lb[s]);
    totR += __popcll(Rb[s]);
  }
  bool swl[S], swr[S];
  int rank[S];
  uint64_t SWL[S], SWR[S];
  int msw = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const bool isl = (Lb[s] >> lane) & 1ull, isr = (Rb[s] >> lane) & 1ull;
    const int a = cl[s] + (int)mbcnt(Lb[s]);
    const int bgt = totR - cr[s] - (int)mbcnt(Rb[s]) - (isr ? 1 : 0);
    swl[s] = isl && bgt > a;
    swr[s] = isr && a > bgt;
    rank[s] = swl[s] ? a : bgt;
    SWL[s] = __ballot(swl[s]);
    SWR[s] = __ballot(swr[s]);
    msw += __popcll(SWL[s]);
  }
  // the pivot swap is a real move even when the partition swaps nothing
  if (m != first && lane == 0) {
    A[first] = vm;
    A[m] = vf;
  }
  if (msw > 0) {
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (swl[s]) sc.xa[rank[s]] = v[s];
      if (swr[s]) sc.xb[rank[s]] = v[s];
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (swl[s] || swr[s]) A[first + 64 * s + lane] = swl[s] ? sc.xb[rank[s]] : sc.xa[rank[s]];
    }
  }
  wave_lds_sync();
  // cut = min(first non-swapping left stop, lowest swapping right stop | last)
  int c1 = 1 << 30, c2 = last;
  bool f1 = false, f2 = msw == 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint64_t nsl = Lb[s] & ~SWL[s];
    if (!f1 && nsl) {
      c1 = first + 64 * s + __ffsll((unsigned long long)nsl) - 1;
      f1 = true;
    }
    if (!f2 && SWR[s]) {
      c2 = first + 64 * s + __ffsll((unsigned long long)SWR[s]) - 1;
      f2 = true;
    }
  }
  return c1 < c2 ? c1 : c2;
}

// Dispatch on the number of slots the range needs (uniform).
template <int S>
__device__ __forceinline__ int lds_partition_any(const TopkLdsV2& sc, int first, int last, int lane) {
  const int len = last - first;
  if (len <= 64) return lds_partition<1>(sc, first, last, lane);
  if (S >= 2 && len <= 128) return lds_partition<(S >= 2 ? 2 : 1)>(sc, first, last, lane);
  if (S >= 4 && len <= 256) return lds_partition<(S >= 4 ? 4 : 1)>(sc, first, last, lane);
  return lds_partition<S>(sc, first, last, lane);
}

// Stable sort (key descending) of positions [0, m) within the segments recorded in
// sc.seg (lo | hi << 16 per position): rank inside the segment by a scan of <= maxlen.
template <int S>
__device__ void lds_segment_sort(const TopkLdsV2& sc, int m, int maxlen, int lane) {
  uint64_t v[S];
  int dst[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = 64 * s + lane;
    dst[s] = -1;
    v[s] = 0ull;
    if (pos < m) {
      v[s] = sc.A[pos];
      const uint32_t sg = sc.seg[pos];
      const int lo = (int)(sg & 0xFFFFu), hi = (int)(sg >> 16);
      if (hi > lo + 1) {
        const uint32_t k = key_of(v[s]);
        int r = 0;
        for (int j = 0; j < maxlen; ++j) {
          const int q = lo + j;
          if (q >= hi) break;
          const uint32_t kj = key_of(sc.A[q]);
          r += (kj > k || (kj == k && q < pos)) ? 1 : 0;
        }
        dst[s] = lo + r;
      }
    }
  }
  wave_lds_sync();
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (dst[s] >= 0) sc.A[dst[s]] = v[s];
  wave_lds_sync();
}

// std::nth_element(begin, begin+k-1, end) -- or, when k*64 <= n, the whole
// std::partial_sort(begin, begin+k, end).  Returns true when [0, k) is final.
template <int S>
__device__ bool lds_select(const TopkLdsV2& sc, int n, int k, int lane) {
  uint64_t* A = sc.A;
  if (k <= 0) return true;
  if (k * 64 <= n) {  // std::partial_sort(begin, begin+k, end)
    if (lane == 0) {
      s_heap_select(A, 0, k, n);
      s_sort_heap(A, 0, k);
    }
    wave_lds_sync();
    return true;
  }
  // __introselect
  int first = 0, last = n;
  const int nth = k - 1;
  int depth = 2 * ilog2(n);
  while (last - first > 3) {
    if (depth == 0) {
      if (lane == 0) {
        s_heap_select(A, first, nth + 1, last);
        const uint64_t t = A[first];
        A[first] = A[nth];
        A[nth] = t;
      }
      wave_lds_sync();
      return false;
    }
    --depth;
    const int cut = lds_partition_any<S>(sc, first, last, lane);
    if (cut <= nth) first = cut;
    else last = cut;
  }
  if (last - first > 1) {  // __insertion_sort(first, last): <= 3 elements, stable
    if (lane == 0) {
      for (int i = first + 1; i < last; ++i) {
        const uint64_t x = A[i];
        int j = i;
        while (j > first && key_of(x) > key_of(A[j - 1])) {
          A[j] = A[j - 1];
          --j;
        }
        A[j] = x;
      }
    }
    wave_lds_sync();
  }
  return false;
}

// std::sort(begin, begin+m): __introsort_loop + __final_insertion_sort
template <int S>
__device__ void lds_sort_prefix(const TopkLdsV2& sc, int m, int lane) {
  uint64_t* A = sc.A;
  if (m <= 1) return;
  // every position starts in its own (trivial) segment
  for (int pos = lane; pos < m; pos += 64) sc.seg[pos] = (uint32_t)pos | ((uint32_t)(pos + 1) << 16);
  int sp = 0;
  sc.stk[sp++] = 0 | (m << 10) | ((2 * ilog2(m)) << 20);
  while (sp > 0) {
    --sp;
    const int e = sc.stk[sp];
    const int f = e & 1023;
    int l = (e >> 10) & 1023;
    int d = e >> 20;
    bool heaped = false;
    while (l - f > 16) {
      if (d == 0) {  // std::__partial_sort(f, l, l): heapsort leaves [f, l) sorted
        if (lane == 0) {
          s_heap_select(A, f, l, l);
          s_sort_heap(A, f, l);
        }
        wave_lds_sync();
        heaped = true;
        break;
      }
      --d;
      const int cut = lds_partition_any<S>(sc, f, l, lane);
      if (lane == 0) sc.stk[sp] = cut | (l << 10) | (d << 20);
      ++sp;
      wave_lds_sync();
      l = cut;
    }
    if (!heaped && l - f > 1)
      for (int pos = f + lane; pos < l; pos += 64) sc.seg[pos] = (uint32_t)f | ((uint32_t)l << 16);
  }
  wave_lds_sync();
  lds_segment_sort<S>(sc, m, 16, lane);
}

// Full top-k of the row in sc.A[0, n) (TopKImpl.h:45-86).  On return positions
// [0, k) hold torch's order.
template <int S>
__device__ void lds_topk(const TopkLdsV2& sc, int n, int k, int lane) {
  if (!lds_select<S>(sc, n, k, lane)) lds_sort_prefix<S>(sc, k - 1, lane);
}

}  // namespace mxa
