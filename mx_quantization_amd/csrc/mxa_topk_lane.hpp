// Lane-per-row tail of the exact-order top-k.
//
// The wave-wide restatement (mxa_topk_reg.hpp) spends ~100 wave instructions on
// every partition step whatever the range length, and most steps of torch's CPU
// topk run on short ranges (DeiT-base, k = 20: ~5 of ~7 introselect steps are on
// <= 64 positions, and std::sort of the k-1 prefix is all short ranges).  Those
// steps are cheaper as plain serial code, one ROW per LANE: the wave-wide pass
// narrows each row until its pending work lies inside positions [0, W), parks that
// window in LDS, and afterwards every lane runs libstdc++ 11 itself on its own
// window -- the same element movements as torch's build, one
// instruction stream amortised over up to 64 rows.
//
// Followed literally (stl_algo.h / stl_heap.h of GCC 11, the code behind
// aten/src/ATen/native/TopKImpl.h:45-86):
//   __introselect, __unguarded_partition_pivot, __move_median_to_first,
//   __unguarded_partition, __insertion_sort (== __final_insertion_sort's two
//   halves: the unguarded half stops at the same element), __introsort_loop,
//   __partial_sort (heap fallback), __heap_select, __sort_heap.
// Elements are pack_ki(order key, index); comp(x, y) = key(x) > key(y).
#pragma once
#include "mxa_topk.hpp"

namespace mxa {

typedef __attribute__((address_space(3))) uint64_t lu64;
typedef __attribute__((address_space(3))) int li32;

__device__ __forceinline__ bool lgt(uint64_t x, uint64_t y) { return (uint32_t)(x >> 32) > (uint32_t)(y >> 32); }

// ---- stl_heap.h on one lane's row ------------------------------------------
__device__ __forceinline__ void ln_push_heap(lu64* f, int hole, int top, uint64_t v) {
  int parent = (hole - 1) / 2;
  while (hole > top && lgt(f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
__device__ __forceinline__ void ln_adjust_heap(lu64* f, int hole, int len, uint64_t v) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (lgt(f[second], f[second - 1])) second--;
    f[hole] = f[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    f[hole] = f[second - 1];
    hole = second - 1;
  }
  ln_push_heap(f, hole, top, v);
}
__device__ __forceinline__ void ln_pop_heap(lu64* first, int len, lu64* result) {
  const uint64_t v = *result;
  *result = *first;
  ln_adjust_heap(first, 0, len, v);
}
// __heap_select(first, middle, last) on a[first..last)
__device__ inline void ln_heap_select(lu64* a, int first, int middle, int last) {
  lu64* f = a + first;
  const int len = middle - first;
  if (len >= 2) {  // __make_heap
    int parent = (len - 2) / 2;
    while (true) {
      ln_adjust_heap(f, parent, len, f[parent]);
      if (parent == 0) break;
      parent--;
    }
  }
  for (int i = middle; i < last; ++i)
    if (lgt(a[i], f[0])) ln_pop_heap(f, len, a + i);
}
__device__ inline void ln_sort_heap(lu64* a, int first, int last) {
  while (last - first > 1) {
    --last;
    ln_pop_heap(a + first, last - first, a + last);
  }
}

// ---- stl_algo.h --------------------------------------------------------------
// __insertion_sort(first, last) (guarded form; the unguarded inner loop of
// __final_insertion_sort stops at the same element)
__device__ __forceinline__ void ln_insertion_sort(lu64* a, int f, int l) {
  for (int i = f + 1; i < l; ++i) {
    const uint64_t v = a[i];
    int j = i;
    uint64_t prev = a[j - 1];
    while (lgt(v, prev)) {
      a[j] = prev;
      --j;
      if (j == f) break;
      prev = a[j - 1];
    }
    a[j] = v;
  }
}

// __unguarded_partition_pivot(first, last): median of (first+1, mid, last-1) to
// first, then Hoare partition of [first+1, last) around it
__device__ __forceinline__ int ln_partition_pivot(lu64* a, int f, int l) {
  const int mid = f + (l - f) / 2;
  const uint64_t xa = a[f + 1], xb = a[mid], xc = a[l - 1];
  int m;
  uint64_t xm;
  if (lgt(xa, xb)) {
    if (lgt(xb, xc)) m = mid, xm = xb;
    else if (lgt(xa, xc)) m = l - 1, xm = xc;
    else m = f + 1, xm = xa;
  } else if (lgt(xa, xc)) m = f + 1, xm = xa;
  else if (lgt(xb, xc)) m = l - 1, xm = xc;
  else m = mid, xm = xb;
  const uint64_t xf = a[f];
  a[m] = xf;  // iter_swap(first, median)
  a[f] = xm;
  const uint32_t p = (uint32_t)(xm >> 32);
  int i = f + 1, j = l;
  while (true) {
    uint64_t xi = a[i];
    while ((uint32_t)(xi >> 32) > p) xi = a[++i];
    uint64_t xj = a[--j];
    while (p > (uint32_t)(xj >> 32)) xj = a[--j];
    if (!(i < j)) return i;
    a[i] = xj;
    a[j] = xi;
    ++i;
  }
}

// state of a row handed from the wave-wide pass to its lane
struct LaneTask {
  int first, last, depth;  // pending __introselect range (first == last: done)
  int nth, k;              // k - 1 == nth; the sorted prefix is [0, k - 1)
};

// __introselect's remainder on [first, last), then std::sort of [0, m), m = k - 1
// (TopKImpl.h:45-86): __introsort_loop down to 16-element segments with the depth
// limit, each segment finished by the (stable) insertion sort.  stk: this lane's
// stack of pending segments (>= 2 * lg(m) entries).
__device__ inline void lane_topk_tail(lu64* a, LaneTask t, li32* stk) {
  int first = t.first, last = t.last, depth = t.depth;
  const int nth = t.nth;
  bool sel_done = first == last;
  while (!sel_done && last - first > 3) {
    if (depth == 0) {  // __heap_select(first, nth + 1, last); iter_swap(first, nth)
      ln_heap_select(a, first, nth + 1, last);
      const uint64_t x = a[first];
      a[first] = a[nth];
      a[nth] = x;
      sel_done = true;
      break;
    }
    --depth;
    const int cut = ln_partition_pivot(a, first, last);
    if (cut <= nth) first = cut;
    else last = cut;
  }
  if (!sel_done) ln_insertion_sort(a, first, last);

  const int m = t.k - 1;  // std::sort(begin, begin + k - 1)
  if (m < 2) return;
  int sp = 0;
  int f = 0, l = m, d = 2 * ilog2(m);
  while (true) {
    while (l - f > 16) {
      if (d == 0) {  // std::__partial_sort(f, l, l): heapsort of the segment
        ln_heap_select(a, f, l, l);
        ln_sort_heap(a, f, l);
        f = l;
        break;
      }
      --d;
      const int cut = ln_partition_pivot(a, f, l);
      stk[sp++] = cut | (l << 10) | (d << 20);  // __introsort_loop(cut, last, depth)
      l = cut;
    }
    if (l - f > 1) ln_insertion_sort(a, f, l);
    if (sp == 0) break;
    const int e = stk[--sp];
    f = e & 1023;
    l = (e >> 10) & 1023;
    d = e >> 20;
  }
}

}  // namespace mxa
