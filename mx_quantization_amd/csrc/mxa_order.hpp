// Order keys and the serial libstdc++ 11 helpers of the exact-order top-k.
//
// torch.topk on CPU (aten/src/ATen/native/TopKImpl.h:45-86) sorts pair<double,int64>
// with cmp(x, y) = (isnan(x) && !isnan(y)) || x > y.  Here an element is
// pack_ki(order key, index) and cmp is an unsigned compare of the keys.
// The serial helpers below follow stl_heap.h / stl_algo.h of GCC 11 literally (the
// code behind torch's build); the group top-k (mxa_topk_grp.hpp) runs
// them on one lane of a row for the rare paths: depth-limit heap fallbacks,
// partial_sort (k*64 <= n) and __insertion_sort of <= 3 elements.
#pragma once
#include "mxa_common.hpp"

namespace mxa {

// Order-preserving key for cmp: NaN largest (all NaNs tie), -0 == +0.  Every key
// of a real element is >= 0x007FFFFF (-inf), so 0 sorts after all of them.
__device__ __forceinline__ uint32_t order_key(float f) {
  uint32_t b = __float_as_uint(f);
  const uint32_t a = b & 0x7FFFFFFFu;
  if (a > 0x7F800000u) return 0xFFFFFFFFu;
  if (a == 0u) b = 0u;
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ uint64_t pack_ki(uint32_t key, uint32_t idx) { return ((uint64_t)key << 32) | idx; }
// the packed element of a row of <= 256 keys: (order key & 0xFFFFFF00) | index
__device__ __forceinline__ uint32_t qelem(uint32_t key, uint32_t idx) { return (key & 0xFFFFFF00u) | idx; }
// nonzero when a score's fp32 bits need the key's low byte (a nonzero low mantissa byte;
// NaN keys are all ones and pack)
__device__ __forceinline__ uint32_t q_bad_bits(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u & 0x7FFFFFFFu) > 0x7F800000u ? 0u : (u & 0xFFu);
}
// nonzero for the values a packed element does not give back bit for bit (q_value): NaN
// (payload) and -0 (its order key is +0's)
__device__ __forceinline__ uint32_t q_val_bad(float v) {
  const uint32_t u = __float_as_uint(v);
  return (uint32_t)((u & 0x7FFFFFFFu) > 0x7F800000u || u == 0x80000000u);
}
// the value of a packed element whose value packs (q_bad_bits == 0) and is neither NaN nor
// -0: the order key's low byte is 0x00 (positive) or 0xFF (negative), then order_key undone
__device__ __forceinline__ float q_value(uint32_t e) {
  const uint32_t key = (e & 0x80000000u) ? (e & 0xFFFFFF00u) : (e | 0xFFu);
  return __uint_as_float((key & 0x80000000u) ? (key & 0x7FFFFFFFu) : ~key);
}

__device__ __forceinline__ int ilog2(int n) { return 31 - __clz(n); }

typedef __attribute__((address_space(3))) uint64_t lu64;
typedef __attribute__((address_space(3))) int li32;

// cmp on elements: (key << 32 | index), or the packed (key & ~0xFF) | index of
// mxa_topk_grp.hpp (key(x) > key(y) <=> x > (y | 0xFF))
__device__ __forceinline__ bool lgt(uint64_t x, uint64_t y) { return (uint32_t)(x >> 32) > (uint32_t)(y >> 32); }
__device__ __forceinline__ bool lgt(uint32_t x, uint32_t y) { return x > (y | 0xFFu); }

// ---- stl_heap.h on one lane's row (LP: an LDS element type) ---------------------
template <typename LP, typename V>
__device__ __forceinline__ void ln_push_heap(LP* f, int hole, int top, V v) {
  int parent = (hole - 1) / 2;
  while (hole > top && lgt((V)f[parent], v)) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
template <typename LP, typename V>
__device__ __forceinline__ void ln_adjust_heap(LP* f, int hole, int len, V v) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (lgt((V)f[second], (V)f[second - 1])) second--;
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
template <typename LP>
__device__ __forceinline__ void ln_pop_heap(LP* first, int len, LP* result) {
  const auto v = +*result;
  *result = *first;
  ln_adjust_heap(first, 0, len, v);
}
// __heap_select(first, middle, last) on a[first..last)
template <typename LP>
__device__ inline void ln_heap_select(LP* a, int first, int middle, int last) {
  LP* f = a + first;
  const int len = middle - first;
  if (len >= 2) {  // __make_heap
    int parent = (len - 2) / 2;
    while (true) {
      ln_adjust_heap(f, parent, len, +f[parent]);
      if (parent == 0) break;
      parent--;
    }
  }
  for (int i = middle; i < last; ++i)
    if (lgt(+a[i], +f[0])) ln_pop_heap(f, len, a + i);
}
template <typename LP>
__device__ inline void ln_sort_heap(LP* a, int first, int last) {
  while (last - first > 1) {
    --last;
    ln_pop_heap(a + first, last - first, a + last);
  }
}

// ---- stl_algo.h --------------------------------------------------------------
// __insertion_sort(first, last) (guarded form; the unguarded inner loop of
// __final_insertion_sort stops at the same element)
template <typename LP>
__device__ __forceinline__ void ln_insertion_sort(LP* a, int f, int l) {
  for (int i = f + 1; i < l; ++i) {
    const auto v = +a[i];
    int j = i;
    auto prev = +a[j - 1];
    while (lgt(v, prev)) {
      a[j] = prev;
      --j;
      if (j == f) break;
      prev = +a[j - 1];
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

}  // namespace mxa
