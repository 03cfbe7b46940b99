// The exact-order top-k's tail, ONE LANE PER ROW, for rows whose remaining work fits a
// prefix of TW <= 64 positions (k - 1 small: DeiT's k = 20 / 30, PixArt's 20).
//
// The selection kernel (mxa_select.hpp, packed elements) runs the wide partition steps of
// torch's CPU topk (TopKImpl.h:45-86: nth_element(k-1) then sort(k-1), libstdc++ 11) on
// sixteen lanes per row, four rows per wave in lockstep; once a row's introselect range
// [f, l) lies inside [0, TW) -- everything left of it (the sort of [0, k-1), the last
// partitions of the selection) happens in that prefix -- it hands the row over: the TW
// packed elements and the state (f, l, depth, phase) go to a staging record (TailRec).
// Here every lane takes one row and finishes it serially, in lockstep with the other 63
// rows of its wave only at the step level: the same Hoare partition in rank form as the
// 16-lane engine (median of three moved to f; left stops key <= p, right stops key >= p;
// cut = f + 1 + #{z in (f, l): T(z) <= totR}; the left stops below the cut trade places,
// in order, with the highest right stops), the depth-limit heap fallbacks of stl_heap.h,
// the <= 3-element insertion sort, std::sort's introsort loop (segments > 16 split, a
// depth limit heapsorts) and its final insertion sort as a stable rank; then the row's k
// indices and prune-mask words go out.  Why: the small partition steps cost the 16-lane
// engine a whole lockstep trip each (median, scans, cut search, exchange) for ~30
// positions of four rows; one lane per row pays a step's fixed work once per 64 rows.
//
// The row's prefix lives in LDS lane-interleaved, element z of lane i at [z][i]: every
// lane addresses its own row with a per-lane position and no two lanes ever share a bank.
#pragma once
#include "mxa_topk_grp.hpp"

namespace mxa {

typedef __attribute__((address_space(3))) uint32_t tl32;

// staging record of a handed-over row: state word, then the TW packed elements
// state: f | l << 8 | depth << 16 | phase << 24 | kTailPending
constexpr uint32_t kTailPending = 0x80000000u;  // (tail_rec_words: mxa_rows2.hpp)

// a lane's row in LDS: element z at base[64 z]
struct TRef {
  tl32* p;
  __device__ operator uint32_t() const { return *p; }
  __device__ TRef& operator=(uint32_t v) {
    *p = v;
    return *this;
  }
  __device__ TRef& operator=(const TRef& o) {
    *p = (uint32_t)o;
    return *this;
  }
};
struct TPtr {
  tl32* p;
  __device__ TRef operator[](int i) const { return TRef{p + 64 * i}; }
  __device__ TPtr operator+(int i) const { return TPtr{p + 64 * i}; }
  __device__ TRef operator*() const { return TRef{p}; }
};
// stl_heap.h / stl_algo.h on a lane's strided row (mxa_order.hpp's ln_* take pointer-like
// types; these are the same algorithms for TPtr)
__device__ __forceinline__ void tn_push_heap(TPtr f, int hole, int top, uint32_t v) {
  int parent = (hole - 1) / 2;
  while (hole > top && lgt((uint32_t)f[parent], v)) {
    f[hole] = (uint32_t)f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}
__device__ __forceinline__ void tn_adjust_heap(TPtr f, int hole, int len, uint32_t v) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (lgt((uint32_t)f[second], (uint32_t)f[second - 1])) second--;
    f[hole] = (uint32_t)f[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    f[hole] = (uint32_t)f[second - 1];
    hole = second - 1;
  }
  tn_push_heap(f, hole, top, v);
}
__device__ __forceinline__ void tn_pop_heap(TPtr first, int len, TPtr result) {
  const uint32_t v = *result;
  *result = (uint32_t)*first;
  tn_adjust_heap(first, 0, len, v);
}
__device__ inline void tn_heap_select(TPtr a, int first, int middle, int last) {
  TPtr f = a + first;
  const int len = middle - first;
  if (len >= 2) {
    int parent = (len - 2) / 2;
    while (true) {
      tn_adjust_heap(f, parent, len, (uint32_t)f[parent]);
      if (parent == 0) break;
      parent--;
    }
  }
  for (int i = middle; i < last; ++i)
    if (lgt((uint32_t)a[i], (uint32_t)f[0])) tn_pop_heap(f, len, a + i);
}
__device__ inline void tn_sort_heap(TPtr a, int first, int last) {
  while (last - first > 1) {
    --last;
    tn_pop_heap(a + first, last - first, a + last);
  }
}
__device__ __forceinline__ void tn_insertion_sort(TPtr a, int f, int l) {
  for (int i = f + 1; i < l; ++i) {
    const uint32_t v = a[i];
    int j = i;
    uint32_t prev = a[j - 1];
    while (lgt(v, prev)) {
      a[j] = prev;
      --j;
      if (j == f) break;
      prev = a[j - 1];
    }
    a[j] = v;
  }
}

template <int W>
using TMask = std::conditional_t<(W > 32), uint64_t, uint32_t>;
template <typename M>
__device__ __forceinline__ M t_low(int n) {
  constexpr int B = sizeof(M) * 8;
  return n >= B ? ~(M)0 : (((M)1 << n) - (M)1);
}
template <typename M>
__device__ __forceinline__ int t_popc(M x) {
  if constexpr (sizeof(M) == 8) return __popcll(x);
  else return __popc(x);
}

// One partition step of [f, l) (act: l - f >= 4) on every lane's own row, window of W
// positions from a base b (b <= f, l <= b + W): returns the cut.  Masks shift in the
// highest position first so bit e <-> position b + e.
template <int W>
__device__ __forceinline__ int t_partition(TPtr A, int f, int l, int b, bool act) {
  using M = TMask<W>;
  const int fa = act ? f : 0, la = act ? l : 4;
  const int mid = fa + ((la - fa) >> 1);
  // the median candidates and the window in one LDS round trip; the median's iter_swap
  // is applied to the stop masks (position f is never a stop; position m holds old f)
  const uint32_t xf = A[fa], xa = A[fa + 1], xb = A[mid], xc = A[la - 1];
  uint32_t K[W];
#pragma unroll
  for (int e = 0; e < W; ++e) K[e] = A[b + e];
  const bool ab = lgt(xa, xb), bc = lgt(xb, xc), ac = lgt(xa, xc);
  const bool pick_b = ab ? bc : (!ac && !bc);
  const bool pick_c = ab ? (!bc && ac) : (!ac && bc);
  int m = pick_c ? la - 1 : fa + 1;
  uint32_t xm = pick_c ? xc : xa;
  m = pick_b ? mid : m;
  xm = pick_b ? xb : xm;
  if (act) {  // iter_swap(f, median)
    A[fa] = xm;
    A[m] = xf;
  }
  const uint32_t pl = xm | 0xFFu, pr = xm & ~0xFFu;
  M Lm, Rm;
  if constexpr (W > 32) {
    uint32_t Lh = 0, Rh = 0, Ll = 0, Rl = 0;
#pragma unroll
    for (int e = W - 1; e >= 32; e -= 2) g_stops2(Lh, Rh, K[e], K[e - 1], pl, pr);
#pragma unroll
    for (int e = 31; e >= 0; e -= 2) g_stops2(Ll, Rl, K[e], K[e - 1], pl, pr);
    Lm = ((uint64_t)Lh << 32) | Ll;
    Rm = ((uint64_t)Rh << 32) | Rl;
  } else {
    uint32_t Lw = 0, Rw = 0;
#pragma unroll
    for (int e = W - 1; e >= 0; e -= 2) g_stops2(Lw, Rw, K[e], K[e - 1], pl, pr);
    Lm = Lw;
    Rm = Rw;
  }
  {  // position m holds old f now
    const int em = m - b;
    const M bm = (uint32_t)em < (uint32_t)W ? (M)1 << em : (M)0;
    Lm = (Lm & ~bm) | (xf <= pl ? bm : (M)0);
    Rm = (Rm & ~bm) | (xf >= pr ? bm : (M)0);
  }
  const M rng = act ? (t_low<M>(l - b) & ~t_low<M>(f + 1 - b)) : (M)0;
  Lm &= rng;
  Rm &= rng;
  const int totR = t_popc(Rm);
  // js = the positions z of the window (a prefix: T non-decreasing) with T(z) <= totR
  int js = 0;
#pragma unroll
  for (int st = W >= 64 ? 64 : W >= 32 ? 32 : W >= 16 ? 16 : 8; st >= 1; st >>= 1) {
    const int c = js + st;
    const M lw = t_low<M>(c);
    const bool ok = c <= W && t_popc(Lm & lw) + t_popc(Rm & lw) <= totR;
    js = ok ? c : js;
  }
  M SL = Lm & t_low<M>(js);  // the swapping left stops
  const int nsw = t_popc(SL);
  M SR = Rm;  // the nsw highest right stops, taken from the top
  // the swaps four at a time: their positions first, then all reads, then all writes (the
  // swapping positions are distinct, so one LDS round trip per four swaps)
  for (int t = 0; __builtin_amdgcn_ballot_w64(t < nsw) != 0; t += 4) {
    int x[4], y[4];
    bool on[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      on[i] = t + i < nsw;
      x[i] = sizeof(M) == 8 ? __ffsll((long long)SL) - 1 : __ffs((int)SL) - 1;
      y[i] = sizeof(M) == 8 ? 63 - __clzll((long long)SR) : 31 - __clz((int)SR);
      x[i] = on[i] ? x[i] : 0;
      y[i] = on[i] ? y[i] : 0;
      SL = on[i] ? (SL & (SL - (M)1)) : SL;
      SR = on[i] ? (SR ^ ((M)1 << y[i])) : SR;
    }
    uint32_t ex[4], ey[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ex[i] = on[i] ? (uint32_t)A[b + x[i]] : 0u;
      ey[i] = on[i] ? (uint32_t)A[b + y[i]] : 0u;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (on[i]) {
        A[b + x[i]] = ey[i];
        A[b + y[i]] = ex[i];
      }
  }
  return b + js;
}

// one partition of [f, l) per acting lane in the narrowest window that holds every
// acting lane's range (base min(f & ~1, TW - W))
template <int TW>
__device__ __forceinline__ int t_partition_any(TPtr A, int f, int l, bool act) {
  const int need = act ? l - (f & ~1) : 0;
  if (__builtin_amdgcn_ballot_w64(need > 8) == 0) return t_partition<8>(A, f, l, min(f & ~1, TW - 8), act);
  if (__builtin_amdgcn_ballot_w64(need > 16) == 0) return t_partition<16>(A, f, l, min(f & ~1, TW - 16), act);
  if (TW <= 32 || __builtin_amdgcn_ballot_w64(need > 32) == 0)
    return t_partition<(TW < 32 ? TW : 32)>(A, f, l, min(f & ~1, TW - (TW < 32 ? TW : 32)), act);
  return t_partition<TW>(A, f, l, 0, act);
}

// stable rank of [0, m) (std::sort's final insertion sort) on the lane's row: position i
// goes to #{j : key_j > key_i} + #{j < i : key_j == key_i}; MW >= m positions held
template <int MW>
__device__ __forceinline__ void t_rank(TPtr A, int m) {
  uint32_t x[MW], r[MW];
#pragma unroll
  for (int i = 0; i < MW; ++i) {
    x[i] = i < m ? (uint32_t)A[i] : 0u;  // 0: a key below every real key
    r[i] = (uint32_t)i;
  }
#pragma unroll
  for (int i = 0; i < MW; ++i) {
    const uint32_t ki = x[i] | 0xFFu;
#pragma unroll
    for (int j = i + 1; j < MW; ++j) g_pair_rank(r[i], r[j], x[j], ki);
  }
#pragma unroll
  for (int i = 0; i < MW; ++i)
    if (i < m) A[r[i]] = x[i];
}

struct TailArgs {
  const uint32_t* rec;  // staging records [rows][tail_rec_words(TW)]
  int64_t rows;
  int k;
  int ntw;              // prune-mask words per row (ceil(T / 32))
  int64_t* idx_out;     // nullable: then idx16
  uint16_t* idx16;
  uint32_t* mask_out;   // nullable
  // the standalone top-k (mxa_topk_ws): the values at the kept indices (nullable out_vals)
  const void* vals;     // dtype dt, row stride ld
  int64_t ld;
  int dt;
  void* out_vals;
};

// The introsort stack of a lane, in registers: 16-bit entries (cut | depth << 8), the top in
// the low bits of s0.  A pushed segment [cut, l) always ends where the entry below it starts
// (or at m for the bottom entry), so its end is not stored (the pop reads it from the next
// entry).  At most 2 lg(32) = 10 entries are live (one push per partition step, each costing a
// level of the depth limit), 12 fit.
struct TStack {
  uint64_t s0, s1, s2;
  __device__ void push(uint32_t e) {
    s2 = (s2 << 16) | (s1 >> 48);
    s1 = (s1 << 16) | (s0 >> 48);
    s0 = (s0 << 16) | e;
  }
  __device__ uint32_t pop() {
    const uint32_t e = (uint32_t)s0 & 0xFFFFu;
    s0 = (s0 >> 16) | (s1 << 48);
    s1 = (s1 >> 16) | (s2 << 48);
    s2 >>= 16;
    return e;
  }
  __device__ uint32_t top() const { return (uint32_t)s0 & 0xFFFFu; }
};

// one lane per row; a workgroup of kTailWaves waves, each wave's 64 rows' prefixes in LDS
// (TW words per lane: the introsort stack lives in registers, the prune-mask words are set
// in the prefix's positions [k, k + ntw) once the kept elements are in registers)
constexpr int kTailWaves = 1;
constexpr int kTailMaxK = 33;  // k handed to the tail (k - 1 <= 32: the final rank's width)
// the record's positions the tail reads: [0, l) of an introselect hand-over (nothing past the
// range is read again: the window loads beyond l are masked out of the stop masks), [0, k - 1)
// of a sort hand-over
__device__ __forceinline__ int tail_rec_len(uint32_t state, int k) {
  return ((state >> 24) & 3u) ? k - 1 : (int)((state >> 8) & 0xFFu);
}
template <int TW>
__global__ __launch_bounds__(64 * kTailWaves) void topk_tail_kernel(TailArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (64 * kTailWaves) + threadIdx.x;
  const TPtr A{(tl32*)(lu32*)(smem) + (size_t)wave * 64 * TW + lane};
  const int k = a.k, nth = k - 1, m = k - 1;
  uint32_t st = 0u;
  if (row < a.rows) {
    const uint32_t* src = a.rec + row * tail_rec_words(TW);
    st = src[0];
    if (st & kTailPending) {  // all loads first, then the LDS stores (one wait)
      const int len = tail_rec_len(st, k);
      uint4 v[TW / 4];
#pragma unroll
      for (int e = 0; e < TW; e += 4)
        v[e / 4] = e < len ? *reinterpret_cast<const uint4*>(src + 4 + e) : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < TW; e += 4) {
        A[e] = v[e / 4].x;
        A[e + 1] = v[e / 4].y;
        A[e + 2] = v[e / 4].z;
        A[e + 3] = v[e / 4].w;
      }
    }
  }
  const bool pend = (st & kTailPending) != 0;
#ifdef MXA_TAIL_SKIP  // tools-only phase timing (build_native defines): 4 = the record loads alone
  if ((MXA_TAIL_SKIP) & 4) {
    if (pend && row < a.rows) {
      if (a.idx_out) a.idx_out[row * k] = (int64_t)((uint32_t)A[0] & 0xFFu);
      else a.idx16[row * k] = (uint16_t)((uint32_t)A[0] & 0xFFu);
    }
    return;
  }
#endif
  int f = (int)(st & 0xFFu), l = (int)((st >> 8) & 0xFFu), d = (int)((st >> 16) & 0xFFu);
  int ph = pend ? (int)((st >> 24) & 0x3u) : 2;  // 0 introselect, 1 introsort loop, 2 done
  int sp = 0;
  TStack stk{0, 0, 0};
  if (ph == 1) {
    f = 0;
    l = m;
    d = m > 1 ? 2 * ilog2(m) : 0;
  }
  while (true) {
    if (ph == 0 && (l - f <= 3 || d == 0)) {  // the selection ends
#ifdef MXA_TAIL_SKIP  // 2 = no sort of [0, k-1) (and no rank)
      if ((MXA_TAIL_SKIP) & 2) {
        ph = 2;
        continue;
      }
#endif
      if (l - f > 3) {  // depth limit: __heap_select(f, nth + 1, l); iter_swap(f, nth)
        tn_heap_select(A, f, nth + 1, l);
        const uint32_t tt = A[f];
        A[f] = (uint32_t)A[nth];
        A[nth] = tt;
      } else if (l - f > 1) {
        tn_insertion_sort(A, f, l);
      }
      ph = 1;
      f = 0;
      l = m;
      d = m > 1 ? 2 * ilog2(m) : 0;
    }
    if (ph == 1) {  // settle: finished segments (<= 16, or heapsorted at the depth limit)
      while (l - f <= 16 || d == 0) {
        if (l - f > 16) {
          tn_heap_select(A, f, l, l);
          tn_sort_heap(A, f, l);
        }
        if (sp == 0) {
          ph = 3;  // the final stable rank is left
          break;
        }
        --sp;
        const uint32_t e = stk.pop();
        f = (int)(e & 0xFFu);
        d = (int)(e >> 8);
        l = sp > 0 ? (int)(stk.top() & 0xFFu) : m;  // the segment ends where the next one starts
      }
    }
    const bool act = ph < 2;
    if (__builtin_amdgcn_ballot_w64(act) == 0) break;
    const int cut = t_partition_any<TW>(A, f, l, act);
    if (act) {
      --d;
      if (ph == 0) {
        if (cut <= nth) f = cut;
        else l = cut;
      } else {
        stk.push((uint32_t)cut | ((uint32_t)d << 8));  // __introsort_loop(cut, l)
        ++sp;
        l = cut;
      }
    }
  }
  // std::sort's final insertion sort = a stable rank of [0, m) (segments mutually ordered)
#ifdef MXA_TAIL_SKIP  // 1 = no final rank
  if ((MXA_TAIL_SKIP) & 1) ph = 2;
#endif
  if (__builtin_amdgcn_ballot_w64(ph == 3 && m >= 2) != 0) {  // (m <= 32: sel_tail_width)
    if (m <= 16) {
      if (ph == 3) t_rank<16>(A, m);
    } else if (m <= 20) {  // DeiT's k = 20
      if (ph == 3) t_rank<20>(A, m);
    } else if (m <= 24) {
      if (ph == 3) t_rank<24>(A, m);
    } else {
      if (ph == 3) t_rank<32>(A, m);
    }
  }
  if (!pend) return;
  // the kept elements (k <= kTailMaxK: sel_tail_width / topk_ws_tw) into registers, then the
  // prune-mask words (zeros.scatter_(-1, idx, 1) as bits) set by LDS ORs in the prefix's free
  // positions [k, k + ntw) (k + ntw <= TW: sel_tail_width); the standalone top-k's values at the
  // kept indices come back from the packed elements themselves (q_value: no gather from the
  // input rows)
  uint32_t x[kTailMaxK];
#pragma unroll
  for (int p = 0; p < kTailMaxK; ++p) x[p] = p < k ? (uint32_t)A[p] : 0u;
  const int ntw = a.mask_out ? a.ntw : 0;
  for (int w = 0; w < ntw; ++w) A[k + w] = 0u;
#pragma unroll
  for (int p = 0; p < kTailMaxK; ++p) {
    if (p < k) {
      const uint32_t ix = x[p] & 0xFFu;
      if (a.idx_out) a.idx_out[row * k + p] = (int64_t)ix;
      else a.idx16[row * k + p] = (uint16_t)ix;
      if (ntw) __hip_atomic_fetch_or(A[k + (int)(ix >> 5)].p, 1u << (ix & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
  }
  for (int w = 0; w < ntw; ++w) a.mask_out[row * ntw + w] = (uint32_t)A[k + w];
  if (a.out_vals)  // (the packed pass sent no row with a NaN or -0 value: q_val_bad)
#pragma unroll
    for (int p = 0; p < kTailMaxK; ++p)
      if (p < k) store_dt(a.out_vals, row * k + p, q_value(x[p]), a.dt);
}

__host__ __device__ constexpr size_t tail_lds(int TW) { return (size_t)kTailWaves * 64 * TW * 4; }

}  // namespace mxa
