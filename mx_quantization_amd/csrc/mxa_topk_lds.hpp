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

// LDS bytes of one wave's scratch for rows of <= 64*S values (16-B multiple).
// big = false: no segment array (only the level-parallel sort of prefixes longer
// than 64 uses it)
// After xb: 64 per-lane trash entries, so that the exchange writes of lanes that
// do not swap need no exec-mask branch (mxa_topk_reg.hpp exchange()).
__host__ __device__ constexpr size_t topk_scratch_bytes(int S, bool big = true) {
  return (size_t)64 * S * 8 + (size_t)2 * 32 * S * 8 + (size_t)64 * 8 + (big ? (size_t)64 * S * 4 : 0) +
         (size_t)kTopkStack * 4 + 0;
}
__device__ __forceinline__ TopkLdsV2 carve_topk(unsigned char* base, int S, bool big = true) {
  TopkLdsV2 sc;
  sc.A = reinterpret_cast<uint64_t*>(base);
  sc.xa = sc.A + 64 * S;
  sc.xb = sc.xa + 32 * S;
  sc.seg = reinterpret_cast<uint32_t*>(sc.xb + 32 * S + 64);
  sc.stk = reinterpret_cast<int*>(sc.seg + (big ? 64 * S : 0));
  return sc;
}

__device__ __forceinline__ uint32_t key_of(uint64_t v) { return (uint32_t)(v >> 32); }

// __unguarded_partition_pivot(first, last) with cmp = greater; returns the cut.
template <int S>
__device__ __forceinline__ int lds_partition(const TopkLdsV2& sc, int first, int last, int lane) {
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
    Lb[s] = ballot64(in && rel > 0 && !(k > p));
    Rb[s] = ballot64(in && !(p > k));
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
    SWL[s] = ballot64(swl[s]);
    SWR[s] = ballot64(swr[s]);
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
// sc.seg (lo | hi << 16 per position, segments of <= 16): rank inside the segment
// by a fully unrolled scan (all 16 key reads in flight).
template <int S>
__device__ __forceinline__ void lds_segment_sort(const TopkLdsV2& sc, int m, int lane) {
  const uint32_t* keys = reinterpret_cast<const uint32_t*>(sc.A);  // key of position q at [2q + 1]
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
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int q = lo + j;
          const uint32_t kj = keys[2 * min(q, 64 * S - 1) + 1];
          r += (q < hi && (kj > k || (kj == k && q < pos))) ? 1 : 0;
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

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// A register window over positions [base, base + 64) of the row: lane i holds
// position base + i.  Once an introselect / introsort range fits 64 positions,
// every later range of that chain is a sub-range, so the steps run on the
// window without LDS loads or write-backs; flush() stores it back.
struct TopkWindow {
  int base;  // -1: no window
  uint64_t w;
  __device__ __forceinline__ void load(const TopkLdsV2& sc, int b, int n, int lane) {
    base = b;
    w = b + lane < n ? sc.A[b + lane] : 0ull;
  }
  __device__ __forceinline__ void flush(const TopkLdsV2& sc, int n, int lane) {
    if (base >= 0) {
      if (base + lane < n) sc.A[base + lane] = w;
      wave_lds_sync();
      base = -1;
    }
  }
  __device__ __forceinline__ bool covers(int f, int l) const { return base >= 0 && f >= base && l <= base + 64; }
};

// __unguarded_partition_pivot(first, last) on the window (same rule as lds_partition)
__device__ __forceinline__ int win_partition(TopkWindow& win, int first, int last, const TopkLdsV2& sc, int lane) {
  const int base = win.base;
  const int len = last - first, mid = first + len / 2;
  const uint32_t hi = (uint32_t)(win.w >> 32);
  const uint32_t ka = (uint32_t)__builtin_amdgcn_readlane((int)hi, first + 1 - base);
  const uint32_t kb = (uint32_t)__builtin_amdgcn_readlane((int)hi, mid - base);
  const uint32_t kc = (uint32_t)__builtin_amdgcn_readlane((int)hi, last - 1 - base);
  int m;  // __move_median_to_first(first, first+1, mid, last-1)
  if (ka > kb) {
    if (kb > kc) m = mid;
    else if (ka > kc) m = last - 1;
    else m = first + 1;
  } else if (ka > kc) m = first + 1;
  else if (kb > kc) m = last - 1;
  else m = mid;
  const uint32_t p = m == first + 1 ? ka : (m == mid ? kb : kc);
  const uint64_t vf = readlane64(win.w, first - base), vm = readlane64(win.w, m - base);
  const int pos = base + lane;
  uint64_t v = pos == first ? vm : (pos == m ? vf : win.w);  // iter_swap(first, m)
  const uint32_t k = key_of(v);
  const bool in = pos >= first && pos < last;
  const bool isl = in && pos > first && !(k > p);
  const bool isr = in && !(p > k);
  const uint64_t Lb = ballot64(isl), Rb = ballot64(isr);
  const int a = (int)mbcnt(Lb);
  const int bgt = (int)__popcll(Rb) - (int)mbcnt(Rb) - (isr ? 1 : 0);
  const bool swl = isl && bgt > a, swr = isr && a > bgt;
  const uint64_t SWL = ballot64(swl), SWR = ballot64(swr);
  if (SWL) {  // exchange the t-th swapping left stop with the t-th swapping right stop
    const int rank = swl ? a : bgt;
    if (swl) sc.xa[rank] = v;
    if (swr) sc.xb[rank] = v;
    wave_lds_sync();
    if (swl) v = sc.xb[rank];
    if (swr) v = sc.xa[rank];
    wave_lds_sync();
  }
  win.w = v;
  const uint64_t nsl = Lb & ~SWL;
  const int c1 = nsl ? base + __ffsll((unsigned long long)nsl) - 1 : (1 << 30);
  const int c2 = SWR ? base + __ffsll((unsigned long long)SWR) - 1 : last;
  return c1 < c2 ? c1 : c2;
}

// std::nth_element(begin, begin+k-1, end) -- or, when k*64 <= n, the whole
// std::partial_sort(begin, begin+k, end).  Returns true when [0, k) is final.
template <int S>
__device__ __forceinline__ bool lds_select(const TopkLdsV2& sc, int n, int k, int lane) {
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
  TopkWindow win{-1, 0ull};
  while (last - first > 3) {
    if (depth == 0) {
      win.flush(sc, n, lane);
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
    int cut;
    if (last - first <= 64) {
      if (!win.covers(first, last)) {
        win.flush(sc, n, lane);
        win.load(sc, first, n, lane);
      }
      cut = win_partition(win, first, last, sc, lane);
    } else {
      cut = lds_partition_any<S>(sc, first, last, lane);
    }
    if (cut <= nth) first = cut;
    else last = cut;
  }
  win.flush(sc, n, lane);
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
__device__ __forceinline__ void lds_sort_prefix(const TopkLdsV2& sc, int m, int lane) {
  uint64_t* A = sc.A;
  if (m <= 1) return;
  // every position starts in its own (trivial) segment
  for (int pos = lane; pos < m; pos += 64) sc.seg[pos] = (uint32_t)pos | ((uint32_t)(pos + 1) << 16);
  int sp = 0;
  sc.stk[sp++] = 0 | (m << 10) | ((2 * ilog2(m)) << 20);
  TopkWindow win{-1, 0ull};
  while (sp > 0) {
    --sp;
    const int e = sc.stk[sp];
    const int f = e & 1023;
    int l = (e >> 10) & 1023;
    int d = e >> 20;
    bool heaped = false;
    while (l - f > 16) {
      if (d == 0) {  // std::__partial_sort(f, l, l): heapsort leaves [f, l) sorted
        win.flush(sc, m, lane);
        if (lane == 0) {
          s_heap_select(A, f, l, l);
          s_sort_heap(A, f, l);
        }
        wave_lds_sync();
        heaped = true;
        break;
      }
      --d;
      int cut;
      if (l - f <= 64) {
        if (!win.covers(f, l)) {
          win.flush(sc, m, lane);
          win.load(sc, f, m, lane);
        }
        cut = win_partition(win, f, l, sc, lane);
      } else {
        win.flush(sc, m, lane);
        cut = lds_partition_any<S>(sc, f, l, lane);
      }
      if (lane == 0) sc.stk[sp] = cut | (l << 10) | (d << 20);
      ++sp;
      wave_lds_sync();
      l = cut;
    }
    if (!heaped && l - f > 1)
      for (int pos = f + lane; pos < l; pos += 64) sc.seg[pos] = (uint32_t)f | ((uint32_t)l << 16);
  }
  win.flush(sc, m, lane);
  wave_lds_sync();
  lds_segment_sort<S>(sc, m, lane);
}

// std::sort(begin, begin+m) for m > 64, level-parallel.  __introsort_loop's
// pending segments are disjoint and each partition / heapsort moves elements only
// inside its own segment, so the order in which the stack processes them does not
// matter: here all segments of one recursion level are partitioned in one
// wave-wide step (segmented ranks: prefix counts of the stop flags, differenced
// at the segment ends; pairs exchanged through xa / xb at index f/2 + rank, which
// stays inside the segment's own share).  Each position carries its segment
// [f, l) and depth budget d.  Then __final_insertion_sort as the segment sort.
template <int S>
__device__ __forceinline__ void lds_sort_prefix_par(const TopkLdsV2& sc, int m, int lane, int dbg = 0) {
  uint64_t* A = sc.A;
  uint32_t* PLR = sc.seg;                               // prefix counts (left | right << 16), then segments
  uint32_t* CUT = reinterpret_cast<uint32_t*>(sc.xa);   // per segment start: min cut candidate
  int f[S], l[S], d[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    f[s] = 0;
    l[s] = m;
    d[s] = 2 * ilog2(m);
  }
  while (true) {
    bool act[S], heap[S];
    uint64_t any_act = 0ull, any_heap = 0ull;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      const bool big = pos < m && l[s] - f[s] > 16;
      act[s] = big && d[s] > 0;
      heap[s] = big && d[s] == 0;
      any_act |= ballot64(act[s]);
      any_heap |= ballot64(heap[s]);
    }
    if (!any_act && !any_heap) break;
    if (any_heap) {  // std::__partial_sort(f, l, l) per exhausted segment, serial, one lane each
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (heap[s] && 64 * s + lane == f[s]) {
          s_heap_select(A, f[s], l[s], l[s]);
          s_sort_heap(A, f[s], l[s]);
        }
        if (heap[s]) {  // sorted: final, a trivial segment for the insertion sort
          f[s] = 64 * s + lane;
          l[s] = f[s] + 1;
        }
      }
      wave_lds_sync();
    }
    if (!any_act) continue;
    // ---- __unguarded_partition_pivot on every active segment ----------------
    uint64_t v[S];
    uint32_t p[S];
    bool isl[S], isr[S];
    int mp[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      v[s] = pos < m ? A[pos] : 0ull;
      p[s] = 0u;
      mp[s] = -1;
      if (act[s]) {
        const int mid = f[s] + (l[s] - f[s]) / 2;
        const uint32_t ka = key_of(A[f[s] + 1]), kb = key_of(A[mid]), kc = key_of(A[l[s] - 1]);
        int mm;
        if (ka > kb) {
          if (kb > kc) mm = mid;
          else if (ka > kc) mm = l[s] - 1;
          else mm = f[s] + 1;
        } else if (ka > kc) mm = f[s] + 1;
        else if (kb > kc) mm = l[s] - 1;
        else mm = mid;
        p[s] = mm == f[s] + 1 ? ka : (mm == mid ? kb : kc);
        mp[s] = mm;
        if (pos == f[s]) v[s] = A[mm];  // iter_swap(first, median)
        else if (pos == mm) v[s] = A[f[s]];
      }
    }
    int totL = 0, totR = 0;
    int pl[S], pr[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      const uint32_t k = key_of(v[s]);
      isl[s] = act[s] && pos > f[s] && !(k > p[s]);
      isr[s] = act[s] && !(p[s] > k);
      const uint64_t Lb = ballot64(isl[s]), Rb = ballot64(isr[s]);
      pl[s] = totL + (int)mbcnt(Lb);
      pr[s] = totR + (int)mbcnt(Rb);
      totL += (int)__popcll(Lb);
      totR += (int)__popcll(Rb);
    }
    wave_lds_sync();  // the median / first reads above are done before any write
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      if (pos < m) PLR[pos] = (uint32_t)pl[s] | ((uint32_t)pr[s] << 16);
      if (act[s] && pos == f[s]) CUT[pos] = (uint32_t)l[s];
    }
    if (lane == 0) PLR[m] = (uint32_t)totL | ((uint32_t)totR << 16);
    wave_lds_sync();
    bool swl[S], swr[S];
    int xi[S];
    uint64_t any_sw = 0ull;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      swl[s] = swr[s] = false;
      xi[s] = 0;
      if (act[s]) {
        const int a = pl[s] - (int)(PLR[f[s]] & 0xFFFFu);
        const int bgt = (int)(PLR[l[s]] >> 16) - pr[s] - (isr[s] ? 1 : 0);
        swl[s] = isl[s] && bgt > a;
        swr[s] = isr[s] && a > bgt;
        xi[s] = f[s] / 2 + (swl[s] ? a : bgt);
      }
      any_sw |= ballot64(swl[s] || swr[s]);
    }
    // the write of the swapped / pivot-moved values happens after the exchange
    if (any_sw) {
      uint64_t* XA = sc.xa;
      uint64_t* XB = sc.xb;
      wave_lds_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (swl[s]) XA[xi[s]] = v[s];
        if (swr[s]) XB[xi[s]] = v[s];
      }
      wave_lds_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if (swl[s]) v[s] = XB[xi[s]];
        if (swr[s]) v[s] = XA[xi[s]];
      }
      wave_lds_sync();
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int pos = 64 * s + lane;
        if (act[s] && pos == f[s]) CUT[pos] = (uint32_t)l[s];  // CUT aliases XA: re-initialise
      }
      wave_lds_sync();
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      if (act[s]) {
        A[pos] = v[s];
        // cut = min(first non-swapping left stop, lowest swapping right stop | last)
        if ((isl[s] && !swl[s]) || swr[s]) atomicMin(&CUT[f[s]], (uint32_t)pos);
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const int pos = 64 * s + lane;
      if (act[s]) {
        const int cut = (int)CUT[f[s]];
        if (pos < cut) l[s] = cut;
        else f[s] = cut;
        d[s] -= 1;
      }
    }
    wave_lds_sync();
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = 64 * s + lane;
    if (pos < m) sc.seg[pos] = (uint32_t)f[s] | ((uint32_t)l[s] << 16);
  }
  wave_lds_sync();
  if (!(dbg & 32)) lds_segment_sort<S>(sc, m, lane);
}

// std::sort(begin, begin+m): the windowed sequential introsort for short prefixes,
// the level-parallel one when the prefix spans several slots
template <int S>
__device__ __forceinline__ void lds_sort_head(const TopkLdsV2& sc, int m, int lane, int dbg = 0) {
  if (S > 1 && m > 64) lds_sort_prefix_par<S>(sc, m, lane, dbg);
  else lds_sort_prefix<S>(sc, m, lane);
}

// Full top-k of the row in sc.A[0, n) (TopKImpl.h:45-86).  On return positions
// [0, k) hold torch's order.
template <int S>
__device__ __forceinline__ void lds_topk(const TopkLdsV2& sc, int n, int k, int lane) {
  if (!lds_select<S>(sc, n, k, lane)) lds_sort_head<S>(sc, k - 1, lane);
}

}  // namespace mxa
