// Wave-per-row top-k in torch's CPU index order, row held in REGISTERS.
//
// Same algorithm restatement as mxa_topk.hpp / mxa_topk_lds.hpp (libstdc++ 11
// __introselect + __introsort_loop + __final_insertion_sort behind torch's CPU
// topk, TopKImpl.h:45-86; ballot/rank form of __unguarded_partition, executable
// model tools/topk_model.py), organised to issue as few instructions as possible:
//
//   * the row lives in VGPRs: key K[s] (order key, u32) and original index I[s]
//     of position 64 s + lane -- the layout the scores are produced in, so the
//     first partition steps need no LDS traffic at all;
//   * a partition step over a range longer than 64 works on the slots it spans;
//     once an introselect / introsort range fits 64 positions every later range
//     of that chain is a sub-range, so the row is moved ONCE into a 64-wide
//     register window (base b: lane i <-> position b + i) and the remaining steps
//     run on one register pair with readlane / writelane pivots, s_bfm-style range
//     masks and one LDS round trip for the swap exchange;
//   * the final insertion sort of std::sort is a stable sort of the arrangement
//     the introsort loop leaves (see lds_sort_prefix), computed as a stable rank;
//   * depth-limit heap fallbacks, partial_sort (k*64 <= n) and prefixes longer
//     than 64 (std::sort of k-1 > 64 elements) go through the LDS row
//     (mxa_topk_lds.hpp), materialised only on those paths.
#pragma once
#include "mxa_topk_lds.hpp"
#include "mxa_topk_lane.hpp"

namespace mxa {

// LDS pointers with the address space spelled out: the compiler does not infer it
// through the RegTopk member and would otherwise emit FLAT accesses
typedef __attribute__((address_space(3))) uint64_t lds_u64;
typedef __attribute__((address_space(3))) int lds_i32;

// S slot registers as one vector value: element access never needs memory, so
// the row cannot be demoted to scratch whatever the index
template <int S> struct SlotVec;
template <> struct SlotVec<1> { typedef uint32_t __attribute__((ext_vector_type(1))) T; };
template <> struct SlotVec<2> { typedef uint32_t __attribute__((ext_vector_type(2))) T; };
template <> struct SlotVec<4> { typedef uint32_t __attribute__((ext_vector_type(4))) T; };
template <> struct SlotVec<8> { typedef uint32_t __attribute__((ext_vector_type(8))) T; };

__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
// writelane: lane l takes the uniform value v (v_cmp + v_cndmask)
__device__ __forceinline__ uint32_t wrl(uint32_t old, uint32_t v, int l) {
  return __builtin_amdgcn_inverse_ballot_w64(1ull << l) ? v : old;
}
__device__ __forceinline__ int ffs64(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }

// __move_median_to_first(first, a = first+1, b = mid, c = last-1) with cmp = greater:
// returns the position moved to `first` and its key.
__device__ __forceinline__ int median3(uint32_t ka, uint32_t kb, uint32_t kc, int a, int b, int c, uint32_t* p) {
  int m;
  if (ka > kb) {
    if (kb > kc) m = b;
    else if (ka > kc) m = c;
    else m = a;
  } else if (ka > kc) m = a;
  else if (kb > kc) m = c;
  else m = b;
  *p = m == a ? ka : (m == b ? kb : kc);
  return m;
}

// uniform-position access to a slot array
template <class V>
__device__ __forceinline__ uint32_t uget(const V& a, int pos) {
  constexpr int S = sizeof(V) / 4;
  const int s = pos >> 6, ln = pos & 63;
  uint32_t v = rdl(a[0], ln);
#pragma unroll
  for (int t = 1; t < S; ++t) {
    const uint32_t w = rdl(a[t], ln);
    v = s == t ? w : v;
  }
  return v;
}
template <class V>
__device__ __forceinline__ void uset(V& a, int pos, uint32_t val) {
  constexpr int S = sizeof(V) / 4;
  const int s = pos >> 6, ln = pos & 63;
  const bool me = lane_id() == ln;
#pragma unroll
  for (int t = 0; t < S; ++t) a[t] = (me && s == t) ? val : a[t];
}

// The swap exchange of one Hoare partition: the t-th swapping left stop and the
// t-th swapping right stop (counted from the right) trade places.  Left stops
// publish at X[t], right stops at X[half + t]; each reads its partner's slot.
// Branch-free: lanes that do not swap write and read their own trash entry
// X[2 half + lane] (no exec-mask save / restore on the SALU).
__device__ __forceinline__ void exchange(uint32_t& k, uint32_t& i, bool swl, bool swr, int rank, lds_u64* X, int half,
                                         int lane) {
  const bool sw = swl || swr;
  X[sw ? (swl ? rank : half + rank) : 2 * half + lane] = pack_ki(k, i);
  wave_lds_sync();
  const uint64_t v = X[sw ? (swl ? half + rank : rank) : 2 * half + lane];
  k = (uint32_t)(v >> 32);
  i = (uint32_t)v;
}

// ---- one partition step on the 64-wide window -------------------------------
struct RWin {
  int b;       // base position (uniform)
  uint32_t k;  // key of position b + lane
  uint32_t i;  // index of position b + lane
};

// a uniform scalar copied into a VGPR the compiler treats as divergent: the logic
// on it is issued on the VALU (the scalar unit is the selection kernel's limiter)
__device__ __forceinline__ uint32_t to_vgpr(uint32_t x) {
  uint32_t v;
  asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
  return v;
}

__device__ __forceinline__ int win_step(RWin& w, int f, int l, lds_u64* X, int half, int lane) {
  const int rf = f - w.b, rl = l - w.b;
  const int ra = rf + 1, rb = rf + (l - f) / 2, rc = rl - 1;
  // __move_median_to_first on the VALU: branch-free selects on VGPR copies
  const uint32_t ka = to_vgpr(rdl(w.k, ra)), kb = to_vgpr(rdl(w.k, rb)), kc = to_vgpr(rdl(w.k, rc));
  const bool ab = ka > kb, bc = kb > kc, ac = ka > kc;
  const int rmv = ab ? (bc ? rb : (ac ? rc : ra)) : (ac ? ra : (bc ? rc : rb));
  const uint32_t p = ab ? (bc ? kb : (ac ? kc : ka)) : (ac ? ka : (bc ? kc : kb));
  const int rm = __builtin_amdgcn_readfirstlane(rmv);
  {  // iter_swap(first, median)
    const uint32_t kf = rdl(w.k, rf), jf = rdl(w.i, rf), jm = rdl(w.i, rm);
    const bool atf = lane == rf, atm = lane == rm;
    w.k = atf ? p : (atm ? kf : w.k);
    w.i = atf ? jm : (atm ? jf : w.i);
  }
  // stops as lane masks straight from VALU compares (ranges as lane offsets)
  const uint64_t inl = ballot64((unsigned)(lane - rf - 1) < (unsigned)(rl - rf - 1));  // [first+1, last)
  const uint64_t inr = ballot64((unsigned)(lane - rf) < (unsigned)(rl - rf));          // [first, last)
  const uint64_t Lb = ballot64(!(w.k > p)) & inl;  // left stops
  const uint64_t Rb = ballot64(!(p > w.k)) & inr;  // right stops
  const int a = mbcnt(Lb);                                          // left stops below
  const int u = (int)__popcll(Rb) - mbcnt_incl(Rb);                 // right stops above
  const uint64_t SWL = ballot64(u > a) & Lb, SWR = ballot64(a > u) & Rb;
  if (SWL) {
    const bool swl = __builtin_amdgcn_inverse_ballot_w64(SWL);
    exchange(w.k, w.i, swl, __builtin_amdgcn_inverse_ballot_w64(SWR), swl ? a : u, X, half, lane);
  }
  // cut = min(first non-swapping left stop, lowest swapping right stop | last)
  const uint64_t nsl = Lb & ~SWL;
  const int c1 = nsl ? ffs64(nsl) : 1 << 20;
  const int c2 = SWR ? ffs64(SWR) : rl;
  return w.b + (c1 < c2 ? c1 : c2);
}

// ---- one partition step on the slot registers (ranges longer than 64) --------
// A mirrors the row in LDS while the steps run on the slot registers (the caller
// writes it before the first step; every step rewrites it): the pivot candidates
// are broadcast LDS reads instead of S readlanes + selects each.
template <int S>
__device__ __forceinline__ int slots_step(typename SlotVec<S>::T& K, typename SlotVec<S>::T& I, int f, int l,
                                          lds_u64* X, int half, int lane, lds_u64* A) {
  const int a_ = f + 1, b_ = f + (l - f) / 2, c_ = l - 1;
  const uint64_t xa = A[a_], xb = A[b_], xc = A[c_], xf = A[f];
  // __move_median_to_first on the VALU (branch-free selects on the broadcast values)
  uint32_t ka = (uint32_t)(xa >> 32), kb = (uint32_t)(xb >> 32), kc = (uint32_t)(xc >> 32);
  asm volatile("" : "+v"(ka), "+v"(kb), "+v"(kc));
  const bool ab = ka > kb, bc = kb > kc, ac = ka > kc;
  const int mv = ab ? (bc ? b_ : (ac ? c_ : a_)) : (ac ? a_ : (bc ? c_ : b_));
  const uint32_t p = ab ? (bc ? kb : (ac ? kc : ka)) : (ac ? ka : (bc ? kc : kb));
  const int m = __builtin_amdgcn_readfirstlane(mv);
  {  // iter_swap(first, median)
    const uint32_t kf = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(xf >> 32));
    const uint32_t jf = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xf);
    const uint32_t ja = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xa);
    const uint32_t jb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xb);
    const uint32_t jc = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)xc);
    const uint32_t jm = m == a_ ? ja : (m == b_ ? jb : jc);
    uset(K, f, p);
    uset(I, f, jm);
    uset(K, m, kf);
    uset(I, m, jf);
  }
  // stops as lane masks: single compares straight to SGPRs, combined by SALU
  uint64_t Lb[S], Rb[S];
  int cl[S], cr[S];
  int totL = 0, totR = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int pos = 64 * s + lane;
    const uint64_t inl = ballot64((unsigned)(pos - f - 1) < (unsigned)(l - f - 1));  // [first+1, last)
    const uint64_t inr = ballot64((unsigned)(pos - f) < (unsigned)(l - f));          // [first, last)
    Lb[s] = inl & ballot64(!(K[s] > p));  // left stops
    Rb[s] = inr & ballot64(!(p > K[s]));  // right stops
    cl[s] = totL;
    cr[s] = totR;
    totL += (int)__popcll(Lb[s]);
    totR += (int)__popcll(Rb[s]);
  }
  int rank[S];
  uint64_t SWL[S], SWR[S];
  uint64_t anysw = 0ull;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int a = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(Lb[s] >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)Lb[s], (uint32_t)cl[s]));
    const int u = totR - cr[s] - mbcnt_incl(Rb[s]);
    SWL[s] = ballot64(u > a) & Lb[s];
    SWR[s] = ballot64(a > u) & Rb[s];
    rank[s] = __builtin_amdgcn_inverse_ballot_w64(SWL[s]) ? a : u;
    anysw |= SWL[s];
  }
  if (anysw) {  // branch-free per slot: non-swapping lanes write / read the trash entry
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const bool sw = __builtin_amdgcn_inverse_ballot_w64(SWL[s] | SWR[s]);
      const bool swl = __builtin_amdgcn_inverse_ballot_w64(SWL[s]);
      X[sw ? (swl ? rank[s] : half + rank[s]) : 2 * half + lane] = pack_ki(K[s], I[s]);
    }
    wave_lds_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const bool sw = __builtin_amdgcn_inverse_ballot_w64(SWL[s] | SWR[s]);
      const bool swl = __builtin_amdgcn_inverse_ballot_w64(SWL[s]);
      const uint64_t v = X[sw ? (swl ? half + rank[s] : rank[s]) : 2 * half + lane];
      K[s] = sw ? (uint32_t)(v >> 32) : K[s];
      I[s] = sw ? (uint32_t)v : I[s];
    }
  }
  // the mirror for the next step
#pragma unroll
  for (int s = 0; s < S; ++s) A[64 * s + lane] = pack_ki(K[s], I[s]);
  wave_lds_sync();
  // cut = min(first non-swapping left stop, lowest swapping right stop | last):
  // per-lane candidates and a DPP min-reduction (VALU) instead of per-slot s_ff1
  uint32_t cand = 1u << 20;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint32_t pos = (uint32_t)(64 * s + lane);
    cand = min(cand, __builtin_amdgcn_inverse_ballot_w64(Lb[s] & ~SWL[s]) ? pos : (1u << 20));
    cand = min(cand, __builtin_amdgcn_inverse_ballot_w64(SWR[s]) ? pos : (1u << 20));
  }
  const int c = (int)wave_reduce(cand, [](uint32_t x, uint32_t y) { return x < y ? x : y; });
  return c < l ? c : l;
}

// ---- row state ---------------------------------------------------------------
// mode kSlots: K/I hold the row.  kWin: w holds positions [w.b, w.b+64), sc.A the
// rest.  kLds: sc.A holds the row.
enum { kSlots = 0, kWin = 1, kLds = 2 };

// BIG: sorted prefixes longer than 64 possible (k > 65): level-parallel LDS sort
template <int S, bool BIG = true>
struct RegTopk {
  typename SlotVec<S>::T K, I;
  RWin w;
  int mode;
  int n;
  int lane;
  lds_u64* A;    // [64 S] the row (realignments, fallbacks, long prefixes)
  lds_u64* X;    // [64 S] swap exchange (left stops [0, 32 S), right stops [32 S, 64 S))
  uint32_t* seg; // [64 S] segments of the level-parallel sort (BIG only)
  lds_i32* stk;  // [kTopkStack] pending introsort segments

  __device__ __forceinline__ void init(unsigned char* base, int n_, int lane_) {
    const TopkLdsV2 t = carve_topk(base, S, BIG);
    A = (lds_u64*)t.A;
    X = (lds_u64*)t.xa;
    seg = t.seg;
    stk = (lds_i32*)t.stk;
    n = n_;
    lane = lane_;
    mode = kSlots;
  }
  // the generic-pointer view for the shared LDS helpers (mxa_topk*.hpp)
  __device__ __forceinline__ TopkLdsV2 sc() const {
    TopkLdsV2 t;
    t.A = (uint64_t*)A;
    t.xa = (uint64_t*)X;
    t.xb = t.xa + 32 * S;
    t.seg = (uint32_t*)(__attribute__((address_space(3))) uint32_t*)seg;
    t.stk = (int*)stk;
    return t;
  }

  __device__ __forceinline__ void slots_to_lds() {
#pragma unroll
    for (int s = 0; s < S; ++s) A[64 * s + lane] = pack_ki(K[s], I[s]);
  }
  __device__ __forceinline__ void win_to_lds() {
    if (w.b + lane < 64 * S) A[w.b + lane] = pack_ki(w.k, w.i);
  }
  __device__ __forceinline__ void lds_to_win(int b) {
    w.b = b;
    const uint64_t v = b + lane < 64 * S ? A[b + lane] : 0ull;
    w.k = (uint32_t)(v >> 32);
    w.i = (uint32_t)v;
  }
  // the whole row into sc.A (mode kLds)
  __device__ __forceinline__ void to_lds() {
    if (mode == kSlots) slots_to_lds();
    else if (mode == kWin) win_to_lds();
    wave_lds_sync();
    mode = kLds;
  }
  // window at base b; sc.A holds every position outside it afterwards
  __device__ __forceinline__ void to_win(int b) {
    if (mode == kWin && w.b == b) return;
    if (mode == kSlots) {
      if (S == 1 && b == 0) {  // the window is the whole row
        w.b = 0;
        w.k = K[0];
        w.i = I[0];
        mode = kWin;
        return;
      }
      slots_to_lds();
    } else if (mode == kWin) {
      win_to_lds();
    }
    wave_lds_sync();
    lds_to_win(b);
    mode = kWin;
  }
  __device__ __forceinline__ int win_base(int f) const { return f < 64 * S - 64 ? f : 64 * S - 64; }

  // __insertion_sort on [f, l), l - f <= 3 (stable), inside the window
  __device__ __forceinline__ void small_insertion(int f, int l) {
    const int rf = f - w.b;
    uint32_t k0 = rdl(w.k, rf), k1 = rdl(w.k, rf + 1);
    uint32_t i0 = rdl(w.i, rf), i1 = rdl(w.i, rf + 1);
    if (k1 > k0) {
      uint32_t t = k0; k0 = k1; k1 = t;
      t = i0; i0 = i1; i1 = t;
    }
    if (l - f == 3) {
      uint32_t k2 = rdl(w.k, rf + 2), i2 = rdl(w.i, rf + 2);
      if (k2 > k1) {
        uint32_t t = k1; k1 = k2; k2 = t;
        t = i1; i1 = i2; i2 = t;
        if (k1 > k0) {
          t = k0; k0 = k1; k1 = t;
          t = i0; i0 = i1; i1 = t;
        }
      }
      w.k = wrl(w.k, k2, rf + 2);
      w.i = wrl(w.i, i2, rf + 2);
    }
    w.k = wrl(w.k, k0, rf);
    w.i = wrl(w.i, i0, rf);
    w.k = wrl(w.k, k1, rf + 1);
    w.i = wrl(w.i, i1, rf + 1);
  }

  // std::nth_element(begin, begin + k - 1, end) or, when k*64 <= n, the whole
  // std::partial_sort.  Returns true when [0, k) is final (no sort needed).
  __device__ __forceinline__ bool select(int k) {
    const int half = 32 * S;
    if (k * 64 <= n) {  // std::partial_sort(begin, begin+k, end)
      to_lds();
      if (lane == 0) {
        s_heap_select(sc().A, 0, k, n);
        s_sort_heap(sc().A, 0, k);
      }
      wave_lds_sync();
      return true;
    }
    int first = 0, last = n;
    bool mirror = false;  // A holds the row (slots_step's pivot reads)
    const int nth = k - 1;
    int depth = 2 * ilog2(n);
    while (last - first > 3) {
      if (depth == 0) {  // std::__heap_select(first, nth+1, last); iter_swap(first, nth)
        to_lds();
        if (lane == 0) {
          s_heap_select(sc().A, first, nth + 1, last);
          const uint64_t t = A[first];
          A[first] = A[nth];
          A[nth] = t;
        }
        wave_lds_sync();
        return false;
      }
      --depth;
      int cut;
      if (mode == kWin || last - first <= 64) {
        if (mode != kWin) to_win(win_base(first));
        cut = win_step(w, first, last, X, half, lane);
      } else {
        if (!mirror) {
          slots_to_lds();
          wave_lds_sync();
          mirror = true;
        }
        cut = slots_step<S>(K, I, first, last, X, half, lane, A);
      }
      if (cut <= nth) first = cut;
      else last = cut;
    }
    if (last - first > 1) {
      if (mode != kWin) to_win(win_base(first));
      small_insertion(first, last);
    }
    return false;
  }

  // The wave-wide part of run(k) when the lanes finish the row (mxa_topk_lane.hpp):
  // __introselect steps only while the pending range reaches past position W
  // (k <= W <= 64).  Returns the hand-off state; first == last when selection is
  // complete (depth-limit fallback, a final <= 3 range past W, or partial_sort,
  // which also leaves the prefix sorted: then k = 0 in the task).
  __device__ __forceinline__ LaneTask select_big(int k, int W) {
    const int half = 32 * S;
    LaneTask t;
    t.nth = k - 1;
    t.k = k;
    t.first = t.last = t.depth = 0;
    if (k * 64 <= n) {  // std::partial_sort(begin, begin+k, end)
      to_lds();
      if (lane == 0) {
        s_heap_select(sc().A, 0, k, n);
        s_sort_heap(sc().A, 0, k);
      }
      wave_lds_sync();
      t.k = 0;
      return t;
    }
    int first = 0, last = n;
    bool mirror = false;  // A holds the row (slots_step's pivot reads)
    const int nth = k - 1;
    int depth = 2 * ilog2(n);
    while (last - first > 3 && last > W) {
      if (depth == 0) {  // std::__heap_select(first, nth+1, last); iter_swap(first, nth)
        to_lds();
        if (lane == 0) {
          s_heap_select(sc().A, first, nth + 1, last);
          const uint64_t x = A[first];
          A[first] = A[nth];
          A[nth] = x;
        }
        wave_lds_sync();
        return t;
      }
      --depth;
      int cut;
      if (mode == kWin || last - first <= 64) {
        if (mode != kWin) to_win(win_base(first));
        cut = win_step(w, first, last, X, half, lane);
      } else {
        if (!mirror) {
          slots_to_lds();
          wave_lds_sync();
          mirror = true;
        }
        cut = slots_step<S>(K, I, first, last, X, half, lane, A);
      }
      if (cut <= nth) first = cut;
      else last = cut;
    }
    if (last > W) {  // a final <= 3 range that reaches past W: __insertion_sort here
      if (last - first > 1) {
        if (mode != kWin) to_win(win_base(first));
        small_insertion(first, last);
      }
      return t;
    }
    t.first = first;
    t.last = last;
    t.depth = depth;
    return t;
  }

  // positions [0, W) of the row to dst[0, W) (W <= 64)
  __device__ __forceinline__ void stage_out(lu64* dst, int W) {
    if (mode == kWin && w.b != 0) to_lds();
    uint64_t v;
    if (mode == kSlots) v = pack_ki(K[0], I[0]);
    else if (mode == kWin) v = pack_ki(w.k, w.i);
    else v = A[lane];
    if (lane < W) dst[lane] = v;
  }

  // std::sort(begin, begin + m) for m <= 64 on the window at base 0:
  // __introsort_loop on a stack of pending segments, then the final insertion
  // sort as a stable rank of [0, m).
  __device__ __forceinline__ void sort_head_win(int m) {
    const int half = 32 * S;
    to_win(0);
    int sp = 0;
    int f = 0, l = m, d = 2 * ilog2(m);
    while (true) {
      while (l - f > 16) {
        if (d == 0) {  // std::__partial_sort(f, l, l): heapsort, [f, l) left sorted
          win_to_lds();
          wave_lds_sync();
          if (lane == 0) {
            s_heap_select(sc().A, f, l, l);
            s_sort_heap(sc().A, f, l);
          }
          wave_lds_sync();
          lds_to_win(0);
          break;
        }
        --d;
        const int cut = win_step(w, f, l, X, half, lane);
        stk[sp] = cut | (l << 10) | (d << 20);  // every lane the same value: no exec branch
        ++sp;
        l = cut;
      }
      if (sp == 0) break;
      --sp;
      wave_lds_sync();
      const int e = __builtin_amdgcn_readfirstlane(stk[sp]);
      f = e & 1023;
      l = (e >> 10) & 1023;
      d = e >> 20;
    }
    // stable rank of every position of [0, m): keys greater, or equal and earlier
    // (4 positions per loop trip: the loop control is scalar work; lanes >= m
    // write / read their trash entry, no exec branch)
    const uint32_t mk = w.k;
    int r = 0;
    for (int j0 = 0; j0 < m; j0 += 4) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int j = j0 + t;
        const uint32_t kj = rdl(w.k, j & 63);
        r += (j < m && (kj > mk || (kj == mk && j < lane))) ? 1 : 0;
      }
    }
    const bool in = lane < m;
    X[in ? r : 2 * half + lane] = pack_ki(w.k, w.i);
    wave_lds_sync();
    const uint64_t v = X[in ? lane : 2 * half + lane];
    w.k = (uint32_t)(v >> 32);
    w.i = (uint32_t)v;
    wave_lds_sync();
  }

  // Full top-k (TopKImpl.h:45-86): afterwards position p < k holds torch's p-th
  // index; read it with out_idx().
  __device__ __forceinline__ void run(int k) {
    if (k <= 0) return;
    if (select(k)) return;
    const int m = k - 1;
    if (m <= 1) return;
    if (!BIG || m <= 64) {
      sort_head_win(m);
    } else {
      to_lds();
      lds_sort_prefix_par<S>(sc(), m, lane);
    }
  }

  // after run(): the result is in the slots, in a window at base 0 (positions
  // >= 64 in sc.A), or in sc.A
  __device__ __forceinline__ void finalize() {
    if (mode == kWin && w.b != 0) to_lds();
  }
  // index at position 64 s + lane (valid for positions < k after run(k) + finalize())
  __device__ __forceinline__ uint32_t out_idx(int s) const {
    if (mode == kSlots) return I[s];
    if (mode == kWin && s == 0) return w.i;
    return (uint32_t)A[64 * s + lane];
  }
};

}  // namespace mxa
