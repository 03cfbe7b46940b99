// Exact-order top-k with ONE DPP ROW (16 lanes) PER ROW: four rows per wave.
//
// torch's CPU topk(k, largest, sorted) runs, per row of pair<double,int64>
// (aten/src/ATen/native/TopKImpl.h:45-86, libstdc++ 11):
//     k*64 <= n : std::partial_sort(begin, begin+k, end, cmp)
//     else      : std::nth_element(begin, begin+k-1, end, cmp); std::sort(begin, begin+k-1, cmp)
// and ties are the norm for the approximate scores, so the element
// MOVEMENTS of __introselect / __introsort_loop / __unguarded_partition have to be
// reproduced, not just the selected set.
//
// Each Hoare partition step is computed from stop flags and prefix counts (the rank
// form derived in tools/topk_model.py and checked against libstdc++ by
// tests/test_topk_model.py).  For pivot p at `first` (cmp = greater on order keys):
//   left stop  x in (first, last): a[x] <= p      right stop y in (first, last): a[y] >= p
//   (the pivot position never swaps and never counts)
//   T(z) = left stops <= z + right stops <= z  (non-decreasing, +1 at least per position)
//   cut  = first + 1 + #{z in (first,last) : T(z) <= totR}
//   swaps: the left stops below the cut (nsw of them) trade places, in order, with the
//   nsw highest right stops taken from the top.
// Why this layout: the per-row work is a few prefix counts and a scatter, which a DPP
// row does with row_shr scans and row_newbcast broadcasts (no SALU, no readlane);
// the 16 lanes of a row hold E contiguous positions each (E = 2 .. 32, the narrowest
// window that holds every pending range of the wave), so a step costs ~E
// instructions per lane for FOUR rows at once instead of ~100+ per row for a
// wave-wide step.  The row itself lives in an LDS mirror A (order key << 32 | index);
// swaps publish their positions in P, then the pairs trade elements.
//
// Elements: El = uint64_t, (order key << 32) | index, for any row; or El = uint32_t, the
// packed form (order key & 0xFFFFFF00) | index for rows of <= 256 keys whose scores all
// have a zero low mantissa byte (then the key's low byte is 0x00 / 0xFF and carries no
// order; the approximate scores of ex_pred / MXINT4 / EXION / partial / true_ex are such
// sums of a few small integers times powers of two): half the LDS per row and 32-bit
// compares, key(a) > key(b) <=> a > (b | 0xFF) (GEl below).
//
// std::sort's final insertion sort is a stable sort of the arrangement the introsort
// loop leaves; because those segments are mutually ordered it equals a stable sort of
// each <= 16-element segment (or of the whole prefix when k-1 <= 64), computed as a
// stable rank.  Depth-limit heap fallbacks and partial_sort run serially on the
// row's first lane (mxa_order.hpp, stl_heap.h semantics).
#pragma once
#include "mxa_order.hpp"

namespace mxa {

typedef __attribute__((address_space(3))) uint32_t lu32;
typedef __attribute__((address_space(3))) uint16_t lu16;
typedef __attribute__((address_space(3))) uint8_t lu8;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lu128;

constexpr int kGStk = 24;  // pending introsort segments (>= depth limit 2*lg(511) + 1)
constexpr int kGSeg = 16;  // final sort segments queued for one ranking pass

// Row capacity: NP (128, 256 or 512, a template parameter: the exchange slots'
// width and the swap-rank split HP = NP/2) and the mirror's allocated positions NPA
// (runtime: T rounded up to a window width, so that the LDS per row -- and with it
// the resident waves -- follows the row length)
// per-row LDS: mirror A[NPA] (El), exchange slots P[NP] + 16 trash slots (u8 for
// NP <= 256, else u16), introsort stack, queue of final segments
__host__ __device__ constexpr int grp_pbytes(int NP) { return ((NP <= 256 ? 1 : 2) * (NP + 16) + 15) & ~15; }
__host__ __device__ constexpr size_t grp_row_bytes(int NPA, int NP, int elb = 8) {
  // packed rows: a stride of 128 mod 256 bytes, so the two rows a 32-lane LDS access
  // group holds sit half the 64 banks apart (their windows' element reads do not collide)
  return elb == 4 ? (((size_t)4 * NPA + grp_pbytes(NP) + 4 * kGStk + 4 * kGSeg + 127) / 256) * 256 + 128
                  : (size_t)elb * NPA + grp_pbytes(NP) + 4 * kGStk + 4 * kGSeg;
}
// (the window widths 16 E are 32, 64, ..., 256, 384, 512, so NPA is one of them)
__host__ __device__ constexpr int grp_alloc(int T) { return T <= 256 ? (T + 31) & ~31 : (T <= 384 ? 384 : 512); }

// element traits: key for the stop compares, order, index
template <typename El>
struct GEl;
template <>
struct GEl<uint64_t> {
  typedef __attribute__((address_space(3))) uint64_t LT;
  __device__ static uint32_t key(uint64_t x) { return (uint32_t)(x >> 32); }
  __device__ static bool gt(uint64_t a, uint64_t b) { return key(a) > key(b); }
  __device__ static uint32_t thr_le(uint32_t pk) { return pk; }  // key(x) <= p  <=>  key(x) <= thr_le
  __device__ static uint32_t thr_ge(uint32_t pk) { return pk; }  // key(x) >= p  <=>  key(x) >= thr_ge
  __device__ static uint32_t idx(uint64_t x) { return (uint32_t)x; }
};
template <>
struct GEl<uint32_t> {
  typedef __attribute__((address_space(3))) uint32_t LT;
  __device__ static uint32_t key(uint32_t x) { return x; }
  __device__ static bool gt(uint32_t a, uint32_t b) { return a > (b | 0xFFu); }
  __device__ static uint32_t thr_le(uint32_t pk) { return pk | 0xFFu; }
  __device__ static uint32_t thr_ge(uint32_t pk) { return pk & ~0xFFu; }
  __device__ static uint32_t idx(uint32_t x) { return x & 0xFFu; }
};

template <typename El = uint64_t>
struct GrpRow {
  typename GEl<El>::LT* A;
  unsigned char __attribute__((address_space(3)))* P;
  lu32* stk;
  lu32* seg;
  int npa;  // allocated mirror positions
};
template <typename El = uint64_t>
__device__ __forceinline__ GrpRow<El> carve_grp(unsigned char* base, int npa, int NP) {
  GrpRow<El> g;
  constexpr int B = (int)sizeof(El);
  g.A = (typename GEl<El>::LT*)(lu32*)(base);
  g.P = (unsigned char __attribute__((address_space(3)))*)(base + B * npa);
  g.stk = (lu32*)(base + B * npa + grp_pbytes(NP));
  g.seg = (lu32*)(base + B * npa + grp_pbytes(NP) + 4 * kGStk);
  g.npa = npa;
  return g;
}
template <int NP, typename El>
__device__ __forceinline__ void p_put(const GrpRow<El>& g, uint32_t i, uint32_t v) {
  if constexpr (NP <= 256) ((lu8*)g.P)[i] = (uint8_t)v;
  else ((lu16*)g.P)[i] = (uint16_t)v;
}
template <int NP, typename El>
__device__ __forceinline__ uint32_t p_get(const GrpRow<El>& g, uint32_t i) {
  if constexpr (NP <= 256) return ((lu8*)g.P)[i];
  else return ((lu16*)g.P)[i];
}

__device__ __forceinline__ uint32_t hi32(uint64_t x) { return (uint32_t)(x >> 32); }
__device__ __forceinline__ uint32_t lowbits(int n) { return n >= 32 ? ~0u : ((1u << n) - 1u); }

// acc * 2 + (a <= b): one compare and one add-with-carry (the compiler would emit a
// compare, a select and an or)
__device__ __forceinline__ uint32_t g_shl_le(uint32_t acc, uint32_t a, uint32_t b) {
  asm("v_cmp_le_u32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, %0, vcc" : "+v"(acc) : "v"(a), "v"(b) : "vcc");
  return acc;
}
// the stop masks of two positions at once: L = 4 L + 2 (k0 <= pl) + (k1 <= pl),
// R = 4 R + 2 (pr <= k0) + (pr <= k1) (pl = pr = p on 64-bit elements; the packed ones
// compare against p | 0xFF and p & ~0xFF).  The four compares go to four SGPR pairs
// first, so each add-with-carry reads a carry written three instructions earlier: no
// wait states (one compare + add-with-carry pair at a time needs an s_nop between them)
__device__ __forceinline__ void g_stops2(uint32_t& L, uint32_t& R, uint32_t k0, uint32_t k1, uint32_t pl, uint32_t pr) {
  uint64_t c0, c1, c2, c3;
  asm("v_cmp_le_u32_e64 %2, %6, %8\n\t"
      "v_cmp_le_u32_e64 %3, %9, %6\n\t"
      "v_cmp_le_u32_e64 %4, %7, %8\n\t"
      "v_cmp_le_u32_e64 %5, %9, %7\n\t"
      "v_addc_co_u32_e64 %0, %2, %0, %0, %2\n\t"
      "v_addc_co_u32_e64 %1, %3, %1, %1, %3\n\t"
      "v_addc_co_u32_e64 %0, %4, %0, %0, %4\n\t"
      "v_addc_co_u32_e64 %1, %5, %1, %1, %5"
      : "+v"(L), "+v"(R), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3)
      : "v"(k0), "v"(k1), "v"(pl), "v"(pr));
}

// r + (a > b) for 64-bit a, b: a compare and an add-with-carry
__device__ __forceinline__ uint32_t g_add_gt(uint32_t r, uint64_t a, uint64_t b) {
  asm("v_cmp_gt_u64 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, 0, vcc" : "+v"(r) : "v"(a), "v"(b) : "vcc");
  return r;
}
// r + (a > b) for 32-bit a, b
__device__ __forceinline__ uint32_t g_add_gt32(uint32_t r, uint32_t a, uint32_t b) {
  asm("v_cmp_gt_u32 vcc, %1, %2\n\tv_addc_co_u32 %0, vcc, %0, 0, vcc" : "+v"(r) : "v"(a), "v"(b) : "vcc");
  return r;
}
// ri += (kj > ki), rj -= (kj > ki): one compare, an add-with-carry and a
// subtract-with-borrow (left to itself the compiler keeps every compare mask live and
// sums them at the end)
__device__ __forceinline__ void g_pair_rank(uint32_t& ri, uint32_t& rj, uint32_t cj, uint32_t ci) {
  uint64_t t;
  asm("v_cmp_gt_u32 vcc, %3, %4\n\tv_addc_co_u32_e64 %0, %2, %0, 0, vcc\n\tv_subb_co_u32_e64 %1, %2, %1, 0, vcc"
      : "+v"(ri), "+v"(rj), "=&s"(t)
      : "v"(cj), "v"(ci)
      : "vcc");
}

// DPP within each 16-lane row: row_shr with zero fill, row_newbcast:15
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_z(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t g_scan(uint32_t x) {  // inclusive prefix sum over the row
  x += dpp_z<0x111>(x);
  x += dpp_z<0x112>(x);
  x += dpp_z<0x114>(x);
  x += dpp_z<0x118>(x);
  return x;
}
__device__ __forceinline__ uint32_t g_last(uint32_t x) {  // lane 15 of the row, to every lane of it
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x15F, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t g_sum(uint32_t x) { return g_last(g_scan(x)); }

template <int E>
constexpr int pow2_floor() { return E >= 32 ? 32 : E >= 16 ? 16 : E >= 8 ? 8 : E >= 4 ? 4 : E >= 2 ? 2 : 1; }

// ---- one partition step ------------------------------------------------------
// libstdc++ __unguarded_partition_pivot(first = f, last = l) (stl_algo.h: median of
// (f+1, mid, l-1) moved to f, then __unguarded_partition of (f, l)) on every row of
// the wave with act set (l - f >= 4), all rows in lockstep.  Window: lane gl holds
// positions lb + e, lb = b + E*gl, e < E (b even, b <= f, l <= b + 16E <= NPA).
// HP = NP / 2 (>= any swap count).  Returns the cut.
template <int E, int NP, typename El>
__device__ __forceinline__ int grp_partition(const GrpRow<El>& g, int f, int l, int b, bool act, int gl) {
  using T = GEl<El>;
  static_assert(E % 2 == 0, "window widths are even");
  constexpr int HP = NP / 2;
  const int fa = act ? f : 0, la = act ? l : 4;  // idle rows read harmless positions
  const int mid = fa + (int)((uint32_t)(la - fa) >> 1);
  const int lb = b + E * gl;
  // the median candidates (whole elements) and the window, all in one LDS round trip:
  // the median's iter_swap is applied to the stop masks in registers and written back
  // while the masks are formed (position f is never a stop; position m holds old f)
  const El xf = g.A[fa], xa = g.A[fa + 1], xb = g.A[mid], xc = g.A[la - 1];
  uint32_t K[E];  // the window's keys (packed elements: the elements)
#pragma unroll
  for (int e = 0; e < E; e += 2) {
    if constexpr (sizeof(El) == 8) {
      const u32x4 v = *(const lu128*)(g.A + lb + e);
      K[e] = v.y;
      K[e + 1] = v.w;
    } else {
      const uint64_t v = *(const __attribute__((address_space(3))) uint64_t*)(g.A + lb + e);
      K[e] = (uint32_t)v;
      K[e + 1] = (uint32_t)(v >> 32);
    }
  }
  // __move_median_to_first(f, f+1, mid, l-1) with cmp = greater, branch-free:
  //   a>b: (b>c ? mid : a>c ? l-1 : f+1);  else: (a>c ? f+1 : b>c ? l-1 : mid)
  const uint32_t ab = T::gt(xa, xb), bc = T::gt(xb, xc), ac = T::gt(xa, xc);
  const uint32_t pick_b = (ab & bc) | (~ab & ~ac & ~bc & 1u);
  const uint32_t pick_c = (ab & ~bc & ac) | (~ab & ~ac & bc & 1u);
  int m = fa + 1;
  El xm = xa;
  m = pick_c ? la - 1 : m;
  xm = pick_c ? xc : xm;
  m = pick_b ? mid : m;
  xm = pick_b ? xb : xm;
  const uint32_t pl = T::thr_le(T::key(xm)), pr = T::thr_ge(T::key(xm)), kf = T::key(xf);
  if (act) {  // iter_swap(f, median)
    g.A[f] = xm;
    g.A[m] = xf;
  }
  // stop masks, bit (E-1-e) <-> position lb + e
  uint32_t Lm = 0, Rm = 0;
#pragma unroll
  for (int e = 0; e < E; e += 2) g_stops2(Lm, Rm, K[e], K[e + 1], pl, pr);
  {  // position m now holds old f (key kf)
    const int em = m - lb;
    const uint32_t bm = (uint32_t)em < (uint32_t)E ? 1u << (E - 1 - em) : 0u;
    Lm = (Lm & ~bm) | (kf <= pl ? bm : 0u);
    Rm = (Rm & ~bm) | (pr <= kf ? bm : 0u);
  }
  const int lo = min(max(f + 1 - lb, 0), E), hi = min(max(l - lb, 0), E);
  const uint32_t rng = act ? (lowbits(E - lo) & ~lowbits(E - hi)) : 0u;
  Lm &= rng;
  Rm &= rng;
  const uint32_t cnt = (uint32_t)__popc(Lm) | ((uint32_t)__popc(Rm) << 16);
  const uint32_t incl = g_scan(cnt);
  const uint32_t tot = g_last(incl), excl = incl - cnt;
  const uint32_t PL = excl & 0xFFFFu, PR = excl >> 16, PLR = PL + PR, totR = tot >> 16;
  // cut = b + #{window positions z : T(z) <= totR}; per lane those are a prefix of
  // its positions (T is non-decreasing), found by binary search on the prefix length
  int j = 0;
#pragma unroll
  for (int st = pow2_floor<E>(); st >= 1; st >>= 1) {
    const int c = j + st, sh = c <= E ? E - c : 0;
    const bool ok = c <= E && PLR + (uint32_t)__popc(Lm >> sh) + (uint32_t)__popc(Rm >> sh) <= totR;
    j = ok ? c : j;
  }
  // the swapping left stops are the left stops below the cut: in this lane the left
  // stops of its first j positions.  One scan gives the cut and their count nsw.
  const uint32_t SLm = Lm & ~lowbits(E - j);
  const uint32_t cj = (uint32_t)j | ((uint32_t)__popc(SLm) << 16);
  const uint32_t sums = g_sum(cj);
  const int cut = b + (int)(sums & 0xFFFFu);
  const uint32_t nsw = sums >> 16;
  // the exchange: every swapping left stop publishes its position at HP + its rank,
  // every swapping right stop (the nsw highest right stops) at its rank from the top,
  // the rest at the lane's trash slot; then the t-th pairs trade elements, 16 pairs a
  // row at a time (only the swaps move: ~range/4 of the positions)
  // (u8 slots: the slot values are LDS byte addresses, the base folded into the
  // popcount accumulations)
  const uint32_t ob = NP <= 256 ? (uint32_t)(size_t)g.P : 0u;
  const uint32_t trash = ob + 2 * HP + gl, lbase = ob + HP + PL, rbase = ob + totR - PR, rlim = ob + nsw;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int sh = E - 1 - e;
    const uint32_t tl = lbase + (uint32_t)__popc((Lm >> sh) >> 1);
    const uint32_t tr = rbase - (uint32_t)__popc(Rm >> sh);
    // branch-free: slot = swapping left stop ? tl : (swapping right stop ? tr : trash)
    const uint32_t rsw = ((Rm >> sh) & 1u) & (uint32_t)(tr < rlim);
    uint32_t slot = rsw ? tr : trash;
    slot = ((SLm >> sh) & 1u) ? tl : slot;
    if constexpr (NP <= 256) *(lu8*)(size_t)slot = (uint8_t)(lb + e);
    else p_put<NP>(g, slot, (uint32_t)(lb + e));
  }
  wave_lds_sync();
  for (uint32_t t = gl; __builtin_amdgcn_ballot_w64(t < nsw) != 0; t += 16) {
    if (t < nsw) {
      const uint32_t y = p_get<NP>(g, t), x = p_get<NP>(g, HP + t);
      const El ax = g.A[x], ay = g.A[y];
      g.A[x] = ay;
      g.A[y] = ax;
    }
  }
  wave_lds_sync();
  return cut;
}

// one partition of [f, l) on every row with act, in the narrowest window (16 E
// positions from an even base at or below f) that holds every acting row's range.
// The base is min(f & ~1, NPA - 16 E); a range fits iff need = l - (f & ~1) <= 16 E
// (when the base is clamped, l <= NPA makes it fit anyway), so each candidate width
// costs one compare of the precomputed need.
template <int E, int NP, typename El>
__device__ __forceinline__ bool grp_try(const GrpRow<El>& g, int f, int l, int need, bool act, int gl, int& cut) {
  if (16 * E > NP || 16 * E > g.npa) return false;
  if (__builtin_amdgcn_ballot_w64(need > 16 * E) != 0) return false;
  cut = grp_partition<E, NP, El>(g, f, l, min(f & ~1, g.npa - 16 * E), act, gl);
  return true;
}
template <int NP, typename El>
__device__ __forceinline__ int grp_partition_any(const GrpRow<El>& g, int f, int l, bool act, int gl) {
  int cut = 0;
  const int need = act ? l - (f & ~1) : 0;
  if (grp_try<2, NP, El>(g, f, l, need, act, gl, cut) || grp_try<4, NP, El>(g, f, l, need, act, gl, cut) ||
      grp_try<6, NP, El>(g, f, l, need, act, gl, cut) || grp_try<8, NP, El>(g, f, l, need, act, gl, cut) ||
      grp_try<10, NP, El>(g, f, l, need, act, gl, cut) || grp_try<12, NP, El>(g, f, l, need, act, gl, cut) ||
      grp_try<14, NP, El>(g, f, l, need, act, gl, cut) || grp_try<16, NP, El>(g, f, l, need, act, gl, cut) ||
      grp_try<24, NP, El>(g, f, l, need, act, gl, cut))
    return cut;
  if constexpr (NP >= 512) cut = grp_partition<32, NP, El>(g, f, l, min(f & ~1, g.npa - 512), act, gl);
  return cut;
}

// stable rank of [0, m) (m <= 16 EP): lane gl holds positions EP gl + e; a position's
// rank counts the keys greater than its own and the equal keys before it
template <int EP, typename El>
__device__ __forceinline__ void grp_rank_prefix(const GrpRow<El>& g, int m, bool valid, int gl) {
  const int z0 = EP * gl;
  uint32_t r[EP];
  if constexpr (sizeof(El) == 8) {
    uint32_t K[EP], I[EP];
#pragma unroll
    for (int e = 0; e < EP; e += 2) {
      const u32x4 v = *(const lu128*)(g.A + z0 + e);
      I[e] = v.x;
      K[e] = v.y;
      I[e + 1] = v.z;
      K[e + 1] = v.w;
      r[e] = r[e + 1] = 0u;
    }
    // composites (key << 32 | 0xFFFF - position): unique, larger for the earlier of two
    // equal keys, so a position's rank is the number of larger composites
    uint64_t C[EP];
#pragma unroll
    for (int e = 0; e < EP; ++e) C[e] = ((uint64_t)K[e] << 32) | (uint32_t)(0xFFFF - (z0 + e));
    for (int w = 0; w < m; ++w) {
      const uint64_t cw = (g.A[w] & 0xFFFFFFFF00000000ull) | (uint32_t)(0xFFFF - w);
#pragma unroll
      for (int e = 0; e < EP; ++e) r[e] = g_add_gt(r[e], cw, C[e]);
    }
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < EP; ++e)
      if (valid && z0 + e < m) g.A[r[e]] = pack_ki(K[e], I[e]);
  } else {
    // packed: composites (element & ~0xFF) | 255 - position (m <= 64)
    uint32_t X[EP], C[EP];
#pragma unroll
    for (int e = 0; e < EP; e += 2) {
      const uint64_t v = *(const __attribute__((address_space(3))) uint64_t*)(g.A + z0 + e);
      X[e] = (uint32_t)v;
      X[e + 1] = (uint32_t)(v >> 32);
      r[e] = r[e + 1] = 0u;
    }
#pragma unroll
    for (int e = 0; e < EP; ++e) C[e] = (X[e] & ~0xFFu) | (uint32_t)(255 - (z0 + e));
    for (int w = 0; w < m; ++w) {
      const uint32_t cw = (g.A[w] & ~0xFFu) | (uint32_t)(255 - w);
#pragma unroll
      for (int e = 0; e < EP; ++e) r[e] = g_add_gt32(r[e], cw, C[e]);
    }
    wave_lds_sync();
#pragma unroll
    for (int e = 0; e < EP; ++e)
      if (valid && z0 + e < m) g.A[r[e]] = X[e];
  }
}

// stable rank of each queued segment (2..16 elements), one lane per segment: the rank
// of element i counts the later elements with a larger key and the earlier ones with a
// larger or equal key -- r[i] starts at i and each pair (i < j) moves one count with
// one 32-bit compare (few registers live: the elements are re-read for the moves)
template <typename El>
__device__ __forceinline__ void grp_rank_segments(const GrpRow<El>& g, int ns, int gl) {
  if (gl < ns) {
    const uint32_t sg = g.seg[gl];
    const int f = (int)(sg & 0xFFFFu), len = (int)(sg >> 16) - f;
    uint32_t kk[16], kr[16], r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (sizeof(El) == 8) {
        kk[i] = i < len ? ((const lu32*)g.A)[2 * (f + i) + 1] : 0u;  // key 0 sorts after every real key
        kr[i] = kk[i];
      } else {
        kk[i] = i < len ? (uint32_t)g.A[f + i] : 0u;  // packed: key(j) > key(i) <=> x_j > (x_i | 0xFF)
        kr[i] = kk[i] | 0xFFu;
      }
      r[i] = (uint32_t)i;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) {
#pragma unroll
      for (int j = i + 1; j < 16; ++j) g_pair_rank(r[i], r[j], kk[j], kr[i]);
    }
    El x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = i < len ? (El)g.A[f + i] : (El)0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (i < len) g.A[f + r[i]] = x[i];
  }
}

// ---- the whole top-k ----------------------------------------------------------
// std::nth_element(begin, begin + k - 1, end) then std::sort(begin, begin + k - 1)
// (or std::partial_sort when k*64 <= n) on every row of the wave.  One loop drives
// both: each trip, every row settles its bookkeeping (exec-divergent, cheap) and then
// every row with a pending range takes part in ONE partition step, so rows still in
// the selection and rows already sorting share the wave's steps.  Afterwards
// GEl<El>::idx(g.A[p]), p < k, is torch's p-th index.
// QM: 0 = the final sort decided at run time, 1 = k - 1 <= 64 (the whole prefix ranked
// at once), 2 = k - 1 > 64 (final segments queued and ranked one lane each) -- the fixed
// forms leave the other ranking code (and its registers) out of the kernel.
// TW > 0 (packed rows, k + 2 <= TW): once a row's introselect range lies in [0, TW) --
// or its selection ended at the depth limit -- the row is handed over to the one-lane
// tail (mxa_tail.hpp) instead of finished here: *hand = its tail state (f | l << 8 |
// d << 16 | phase << 24, phase 0 the introselect on [f, l), 1 the sort of [0, k-1)),
// g.A[0, TW) its prefix; the sort phase and the final ranks never run here.
struct GrpHand {
  uint32_t state;
  bool on;
};
template <int NP, typename El = uint64_t, int QM = 0, int TW = 0>
__device__ __forceinline__ void grp_topk(const GrpRow<El>& g, int n, int k, bool valid, int gl, GrpHand* hand = nullptr) {
  if (k <= 0) return;
  if (k * 64 <= n) {  // std::partial_sort(begin, begin + k, end)
    if (valid && gl == 0) {
      ln_heap_select(g.A, 0, k, n);
      ln_sort_heap(g.A, 0, k);
    }
    wave_lds_sync();
    return;
  }
  const int nth = k - 1, m = k - 1;
  const bool queue = QM == 0 ? m > 64 : QM == 2;  // final sort segments ranked one lane each (else the whole prefix)
  int ph = valid ? 0 : 2;     // 0 __introselect, 1 __introsort_loop, 2 done
  int f = 0, l = n, d = 2 * ilog2(n), sp = 0, ns = 0;
  while (true) {
    if (TW > 0 && ph == 0 && l <= TW) {  // the rest fits the tail's prefix: hand it over
      hand->state = (uint32_t)f | ((uint32_t)l << 8) | ((uint32_t)d << 16);
      hand->on = true;
      ph = 2;
    }
    if (ph == 0 && (l - f <= 3 || d == 0)) {  // the selection ends
      if (l - f > 3) {  // depth limit: __heap_select(f, nth + 1, l); iter_swap(f, nth)
        if (gl == 0) {
          ln_heap_select(g.A, f, nth + 1, l);
          const El t = g.A[f];
          g.A[f] = g.A[nth];
          g.A[nth] = t;
        }
      } else if (l - f > 1 && gl == 0) {
        ln_insertion_sort(g.A, f, l);  // __insertion_sort(f, l)
      }
      ph = m > 16 ? 1 : 2;
      f = 0;
      l = m;
      d = m > 1 ? 2 * ilog2(m) : 0;
      if (TW > 0) {  // the sort of [0, k-1) to the tail
        hand->state = 1u << 24;
        hand->on = true;
        ph = 2;
      }
    }
    if (ph == 1) {
      // settle: finished segments (<= 16 elements, or heap-sorted at the depth limit)
      while (l - f <= 16 || d == 0) {
        if (l - f > 16) {  // std::__partial_sort(f, l, l): heapsort, final as it stands
          if (gl == 0) {
            ln_heap_select(g.A, f, l, l);
            ln_sort_heap(g.A, f, l);
          }
        } else if (QM != 1 && queue && l - f >= 2) {
          g.seg[ns] = (uint32_t)f | ((uint32_t)l << 16);
          ++ns;
          if (ns == kGSeg) {
            wave_lds_sync();
            grp_rank_segments(g, ns, gl);
            ns = 0;
          }
        }
        if (sp == 0) {
          ph = 2;
          break;
        }
        --sp;
        const uint32_t e = g.stk[sp];
        f = (int)(e & 1023u);
        l = (int)((e >> 10) & 1023u);
        d = (int)(e >> 20);
      }
    }
    const bool act = ph < 2;
    if (__builtin_amdgcn_ballot_w64(act) == 0) break;
    wave_lds_sync();
    const int cut = grp_partition_any<NP>(g, f, l, act, gl);
    if (act) {
      --d;
      if (ph == 0) {
        if (cut <= nth) f = cut;
        else l = cut;
      } else {
        g.stk[sp] = (uint32_t)cut | ((uint32_t)l << 10) | ((uint32_t)d << 20);  // __introsort_loop(cut, l)
        ++sp;
        l = cut;
      }
    }
  }
  wave_lds_sync();
  if constexpr (TW == 0) {
    if (QM != 1 && queue) {
      if (valid && ns > 0) grp_rank_segments(g, ns, gl);
    } else if (QM != 2 && m >= 2) {
      if (m <= 32) grp_rank_prefix<2>(g, m, valid, gl);
      else grp_rank_prefix<4>(g, m, valid, gl);
    }
    wave_lds_sync();
  }
}

}  // namespace mxa
