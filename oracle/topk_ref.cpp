// ORACLE — test infrastructure only.  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker.
//
// CPU restatement of torch's CPU top-k (the call the reference's attention
// modules make: `torch.topk(pred, k, dim=-1, largest=True, sorted=True)`,
// workloads/deit/scripts/main.py:123, workloads/DiT/models.py:194,
// workloads/PixArt/models/MX_transformer_block.py:678,:825).
//
// Third-party algorithm (absent from /root/reference): PyTorch 2.10
// aten/src/ATen/native/TopKImpl.h:45-86, compiled by PyTorch with
// gcc-toolset-11 (libstdc++ 11).  Per row it fills a vector of
// pair<double,int64> and calls
//     k*64 <= n : std::partial_sort(begin, begin+k, end, cmp)
//     else      : std::nth_element(begin, begin+k-1, end, cmp);
//                 if sorted: std::sort(begin, begin+k-1, cmp)
// with cmp(x,y) = (isnan(x) && !isnan(y)) || x > y   (largest=True).
// We call the same libstdc++ algorithms (g++ 11.4 here), which reproduced
// torch's index order for 100% of probe rows and is pinned by
// tests/golden/topk_ties.npz.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

namespace {
using elem_t = std::pair<double, int64_t>;

inline bool cmp_largest(const elem_t& x, const elem_t& y) {
  return (std::isnan(x.first) && !std::isnan(y.first)) || (x.first > y.first);
}
inline bool cmp_smallest(const elem_t& x, const elem_t& y) {
  return (!std::isnan(x.first) && std::isnan(y.first)) || (x.first < y.first);
}
}  // namespace

extern "C" {

// vals: rows x n float32 (row stride `ld` elements).  Writes k indices (int64)
// and values (float32) per row.  Returns 0 on success.
int oracle_topk_f32(const float* vals, int64_t rows, int64_t n, int64_t ld, int64_t k,
                    int largest, int sorted, int64_t* out_idx, float* out_vals) {
  if (k < 0 || k > n) return -1;
  if (k == 0) return 0;
  std::vector<elem_t> queue(n);
  const bool use_partial_sort = k * 64 <= n;
  for (int64_t r = 0; r < rows; ++r) {
    const float* row = vals + r * ld;
    for (int64_t j = 0; j < n; ++j) {
      queue[j].first = row[j];
      queue[j].second = j;
    }
    if (use_partial_sort) {
      if (largest)
        std::partial_sort(queue.begin(), queue.begin() + k, queue.end(), cmp_largest);
      else
        std::partial_sort(queue.begin(), queue.begin() + k, queue.end(), cmp_smallest);
    } else {
      if (largest) {
        std::nth_element(queue.begin(), queue.begin() + k - 1, queue.end(), cmp_largest);
        if (sorted) std::sort(queue.begin(), queue.begin() + k - 1, cmp_largest);
      } else {
        std::nth_element(queue.begin(), queue.begin() + k - 1, queue.end(), cmp_smallest);
        if (sorted) std::sort(queue.begin(), queue.begin() + k - 1, cmp_smallest);
      }
    }
    for (int64_t j = 0; j < k; ++j) {
      if (out_idx) out_idx[r * k + j] = queue[j].second;
      if (out_vals) out_vals[r * k + j] = static_cast<float>(queue[j].first);
    }
  }
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Test-input generator: McIlroy's "killer adversary" (A Killer Adversary for
// Quicksort, 1999) run against the same libstdc++ nth_element + sort that
// torch's top-k uses.  Produces rows that exhaust introselect's/introsort's
// depth limit, so the heap_select / heapsort fallbacks get exercised.
// out[n] receives values such that std::nth_element(.., k-1, .., greater) on
// them degenerates.
namespace {
struct Adversary {
  std::vector<int64_t> val;
  int64_t gas, nsolid = 0, candidate = 0;
  explicit Adversary(int64_t n) : val(n, n), gas(n) {}
  void freeze(int64_t x) { val[x] = nsolid++; }
  // "less" on item ids with lazy value assignment
  bool less(int64_t x, int64_t y) {
    if (val[x] == gas && val[y] == gas) {
      if (x == candidate) freeze(x); else freeze(y);
    }
    if (val[x] == gas) candidate = x;
    else if (val[y] == gas) candidate = y;
    return val[x] < val[y];
  }
};
}  // namespace

extern "C" int oracle_antiqsort(int64_t n, int64_t k, int with_sort, float* out) {
  if (k < 1 || k > n) return -1;
  Adversary adv(n);
  std::vector<int64_t> ids(n);
  for (int64_t i = 0; i < n; ++i) ids[i] = i;
  auto cmp = [&](int64_t x, int64_t y) { return adv.less(x, y); };
  std::nth_element(ids.begin(), ids.begin() + k - 1, ids.end(), cmp);
  if (with_sort) std::sort(ids.begin(), ids.begin() + k - 1, cmp);
  // the adversary built an input bad for "less"; negate for torch's "greater"
  for (int64_t i = 0; i < n; ++i) out[i] = -static_cast<float>(adv.val[i]);
  return 0;
}
