"""Executable model of the HIP top-k (mx_quantization_amd/csrc/mxa_topk.hip).

It reproduces torch's CPU `topk(largest=True, sorted=True)` index order
(TopKImpl.h:45-86 -> libstdc++ 11 nth_element + sort, or partial_sort when
k*64 <= n) WITHOUT running the serial algorithms element by element: every
Hoare partition step is computed from per-position flags and prefix counts,
which is what one wavefront does with ballots (SURVEY.md §7 "Hard parts").

Partition of [first, last) around the pivot p at `first` (stl_algo.h
__unguarded_partition, with comp(x, y) = x > y):
  left stop  x in [first+1, last):  !(a[x] > p)
  right stop y in [first, last):    !(p > a[y])
  A(x)   = # left stops  at positions < x      (rank of a left stop)
  Bgt(y) = # right stops at positions > y      (rank of a right stop)
  left stop x swaps  iff Bgt(x) > A(x);  right stop y swaps iff A(y) > Bgt(y)
  the t-th swapping left stop exchanges with the t-th swapping right stop
  cut = min(first non-swapping left stop, lowest swapping right stop)
        (lowest swapping right stop := last when nothing swaps)

std::sort's final insertion sort is a stable sort; because introsort leaves
segments of <= 16 elements that are mutually ordered, it equals a stable sort
of each segment.  The depth-limit fallbacks (heap_select / heapsort) and the
partial_sort branch are serial in the kernel too; here they are restated from
stl_heap.h.

Used by tests/test_topk_model.py to check the model against oracle/topk_ref.cpp.
"""
from __future__ import annotations

import numpy as np


def keys_from_f32(x: np.ndarray) -> np.ndarray:
    """Order-preserving uint32 keys for torch's comparator: NaN largest (all NaNs
    equal), -0 == +0."""
    x = np.asarray(x, dtype=np.float32).copy()
    x[x == 0] = 0.0
    b = x.view(np.uint32).astype(np.uint64)
    k = np.where(b >> 31, (~b) & 0xFFFFFFFF, b | 0x80000000)
    k = np.where(np.isnan(x), 0xFFFFFFFF, k)
    return k.astype(np.uint64)


def lg(n: int) -> int:
    return n.bit_length() - 1


class Row:
    def __init__(self, keys):
        self.k = np.array(keys, dtype=np.uint64)
        self.i = np.arange(len(keys), dtype=np.int64)
        self.fallbacks = 0

    def gt(self, a, b):  # comp(a, b) on positions
        return self.k[a] > self.k[b]

    def swap(self, a, b):
        self.k[[a, b]] = self.k[[b, a]]
        self.i[[a, b]] = self.i[[b, a]]

    # -- parallel-rule partition -------------------------------------------------
    def partition_pivot(self, first, last):
        mid = first + (last - first) // 2
        a, b, c = first + 1, mid, last - 1
        if self.gt(a, b):
            if self.gt(b, c):
                self.swap(first, b)
            elif self.gt(a, c):
                self.swap(first, c)
            else:
                self.swap(first, a)
        elif self.gt(a, c):
            self.swap(first, a)
        elif self.gt(b, c):
            self.swap(first, c)
        else:
            self.swap(first, b)
        p = self.k[first]
        pos = np.arange(first, last)
        seg = self.k[first:last]
        lstop = (seg <= p) & (pos >= first + 1)
        rstop = seg >= p
        A = np.cumsum(lstop) - lstop  # exclusive prefix
        Bgt = rstop[::-1].cumsum()[::-1] - rstop
        swl = lstop & (Bgt > A)
        swr = rstop & (A > Bgt)
        m = int(swl.sum())
        assert m == int(swr.sum())
        lpos = pos[swl]  # ascending: rank t = A
        rpos = pos[swr][::-1]  # descending: rank t = Bgt
        kk, ii = self.k.copy(), self.i.copy()
        self.k[lpos], self.k[rpos] = kk[rpos], kk[lpos]
        self.i[lpos], self.i[rpos] = ii[rpos], ii[lpos]
        nl = pos[lstop & ~swl]
        c1 = int(nl[0]) if len(nl) else 1 << 30
        c2 = int(rpos[-1]) if m else last
        return min(c1, c2)

    def stable_sort(self, first, last):
        if last - first < 2:
            return
        o = np.argsort(-self.k[first:last].astype(np.float64), kind="stable")
        self.k[first:last] = self.k[first:last][o]
        self.i[first:last] = self.i[first:last][o]

    # -- serial heap algorithms (stl_heap.h) ---------------------------------------
    def _push_heap(self, base, hole, top, vk, vi):
        parent = (hole - 1) // 2
        while hole > top and self.k[base + parent] > vk:
            self.k[base + hole], self.i[base + hole] = self.k[base + parent], self.i[base + parent]
            hole = parent
            parent = (hole - 1) // 2
        self.k[base + hole], self.i[base + hole] = vk, vi

    def _adjust_heap(self, base, hole, ln, vk, vi):
        top = hole
        second = hole
        while second < (ln - 1) // 2:
            second = 2 * (second + 1)
            if self.k[base + second] > self.k[base + second - 1]:
                second -= 1
            self.k[base + hole], self.i[base + hole] = self.k[base + second], self.i[base + second]
            hole = second
        if (ln & 1) == 0 and second == (ln - 2) // 2:
            second = 2 * (second + 1)
            self.k[base + hole], self.i[base + hole] = self.k[base + second - 1], self.i[base + second - 1]
            hole = second - 1
        self._push_heap(base, hole, top, vk, vi)

    def _make_heap(self, first, last):
        ln = last - first
        if ln < 2:
            return
        parent = (ln - 2) // 2
        while True:
            self._adjust_heap(first, parent, ln, self.k[first + parent], self.i[first + parent])
            if parent == 0:
                return
            parent -= 1

    def _pop_heap(self, first, last, result):
        vk, vi = self.k[result], self.i[result]
        self.k[result], self.i[result] = self.k[first], self.i[first]
        self._adjust_heap(first, 0, last - first, vk, vi)

    def heap_select(self, first, middle, last):
        self._make_heap(first, middle)
        for i in range(middle, last):
            if self.k[i] > self.k[first]:
                self._pop_heap(first, middle, i)

    def sort_heap(self, first, last):
        while last - first > 1:
            last -= 1
            self._pop_heap(first, last, last)

    # -- algorithms -------------------------------------------------------------
    def nth_element(self, nth, first=0, last=None):
        last = len(self.k) if last is None else last
        if first == last or nth == last:
            return
        depth = 2 * lg(last - first)
        while last - first > 3:
            if depth == 0:
                self.fallbacks += 1
                self.heap_select(first, nth + 1, last)
                self.swap(first, nth)
                return
            depth -= 1
            cut = self.partition_pivot(first, last)
            if cut <= nth:
                first = cut
            else:
                last = cut
        self.stable_sort(first, last)

    def sort(self, first, last):
        if first == last:
            return
        stack = [(first, last, 2 * lg(last - first))]
        while stack:  # segment order is irrelevant: segments are disjoint
            f, l, depth = stack.pop()
            while l - f > 16:
                if depth == 0:
                    self.fallbacks += 1
                    self.heap_select(f, l, l)
                    self.sort_heap(f, l)
                    l = f  # segment finished (heapsort is a full sort)
                    break
                depth -= 1
                cut = self.partition_pivot(f, l)
                stack.append((cut, l, depth))
                l = cut
            if l > f:
                self.stable_sort(f, l)

    def partial_sort(self, middle):
        self.heap_select(0, middle, len(self.k))
        self.sort_heap(0, middle)


def topk_model(vals: np.ndarray, k: int):
    """Index order of torch.topk(vals, k, largest=True, sorted=True) on CPU."""
    r = Row(keys_from_f32(vals))
    n = len(vals)
    if k * 64 <= n:
        r.partial_sort(k)
    else:
        r.nth_element(k - 1)
        r.sort(0, k - 1)
    return r.i[:k].copy(), r.fallbacks
