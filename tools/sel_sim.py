"""Trip statistics of the selection kernel's exact-order top-k (tools-only cost model).

Replays grp_topk (mxa_topk_grp.hpp) on ex_pred score rows with the partition model
of tools/topk_model.py: per group of G rows in lockstep, each trip every row with a
pending range takes one partition step in the narrowest common window.  Prints trips
per group and the window-width histogram, per policy.

  python tools/sel_sim.py deit_base|dit_xl2 [images] [G]
"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import mx_oracle as O  # noqa: E402
from tools.topk_model import Row, keys_from_f32, lg  # noqa: E402

WIDTHS = (2, 4, 6, 8, 10, 12, 14, 16, 24, 32)


def rows_of(cfg, images):
    import bench
    c = bench.CONFIGS[cfg]
    out = []
    for i in range(images):
        q, k, _ = bench.image_inputs(c, i)
        aq, ak = O.approx_operands(q, k, "ex_pred")
        pred = O.exact_matmul_f32(aq, np.swapaxes(ak, -1, -2))
        out.append(pred.reshape(-1, c["T"]))
    return np.concatenate(out), c["k"]


class RowState:
    """One row's grp_topk bookkeeping; step() is one partition of the pending range."""

    def __init__(self, vals, k):
        self.r = Row(keys_from_f32(vals))
        n = len(vals)
        self.n, self.k, self.nth, self.m = n, k, k - 1, k - 1
        self.ph, self.f, self.l, self.d = 0, 0, n, 2 * lg(n)
        self.stk = []
        self.queue = self.m > 64
        self.steps = collections.Counter()

    def settle(self):
        if self.ph == 0 and (self.l - self.f <= 3 or self.d == 0):
            if self.l - self.f > 3:
                self.r.heap_select(self.f, self.nth + 1, self.l)
                self.r.swap(self.f, self.nth)
            else:
                self.r.stable_sort(self.f, self.l)
            self.ph = 1 if self.m > 16 else 2
            self.f, self.l = 0, self.m
            self.d = 2 * lg(self.m) if self.m > 1 else 0
        if self.ph == 1:
            while self.l - self.f <= 16 or self.d == 0:
                if self.l - self.f > 16:
                    self.r.heap_select(self.f, self.l, self.l)
                    self.r.sort_heap(self.f, self.l)
                if not self.stk:
                    self.ph = 2
                    break
                self.f, self.l, self.d = self.stk.pop()

    def need(self):
        return self.l - (self.f & ~1)

    def step(self):
        cut = self.r.partition_pivot(self.f, self.l)
        self.d -= 1
        if self.ph == 0:
            if cut <= self.nth:
                self.f = cut
            else:
                self.l = cut
        else:
            self.stk.append((cut, self.l, self.d))
            self.l = cut


def simulate(P, k, G):
    trips = []
    hist = collections.Counter()
    per_row = []
    for g0 in range(0, len(P), G):
        rs = [RowState(v, k) for v in P[g0:g0 + G]]
        t = 0
        while True:
            for s in rs:
                s.settle()
            act = [s for s in rs if s.ph < 2]
            if not act:
                break
            need = max(s.need() for s in act)
            E = next((e for e in WIDTHS if 16 * e >= need), 32)
            hist[E] += 1
            for s in act:
                s.step()
            t += 1
        trips.append(t)
    for v in P[:min(len(P), 4096)]:
        s = RowState(v, k)
        n = 0
        while True:
            s.settle()
            if s.ph == 2:
                break
            s.step()
            n += 1
        per_row.append(n)
    return np.array(trips), hist, np.array(per_row)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "deit_base"
    images = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    G = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    P, k = rows_of(cfg, images)
    trips, hist, per_row = simulate(P, k, G)
    print(f"{cfg}: rows {len(P)}, k {k}, G {G}: trips/group mean {trips.mean():.2f} max {trips.max()}; "
          f"steps/row alone mean {per_row.mean():.2f}; lockstep overhead {trips.mean() / per_row.mean() - 1:.1%}")
    tot = sum(hist.values())
    print("window E histogram (per group trip):", {e: round(c / len(trips), 2) for e, c in sorted(hist.items())},
          "positions/trip", round(sum(16 * e * c for e, c in hist.items()) / tot, 1))


if __name__ == "__main__":
    main()
