"""Executable model of the one-wave-per-row top-k (mx_quantization_amd/csrc/mxa_topk_wave.hpp),
step for step: the rank-form partition (stop masks, inclusive prefix counts, slot
tables, cut = first + 1 + #{T <= totR}), the introselect / introsort drivers with the
pending-range stack, the boundary bits and the stable rank within each final segment.
tests/test_topk_model.py checks it against oracle/topk_ref.cpp (libstdc++)."""
from __future__ import annotations

import numpy as np

from tools.topk_model import Row, keys_from_f32, lg


def w_partition(r: Row, f: int, l: int) -> int:
    mid = f + ((l - f) >> 1)
    ka, kb, kc = r.k[f + 1], r.k[mid], r.k[l - 1]
    if ka > kb:
        ms = 2 if kb > kc else (3 if ka > kc else 1)
    else:
        ms = 1 if ka > kc else (3 if kb > kc else 2)
    m = {1: f + 1, 2: mid, 3: l - 1}[ms]
    r.swap(f, m)
    p = r.k[f]
    pos = np.arange(f + 1, l)
    key = r.k[f + 1:l]
    isL, isR = key <= p, key >= p
    totR = int(isR.sum())
    PLi, PRi = np.cumsum(isL), np.cumsum(isR)
    ok = PLi + PRi <= totR
    ncut, nsw = int(ok.sum()), int((ok & isL).sum())
    SL = np.zeros(l - f, dtype=np.int64)
    SR = np.zeros(l - f, dtype=np.int64)
    SL[PLi[isL] - 1] = pos[isL]
    SR[totR - PRi[isR]] = pos[isR]
    x, y = SL[:nsw], SR[:nsw]
    assert len(set(x.tolist()) | set(y.tolist())) == 2 * nsw
    kk, ii = r.k.copy(), r.i.copy()
    r.k[x], r.k[y] = kk[y], kk[x]
    r.i[x], r.i[y] = ii[y], ii[x]
    return f + 1 + ncut


def wave_topk(vals, k: int) -> np.ndarray:
    r = Row(keys_from_f32(vals))
    n = len(vals)
    if k * 64 <= n:
        r.partial_sort(k)
        return r.i[:k].copy()
    nth = m = k - 1
    f, l, d = 0, n, 2 * lg(n)
    heap = False
    while l - f > 3:
        if d == 0:
            heap = True
            break
        d -= 1
        cut = w_partition(r, f, l)
        if cut <= nth:
            f = cut
        else:
            l = cut
    if heap:
        r.heap_select(f, nth + 1, l)
        r.swap(f, nth)
    elif l - f > 1:
        r.stable_sort(f, l)
    if m < 2:
        return r.i[:k].copy()
    bnd = {0, m}
    maxlen = 0
    stk = []
    f, l, d = 0, m, 2 * lg(m)
    while True:
        while l - f > 16 and d > 0:
            d -= 1
            cut = w_partition(r, f, l)
            bnd.add(cut)
            stk.append((cut, l, d))
            l = cut
        if l - f > 16:
            r.heap_select(f, l, l)
            r.sort_heap(f, l)
            bnd.update(range(f + 1, l))
        else:
            maxlen = max(maxlen, l - f)
        if not stk:
            break
        f, l, d = stk.pop()
    if maxlen >= 2:
        b = sorted(bnd)
        kk, ii = r.k.copy(), r.i.copy()
        for s, t in zip(b[:-1], b[1:]):
            assert t - s <= 16 or all(c in bnd for c in range(s, t))
            comp = [(int(kk[z]) << 32) | (0xFFFF - z) for z in range(s, t)]
            for zi, z in enumerate(range(s, t)):
                rank = s + sum(1 for w in comp if w > comp[zi])
                r.k[rank], r.i[rank] = kk[z], ii[z]
    return r.i[:k].copy()
