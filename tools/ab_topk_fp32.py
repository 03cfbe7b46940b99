"""ops.topk on arbitrary float32 rows (random normal: almost no value leaves the packed key's
low byte free) through the workspace path (mxa_topk_ws: packed pass, tail, 64-bit pass over the
rows it leaves) against mxa_topk alone (the 64-bit pass), and on ex_pred-like rows that pack
(small integers times powers of two).  ADVICE round 5; tools-only timing."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mx_quantization_amd as M

rows, n, k = 256 * 12 * 197, 197, 20
g = torch.Generator(device="cuda").manual_seed(0)
cases = {"randn": torch.randn(rows, n, device="cuda", generator=g),
         "packable": torch.randint(-32, 33, (rows, n), device="cuda", generator=g).float() *
         torch.exp2(torch.randint(-4, 4, (rows, n), device="cuda", generator=g).float())}
for name, x in cases.items():
    def direct():
        return M.topk(x, k, packed=False)

    res = {}
    for lbl, fn in (("ws", lambda: M.topk(x, k)), ("direct", direct)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        res[lbl] = (time.perf_counter() - t) / 5 * 1e3
    same = torch.equal(M.topk(x, k)[1], direct()[1])
    print(name, {k_: round(v, 3) for k_, v in res.items()}, "ms", "idx equal:", same)
