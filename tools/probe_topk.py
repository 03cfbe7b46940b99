"""GPU probe: time the phases of the fused op and the standalone top-k variants
(DeiT-base / DiT-XL/2 shapes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import mx_quantization_amd as M


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def with_env(var, val, fn):
    old = os.environ.get(var)
    os.environ[var] = val
    try:
        return fn()
    finally:
        if old is None:
            os.environ.pop(var)
        else:
            os.environ[var] = old


for name, (B, H, N, D, k, sc) in {"deit": (256, 12, 197, 64, 20, 0.125),
                                   "dit": (64, 16, 256, 72, 154, 72 ** -0.5)}.items():
    q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, N, D), dtype=np.float32)).cuda()
                for s in range(3))
    out, idx, t, p = M.mx_topk_attention(q, kk, v, sc, k_top=k, return_scores=True)
    rows = p.reshape(-1, N).contiguous()
    r = {}
    r["fused_rows"] = timeit(lambda: M.mx_topk_attention(q, kk, v, sc, k_top=k))
    r["fused_tiles"] = with_env("MXA_ATTN_PATH", "tiles", lambda: timeit(lambda: M.mx_topk_attention(q, kk, v, sc, k_top=k)))
    r["fused_dense"] = timeit(lambda: M.mx_topk_attention(q, kk, v, sc, k_top=k, top_k=False))
    r["topk_v2"] = timeit(lambda: M.topk(rows, k))
    r["topk_v1"] = with_env("MXA_TOPK_V1", "1", lambda: timeit(lambda: M.topk(rows, k)))
    r["torch_topk_gpu"] = timeit(lambda: torch.topk(rows, k, dim=-1))
    i2 = M.topk(rows, k)[1]
    i1 = with_env("MXA_TOPK_V1", "1", lambda: M.topk(rows, k)[1])
    iw = with_env("MXA_ATTN_PATH", "tiles", lambda: M.mx_topk_attention(q, kk, v, sc, k_top=k)[1])
    print(name, {a: round(b, 3) for a, b in r.items()}, "v1==v2", bool(torch.equal(i1, i2)),
          "fused==standalone", bool(torch.equal(i2.view(idx.shape), idx)), "rows==tiles", bool(torch.equal(iw, idx)),
          flush=True)
