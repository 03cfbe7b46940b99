"""Time the standalone top-k implementations (MXA_TOPK_IMPL reg / lds) on the
kernel's own DeiT-base / DiT approximate scores, and the fused op per path."""
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
    return round(s.elapsed_time(e) / reps, 3)


cfgs = {"deit_base": (256, 12, 197, 64, 20), "dit_xl2": (64, 16, 256, 72, 154)}
for cfg in sys.argv[1].split(",") if len(sys.argv) > 1 else cfgs:
    B, H, N, D, k = cfgs[cfg]
    q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, N, D), dtype=np.float32)).cuda()
                for s in range(3))
    out, idx, t, p = M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k, return_scores=True)
    rows = p.reshape(-1, N).contiguous()
    res = {}
    for impl in ("lane", "reg", "lds"):
        os.environ["MXA_TOPK_IMPL"] = impl
        res["topk_" + impl] = timeit(lambda: M.topk(rows, k))
    os.environ.pop("MXA_TOPK_IMPL")
    for path in ("rows", "rows1"):
        os.environ["MXA_ATTN_PATH"] = path
        res["attn_" + path] = timeit(lambda: M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k))
    os.environ.pop("MXA_ATTN_PATH")
    print(cfg, res, flush=True)
