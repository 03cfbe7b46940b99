"""Time the row-oriented fused kernel with phases switched off (instrumented
build libmxa_prof.so, MXA_DBG_SKIP bits: 1 top-k, 2 P quant/store, 4 scoring,
8 true-score gather, 16 the sort of the kept prefix) -- shows which phase the kernel's time depends on."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MXA_LIB"] = os.path.join(ROOT, "mx_quantization_amd", "libmxa_prof.so")
sys.path.insert(0, ROOT)
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


for cfg, (B, H, Nq, D, k) in {"deit_base": (256, 12, 197, 64, 20), "dit_xl2": (64, 16, 256, 72, 154)}.items():
    q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, Nq, D), dtype=np.float32)).cuda()
                for s in range(3))
    res = {}
    for skip in [int(x) for x in os.environ.get("SKIPS", "0,1,2,4,8,16,3,9,11,15").split(",")]:
        os.environ["MXA_DBG_SKIP"] = str(skip)
        res[skip] = round(timeit(lambda: M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k)), 3)
    os.environ.pop("MXA_DBG_SKIP")
    print(cfg, "ms by skipped phases:", res, flush=True)
