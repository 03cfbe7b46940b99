"""Time the lane-per-row top-k (MXA_LANE_CFG = WAVESxTAILW, MXA_TOPK_DBG skip bits)
against the register-resident one on the kernel's DeiT-base / DiT approximate scores."""
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


cfgs = {"deit_base": (256, 12, 197, 64, 20), "dit_xl2": (64, 16, 256, 72, 154), "deit30": (256, 12, 197, 64, 30)}
for cfg in sys.argv[1].split(",") if len(sys.argv) > 1 else ["deit_base"]:
    B, H, N, D, k = cfgs[cfg]
    q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, N, D), dtype=np.float32)).cuda()
                for s in range(3))
    out, idx, t, p = M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k, return_scores=True)
    rows = p.reshape(-1, N).contiguous()
    res = {}
    os.environ["MXA_TOPK_IMPL"] = "reg"
    res["reg"] = timeit(lambda: M.topk(rows, k))
    ref = M.topk(rows, k)[1]
    os.environ["MXA_TOPK_IMPL"] = "lane"
    for lc in os.environ.get("LANE_CFGS", "4x1,4x4,8x1,8x2,8x8,16x16").split(","):
        os.environ["MXA_LANE_CFG"] = lc
        for dbg in (0, 1, 2, 3):
            os.environ["MXA_TOPK_DBG"] = str(dbg)
            res[f"{lc}/d{dbg}"] = timeit(lambda: M.topk(rows, k))
        os.environ["MXA_TOPK_DBG"] = "0"
        assert torch.equal(M.topk(rows, k)[1], ref), lc
    print(cfg, res, flush=True)
