"""Fused attention on a bench config through both fused kernels (for rocprofv3
--pmc / --kernel-trace): the row-oriented kernel and the MFMA score-tile kernel
(MXA_ATTN_PATH=tiles); plus the standalone top-k on the same approximate scores."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import mx_quantization_amd as M

cfg = sys.argv[1] if len(sys.argv) > 1 else "deit_base"
paths = sys.argv[2].split(",") if len(sys.argv) > 2 else ["rows", "tiles"]
B, H, N, D, k = {"deit_base": (256, 12, 197, 64, 20), "dit_xl2": (64, 16, 256, 72, 154)}[cfg]
q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, N, D), dtype=np.float32)).cuda()
            for s in range(3))
for path in paths:
    if path == "tiles":
        os.environ["MXA_ATTN_PATH"] = "tiles"
    else:
        os.environ.pop("MXA_ATTN_PATH", None)
    for _ in range(2):
        out, idx = M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k)
    torch.cuda.synchronize()
os.environ.pop("MXA_ATTN_PATH", None)
out, idx, t, p = M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k, return_scores=True)
rows = p.reshape(-1, N).contiguous()
for _ in range(2):
    M.topk(rows, k)
torch.cuda.synchronize()
print("done", cfg, paths)
