"""Standalone top-k on the kernel's DeiT-base / DiT approximate scores (for rocprofv3 --pmc)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import mx_quantization_amd as M

cfg = sys.argv[1] if len(sys.argv) > 1 else "deit_base"
B, H, N, D, k = {"deit_base": (256, 12, 197, 64, 20), "dit_xl2": (64, 16, 256, 72, 154)}[cfg]
q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, N, D), dtype=np.float32)).cuda()
            for s in range(3))
out, idx, t, p = M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k, return_scores=True)
rows = p.reshape(-1, N).contiguous()
for _ in range(2):
    M.topk(rows, k)
torch.cuda.synchronize()
