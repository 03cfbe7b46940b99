"""Standalone exact top-k on DeiT-base-shaped ex_pred score rows (for rocprofv3 --pmc)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import mx_quantization_amd as M
B, H, N, D, k = 256, 12, 197, 64, 20
q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, N, D), dtype=np.float32)).cuda() for s in range(3))
out, idx, t, p = M.mx_topk_attention(q, kk, v, 0.125, k_top=k, return_scores=True)
rows = p.reshape(-1, N).contiguous()
for _ in range(3):
    M.topk(rows, k)
torch.cuda.synchronize()
print("rows", rows.shape[0])
