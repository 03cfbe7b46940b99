"""Run the fused qkv-projection attention (DeiT-base or DiT block shape) a few times,
for rocprofv3 kernel traces / PMC passes (tools-only)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mx_quantization_amd as M

cfg = sys.argv[1] if len(sys.argv) > 1 else "deit_base"
B, N, H, D, k = (256, 197, 12, 64, 20) if cfg == "deit_base" else (64, 256, 16, 72, 154)
C = H * D
rng = np.random.default_rng(1)
x = torch.from_numpy(rng.standard_normal((B, N, C), dtype=np.float32)).cuda()
W = torch.from_numpy(rng.standard_normal((3 * C, C), dtype=np.float32) * np.float32(C ** -0.5)).cuda()
b = torch.from_numpy(rng.standard_normal(3 * C, dtype=np.float32) * np.float32(0.02)).cuda()
wq = M.LinearWeightMX(W, D)
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    out, idx = M.mx_qkv_attention(x, wq, b, H, D ** -0.5, k_top=k)
torch.cuda.synchronize()
print("ok", float(out.float().abs().mean()))
