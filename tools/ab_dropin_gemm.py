"""Same-box timing of mx.matmul at the drop-in's DeiT-base shapes (QK^T 197 x 197 x 64 and
P.V 197 x 64 x 197, 3072 heads) for the library in MXA_LIB (tools-only A/B)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import mx_quantization_amd as M

mx, _ = M.install_dropin()
specs = {"a_elem_format": "int8", "w_elem_format": "int8", "block_size": 32, "scale_bits": 8, "bfloat": 32}
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(256, 12, 197, 64, device="cuda", generator=g)
k = torch.randn(256, 12, 197, 64, device="cuda", generator=g)
v = torch.randn(256, 12, 197, 64, device="cuda", generator=g)
p = torch.rand(256, 12, 197, 197, device="cuda", generator=g)
p = p * (p > 0.9)
for name, fn in (("qk", lambda: mx.matmul(q, k.transpose(-2, -1), mx_specs=specs)),
                 ("pv", lambda: mx.matmul(p, v, mx_specs=specs))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    print(os.environ.get("MXA_LIB", "default"), name, f"{(time.perf_counter() - t) / 10 * 1e3:.3f} ms")
