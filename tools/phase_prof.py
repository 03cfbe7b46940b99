"""Per-phase cycle shares of the row-oriented fused kernel (instrumented build
libmxa_prof.so: python -m mx_quantization_amd.build_native --phase-prof)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MXA_LIB"] = os.path.join(ROOT, "mx_quantization_amd", "libmxa_prof.so")
sys.path.insert(0, ROOT)
import numpy as np
import torch

import mx_quantization_amd as M
from mx_quantization_amd import _native as N

fn = N.lib().mxa_debug_phase_cycles
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
names = ["stage", "scores", "select", "gather+softmax", "P quant", "PV+store", "sort", "-"]
skips = [int(x) for x in os.environ.get("PHASE_SKIPS", "0").split(",")]
for cfg, (B, H, Nq, D, k) in {"deit_base": (256, 12, 197, 64, 20), "dit_xl2": (64, 16, 256, 72, 154)}.items():
    q, kk, v = (torch.from_numpy(np.random.default_rng(s).standard_normal((B, H, Nq, D), dtype=np.float32)).cuda()
                for s in range(3))
    for sk in skips:
        os.environ["MXA_DBG_SKIP"] = str(sk)
        M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 16)()
        fn(buf, 1)
        M.mx_topk_attention(q, kk, v, D ** -0.5, k_top=k)
        torch.cuda.synchronize()
        fn(buf, 1)
        tot = sum(buf[i] for i in range(8))
        rows = B * H * Nq
        print(cfg, "skip", sk, "cycles/row by phase:", {names[i]: round(buf[i] / rows) for i in range(8)},
              "shares:", {names[i]: round(buf[i] / tot, 3) for i in range(8)}, flush=True)
