"""Step time of the fused op at a bench config three ways (tools-only): mxa_attention_timed
(HIP events between the kernels: the bench's stage breakdown), an eager loop of
mxa_attention, and a HIP graph of one call replayed (no launch gaps)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import bench
import mx_quantization_amd as M
from mx_quantization_amd import _native as N
from mx_quantization_amd.ops import _workspace

cfg = sys.argv[1] if len(sys.argv) > 1 else "deit_base"
c = bench.CONFIGS[cfg]
dev = torch.device("cuda", 0)
images = list(range(c["B"]))
q, k, v, bias = (None if a is None else torch.from_numpy(a).to(dev) for a in bench.make_inputs(c, images))
out, idx = M.mx_topk_attention(q, k, v, c["scale"], k_top=c["k"], pred_mode=c["mode"], bias=bias,
                               flush_subnormals=c["bias"])
p = N.AttnParams()
p.q, p.k, p.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
p.q_strides[:] = q.stride()[:3]
p.k_strides[:] = k.stride()[:3]
p.v_strides[:] = v.stride()[:3]
p.B, p.H, p.N, p.T, p.D = c["B"], c["H"], c["N"], c["T"], c["D"]
p.k_top, p.scale = c["k"], float(np.float32(c["scale"]))
p.pred_mode, p.top_k, p.approx = N.PRED_MODES[c["mode"]], 1, 1
p.flush_subnormals, p.bfloat = int(c["bias"]), 0
if bias is not None:
    b4 = bias.expand(c["B"], c["H"], c["N"], c["T"])
    p.bias, p.bias_strides[:] = b4.data_ptr(), b4.stride()
p.out, p.out_strides[:] = out.data_ptr(), out.stride()[:3]
p.idx_out = idx.data_ptr()
ws = _workspace(dev, N.lib().mxa_attention_workspace_bytes(ctypes.byref(p)))
p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
K = 20
st = (ctypes.c_float * 5)()


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / K * 1e3


s = torch.cuda.current_stream()
print("timed ", round(timeit(lambda: N.lib().mxa_attention_timed(ctypes.byref(p), s.cuda_stream, K, st)), 4), "ms")


def eager():
    for _ in range(K):
        N.check(N.lib().mxa_attention(ctypes.byref(p), torch.cuda.current_stream().cuda_stream), "mxa_attention")


print("eager ", round(timeit(eager), 4), "ms")
g = torch.cuda.CUDAGraph()
side = torch.cuda.Stream()
side.wait_stream(s)
with torch.cuda.stream(side):
    eager()
s.wait_stream(side)
torch.cuda.synchronize()
with torch.cuda.graph(g):
    N.check(N.lib().mxa_attention(ctypes.byref(p), torch.cuda.current_stream().cuda_stream), "mxa_attention")
ref = idx.clone()
idx.zero_()
g.replay()
torch.cuda.synchronize()
print("graph idx equal:", bool(torch.equal(idx, ref)))


def replay():
    for _ in range(K):
        g.replay()


print("graph ", round(timeit(replay), 4), "ms")
