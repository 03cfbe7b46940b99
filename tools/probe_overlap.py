"""Does splitting the batch over two HIP streams overlap the selection kernel (VALU-bound)
with the finishing / prep kernels of the neighbouring chunk?  (tools-only experiment)"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import mx_quantization_amd as M

cfg = sys.argv[1] if len(sys.argv) > 1 else "deit_base"
B, H, N, D, k = (256, 12, 197, 64, 20) if cfg == "deit_base" else (64, 16, 256, 72, 154)
rng = np.random.default_rng(0)
q, kk, v = (torch.from_numpy(rng.standard_normal((B, H, N, D), dtype=np.float32)).cuda() for _ in range(3))
out = torch.empty_like(q)
idx = torch.empty((B, H, N, k), dtype=torch.int64, device="cuda")
streams = [torch.cuda.Stream() for _ in range(4)]


def run(chunks, nstreams):
    cur = torch.cuda.current_stream()
    ev0 = torch.cuda.Event()
    ev0.record(cur)
    bounds = np.linspace(0, B, chunks + 1).astype(int)
    evs = []
    for c in range(chunks):
        s = streams[c % nstreams] if nstreams > 1 else cur
        s.wait_event(ev0)
        with torch.cuda.stream(s):
            b0, b1 = bounds[c], bounds[c + 1]
            o, i = M.mx_topk_attention(q[b0:b1], kk[b0:b1], v[b0:b1], D ** -0.5, k_top=k, out=out[b0:b1])
            idx[b0:b1].copy_(i)
        e = torch.cuda.Event()
        e.record(s)
        evs.append(e)
    for e in evs:
        cur.wait_event(e)


for chunks, ns in ((1, 1), (2, 2), (4, 2), (8, 2), (4, 4), (8, 4)):
    for _ in range(3):
        run(chunks, ns)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        run(chunks, ns)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    print(f"{cfg} chunks={chunks} streams={ns}: {dt*1e3:.3f} ms  {B*N/dt/1e6:.1f} Mtok/s", flush=True)
