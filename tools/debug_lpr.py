"""Debug probe for the ex_pred integer-key path: mismatch pattern of the debug
score outputs and the fallback count in the workspace."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mx_quantization_amd as M
from mx_quantization_amd import ops

d = np.load("tests/golden/attn_deit_tiny.npz")
q, k, v = (torch.from_numpy(d[n]).cuda() for n in ("q", "k", "v"))
out, idx, t, p = M.mx_topk_attention(q, k, v, float(d["scale"]), k_top=20, return_scores=True)
torch.cuda.synchronize()
p = p.cpu().numpy(); t = t.cpu().numpy(); idx = idx.cpu().numpy()
want = d["ex_pred_k20/pred"]
bad = p != want
print("true ok:", np.array_equal(t, d["true"]), "idx ok:", np.array_equal(idx, d["ex_pred_k20/idx"]))
print("pred mismatch frac per head:", bad.mean(axis=(0, 2, 3)))
rows_bad = bad.any(-1)[0]
print("rows with mismatch per head:", rows_bad.sum(-1), "first rows:", np.argwhere(rows_bad)[:10].tolist())
h, r = np.argwhere(rows_bad)[0]
print("row", h, r, "got", p[0, h, r, :12], "\nwant", want[0, h, r, :12])
print("got/want ratio", (p[0, h, r, :12] / want[0, h, r, :12]))
# fallback count: replicate attn_layout
B, H, N, D = d["q"].shape; T = N
al = lambda x: (x + 255) // 256 * 256
nbd = (D + 31) // 32; dpad = nbd * 32; ntb = (T + 31) // 32; tpad = ntb * 32
BH = B * H; qr = BH * N; kr = BH * T
sizes = [qr * dpad, qr * dpad, qr * nbd * 2, qr * nbd * 2, qr * nbd * 4, kr * dpad, kr * dpad, kr * nbd * 2,
         kr * nbd * 2, kr * nbd * 4, BH * D * tpad, BH * ntb * D * 2, qr * tpad, qr * ntb * 2]
off = sum(al(s) for s in sizes)
ws = [w for w in ops._WS.values()] if hasattr(ops, "_WS") else None
print("fb offset", off)
buf = list(ops._WS.values())[0]
print("fb count", buf[off:off + 4].cpu().numpy().view(np.int32))
