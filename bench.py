#!/usr/bin/env python
"""Benchmark of the MX top-k attention hot path on MI355X.

BASELINE.json metric: "MXINT8 attn fwd tokens/s/GPU (DeiT-base, DiT-XL/2); top-k
idx bit-match".  One step = one call of the attention core over one batch of
synthetic q, k, v already resident in HBM: q,k,v (B,H,N,D) fp32 -> out (B,H,N,D)
fp32 + top-k indices (B,H,N,k) int64.  value = B*N tokens per
step summed over all ranks / max-over-ranks wall time.

  python bench.py [--config deit_base|dit_xl2|pixart_cross] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU, RCCL)

Multi-GPU: image batches are independent, so every rank runs the
full per-GPU batch on its own shard of images (weak scaling); the only
collectives are the barriers around the timed region and a MAX all-reduce of the
elapsed time.

Besides the contract fields the JSON line carries
  roofline      the dominant kernel's algorithmic bytes / its mean duration, measured
                with HIP events recorded on the launch stream inside the timed region
  cpu_baseline  the CPU oracle (oracle/, a 1-core port) timed on the host, rank 0 only
  parity        top-k index bit-match and output error of a sample of heads vs the oracle
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MXINT8 attn fwd tokens/s/GPU (DeiT-base, DiT-XL/2); top-k idx bit-match"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)

CONFIGS = {
    # BASELINE.json configs[1]: the metric's headline config on one GPU
    "deit_base": dict(workload="DeiT-base MXINT8 top-k attention core, ex_pred approximator",
                      B=256, H=12, N=197, T=197, D=64, k=20, mode="ex_pred", scale=64 ** -0.5, bias=False),
    # configs[2]
    "dit_xl2": dict(workload="DiT-XL/2 256x256 MXINT8 top-k attention core, ex_pred approximator",
                    B=64, H=16, N=256, T=256, D=72, k=154, mode="ex_pred", scale=72 ** -0.5, bias=False),
    # configs[4]
    "pixart_cross": dict(workload="PixArt-alpha 256x256 cross-attention core, MXINT4 (Sanger) approximator",
                         B=8, H=16, N=256, T=120, D=72, k=20, mode="MXINT4", scale=1 / np.sqrt(72), bias=True),
}
STAGES = ("rows_prep_q", "rows_prep_k", "cols_prep_v", "row kernel(s)", "")  # names: stage_bytes()


def stage_bytes(c, path):
    """Algorithmic HBM bytes each kernel must move per launch, by the
    kernel path mxa_attention_path() reports:
      rows_split  stage 3 = selection kernel (scores + top-k; writes the kept indices),
                  stage 4 = finishing kernel (gather, softmax, P, P.V; writes out)
      rows_fused  stage 3 = the one row kernel, stage 4 empty"""
    h = c["B"] * c["H"]
    N, T, D, k = c["N"], c["T"], c["D"], c["k"]
    nbd = -(-D // 32)
    dpad = 32 * nbd
    ntb = -(-T // 32)
    tpad = 32 * ntb
    codes = lambda rows: rows * (dpad + 2 * nbd)  # MXINT8 codes + int16 block exponents
    if c["mode"] == "ex_pred":  # sign words + int16 block exponents
        apx = lambda rows: rows * (4 * nbd + 2 * nbd)
    else:  # approximator codes + int16 block scales
        apx = lambda rows: rows * (dpad + 2 * nbd)
    vtab = D * tpad + 2 * ntb * D
    by = {
        "rows_prep_q": h * (4 * N * D + codes(N) + apx(N)),
        "rows_prep_k": h * (4 * T * D + codes(T) + apx(T)),
        "cols_prep_v": h * (4 * T * D + vtab),
    }
    if path == "rows_split":
        by["select"] = h * (apx(N) + apx(T) + 8 * N * k + 4 * N * k)
        by["finish"] = h * (codes(N) + codes(T) + vtab + 4 * N * k + 4 * N * D)
    else:
        by["fused"] = h * (codes(N) + codes(T) + apx(N) + apx(T) + vtab + 8 * N * k + 4 * N * D)
        by["-"] = 0
    return by


def fused_min_bytes(c):
    """SURVEY.md §8d fully-fused end-to-end minimum: fp32 q,k,v in, fp32 out, int64 idx out."""
    h = c["B"] * c["H"]
    return h * (4 * (c["N"] * c["D"] + 2 * c["T"] * c["D"]) + 4 * c["N"] * c["D"] + 8 * c["N"] * c["k"])


def make_inputs(c, rank, device=None):
    rng = lambda s: np.random.default_rng(1000 * rank + s)
    q = rng(0).standard_normal((c["B"], c["H"], c["N"], c["D"]), dtype=np.float32)
    k = rng(1).standard_normal((c["B"], c["H"], c["T"], c["D"]), dtype=np.float32)
    v = rng(2).standard_normal((c["B"], c["H"], c["T"], c["D"]), dtype=np.float32)
    bias = None
    if c["bias"]:  # 60 valid text tokens: (1 - mask) * -10000 (MX_pixart_transformer_2d.py:394-397)
        bias = np.where(np.arange(c["T"]) < 60, 0.0, -10000.0).astype(np.float32)[None, None, None, :]
        bias = np.repeat(bias, c["B"], 0)
    if device is None:
        return q, k, v, bias
    t = lambda a: None if a is None else torch.from_numpy(a).to(device)
    return t(q), t(k), t(v), t(bias)


def cpu_baseline(c, images):
    """The oracle (CPU restatement, 1 thread) on `images` images of the same workload."""
    from threadpoolctl import threadpool_limits
    from oracle import mx_oracle as O
    q, k, v, bias = make_inputs(dict(c, B=images), rank=0)
    with threadpool_limits(1):
        O.attention(q[:1], k[:1], v[:1], c["scale"], k_top=c["k"], pred_mode=c["mode"],
                    bias=None if bias is None else bias[:1], flush=c["bias"])  # warm
        t0 = time.perf_counter()
        O.attention(q, k, v, c["scale"], k_top=c["k"], pred_mode=c["mode"], bias=bias, flush=c["bias"])
        dt = time.perf_counter() - t0
    return {"value": images * c["N"] / dt, "unit": "tokens/s", "cores": 1, "kind": "port",
            "sample": f"{images} images x {c['H']} heads of the {c['workload']} workload, same synthetic inputs; "
                      f"oracle/mx_oracle.py (numpy float32 + libstdc++ top-k), 1 thread, {dt:.2f} s"}


def parity_sample(c, q, k, v, bias, out, idx, heads=4):
    """Top-k order bit-match and output error of a few images vs the oracle."""
    from oracle import mx_oracle as O
    rows = match = 0
    errs = []
    for b in sorted({0, c["B"] // 2, c["B"] - 1})[:heads]:
        hb = lambda t: None if t is None else t[b:b + 1].cpu().numpy()
        r = O.attention(hb(q), hb(k), hb(v), c["scale"], k_top=c["k"], pred_mode=c["mode"], bias=hb(bias),
                        flush=c["bias"])
        got = idx[b:b + 1].cpu().numpy()
        rows += got.shape[0] * got.shape[1] * got.shape[2]
        match += int(np.all(got == r["idx"], axis=-1).sum())
        errs.append(O.normwise_rel_err(out[b:b + 1].cpu().numpy(), r["out"]))
    return {"idx_rows_checked": rows, "idx_bitmatch": match / rows, "out_normwise_rel_err_max": max(errs),
            "out_tol": 1e-3}


def timed_region(run, world, sync, device):
    """Barrier + device sync on both sides of `run`, then the MAX of the elapsed
    wall time over ranks (the only collectives of the benchmark)."""
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    run()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="deit_base", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-images", type=int, default=-1, help="images for the CPU baseline (-1: whole batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--traffic-json", default=None, help="PMC-derived HBM bytes per dominant-kernel launch")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local)

    import mx_quantization_amd as M
    from mx_quantization_amd import _native as N
    c = CONFIGS[args.config]
    q, k, v, bias = make_inputs(c, rank, device)
    out = torch.empty_like(q)
    # warmup through the public op (also validates arguments and allocates workspace)
    for _ in range(max(args.warmup, 1)):
        out, idx = M.mx_topk_attention(q, k, v, c["scale"], k_top=c["k"], pred_mode=c["mode"], bias=bias,
                                       flush_subnormals=c["bias"], out=out)
    torch.cuda.synchronize()

    # the same call through the timed C entry point: K steps, events between kernels
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
    from mx_quantization_amd.ops import _workspace
    ws = _workspace(device, N.lib().mxa_attention_workspace_bytes(ctypes.byref(p)))
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    stage_ms = (ctypes.c_float * 5)()
    stream = torch.cuda.current_stream(device).cuda_stream

    elapsed = timed_region(
        lambda: N.check(N.lib().mxa_attention_timed(ctypes.byref(p), stream, args.steps, stage_ms),
                        "mxa_attention_timed"),
        world, torch.cuda.synchronize, device)

    tokens = world * c["B"] * c["N"] * args.steps
    value = tokens / elapsed
    path = N.PATH_NAMES.get(N.lib().mxa_attention_path(ctypes.byref(p)), "?")
    by = stage_bytes(c, path)
    names = list(by)  # stage order of mxa_attention_timed
    stages = {names[i]: float(stage_ms[i]) for i in range(len(STAGES))}
    dom = max(stages, key=stages.get)
    ach = by[dom] / (stages[dom] * 1e-3) / 1e9
    traffic = None
    if args.traffic_json and os.path.exists(args.traffic_json):
        traffic = json.load(open(args.traffic_json)).get(dom)
    res = {
        "metric": METRIC,
        "value": value,
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic (numpy default_rng standard_normal q/k/v, seeds 0/1/2 per rank)",
        "config": {"workload": c["workload"], "batch_per_gpu": c["B"], "heads": c["H"], "seq": c["N"],
                   "keys": c["T"], "head_dim": c["D"], "k": c["k"], "pred_mode": c["mode"],
                   "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "path": path,
                     "limiter": ("instruction issue, scalar ALU (exact-order top-k partition steps; "
                                 "PMC SQ_INSTS_SALU, profiles/r01_pmc_instr_*)") if dom in ("select", "fused") else None, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": by[dom], "mean_ms": stages[dom]},
        "stages_ms": stages,
        "e2e": {"fused_min_bytes": fused_min_bytes(c),
                "achieved_GBs": fused_min_bytes(c) / (sum(stages.values()) * 1e-3) / 1e9,
                "frac": fused_min_bytes(c) / (sum(stages.values()) * 1e-3) / 1e9 / HBM_PEAK_GBS},
    }
    if rank == 0 and not args.no_parity:
        res["parity"] = parity_sample(c, q, k, v, bias, out, idx)
    if rank == 0 and not args.no_cpu_baseline and world == 1:
        res["cpu_baseline"] = cpu_baseline(c, c["B"] if args.cpu_images < 0 else args.cpu_images)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
