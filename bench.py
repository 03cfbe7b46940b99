#!/usr/bin/env python
"""Benchmark of the MX top-k attention hot path on MI355X.

BASELINE.json metric: "MXINT8 attn fwd tokens/s/GPU (DeiT-base, DiT-XL/2); top-k
idx bit-match".  One step = one call of the attention core over one batch of
synthetic q, k, v already resident in HBM: q,k,v (B,H,N,D) fp32 -> out (B,H,N,D)
fp32 + top-k indices (B,H,N,k) int64.  value = B*N tokens per
step summed over all ranks / max-over-ranks wall time.

  python bench.py [--config deit_base|dit_xl2|pixart_cross] [--steps K] [--warmup W]
  python bench.py --gpus N [--scaling weak|strong] ...

Multi-GPU: images are independent, so the batch is sharded over one
process per GPU (RCCL over xGMI; `--gpus N` without WORLD_SIZE starts the N ranks
itself through torch.distributed.run, before anything touches the GPU).  weak: every
rank runs the config's batch (tokens/s grows with N); strong: the config's batch is
split over the ranks.  The only data-path collective is the rank-0 all_gather of a
sample of every rank's indices / outputs for the parity check after timing; the
timed region is bracketed by barriers and its time is the MAX over ranks.

Besides the contract fields the JSON line carries
  roofline      the dominant kernel's algorithmic bytes / its mean duration (HIP events
                on the launch stream inside the timed region), plus
                qa_pass: SURVEY §8d Bytes_qa over the quantize + approx + top-k kernels,
                mfma:    Ops_gemm (dense QK^T + PV) over the finishing kernel's time
  cpu_baseline  the CPU oracle (oracle/, test infrastructure) on the host's cores
  parity        top-k index bit-match and output error of a sample of images per rank
  secondary     the DiT-XL/2 line (the metric names both models) when --config deit_base, the
                qkv-Linear-fused lines (mxa_qkv_attention, + the proj Linear), the dense branch
                (top_k=False) at the config's shape, and the drop-in modules' line
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MXINT8 attn fwd tokens/s/GPU (DeiT-base, DiT-XL/2); top-k idx bit-match"
PROFILE_TAG = "r06v2"  # the profiling session whose committed PMC files the bench line cites
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
I8_PEAK_TOPS = 5000.0  # MI355X_MICROARCH.md: dense I8 MFMA = 2x BF16 (~2.5 PF) per clock

CONFIGS = {
    # BASELINE.json configs[1]: the metric's headline config on one GPU
    "deit_base": dict(workload="DeiT-base MXINT8 top-k attention core, ex_pred approximator",
                      B=256, H=12, N=197, T=197, D=64, k=20, mode="ex_pred", scale=64 ** -0.5, bias=False),
    # configs[2] (configs[3] is the same shape sharded over 8 GPUs: --gpus 8)
    "dit_xl2": dict(workload="DiT-XL/2 256x256 MXINT8 top-k attention core, ex_pred approximator",
                    B=64, H=16, N=256, T=256, D=72, k=154, mode="ex_pred", scale=72 ** -0.5, bias=False),
    # configs[4]
    "pixart_cross": dict(workload="PixArt-alpha 256x256 cross-attention core, MXINT4 (Sanger) approximator",
                         B=8, H=16, N=256, T=120, D=72, k=20, mode="MXINT4", scale=1 / np.sqrt(72), bias=True),
}
# bench stages <- mxa_attention_timed's stage slots (include/mxa.h: 0 the operand builders
# for Q, K and V in one launch; 1, 2 empty; 3 selection; 4 finishing / dense row kernel)
STAGES = ("prep", "select", "finish")
STAGE_SLOTS = (0, 3, 4)
QKV_STAGES = ("x_quant+qkv_proj", "select", "finish")  # mxa_qkv_attention_timed, same slots


def stage_bytes(c, path):
    """Algorithmic HBM bytes each kernel must move per launch:
      prep    the operand builders (Q, K rows, V columns: one launch)
      select  selection kernel (approximate scores + top-k; writes the kept indices)
      finish  finishing kernel (gather, softmax, P, P.V; writes out)  [dense path: the row kernel]"""
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
    by = {"prep": h * (4 * N * D + codes(N) + apx(N)) + h * (4 * T * D + codes(T) + apx(T)) + h * (4 * T * D + vtab)}
    if path == "rows_split":
        by["select"] = h * (apx(N) + apx(T) + 8 * N * k)  # the int64 idx, which the finishing kernel reads
        by["finish"] = h * (codes(N) + codes(T) + vtab + 8 * N * k + 4 * N * D)
    else:  # dense: stage 3 empty, stage 4 the row kernel
        by["select"] = 0
        by["finish"] = h * (codes(N) + codes(T) + vtab + 4 * N * D)
    return by


def bytes_qa(c):
    """SURVEY.md §8d Bytes_qa: read Q,K,V fp32, write int8 codes, E8M0 exponents, idx int32."""
    h = c["B"] * c["H"]
    N, T, D, k = c["N"], c["T"], c["D"], c["k"]
    nb, tb = -(-D // 32), -(-T // 32)
    return h * (4 * (N * D + 2 * T * D) + (N * D + 2 * T * D) + (N * nb + T * nb + D * tb) + 4 * N * k)


def ops_gemm(c):
    """SURVEY.md §8d Ops_gemm: dense QK^T + PV int8 ops (2 per MAC), padding not counted."""
    return c["B"] * c["H"] * 2 * (2 * c["N"] * c["T"] * c["D"])


def fused_min_bytes(c):
    """SURVEY.md §8d fully-fused end-to-end minimum: fp32 q,k,v in, fp32 out, int64 idx out."""
    h = c["B"] * c["H"]
    return h * (4 * (c["N"] * c["D"] + 2 * c["T"] * c["D"]) + 4 * c["N"] * c["D"] + 8 * c["N"] * c["k"])


def image_inputs(c, img):
    """q, k, v (1,H,*,D) of global image `img`: seeded per image, so any rank (and the
    parity check on rank 0) regenerates the same image whatever the sharding."""
    rng = np.random.default_rng([img, 7])
    q = rng.standard_normal((1, c["H"], c["N"], c["D"]), dtype=np.float32)
    k = rng.standard_normal((1, c["H"], c["T"], c["D"]), dtype=np.float32)
    v = rng.standard_normal((1, c["H"], c["T"], c["D"]), dtype=np.float32)
    return q, k, v


def bias_of(c, B):
    if not c["bias"]:
        return None
    # 60 valid text tokens: (1 - mask) * -10000 (MX_pixart_transformer_2d.py:394-397)
    b = np.where(np.arange(c["T"]) < 60, 0.0, -10000.0).astype(np.float32)[None, None, None, :]
    return np.repeat(b, B, 0)


def make_inputs(c, images):
    qs, ks, vs = zip(*(image_inputs(c, i) for i in images))
    return np.concatenate(qs), np.concatenate(ks), np.concatenate(vs), bias_of(c, len(images))


def shard(c, rank, world, scaling):
    """Global image indices of this rank."""
    if scaling == "weak":
        return list(range(rank * c["B"], (rank + 1) * c["B"]))
    base, extra = divmod(c["B"], world)
    lo = rank * base + min(rank, extra)
    return list(range(lo, lo + base + (1 if rank < extra else 0)))


_CPU_INPUTS = None  # images of the CPU-baseline sample, made before the pool forks


def usable_cores():
    """Every core this process may run on: the affinity mask, capped by the cgroup CPU
    quota when one is set (cpu.max; a GPU box's share of a large host shows all the
    host's CPUs in nproc and the affinity mask but runs on its quota only)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    if quota is None:
        for var in ("OMP_NUM_THREADS",):  # the box's advertised share when no quota file exists
            v = os.environ.get(var, "")
            if v.isdigit() and int(v) > 0 and int(v) < aff:
                quota = int(v)
    cores = min(aff, quota) if quota else aff
    return cores, (f"nproc {os.cpu_count()}, affinity {aff}, cgroup/allotment quota {quota}: "
                   f"{cores} worker processes, every usable core")


def _oracle_image(i):
    from threadpoolctl import threadpool_limits
    from oracle import mx_oracle as O
    c, (q, k, v, bias) = _CPU_INPUTS
    with threadpool_limits(1):
        t0 = time.perf_counter()
        O.attention(q[i:i + 1], k[i:i + 1], v[i:i + 1], c["scale"], k_top=c["k"], pred_mode=c["mode"],
                    bias=None if bias is None else bias[i:i + 1], flush=c["bias"])
        return time.perf_counter() - t0


def cpu_baseline(c, images):
    """The oracle (CPU restatement, numpy float32 + libstdc++ top-k; oracle/ is test
    infrastructure) on `images` images of the same workload, one image per task over
    a pool of single-threaded worker processes, one per usable host core (at most 16,
    the GPU box's share).  Runs before anything touches the GPU (fork is safe then);
    the inputs are made beforehand, so the wall time is the oracle's alone."""
    global _CPU_INPUTS
    import multiprocessing as mp
    import torch
    cores, why = usable_cores()
    _CPU_INPUTS = (c, make_inputs(c, list(range(images))))
    _oracle_image(0)  # warm: loads the oracle library before the fork
    with mp.get_context("fork").Pool(cores) as pool:
        t0 = time.perf_counter()
        busy = sum(pool.map(_oracle_image, range(images), chunksize=1))
        dt = time.perf_counter() - t0
    _CPU_INPUTS = None
    return {"value": images * c["N"] / dt, "unit": "tokens/s", "cores": cores, "kind": "port",
            "sample": f"{images} images x {c['H']} heads of the {c['workload']} workload, same synthetic inputs; "
                      f"oracle/mx_oracle.py (numpy float32 + libstdc++ top-k), {cores} worker processes x 1 thread "
                      f"({why}; torch threads "
                      f"{torch.get_num_threads()} unused by the oracle), {dt:.2f} s wall, {busy:.1f} s of CPU work"}


def parity_check(c, got_idx, got_out, images):
    """Top-k order bit-match and output error of gathered images vs the oracle."""
    from oracle import mx_oracle as O
    rows = match = 0
    errs = []
    for i, img in enumerate(images):
        q, k, v, bias = make_inputs(c, [img])
        r = O.attention(q, k, v, c["scale"], k_top=c["k"], pred_mode=c["mode"], bias=bias, flush=c["bias"])
        g = got_idx[i:i + 1]
        rows += g.shape[0] * g.shape[1] * g.shape[2]
        match += int(np.all(g == r["idx"], axis=-1).sum())
        errs.append(O.normwise_rel_err(got_out[i:i + 1], r["out"]))
    return {"images_checked": len(images), "idx_rows_checked": rows, "idx_bitmatch": match / max(rows, 1),
            "out_normwise_rel_err_max": max(errs) if errs else None, "out_tol": 1e-3}


def timed_region(run, world, sync, device):
    """Barrier + device sync on both sides of `run`, then the MAX of the elapsed wall
    time over ranks."""
    import torch
    import torch.distributed as dist
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


def timed_product(call, timed_call, steps, world, device):
    """The measured region: `steps` calls of the product entry point (`call`), bracketed as
    timed_region does.  The stage breakdown comes from one more pass through the entry's
    *_timed twin (`timed_call`: HIP events between the kernels) outside that region -- the
    events cost ~4 % of a DeiT-base step and a third of a PixArt one (tools/probe_graph.py)."""
    import torch
    elapsed = timed_region(lambda: [call() for _ in range(steps)], world, torch.cuda.synchronize, device)
    timed_call()
    torch.cuda.synchronize()
    return elapsed


SIMDS = 1024            # MI355X_MICROARCH.md: 256 CUs x 4 SIMDs
CLK_HZ = 2.4e9          # max engine clock (the chip runs lower under load: the VALU fraction is a floor)
VALU_ISSUE_CYC = 2      # a wave64 VALU instruction occupies a SIMD-32 for 2 cycles


def _unique_kernel(d, stage):
    """The one kernel instantiation of `stage` in a per-kernel profile dict, or None
    (several instantiations never average together: tools/hbm_traffic.py)."""
    names = [n for n in d if stage_of_kernel(n) == stage]
    return names[0] if len(names) == 1 else None


def stage_of_kernel(name):
    """The bench stage (or selection sub-stage) of a kernel instantiation: the selection
    stage's HIP events cover the packed selection kernel ("select"), the one-lane top-k
    tail ("select_tail") and the 64-bit kernel ("select_fb": the rows the packed pass
    leaves, or every row where the scores do not pack)."""
    if "topk_tail_kernel" in name:
        return "select_tail"
    if "select_kernel" in name:
        return "select" if "unsigned int" in name else "select_fb"
    if any(f in name for f in ("finish_kernel", "finish16_kernel", "finish_qk_kernel", "dense_rows_kernel")):
        return "finish"
    if "attn_prep_kernel" in name:
        return "prep"
    if "qkv_proj_kernel" in name:
        return "proj"
    if "mx_gemm" in name:
        return "proj_linear"
    return None


def profile_of(prof, stage, ms, ach_gbs):
    """(traffic bytes per launch or None, limiter block) of the dominant kernel from the
    committed profiles of this config: PMC HBM traffic (tools/hbm_traffic.py output) and
    instruction counters (tools/pmc_summary.py --json output).  bound = the resource with
    the largest measured busy fraction among HBM (PMC traffic / time / peak), VALU issue
    (VALU instructions x 2 cycles / (SIMDs x clock x time)) and MFMA (busy cycles)."""
    prof = prof or {}
    traffic = None
    lim = {"bound": "hbm", "source": None, "fracs": {"hbm_algorithmic": ach_gbs / HBM_PEAK_GBS}}
    tj = prof.get("traffic")
    if tj and os.path.exists(tj):
        with open(tj) as fh:
            t = json.load(fh)
        traffic = t.get("stages", {}).get(stage)
        if traffic is not None:
            lim["fracs"]["hbm_measured"] = traffic / (ms * 1e-3) / (HBM_PEAK_GBS * 1e9)
        lim["source"] = os.path.relpath(tj, ROOT)
    pj = prof.get("pmc")
    if pj and os.path.exists(pj):
        with open(pj) as fh:
            pm = json.load(fh)
        name = _unique_kernel(pm, stage)
        if name:
            k = pm[name]
            sec = ms * 1e-3
            if "SQ_INSTS_VALU" in k:
                lim["fracs"]["valu_issue"] = k["SQ_INSTS_VALU"] * VALU_ISSUE_CYC / (SIMDS * CLK_HZ * sec)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in k:  # counted in cycles, summed over SIMDs
                lim["fracs"]["mfma_busy"] = k["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * CLK_HZ * sec)
            if "SQ_WAIT_ANY" in k and "SQ_WAVE_CYCLES" in k and k["SQ_WAVE_CYCLES"]:
                lim["wait_any_share"] = k["SQ_WAIT_ANY"] / k["SQ_WAVE_CYCLES"]
            if "SQ_LDS_BANK_CONFLICT" in k and k.get("SQ_INSTS_LDS"):
                lim["lds_conflict_cycles_per_lds_instr"] = k["SQ_LDS_BANK_CONFLICT"] / k["SQ_INSTS_LDS"]
            lim["kernel"] = name
            lim["pmc_source"] = os.path.relpath(pj, ROOT)
    f = lim["fracs"]
    cand = {"hbm": max(f.get("hbm_measured", 0.0), f["hbm_algorithmic"]), "valu": f.get("valu_issue", 0.0),
            "mfma": f.get("mfma_busy", 0.0)}
    lim["bound"] = max(cand, key=cand.get)
    if lim["bound"] != "mfma" and max(cand.values()) < 0.5 and lim.get("wait_any_share", 0.0) > 0.3:
        lim["bound"] = "latency"  # no unit near its peak and the waves mostly parked
    return traffic, lim


def run_config(c, images, steps, warmup, device, world, prof=None):
    """Time `steps` calls of the op on this rank's images; returns the elapsed time
    (max over ranks), the stage times, the roofline block and the outputs."""
    import torch
    import mx_quantization_amd as M
    from mx_quantization_amd import _native as N
    t = lambda a: None if a is None else torch.from_numpy(a).to(device)
    q, k, v, bias = (t(a) for a in make_inputs(c, images))
    out = torch.empty_like(q)
    for _ in range(max(warmup, 1)):  # through the public op (validates, allocates the workspace)
        out, idx = M.mx_topk_attention(q, k, v, c["scale"], k_top=c["k"], pred_mode=c["mode"], bias=bias,
                                       flush_subnormals=c["bias"], out=out)
    torch.cuda.synchronize()

    # the same call through the C entry point: K steps timed (the value), then its timed twin
    # (HIP events between the kernels) for the stage breakdown
    B = len(images)
    p = N.AttnParams()
    p.q, p.k, p.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
    p.q_strides[:] = q.stride()[:3]
    p.k_strides[:] = k.stride()[:3]
    p.v_strides[:] = v.stride()[:3]
    p.B, p.H, p.N, p.T, p.D = B, c["H"], c["N"], c["T"], c["D"]
    p.k_top, p.scale = c["k"], float(np.float32(c["scale"]))
    p.pred_mode, p.top_k, p.approx = N.PRED_MODES[c["mode"]], 1, 1
    p.flush_subnormals, p.bfloat = int(c["bias"]), 0
    if bias is not None:
        b4 = bias.expand(B, c["H"], c["N"], c["T"])
        p.bias, p.bias_strides[:] = b4.data_ptr(), b4.stride()
    p.out, p.out_strides[:] = out.data_ptr(), out.stride()[:3]
    p.idx_out = idx.data_ptr()
    from mx_quantization_amd.ops import _workspace
    ws = _workspace(device, N.lib().mxa_attention_workspace_bytes(ctypes.byref(p)))
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    stage_ms = (ctypes.c_float * 5)()
    stream = torch.cuda.current_stream(device).cuda_stream
    elapsed = timed_product(
        lambda: N.check(N.lib().mxa_attention(ctypes.byref(p), stream), "mxa_attention"),
        lambda: N.check(N.lib().mxa_attention_timed(ctypes.byref(p), stream, steps, stage_ms), "mxa_attention_timed"),
        steps, world, device)
    path = N.PATH_NAMES.get(N.lib().mxa_attention_path(ctypes.byref(p)), "?")
    fin = fin_engines(p)
    stages = {name: float(stage_ms[slot]) for name, slot in zip(STAGES, STAGE_SLOTS)}
    cb = dict(c, B=B)
    by = stage_bytes(cb, path)
    dom = max(stages, key=stages.get)
    ach = by[dom] / (stages[dom] * 1e-3) / 1e9
    traffic, lim = profile_of(prof, dom, stages[dom], ach)
    qa_ms = stages["prep"] + stages["select"]
    qa_gbs = bytes_qa(cb) / (qa_ms * 1e-3) / 1e9
    mf_tops = ops_gemm(cb) / (stages["finish"] * 1e-3) / 1e12
    roof = {
        # bound: the resource the PMC profile shows limiting the dominant kernel; the
        # achieved / peak / frac below are its HBM roofline (algorithmic bytes / time)
        "bound": lim["bound"], "frac_of": "hbm", "kernel": dom, "path": path, "limiter": lim,
        "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
        "algorithmic_bytes_per_launch": by[dom], "mean_ms": stages[dom],
        "qa_pass": {"what": "SURVEY §8d Bytes_qa over the prep (Q, K, V) + selection kernels",
                    "bytes": bytes_qa(cb), "ms": qa_ms, "achieved": qa_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": qa_gbs / HBM_PEAK_GBS},
        "mfma": {"what": "SURVEY §8d Ops_gemm (dense QK^T + PV int8 ops) over the finishing kernel's time "
                         "(the dense-equivalent rate; `engine` names the kernel the library launched and the "
                         "units its two contractions run on, from mxa_attention_finish_kernel)",
                 "ops": ops_gemm(cb), "ms": stages["finish"], "achieved": mf_tops, "peak": I8_PEAK_TOPS,
                 "unit": "TOPS", "frac": mf_tops / I8_PEAK_TOPS, "engine": fin},
    }
    e2e = {"fused_min_bytes": fused_min_bytes(cb),
           "achieved_GBs": fused_min_bytes(cb) / (sum(stages.values()) * 1e-3) / 1e9}
    e2e["frac"] = e2e["achieved_GBs"] / HBM_PEAK_GBS
    return elapsed, stages, roof, e2e, out, idx


def fin_engines(p):
    """The finishing kernel mxa_attention(p) launches and the engines of its QK^T and P.V
    (include/mxa.h mxa_attention_finish_kernel: the library's own dispatch decision)."""
    from mx_quantization_amd import _native as N
    kind = N.lib().mxa_attention_finish_kernel(ctypes.byref(p))
    name, qk, pv = N.FIN_KERNELS.get(kind, ("?", "?", "?"))
    return {"kernel": name, "qk": qk, "pv": pv, "code": kind}


def run_dense(c, images, steps, warmup, device, world):
    """The dense branch (top_k=False: DeiT block 11, deit main.py:149-152; DiT's last block,
    models.py:218-225) at the config's shape: attn = softmax(true scores) over every key, then
    MX(P) @ MX(V).  Returns (elapsed, stage_ms, extra)."""
    import torch
    import mx_quantization_amd as M
    from mx_quantization_amd import _native as N
    t = lambda a: None if a is None else torch.from_numpy(a).to(device)
    q, k, v, bias = (t(a) for a in make_inputs(c, images))
    out = torch.empty_like(q)
    for _ in range(max(warmup, 1)):
        out, _ = M.mx_topk_attention(q, k, v, c["scale"], top_k=False, bias=bias, flush_subnormals=c["bias"], out=out)
    torch.cuda.synchronize()
    B = len(images)
    p = N.AttnParams()
    p.q, p.k, p.v = q.data_ptr(), k.data_ptr(), v.data_ptr()
    p.q_strides[:], p.k_strides[:], p.v_strides[:] = q.stride()[:3], k.stride()[:3], v.stride()[:3]
    p.B, p.H, p.N, p.T, p.D = B, c["H"], c["N"], c["T"], c["D"]
    p.k_top, p.scale = 0, float(np.float32(c["scale"]))
    p.pred_mode, p.top_k, p.approx = N.PRED_MODES[c["mode"]], 0, 1
    p.flush_subnormals, p.bfloat = int(c["bias"]), 0
    if bias is not None:
        b4 = bias.expand(B, c["H"], c["N"], c["T"])
        p.bias, p.bias_strides[:] = b4.data_ptr(), b4.stride()
    p.out, p.out_strides[:] = out.data_ptr(), out.stride()[:3]
    from mx_quantization_amd.ops import _workspace
    ws = _workspace(device, N.lib().mxa_attention_workspace_bytes(ctypes.byref(p)))
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    stage_ms = (ctypes.c_float * 5)()
    stream = torch.cuda.current_stream(device).cuda_stream
    elapsed = timed_product(
        lambda: N.check(N.lib().mxa_attention(ctypes.byref(p), stream), "mxa_attention"),
        lambda: N.check(N.lib().mxa_attention_timed(ctypes.byref(p), stream, steps, stage_ms), "mxa_attention_timed"),
        steps, world, device)
    stages = {"prep": float(stage_ms[0]), "dense": float(stage_ms[4])}
    cb = dict(c, B=B)
    tops = ops_gemm(cb) / (stages["dense"] * 1e-3) / 1e12
    by = stage_bytes(cb, "rows_fused")["finish"]
    extra = {"mfma": {"what": "SURVEY §8d Ops_gemm (QK^T + P.V int8 ops, every key) over the dense kernel's time",
                      "ops": ops_gemm(cb), "achieved": tops, "peak": I8_PEAK_TOPS, "unit": "TOPS",
                      "frac": tops / I8_PEAK_TOPS, "engine": fin_engines(p)},
             "hbm": {"algorithmic_bytes_per_launch": by, "achieved": by / (stages["dense"] * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s"}}
    if world == 1:  # one image against the oracle's dense branch (test infrastructure)
        from oracle import mx_oracle as O
        qh, kh, vh, bh = make_inputs(c, [images[0]])
        r = O.attention(qh, kh, vh, c["scale"], top_k=False, pred_mode=c["mode"], bias=bh, flush=c["bias"])
        extra["parity"] = {"out_normwise_rel_err": O.normwise_rel_err(out[:1].cpu().numpy(), r["out"]), "out_tol": 1e-3}
    return elapsed, stages, extra


def run_qkv(c, images, steps, warmup, device, world):
    """The qkv mx.Linear fused in front of the attention core (mxa_qkv_attention): x (B, N,
    H*D) tokens and a (3*H*D, H*D) weight (prepared once, outside the timed region: the
    weights are constant at inference) -> out + idx.  Returns (elapsed, stage_ms, extra)."""
    import torch
    import mx_quantization_amd as M
    from mx_quantization_amd import _native as N
    B, H, Nt, D = len(images), c["H"], c["N"], c["D"]
    C = H * D
    rng = np.random.default_rng(99)
    x = torch.from_numpy(rng.standard_normal((B, Nt, C), dtype=np.float32)).to(device)
    W = torch.from_numpy((rng.standard_normal((3 * C, C), dtype=np.float32) * np.float32(C ** -0.5))).to(device)
    bias = torch.from_numpy(rng.standard_normal(3 * C, dtype=np.float32) * np.float32(0.02)).to(device)
    wq = M.LinearWeightMX(W, D)
    for _ in range(max(warmup, 1)):
        M.mx_qkv_attention(x, wq, bias, H, c["scale"], k_top=c["k"], pred_mode=c["mode"])
    torch.cuda.synchronize()
    p = N.AttnParams()
    p.B, p.H, p.N, p.T, p.D = B, H, Nt, Nt, D
    p.k_top, p.scale = c["k"], float(np.float32(c["scale"]))
    p.pred_mode, p.top_k, p.approx = N.PRED_MODES[c["mode"]], 1, 1
    out = torch.empty((B, H, Nt, D), dtype=torch.float32, device=device)
    idx = torch.empty((B, H, Nt, c["k"]), dtype=torch.int64, device=device)
    p.out, p.out_strides[:] = out.data_ptr(), out.stride()[:3]
    p.idx_out = idx.data_ptr()
    xp = N.QkvParams()
    xp.x, xp.x_row_stride, xp.C, xp.wq, xp.bias = x.data_ptr(), C, C, wq.buf.data_ptr(), bias.data_ptr()
    from mx_quantization_amd.ops import _workspace
    ws = _workspace(device, N.lib().mxa_qkv_attention_workspace_bytes(ctypes.byref(p), ctypes.byref(xp)))
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    stage_ms = (ctypes.c_float * 5)()
    stream = torch.cuda.current_stream(device).cuda_stream
    elapsed = timed_product(
        lambda: N.check(N.lib().mxa_qkv_attention(ctypes.byref(p), ctypes.byref(xp), stream), "mxa_qkv_attention"),
        lambda: N.check(N.lib().mxa_qkv_attention_timed(ctypes.byref(p), ctypes.byref(xp), stream, steps, stage_ms),
                        "mxa_qkv_attention_timed"), steps, world, device)
    stages = {name: float(stage_ms[slot]) for name, slot in zip(QKV_STAGES, STAGE_SLOTS)}
    proj_ms = stages["x_quant+qkv_proj"]
    ops = 2 * B * Nt * C * 3 * C  # int8 ops of the projection GEMM
    extra = {"proj_int8_tops": ops / (proj_ms * 1e-3) / 1e12,
             "proj_bytes_min": B * Nt * C * 4 + 3 * C * C + B * Nt * C * 3 * 1,
             "fp32_qkv_bytes_avoided": B * Nt * 3 * C * 4 * 2}
    return elapsed, stages, extra


def run_qkv_proj(c, images, steps, warmup, device, world):
    """x -> qkv mx.Linear -> attention -> proj mx.Linear in one call (mxa_attention_proj with
    the qkv front end): the attention block's whole MX path from tokens to tokens, weights
    prepared once outside the timed region.  Returns (elapsed, stage_ms, extra)."""
    import torch
    import mx_quantization_amd as M
    from mx_quantization_amd import _native as N
    B, H, Nt, D = len(images), c["H"], c["N"], c["D"]
    C = H * D
    rng = np.random.default_rng(98)
    x = torch.from_numpy(rng.standard_normal((B, Nt, C), dtype=np.float32)).to(device)
    W = torch.from_numpy((rng.standard_normal((3 * C, C), dtype=np.float32) * np.float32(C ** -0.5))).to(device)
    bias = torch.from_numpy(rng.standard_normal(3 * C, dtype=np.float32) * np.float32(0.02)).to(device)
    Wp = torch.from_numpy((rng.standard_normal((C, C), dtype=np.float32) * np.float32(C ** -0.5))).to(device)
    bp = torch.from_numpy(rng.standard_normal(C, dtype=np.float32) * np.float32(0.02)).to(device)
    wq, wp = M.LinearWeightMX(W, D), M.LinearWeightMX(Wp, C)
    for _ in range(max(warmup, 1)):
        y, idx = M.mx_qkv_attention(x, wq, bias, H, c["scale"], k_top=c["k"], pred_mode=c["mode"], proj_weight=wp,
                                    proj_bias=bp)
    torch.cuda.synchronize()
    p = N.AttnParams()
    p.B, p.H, p.N, p.T, p.D = B, H, Nt, Nt, D
    p.k_top, p.scale = c["k"], float(np.float32(c["scale"]))
    p.pred_mode, p.top_k, p.approx = N.PRED_MODES[c["mode"]], 1, 1
    p.idx_out = idx.data_ptr()
    xp = N.QkvParams()
    xp.x, xp.x_row_stride, xp.C, xp.wq, xp.bias = x.data_ptr(), C, C, wq.buf.data_ptr(), bias.data_ptr()
    pj = N.ProjParams()
    pj.wq, pj.out_features, pj.bias = wp.buf.data_ptr(), C, bp.data_ptr()
    yy = y.reshape(B * Nt, C)
    pj.y, pj.y_row_stride = yy.data_ptr(), C
    from mx_quantization_amd.ops import _workspace
    ws = _workspace(device, N.lib().mxa_attention_proj_workspace_bytes(ctypes.byref(p), ctypes.byref(xp),
                                                                       ctypes.byref(pj)))
    p.workspace, p.workspace_bytes = ws.data_ptr(), ws.numel()
    stage_ms = (ctypes.c_float * N.PROJ_STAGES)()
    stream = torch.cuda.current_stream(device).cuda_stream
    elapsed = timed_product(
        lambda: N.check(N.lib().mxa_attention_proj(ctypes.byref(p), ctypes.byref(xp), ctypes.byref(pj), stream),
                        "mxa_attention_proj"),
        lambda: N.check(N.lib().mxa_attention_proj_timed(ctypes.byref(p), ctypes.byref(xp), ctypes.byref(pj), stream,
                                                         steps, stage_ms), "mxa_attention_proj_timed"),
        steps, world, device)
    stages = {name: float(stage_ms[slot]) for name, slot in zip(QKV_STAGES + ("proj_linear",), STAGE_SLOTS + (5,))}
    ops = 2 * B * Nt * C * C  # int8 ops of the proj GEMM
    pms = stages["proj_linear"]
    extra = {"proj_linear_int8_tops": ops / (pms * 1e-3) / 1e12,
             "proj_linear_frac_of_i8_peak": ops / (pms * 1e-3) / 1e12 / I8_PEAK_TOPS,
             "proj_linear_min_bytes": B * Nt * C * (1 + 2 / 32) + C * C + B * Nt * C * 4,
             "proj_input": "MX codes straight from the finishing kernel" if D % 32 == 0 else
                           "fp32 workspace copy + row quantizer (a 32-block of C spans two heads)",
             "fp32_attn_out_bytes_avoided": B * Nt * C * 4 * 2 if D % 32 == 0 else 0}
    return elapsed, stages, extra


def run_dropin(c, images, steps, warmup, device, world):
    """The unchanged attention modules through install_dropin() (workloads/deit/scripts/
    main.py:101-152 restated: mx.matmul QK^T, exponent_approximation operands, aQ @ aK^T,
    the top-k in torch CPU order, gather / softmax / scatter, mx.matmul P.V): what a patched
    module runs when only the imports change.  Returns (elapsed, extra)."""
    import torch
    import mx_quantization_amd as M
    mx, funcs = M.install_dropin()
    from mx_quantization_amd.mx.specs import apply_mx_specs
    specs = apply_mx_specs({"w_elem_format": "int8", "a_elem_format": "int8", "scale_bits": 8,  # deit main.py:716-736
                            "shared_exp_method": "max", "block_size": 32, "bfloat": 32, "fp": 0,
                            "bfloat_subnorms": True, "round": "nearest", "round_mx_output": "nearest",
                            "round_output": "nearest", "round_weight": "nearest",
                            "mx_flush_fp32_subnorms": False, "custom_cuda": False, "quantize_backprop": False})
    t = lambda a: torch.from_numpy(a).to(device)
    q, k, v, _ = (None if a is None else t(a) for a in make_inputs(c, images))

    def step():
        ts = mx.matmul(q, k.transpose(-2, -1), mx_specs=specs, mode_config="aa") * c["scale"]
        aq, ak = funcs.exponent_approximation(Q=q, K=k, mx_specs=specs).exponent_based_sign()
        pred = aq @ ak.transpose(-2, -1)
        _, idx = M.topk(pred, c["k"])
        vals = ts.gather(dim=-1, index=idx)
        attn = torch.zeros_like(ts)
        attn.scatter_(-1, idx, torch.softmax(vals, dim=-1).to(attn.dtype))
        return mx.matmul(attn, v, mx_specs=specs, mode_config="aa"), idx

    for _ in range(max(warmup, 1)):
        out, idx = step()
    torch.cuda.synchronize()

    def timed():
        for _ in range(steps):
            step()
    elapsed = timed_region(timed, world, torch.cuda.synchronize, device)
    ref_out, ref_idx = M.mx_topk_attention(q, k, v, c["scale"], k_top=c["k"], pred_mode=c["mode"])
    return elapsed, {"idx_equal_fused": bool(torch.equal(idx, ref_idx)),
                     "out_max_abs_diff_vs_fused": float((out - ref_out).abs().max())}


def run_secondary(args, c, rank, world, images, lines, run, device, res=None):
    """The secondary lines: `qkv` (the config's fused qkv-Linear line) and `dit` (the
    DiT-XL/2 line of deit_base).  With res None (no main line: profiling passes) the
    secondaries go out as their own JSON line."""
    import torch.distributed as dist
    alone = res is None
    if alone:
        res = {"metric": METRIC, "lines": sorted(lines)}
    if args.config in ("deit_base", "dit_xl2") and "qkv" in lines and run is run_config:
        # the qkv mx.Linear fused in front: x (B, N, C) -> out + idx
        qsteps = max(args.steps // 2, 1)
        qel, qst, qex = run_qkv(c, images, qsteps, 2, device, world)
        qtok = (world * c["B"] if args.scaling == "weak" else c["B"]) * c["N"] * qsteps
        res.setdefault("secondary", []).append(
            {"config": args.config + "+qkv_linear", "workload": "mx.Linear qkv projection (C=%d -> 3C) fused into the "
             "attention core's MX operands, then the same attention" % (c["H"] * c["D"]),
             "value": qtok / qel, "unit": "tokens/s", "ms_per_step": qel / qsteps * 1e3, "stages_ms": qst, **qex})

    if args.config in ("deit_base", "dit_xl2") and "qkvproj" in lines and run is run_config:
        # ... and the proj mx.Linear behind it (both halves): x -> y
        psteps = max(args.steps // 2, 1)
        pel, pst, pex = run_qkv_proj(c, images, psteps, 2, device, world)
        ptok = (world * c["B"] if args.scaling == "weak" else c["B"]) * c["N"] * psteps
        res.setdefault("secondary", []).append(
            {"config": args.config + "+qkv_linear+proj_linear", "workload": "x (B, N, C=%d) -> qkv mx.Linear -> MX "
             "top-k attention -> proj mx.Linear -> y (B, N, C), one call" % (c["H"] * c["D"]),
             "value": ptok / pel, "unit": "tokens/s", "ms_per_step": pel / psteps * 1e3, "stages_ms": pst, **pex})
    if "dense" in lines and run is run_config:
        # the dense branch (top_k=False) at the config's shape: QK^T and P.V over every key
        nsteps = max(args.steps // 2, 1)
        nel, nst, nex = run_dense(c, images, nsteps, 2, device, world)
        ntok = (world * c["B"] if args.scaling == "weak" else c["B"]) * c["N"] * nsteps
        res.setdefault("secondary", []).append(
            {"config": args.config + "+dense", "workload": "the dense branch (top_k=False) of the %s shape: "
             "softmax over every key's true score, MX(P) @ MX(V)" % args.config,
             "value": ntok / nel, "unit": "tokens/s", "ms_per_step": nel / nsteps * 1e3, "stages_ms": nst, **nex})
    if args.config == "deit_base" and "dropin" in lines and run is run_config:
        # the drop-in modules the unchanged attention code imports (install_dropin)
        dsteps = max(args.steps // 4, 1)
        del_, dex = run_dropin(c, images, dsteps, 1, device, world)
        dtok = (world * c["B"] if args.scaling == "weak" else c["B"]) * c["N"] * dsteps
        res.setdefault("secondary", []).append(
            {"config": "deit_base+dropin", "workload": "the unchanged DeiT attention glue (main.py:101-152) on the "
             "install_dropin() mx / funcs modules: mx.matmul QK^T and P.V on the block-scaled MFMA GEMM, "
             "exponent_approximation operands, torch-CPU-order top-k; torch gather / softmax / scatter",
             "value": dtok / del_, "unit": "tokens/s", "ms_per_step": del_ / dsteps * 1e3, **dex})
    if args.config == "deit_base" and "dit" in lines:
        d = CONFIGS["dit_xl2"]
        dimg = shard(d, rank, world, args.scaling)
        dprof = {"traffic": os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_traffic_dit_xl2.json"),
                 "pmc": os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_pmc_dit_xl2.json")}
        delapsed, dst, droof, _, _, _ = run(d, dimg, max(args.steps // 2, 1), 2, device, world, dprof)
        dtok = (world * d["B"] if args.scaling == "weak" else d["B"]) * d["N"] * max(args.steps // 2, 1)
        res.setdefault("secondary", []).append({"config": "dit_xl2", "workload": d["workload"], "value": dtok / delapsed,
                             "unit": "tokens/s", "ms_per_step": delapsed / max(args.steps // 2, 1) * 1e3,
                             "batch_per_gpu": len(dimg), "stages_ms": dst, "roofline": droof})
    if alone:
        if rank == 0:
            print(json.dumps(res), flush=True)
        if world > 1:
            dist.barrier()
        return res if rank == 0 else 0
    return res


def launch_ranks(args):
    """--gpus N without WORLD_SIZE: start the N ranks (one process per GPU) through
    torch.distributed.run from this process, which has not touched the GPU, and exit
    with their status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main(argv=None, run=run_config):
    """`run` is the per-rank timed step (tests substitute a CPU stand-in with the same
    signature to drive the multi-rank path over gloo)."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, or 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="deit_base", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"))
    ap.add_argument("--k", type=int, default=None, help="override the config's k (A/B runs only)")
    ap.add_argument("--cpu-images", type=int, default=-1, help="images for the CPU baseline (-1: the batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the DiT-XL/2 line")
    ap.add_argument("--parity-images", type=int, default=2, help="images per rank checked against the oracle")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC HBM traffic per kernel (tools/hbm_traffic.py; default: the committed "
                         "profiles/<PROFILE_TAG>_traffic_<config>.json)")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC instruction counters per kernel (tools/pmc_summary.py --json; default: the "
                         "committed profiles/<PROFILE_TAG>_pmc_<config>.json)")
    ap.add_argument("--lines", default="main,qkv,qkvproj,dense,dropin,dit",
                    help="which lines to run: main (the config), qkv (its fused qkv-Linear line), qkvproj (x -> "
                         "qkv Linear -> attention -> proj Linear), dense (the top_k=False branch at the config's "
                         "shape), dropin (the drop-in modules' path), dit (the DiT-XL/2 secondary of deit_base)")
    args = ap.parse_args(argv)

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus and args.gpus > 1:
        return launch_ranks(args)
    world = int(env_world or 1)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    c = CONFIGS[args.config] if args.k is None else dict(CONFIGS[args.config], k=args.k)

    cpu = None  # before any HIP call: the pool forks
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(c, c["B"] if args.cpu_images < 0 else args.cpu_images)

    import torch
    import torch.distributed as dist
    backend = os.environ.get("MXA_BENCH_BACKEND", "nccl")  # gloo: the CPU multi-rank tests
    if backend == "nccl":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend, **({"device_id": device} if backend == "nccl" else {}))

    images = shard(c, rank, world, args.scaling)
    lines = set(args.lines.split(","))
    if args.no_secondary:
        lines &= {"main"}
    prof = {"traffic": args.traffic_json or os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_traffic_{args.config}.json"),
            "pmc": args.pmc_json or os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_pmc_{args.config}.json")}
    if "main" not in lines:  # profiling the secondary lines alone
        return run_secondary(args, c, rank, world, images, lines, run, device)
    elapsed, stages, roof, e2e, out, idx = run(c, images, args.steps, args.warmup, device, world, prof)
    tokens = (world * c["B"] if args.scaling == "weak" else c["B"]) * c["N"] * args.steps
    res = {
        "metric": METRIC,
        "value": tokens / elapsed,
        "unit": "tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic (numpy default_rng standard_normal q/k/v, seeded per image)",
        "config": {"workload": c["workload"], "global_batch": world * c["B"] if args.scaling == "weak" else c["B"],
                   "batch_per_gpu": len(images), "heads": c["H"], "seq": c["N"], "keys": c["T"],
                   "head_dim": c["D"], "k": c["k"], "pred_mode": c["mode"], "parallelism": f"dp{world}"},
        "roofline": roof,
        "stages_ms": stages,
        "e2e": e2e,
        "cpu_baseline": cpu,
        # what torch.distributed saw (a SCALE record shows RCCL ran N ranks)
        "dist": {"initialized": dist.is_initialized(),
                 "world_size": dist.get_world_size() if dist.is_initialized() else 1,
                 "backend": dist.get_backend() if dist.is_initialized() else None},
    }

    if not args.no_parity:  # a sample of every rank's shard, gathered to rank 0
        # the same sample size on every rank (all_gather needs equal shapes)
        npar = min([args.parity_images] + [len(shard(c, r, world, args.scaling)) for r in range(world)])
        sel = sorted({0, len(images) - 1})[:npar] if npar > 1 else [0]
        mine_idx = idx[sel].contiguous()
        mine_out = out[sel].contiguous()
        mine_img = torch.tensor([images[i] for i in sel], dtype=torch.int64, device=device)
        if world > 1:
            gi = [torch.empty_like(mine_idx) for _ in range(world)]
            go = [torch.empty_like(mine_out) for _ in range(world)]
            gm = [torch.empty_like(mine_img) for _ in range(world)]
            dist.all_gather(gi, mine_idx)
            dist.all_gather(go, mine_out)
            dist.all_gather(gm, mine_img)
        else:
            gi, go, gm = [mine_idx], [mine_out], [mine_img]
        if rank == 0:
            res["parity"] = parity_check(c, torch.cat(gi).cpu().numpy(), torch.cat(go).cpu().numpy(),
                                         torch.cat(gm).cpu().tolist())
            res["parity"]["ranks_checked"] = world

    run_secondary(args, c, rank, world, images, lines, run, device, res)

    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        if backend == "nccl":
            dist.destroy_process_group()
    return res if rank == 0 else 0


if __name__ == "__main__":
    rc = main()
    sys.exit(rc if isinstance(rc, int) else 0)
