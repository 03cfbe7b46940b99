"""Multi-process path of bench.py on CPU (gloo, world_size 2): each rank builds
its own shard of images (weak scaling, no data-path collective), the timed region
is bracketed by barriers, and the reported time is the MAX over ranks
(SURVEY.md §8e).  The HIP path itself needs a GPU; here the per-rank "step" is a
CPU stand-in with a rank-dependent duration."""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        c = dict(bench.CONFIGS["deit_base"], B=2, H=2)
        q, k, v, bias = bench.make_inputs(c, rank)
        # every rank's shard is its own images: gather a checksum of each
        sums = [torch.zeros(3, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(sums, torch.tensor([q.sum(), k.sum(), v.sum()], dtype=torch.float64))
        delay = 0.05 * (rank + 1)
        elapsed = bench.timed_region(lambda: time.sleep(delay), world, lambda: None, torch.device("cpu"))
        out[rank] = (elapsed, [s.tolist() for s in sums])
    finally:
        dist.destroy_process_group()


def test_bench_timed_region_max_over_ranks_and_sharded_inputs():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    e0, sums0 = out[0]
    e1, sums1 = out[1]
    # both ranks report the same MAX, at least the slowest rank's step
    assert e0 == e1
    assert e0 >= 0.1
    # rank shards differ, and each rank reproduces its shard deterministically
    assert sums0 == sums1
    assert sums0[0] != sums0[1]
    import bench
    c = dict(bench.CONFIGS["deit_base"], B=2, H=2)
    q1, _, _, _ = bench.make_inputs(c, 1)
    assert np.isclose(float(q1.astype(np.float64).sum()), sums0[1][0])


def test_bench_single_rank_timed_region_has_no_collectives():
    import bench
    calls = []
    e = bench.timed_region(lambda: calls.append(1), 1, lambda: calls.append(0), torch.device("cpu"))
    assert calls == [0, 1, 0] and e >= 0.0
    assert not dist.is_initialized()


def test_bench_stage_bytes_by_path():
    """Algorithmic bytes per kernel: the split path's two kernels move
    the fused kernel's inputs plus the 4-byte kept indices written once and read once."""
    import bench
    c = bench.CONFIGS["deit_base"]
    split = bench.stage_bytes(c, "rows_split")
    fused = bench.stage_bytes(c, "rows_fused")
    h, N, k = c["B"] * c["H"], c["N"], c["k"]
    assert list(split)[:3] == list(fused)[:3] == ["rows_prep_q", "rows_prep_k", "cols_prep_v"]
    assert split["select"] + split["finish"] == fused["fused"] + h * 8 * N * k
    assert bench.fused_min_bytes(c) == 716537856  # 716.5 MB at DeiT-base b256


def test_hbm_traffic_kernel_names_map_to_bench_stages():
    import importlib.util
    spec = importlib.util.spec_from_file_location("hbm_traffic", os.path.join(ROOT, "tools", "hbm_traffic.py"))
    ht = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ht)
    assert ht.stage_of("void mxa::attn_rows2_kernel<4, 3, true, false, 1>(mxa::Rows2Args)") == "select"
    assert ht.stage_of("void mxa::attn_rows2_kernel<4, 3, true, true, 2>(mxa::Rows2Args)") == "finish"
    assert ht.stage_of("void mxa::attn_rows2_kernel<4, 0, false, false, 0>(mxa::Rows2Args)") == "fused"
    assert ht.stage_of("mxa::rows_prep_kernel(mxa::RowsPrepArgs)") == "rows_prep"
    assert ht.stage_of("mxa::cols_prep_kernel(mxa::ColsPrepArgs)") == "cols_prep_v"
