"""Multi-process path of bench.py on CPU (gloo, world_size 2), end to end through
bench.main: each rank generates its own shard of images (weak: B images per rank;
strong: the batch split over the ranks), the timed region is bracketed by barriers
and the reported time is the MAX over ranks, and a sample of every rank's indices /
outputs is all_gathered to rank 0 and checked against the oracle.
The HIP op itself needs a GPU: here the per-rank step (bench.run_config) is a CPU
stand-in that produces the op's outputs with the oracle and sleeps a rank-dependent
time."""
import json
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

SMALL = dict(B=3, H=2)  # deit_base shape with 3 images of 2 heads per rank


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stub_run(c, images, steps, warmup, device, world, prof):
    """CPU stand-in for run_config: the op's outputs from the oracle, a timed region of
    rank-dependent length."""
    import bench
    from oracle import mx_oracle as O
    q, k, v, bias = bench.make_inputs(c, images)
    r = O.attention(q, k, v, c["scale"], k_top=c["k"], pred_mode=c["mode"], bias=bias, flush=c["bias"])
    rank = dist.get_rank() if dist.is_initialized() else 0
    elapsed = bench.timed_region(lambda: time.sleep(0.05 * (rank + 1)), world, lambda: None, device)
    stages = {s: 0.0 for s in bench.STAGES}
    roof = {"frac": 0.0, "qa_pass": {"frac": 0.0}}
    return elapsed, stages, roof, {}, torch.from_numpy(r["out"]), torch.from_numpy(r["idx"])


def _worker(rank, world, port, argv, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MXA_BENCH_BACKEND="gloo")
    import bench
    bench.CONFIGS["deit_base"] = dict(bench.CONFIGS["deit_base"], **SMALL)
    res = bench.main(argv, run=_stub_run)
    if rank == 0:
        out["res"] = json.dumps(res)
    dist.destroy_process_group()


def _run_world(argv, world=2):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, argv, out), nprocs=world, join=True)
    return json.loads(out["res"])


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_bench_main_two_ranks_gathers_and_checks_every_shard(scaling):
    res = _run_world(["--gpus", "2", "--steps", "3", "--warmup", "1", "--no-secondary", "--scaling", scaling,
                      "--parity-images", "2"])
    assert res["n_gpus"] == 2 and res["scaling"] == scaling
    assert res["config"]["parallelism"] == "dp2"
    assert res["dist"] == {"initialized": True, "world_size": 2, "backend": "gloo"}
    # the MAX over ranks: at least the slower rank's region (0.1 s)
    assert res["ms_per_step"] * res["steps"] >= 100.0
    par = res["parity"]
    assert par["ranks_checked"] == 2
    assert par["idx_bitmatch"] == 1.0 and par["out_normwise_rel_err_max"] == 0.0
    if scaling == "weak":  # 3 images per rank: ranks hold images 0-2 and 3-5, two checked each
        assert res["config"]["global_batch"] == 6 and res["config"]["batch_per_gpu"] == 3
        assert par["images_checked"] == 4
        assert res["value"] == pytest.approx(6 * 197 * 3 / (res["ms_per_step"] * 3 / 1e3))
    else:  # the 3-image batch split 2 + 1: one image of each rank checked (equal all_gather shapes)
        assert res["config"]["global_batch"] == 3 and res["config"]["batch_per_gpu"] == 2
        assert par["images_checked"] == 2


def test_bench_shards_and_per_image_inputs():
    import bench
    c = dict(bench.CONFIGS["deit_base"], **SMALL)
    assert bench.shard(c, 1, 2, "weak") == [3, 4, 5]
    assert bench.shard(c, 0, 2, "strong") == [0, 1] and bench.shard(c, 1, 2, "strong") == [2]
    assert sum((bench.shard(dict(c, B=256), r, 8, "strong") for r in range(8)), []) == list(range(256))
    # an image is the same whatever shard it is generated in
    q_a = bench.make_inputs(c, [0, 1, 2])[0][2]
    q_b = bench.make_inputs(c, [2])[0][0]
    assert np.array_equal(q_a, q_b)


def test_bench_single_rank_timed_region_has_no_collectives():
    import bench
    calls = []
    e = bench.timed_region(lambda: calls.append(1), 1, lambda: calls.append(0), torch.device("cpu"))
    assert calls == [0, 1, 0] and e >= 0.0
    assert not dist.is_initialized()


def test_bench_byte_and_op_accounting():
    """Algorithmic bytes per kernel and the SURVEY §8d totals."""
    import bench
    c = bench.CONFIGS["deit_base"]
    split = bench.stage_bytes(c, "rows_split")
    dense = bench.stage_bytes(c, "rows_fused")
    h, N, k = c["B"] * c["H"], c["N"], c["k"]
    assert list(split) == list(dense) == list(bench.STAGES)
    assert dense["select"] == 0 and split["finish"] - dense["finish"] == h * 8 * N * k
    assert bench.fused_min_bytes(c) == 716537856  # 716.5 MB at DeiT-base b256
    assert abs(bench.bytes_qa(c) - 633.2e6) < 0.1e6  # SURVEY.md §8d Bytes_qa
    assert abs(bench.ops_gemm(c) - 30.52e9) < 0.01e9  # SURVEY.md §8d Ops_gemm
    assert abs(bench.bytes_qa(bench.CONFIGS["dit_xl2"]) - 446.8e6) < 0.1e6


def test_hbm_traffic_kernel_names_map_to_bench_stages():
    ht = _load_hbm_traffic()
    assert ht.stage_of("void mxa::select_kernel<256, 3, 2, unsigned int, 1, 64>(mxa::Rows2Args)") == "select"
    assert ht.stage_of("void mxa::select_kernel<256, 3, 2, unsigned long, 0, 0>(mxa::Rows2Args)") == "select_fb"
    assert ht.stage_of("void mxa::topk_tail_kernel<64>(mxa::TailArgs)") == "select_tail"
    assert ht.stage_of("void mxa::finish_qk_kernel<3, 8, false>(mxa::Rows2Args)") == "finish"
    assert ht.stage_of("void mxa::finish_kernel<2, 2>(mxa::Rows2Args)") == "finish"
    assert ht.stage_of("void mxa::dense_rows_kernel<4>(mxa::Rows2Args)") == "finish"
    assert ht.stage_of("mxa::attn_prep_kernel(mxa::RowsPrepArgs, mxa::RowsPrepArgs, mxa::ColsPrepArgs, unsigned int, "
                       "unsigned int)") == "prep"
    assert ht.stage_of("void mxa::qkv_proj_kernel<2>(mxa::ProjArgs)") == "proj"


def _load_hbm_traffic():
    import importlib.util
    spec = importlib.util.spec_from_file_location("hbm_traffic", os.path.join(ROOT, "tools", "hbm_traffic.py"))
    ht = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ht)
    return ht


def test_hbm_traffic_never_averages_two_instantiations_of_a_stage():
    """Round 2's DeiT select traffic was the average of DeiT's select_kernel<256,3,2> and
    DiT's select_kernel<256,3,4> dispatches: per-instantiation keys keep them apart, and a
    stage with two instantiations in one run gets no traffic number at all."""
    ht = _load_hbm_traffic()
    deit, dit = ("void mxa::select_kernel<256, 3, 2, unsigned int, 1, 64>(mxa::Rows2Args)",
                 "void mxa::select_kernel<256, 3, 4, unsigned int, 0, 0>(mxa::Rows2Args)")
    fin = "void mxa::finish_kernel<2, 12, true>(mxa::Rows2Args)"
    rows = []
    for name, kib_f, kib_w, n in ((deit, 10.0, 143250.0, 7), (dit, 20.0, 473145.0, 3), (fin, 100.0, 200.0, 7)):
        for _ in range(n):
            rows.append({"Kernel_Name": name, "Counter_Name": "FETCH_SIZE", "Counter_Value": str(kib_f)})
            rows.append({"Kernel_Name": name, "Counter_Name": "WRITE_SIZE", "Counter_Value": str(kib_w)})
    out = ht.combine(ht.per_kernel(rows, "FETCH_SIZE"), ht.per_kernel(rows, "WRITE_SIZE"))
    assert out["kernels"][deit]["write_bytes"] == 143250.0 * 1024 and out["kernels"][deit]["dispatches"] == [7, 7]
    assert out["kernels"][dit]["write_bytes"] == 473145.0 * 1024
    assert out["kernels"][deit]["traffic_bytes"] == (2 * 10.0 + 143250.0) * 1024
    assert "select" not in out["stages"] and sorted(out["ambiguous"]["select"]) == sorted([deit, dit])
    assert out["stages"]["finish"] == (2 * 100.0 + 200.0) * 1024
    # a run with one instantiation per stage maps every stage
    one = ht.combine(ht.per_kernel(rows[:14], "FETCH_SIZE"), ht.per_kernel(rows[:14], "WRITE_SIZE"))
    assert one["stages"] == {"select": (2 * 10.0 + 143250.0) * 1024} and not one["ambiguous"]


def test_hbm_traffic_select_stage_sums_its_kernels():
    """The selection stage's HIP events span the packed kernel, the one-lane tail and the
    64-bit pass: its traffic per launch is the sum of the three."""
    ht = _load_hbm_traffic()
    names = {"void mxa::select_kernel<256, 3, 2, unsigned int, 1, 64>(mxa::Rows2Args)": 100.0,
             "void mxa::topk_tail_kernel<64>(mxa::TailArgs)": 10.0,
             "void mxa::select_kernel<256, 3, 2, unsigned long, 0, 0>(mxa::Rows2Args)": 1.0}
    rows = []
    for name, kib in names.items():
        for _ in range(3):
            rows.append({"Kernel_Name": name, "Counter_Name": "FETCH_SIZE", "Counter_Value": str(kib)})
            rows.append({"Kernel_Name": name, "Counter_Name": "WRITE_SIZE", "Counter_Value": str(kib)})
    out = ht.combine(ht.per_kernel(rows, "FETCH_SIZE"), ht.per_kernel(rows, "WRITE_SIZE"))
    assert out["stages"]["select"] == 3 * 111.0 * 1024
    assert out["stages"]["select_parts"]["select_tail"] == 3 * 10.0 * 1024


def test_bench_limiter_from_profiles(tmp_path):
    import bench
    sel = "void mxa::select_kernel<256, 3, 2, unsigned int, 1, 64>(mxa::Rows2Args)"
    tj, pj = tmp_path / "t.json", tmp_path / "p.json"
    tj.write_text(json.dumps({"stages": {"select": 160e6}}))
    # 0.5 ms: HBM 160 MB -> 0.04 of peak; VALU 436 M instr x 2 cycles over 1024 SIMDs at 2.4 GHz -> 0.71
    pj.write_text(json.dumps({sel: {"SQ_INSTS_VALU": 436e6, "SQ_WAVE_CYCLES": 10.0, "SQ_WAIT_ANY": 4.0,
                                    "SQ_LDS_BANK_CONFLICT": 5.0, "SQ_INSTS_LDS": 10.0}}))
    traffic, lim = bench.profile_of({"traffic": str(tj), "pmc": str(pj)}, "select", 0.5, 320.0)
    assert traffic == 160e6 and lim["bound"] == "valu" and lim["kernel"] == sel
    assert abs(lim["fracs"]["valu_issue"] - 436e6 * 2 / (1024 * 2.4e9 * 0.5e-3)) < 1e-9
    assert lim["lds_conflict_cycles_per_lds_instr"] == 0.5
    # two instantiations of the stage in the PMC file: no kernel is picked
    pj.write_text(json.dumps({sel: {"SQ_INSTS_VALU": 1.0}, sel.replace("1, 64>", "0, 0>"): {"SQ_INSTS_VALU": 1.0}}))
    _, lim = bench.profile_of({"pmc": str(pj)}, "select", 0.5, 320.0)
    assert "kernel" not in lim and lim["bound"] == "hbm"


def _dit_worker(rank, world, port, argv, out):
    """bench.main on the DiT-XL/2 config (2 heads per image to keep the oracle cheap); the
    stand-in records which images this rank generated and checks them against the
    images a 1-rank run generates for the same ids."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), MXA_BENCH_BACKEND="gloo")
    import bench
    bench.CONFIGS["dit_xl2"] = dict(bench.CONFIGS["dit_xl2"], H=2)

    def run(c, images, steps, warmup, device, world_, prof):
        out[f"images{rank}"] = list(images)
        q, k, v, _ = bench.make_inputs(c, images)
        q1, k1, v1, _ = bench.make_inputs(c, list(range(c["B"])))  # the 1-rank run's batch
        out[f"same{rank}"] = bool(np.array_equal(q, q1[images]) and np.array_equal(k, k1[images])
                                  and np.array_equal(v, v1[images]))
        return _stub_run(c, images, steps, warmup, device, world_, prof)

    res = bench.main(argv, run=run)
    if rank == 0:
        out["res"] = json.dumps(res)
    dist.destroy_process_group()


def test_bench_dit_strong_scaling_two_ranks_shard_boundaries():
    """configs[3] (DiT-XL/2 sharded over GPUs, strong scaling): B = 64 over 2 ranks is
    images 0-31 and 32-63, each rank's inputs equal the 1-rank run's images, the job
    reports the whole batch, and rank 0 checks a sample of both shards."""
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    argv = ["--config", "dit_xl2", "--gpus", "2", "--steps", "2", "--warmup", "1", "--no-secondary",
            "--scaling", "strong", "--parity-images", "1", "--no-cpu-baseline"]
    mp.spawn(_dit_worker, args=(2, port, argv, out), nprocs=2, join=True)
    assert out["images0"] == list(range(32)) and out["images1"] == list(range(32, 64))
    assert out["same0"] and out["same1"]
    res = json.loads(out["res"])
    assert res["config"]["global_batch"] == 64 and res["config"]["batch_per_gpu"] == 32
    assert res["scaling"] == "strong" and res["n_gpus"] == 2
    assert res["value"] == pytest.approx(64 * 256 * 2 / (res["ms_per_step"] * 2 / 1e3))
    assert res["parity"]["ranks_checked"] == 2 and res["parity"]["idx_bitmatch"] == 1.0
