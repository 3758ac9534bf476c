"""bench.py's launch decision (CPU): `python bench.py --gpus N` without
torchrun starts N rank processes itself, and a world that differs from
--gpus never produces a result line (VERDICT r02 "next" 1).

The ranks of the dry run (TSG_BENCH_DRYRUN=1) stop before importing torch, so
these tests need no GPU; the failing-rank case runs the real rank code on a
box without (enough) GPUs and must fail loudly.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TSG_BENCH_BACKEND",
                        "TSG_BENCH_DRYRUN", "TSG_BENCH_DRYRUN_FAIL_RANK")}
    env.update(kw)
    return env


def test_launch_mode():
    sys.path.insert(0, REPO)
    import bench
    assert bench.launch_mode(1, {}) == "rank"
    assert bench.launch_mode(8, {}) == "launch"
    assert bench.launch_mode(8, {"WORLD_SIZE": "8"}) == "rank"   # torchrun
    assert bench.launch_mode(2, {"WORLD_SIZE": "1"}) == "rank"   # then refused as a mismatch
    with pytest.raises(SystemExit):
        bench.launch_mode(0, {})


@pytest.mark.parametrize("n", [2, 3])
def test_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n)], env=_env(TSG_BENCH_DRYRUN="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    ranks = [json.loads(ln) for ln in r.stdout.splitlines() if ln.strip()]
    assert sorted(x["rank"] for x in ranks) == list(range(n))
    assert all(x["world"] == n and x["local_rank"] == x["rank"] for x in ranks)
    masters = {x["master"] for x in ranks}
    assert len(masters) == 1 and masters.pop().startswith("127.0.0.1:")


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_failed_rank_stops_the_others(fail_rank):
    """One rank exits non-zero while the others wait (as in an RCCL
    rendezvous): the launcher stops them and returns the failing code."""
    import time
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3"],
                       env=_env(TSG_BENCH_DRYRUN="1", TSG_BENCH_DRYRUN_FAIL_RANK=str(fail_rank)),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 3
    assert time.time() - t0 < 60
    assert "terminating the others" in r.stderr


def test_world_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", TSG_BENCH_DRYRUN="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert r.stdout.strip() == ""
    assert "WORLD_SIZE=2" in r.stderr


def test_missing_gpus_fail_loudly():
    """More ranks than visible GPUs over RCCL: the launcher exits non-zero and
    prints no result line (here: no GPU at all)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("this box has enough GPUs for 2 ranks")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu-rows", "0"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert r.stdout.strip() == ""
    assert "GPU(s) are visible" in r.stderr


def test_deadline_stops_a_hanging_rank():
    """VERDICT r04 "next" 1: a rank that neither exits nor fails (stuck in
    the RCCL rendezvous) must not keep the launcher waiting until the
    driver's limit: at --timeout the launcher stops every running rank by
    PID, names them and exits 124 with no result line."""
    import time
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--timeout", "5"],
                       env=_env(TSG_BENCH_DRYRUN="1", TSG_BENCH_DRYRUN_HANG_RANK="2"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 124, r.stderr
    assert time.time() - t0 < 60
    assert "rank(s) [2] still running" in r.stderr
    assert r.stdout.strip() == ""


def _args(steps=20, warmup=3):
    import argparse
    return argparse.Namespace(steps=steps, warmup=warmup, seed_w=42, seed_x=12345)


def _line(world, gather):
    sys.path.insert(0, REPO)
    import bench
    M, K, Nr, s = 4096, 4096, 16384, 4
    nnz = K * Nr // s
    return bench.build_line(_args(), world=world, mode="weak", backend="nccl" if world > 1 else None, M=M, K=K,
                            Nr=Nr, Ntot=Nr * world, s=s, nnz=nnz, nnz_all=nnz * world, kname="tsg_jit64_kernel",
                            compute_elapsed_max=20 * 1.23e-3, kern_ms_max=1.22, gather=gather)


def test_line_world_gt1_is_compute_plus_allgather():
    """At world > 1 `value` / `ms_per_step` are configs[4]'s whole step (the
    GatherPipeline: compute + all-gather), the compute-only step is a side
    key, and the gather's bandwidth per GPU is reported."""
    P, steps = 8, 20
    gather = {"allgather_ms": 2.5, "pipeline_elapsed_s": steps * 3.1e-3, "columns_match": True,
              "blocks_match": True, "bytes_received_per_gpu": 4 * 4096 * 16384 * (P - 1), "chunks": 4}
    ln = _line(P, gather)
    assert ln["value"] == ln["with_allgather"]["value"]
    assert ln["ms_per_step"] == ln["with_allgather"]["ms_per_step"] == 3.1
    flops_all = 4096 * (4096 * 16384 // 4 * P + 16384 * P)
    assert abs(ln["value"] - flops_all / 3.1e-3 / 1e9) < 1e-3 * ln["value"]
    assert ln["compute_only"]["ms_per_step"] == 1.23
    assert ln["compute_only"]["value"] > ln["value"]
    assert abs(ln["allgather_gbps_per_gpu"] - gather["bytes_received_per_gpu"] / 2.5e-3 / 1e9) < 0.01
    assert "= configs[4]" in ln["config"]["workload"] and "all-gather" in ln["config"]["parallelism"]
    assert ln["binding_roof"]["resource"] == "valu fp32 adds" and 0 < ln["binding_roof"]["frac"] < 1
    sys.path.insert(0, REPO)
    import bench
    with pytest.raises(ValueError):
        bench.headline(2, steps, flops_all, 1.0, None)


def test_line_world1_is_the_compute_step():
    ln = _line(1, None)
    assert ln["ms_per_step"] == 1.23 and ln["compute_only"] is None and ln["with_allgather"] is None
    assert ln["config"]["workload"] == "BASELINE configs[2]"
    assert ln["binding_roof"]["frac"] == ln["roofline"]["binding"]["frac"]
