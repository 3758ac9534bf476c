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
