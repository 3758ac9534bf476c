#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline: effective GFLOP/s (+ achieved HBM GB/s
vs roofline) of the TCSC ternary spGEMM Y = X*W + b on MI355X.

One step = one pass of the hot path over one batch: X [M,K] fp32 (resident in
HBM) -> Y [M,N] through the C-ABI (tcsc_hip_gemm_dev: X^T staging kernel +
the TCSC kernel).  Workload at N=1 = BASELINE.json configs[2]
(M=4096 K=4096 N=16384 s=4).  With --gpus G (torchrun, one process per GPU)
W's columns are sharded: every rank owns N=16384 columns of a
M x K x (16384*G) problem (G=8 -> configs[4], N=131072), no data-path
collective ("scaling": "weak"); --allgather additionally times an RCCL
all-gather of the Y column blocks outside the timed region.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))

import tspgemm as T  # noqa: E402
import tsg_dist as D  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
PROFILE_PMC = os.path.join(REPO, "profiles", "r01d_jit_pmc_summary.json")
# Binding roof of the path: fp32 VALU adds.  v_pk_add_f32 retires 2 IEEE adds per
# lane, 128 adds/clk/CU (measured 121 in scripts/issue_micro.hip), x 256 CUs x
# 2.4 GHz = 78.6 T adds/s (the 157.3 TFLOP/s fp32 vector spec counts an FMA as 2).
VALU_PEAK_TADDS = 128 * 256 * 2.4e9 / 1e12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--N", type=int, default=16384, help="columns PER GPU")
    ap.add_argument("--s", type=int, default=4)
    ap.add_argument("--seed-w", type=int, default=42)
    ap.add_argument("--seed-x", type=int, default=12345)
    ap.add_argument("--cpu-rows", type=int, default=2048,
                    help="rows of the bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--allgather", action="store_true")
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and rank == 0:
        print(f"# note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # one process per GPU; the modulo only matters for a multi-rank rehearsal
    # on a box with fewer GPUs (TSG_BENCH_BACKEND=gloo: RCCL refuses two ranks
    # on one device)
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("TSG_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    M, K, Nr, s = a.M, a.K, a.N, a.s
    Ntot = Nr * world
    n0, n1 = D.column_shard(Ntot, world, rank)  # == [rank*Nr, (rank+1)*Nr)
    assert n1 - n0 == Nr

    # --- synthetic inputs (generateSparseMatrix law), this rank's column shard
    t0 = time.time()
    csp, csn, rip, rin = T.gen_tcsc(K, Ntot, s, a.seed_w, n0, n1)
    h = T.TCSCDevice(csp, csn, rip, rin, K, Nr, device=local)
    kname = h.kernel_name()
    nnz = int(len(rip) + len(rin))
    g = torch.Generator(device=dev)
    g.manual_seed(a.seed_x)
    X = torch.randint(-512, 513, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.float32)
    b = torch.full((Nr,), 2.0, device=dev)  # main.cpp:194
    Y = torch.empty((M, Nr), device=dev)
    h.reserve(M)
    setup_s = time.time() - t0

    stream = torch.cuda.current_stream(dev)
    for _ in range(a.warmup):
        h.gemm_torch(X, b, Y)
    torch.cuda.synchronize()
    h.set_timing(True)
    h.kernel_time(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        h.gemm_torch(X, b, Y)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kern_ms_total, launches = h.kernel_time(reset=True)
    h.set_timing(False)
    stream_ms = ev0.elapsed_time(ev1)

    tt = torch.tensor([elapsed, kern_ms_total / max(launches, 1)], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed_max, kern_ms_max = float(tt[0]), float(tt[1])
    nnz_t = torch.tensor([nnz], device=dev, dtype=torch.int64)
    if world > 1:
        dist.all_reduce(nnz_t)
    nnz_all = int(nnz_t.item())

    # optional: all-gather of Y column blocks over RCCL (outside the timed region)
    allgather_ms = None
    if a.allgather and world > 1:
        Yall = D.allgather_columns(Y, Ntot, world)  # warm RCCL
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(3):
            Yall = D.allgather_columns(Y, Ntot, world)
        torch.cuda.synchronize()
        allgather_ms = (time.perf_counter() - t1) / 3 * 1e3
        del Yall

    # --- end to end through the comp_func surface (host pointers: H2D X, the
    # step, D2H Y; synchronous, as the reference calls it, main.cpp:214-216).
    # PCIe-inclusive, reported beside the headline, never as `value`.
    e2e = None
    if rank == 0 and world == 1:
        Xh, bh = X.cpu().numpy(), b.cpu().numpy()
        Yh = np.empty((M, Nr), np.float32)
        h(Xh, bh, Yh, M, Nr, K)
        reps = 3
        e0 = time.perf_counter()
        for _ in range(reps):
            h(Xh, bh, Yh, M, Nr, K)
        e_ms = (time.perf_counter() - e0) / reps * 1e3
        e2e = {"ms": round(e_ms, 3), "gflops": round(T.flops(M, Nr, nnz) / (e_ms * 1e-3) / 1e9, 1),
               "bytes_over_pcie": 4 * (M * K + Nr + M * Nr)}

    # --- CPU baseline: the oracle (BaseTCSC restatement, 1 thread) on a
    # bounded sample of the same workload; rank 0 at N=1 only.
    cpu = None
    if rank == 0 and world == 1 and a.cpu_rows > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as O
        rows = min(a.cpu_rows, M)
        Xs = X[:rows].cpu().numpy()
        tc = O.TCSC(csp, csn, rip, rin, K, Nr)
        bs = np.full(Nr, 2.0, np.float32)
        c0 = time.perf_counter()
        Ycpu = O.base_tcsc(Xs, tc, bs)
        cpu_s = time.perf_counter() - c0
        parity = bool(np.array_equal(Ycpu.view(np.uint32), Y[:rows].cpu().numpy().view(np.uint32)))
        cpu = {"value": round(T.flops(rows, Nr, nnz) / cpu_s / 1e9, 4), "unit": "GFLOP/s",
               "cores": 1, "kind": "port",
               "sample": f"BaseTCSC restatement (oracle/tcsc_oracle.c, comp.h:25-69), first {rows} of "
                         f"{M} rows, K={K} N={Nr} s={s}, gcc -O3 -fno-tree-vectorize, {cpu_s:.2f} s",
               "seconds": round(cpu_s, 3), "gpu_rows_bit_identical": parity}

    if rank == 0:
        flops_all = M * (nnz_all + Ntot)  # sum over ranks of T.flops(M, Nr, nnz_rank)
        value = flops_all * a.steps / elapsed_max / 1e9
        ms_step = elapsed_max / a.steps * 1e3
        alg_bytes = T.algorithmic_bytes(M, Nr, K, nnz)  # per launch, this rank
        adds = T.flops(M, Nr, nnz)                       # per launch: one IEEE add per (m, nonzero) + bias
        achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9
        traffic = None
        try:
            # HBM bytes per launch of THIS kernel on THIS workload, from the
            # committed rocprofv3 PMC passes (scripts/pmc_summary.py: FETCH_SIZE
            # and WRITE_SIZE with the gfx950 corrections of MI355X_MICROARCH.md)
            pm = json.load(open(PROFILE_PMC))
            if pm.get("workload") == f"{M}x{K}x{Nr}s{s}":
                traffic = pm.get("kernels", {}).get(kname, {}).get("hbm_bytes")
        except Exception:
            pass
        out = {
            "metric": "effective GFLOP/s + achieved HBM GB/s (% roofline), TCSC spGEMM M×K×N at s",
            "value": round(value, 3),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (generateSparseMatrix law, seed_w=%d; X integer U[-512,512], seed_x=%d; b=2)"
                    % (a.seed_w, a.seed_x),
            "config": {"workload": ("BASELINE configs[2]" if world == 1 else
                                    f"BASELINE configs[4]-style column shard, N_total={Ntot}"),
                       "M": M, "K": K, "N_per_gpu": Nr, "N_total": Ntot, "s": s,
                       "nnz_per_gpu": nnz, "parallelism": f"W columns x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": traffic,
                         "kernel": kname, "kernel_ms": round(kern_ms_max, 4),
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "kernel_gflops": round(adds / (kern_ms_max * 1e-3) / 1e9, 2),
                         "traffic_source": (os.path.relpath(PROFILE_PMC, REPO) if traffic is not None else None),
                         "binding": {"resource": "valu fp32 adds (DESIGN.md 5)", "adds_per_launch": adds,
                                     "achieved_Tadds": round(adds / (kern_ms_max * 1e-3) / 1e12, 2),
                                     "peak_Tadds": round(VALU_PEAK_TADDS, 2),
                                     "frac": round(adds / (kern_ms_max * 1e-3) / 1e12 / VALU_PEAK_TADDS, 4)}},
            "cpu_baseline": cpu,
            "stream_ms_per_step": round(stream_ms / a.steps, 4),
            "e2e_host_pointers": e2e,
            "allgather_ms": None if allgather_ms is None else round(allgather_ms, 3),
            "setup_s": round(setup_s, 2),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
