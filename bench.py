#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline: effective GFLOP/s (+ achieved HBM GB/s
vs roofline) of the TCSC ternary spGEMM Y = X*W + b on MI355X.

One step = one pass of the hot path over one batch: X [M,K] fp32 (resident in
HBM) -> Y [M,N] through the C-ABI (tcsc_hip_gemm_dev: X^T staging kernel +
the TCSC kernel).  Workload at N=1 = BASELINE.json configs[2]
(M=4096 K=4096 N=16384 s=4).

Multi-GPU (torchrun, one process per GPU, RCCL): W's columns are sharded
(tsg_dist.py).  `value` is the compute step (every rank's Y column block, no
collective on the compute path); for world > 1 the line also carries the
RCCL all-gather of the Y blocks into the row-major [M, N] result:
`allgather_ms` (the gather alone) and `with_allgather` (the step as
compute + gather pipelined by M chunks, tsg_dist.GatherPipeline).
  * default (weak): every rank owns --N columns (N_total = N * P; P = 8 is
    configs[4], N = 131072); each rank draws only its own column block.
  * --strong: N_total = --N fixed, N/P columns per rank (same W for every P).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strong]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))

import tspgemm as T  # noqa: E402
import tsg_dist as D  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
PROFILE_PMC = os.path.join(REPO, "profiles", "r02final_jit_pmc_summary.json")
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
    ap.add_argument("--N", type=int, default=16384, help="columns per GPU (weak) or in total (--strong)")
    ap.add_argument("--s", type=int, default=4)
    ap.add_argument("--strong", action="store_true", help="N fixed in total, split over the GPUs")
    ap.add_argument("--chunks", type=int, default=4, help="M chunks of the compute/all-gather pipeline")
    ap.add_argument("--clock-warmup", type=float, default=0.3,
                    help="seconds of untimed steps before the warmup steps (GPU clock ramp; 0 = none)")
    ap.add_argument("--seed-w", type=int, default=42)
    ap.add_argument("--seed-x", type=int, default=12345)
    ap.add_argument("--cpu-rows", type=int, default=512,
                    help="rows of the bounded single-thread CPU-baseline samples (0 = skip the CPU legs)")
    return ap.parse_args()


def host_info() -> dict:
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "cpus_in_affinity": avail,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(X, csp, csn, rip, rin, K, N, s, Y_gpu, rows1):
    """The oracle (BaseTCSC restatement, oracle/tcsc_oracle.c) timed with the
    reference's method (perf.cpp:37-71: rdtsc, CALIBRATE to >= 1e8 cycles) on
    the host cores of the GPU box: three legs, each checked bit for bit against
    the GPU's rows of the same workload."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    host = host_info()
    threads = int(host["omp_num_threads_env"] or host["cpus_in_affinity"] or 1)
    M = X.shape[0]
    tc = O.TCSC(csp, csn, rip, rin, K, N)
    bs = np.full(N, 2.0, np.float32)
    Xh = X.cpu().numpy()
    nnz = len(rip) + len(rin)
    legs = []
    for name, kern, th, rows in (("BaseTCSC", "BaseTCSC", 1, rows1),
                                 ("DoubleUnrolledTCSC_K4_M4", "DoubleUnrolledTCSC_K4_M4", 1, rows1),
                                 ("BaseTCSC_omp", "BaseTCSC_omp", threads, M)):
        rows = min(rows, M)
        Xs = np.ascontiguousarray(Xh[:rows])
        sec, runs, cyc, Yc = O.perf_calibrated(kern, Xs, tc, bs, threads=th if kern.endswith("omp") else 0)
        same = bool(np.array_equal(Yc.view(np.uint32), Y_gpu[:rows].cpu().numpy().view(np.uint32)))
        legs.append({"kernel": name, "value": round(T.flops(rows, N, nnz) / sec / 1e9, 4), "unit": "GFLOP/s",
                     "cores": th, "rows": rows, "sec_per_call": round(sec, 4), "runs": runs,
                     "tsc_cycles_per_call": round(cyc), "flops_per_tsc_cycle": round(T.flops(rows, N, nnz) / cyc, 4),
                     "bit_identical_to_gpu_rows": same,
                     "source": {"BaseTCSC": "comp.h:25-69", "DoubleUnrolledTCSC_K4_M4": "comp.h:1227-1438",
                                "BaseTCSC_omp": "comp.h:25-69 + OpenMP over rows (our parallelisation)"}[name]})
    base = legs[0]
    return {"value": base["value"], "unit": "GFLOP/s", "cores": 1, "kind": "port",
            "sample": (f"BaseTCSC restatement (oracle/tcsc_oracle.c, comp.h:25-69), first {base['rows']} of {M} rows, "
                       f"K={K} N={N} s={s}, gcc -O3 -fno-tree-vectorize, timed as perf.cpp:37-71 "
                       f"(rdtsc, calibrated to >= 1e8 cycles, {base['runs']} run(s) of {base['sec_per_call']} s); "
                       f"legs: 1-thread BaseTCSC, 1-thread DoubleUnrolledTCSC<4,4> (the reference's best), "
                       f"BaseTCSC + OpenMP on {threads} threads over all {M} rows"),
            "host": host, "legs": legs}


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
    backend = None
    if world > 1:
        backend = os.environ.get("TSG_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    M, K, s = a.M, a.K, a.s
    mode = "strong" if a.strong else "weak"
    Ntot = a.N if a.strong else a.N * world
    n0, n1 = D.column_shard(Ntot, world, rank)
    Nr = n1 - n0

    # --- synthetic inputs: this rank's column block only (tsg_dist.py)
    t0 = time.time()
    csp, csn, rip, rin = D.ShardedTCSC.draw(K, Ntot, s, a.seed_w, rank, world, mode)
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

    def barrier():
        if world > 1:
            dist.barrier()

    stream = torch.cuda.current_stream(dev)
    # Clock warm-up (untimed, before the W warmup steps): after idle the GPU
    # runs the first ~25 launches at a ramping clock (1.47-1.67 ms -> a steady
    # 1.27-1.29 ms at config 3, profiles/r02c_clock_ramp.txt); the timed
    # region then measures the steady state.  Reported as clock_warmup_s.
    cw0 = time.perf_counter()
    n_clock = 0
    while time.perf_counter() - cw0 < a.clock_warmup:
        for _ in range(8):
            h.gemm_torch(X, b, Y)
        n_clock += 8
        torch.cuda.synchronize()
    clock_warmup_s = time.perf_counter() - cw0
    for _ in range(a.warmup):
        h.gemm_torch(X, b, Y)
    torch.cuda.synchronize()
    h.set_timing(True)
    h.kernel_time(reset=True)
    barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        h.gemm_torch(X, b, Y)
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kern_ms_total, launches = h.kernel_time(reset=True)
    h.set_timing(False)
    stream_ms = ev0.elapsed_time(ev1)

    # --- world > 1: the RCCL all-gather of the Y column blocks (north_star's
    # collective), alone and pipelined with the compute by M chunks
    gather = None
    if world > 1:
        Yfull = torch.empty((M, Ntot), device=dev)
        for _ in range(2):  # warm RCCL
            Yall = D.allgather_columns(Y, Ntot, world)
        del Yall
        torch.cuda.synchronize()
        barrier()
        reps = max(3, a.steps // 4)
        tg = time.perf_counter()
        for _ in range(reps):
            Yall = D.allgather_columns(Y, Ntot, world)
        torch.cuda.synchronize()
        barrier()
        ag_s = (time.perf_counter() - tg) / reps
        del Yall
        pipe = D.GatherPipeline(M, Ntot, world, chunks=a.chunks, device=dev)
        Xc = {(r0, r1): X[r0:r1] for r0, r1 in pipe.ranges}  # row slices: contiguous

        def compute(r0, r1, Yc):
            h.gemm_torch(Xc[(r0, r1)], b, Yc)

        for _ in range(a.warmup):
            pipe.run(compute, Yfull, Nr)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for _ in range(a.steps):
            pipe.run(compute, Yfull, Nr)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        pipe_s = (time.perf_counter() - tp) / a.steps
        # the pipelined result equals the compute-only blocks (this rank's columns)
        ok = torch.equal(Yfull[:, n0:n1].view(torch.int32), Y.view(torch.int32))
        tg = torch.tensor([ag_s, pipe_s, 0.0 if ok else 1.0], device=dev, dtype=torch.float64)
        dist.all_reduce(tg, op=dist.ReduceOp.MAX)
        gather = {"allgather_ms": float(tg[0]) * 1e3, "pipeline_ms": float(tg[1]) * 1e3,
                  "columns_match": float(tg[2]) == 0.0,
                  "bytes_received_per_gpu": 4 * M * (Ntot - Nr), "chunks": len(pipe.ranges)}
        del pipe, Yfull

    tt = torch.tensor([elapsed, kern_ms_total / max(launches, 1)], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed_max, kern_ms_max = float(tt[0]), float(tt[1])
    nnz_t = torch.tensor([nnz], device=dev, dtype=torch.int64)
    if world > 1:
        dist.all_reduce(nnz_t)
    nnz_all = int(nnz_t.item())

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

    # --- CPU baseline (rank 0 at N=1 only): bounded samples of the same workload
    cpu = None
    if rank == 0 and world == 1 and a.cpu_rows > 0:
        cpu = cpu_baseline(X, csp, csn, rip, rin, K, Nr, s, Y, a.cpu_rows)

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
        if world == 1:
            workload = "BASELINE configs[2]" if (M, K, Nr, s) == (4096, 4096, 16384, 4) else "custom"
        elif mode == "weak":
            workload = (f"BASELINE configs[4]-style weak column shard: {Nr} columns per GPU, N_total={Ntot}"
                        + (" (= configs[4])" if (M, K, Ntot, s, world) == (4096, 4096, 131072, 4, 8) else ""))
        else:
            workload = f"strong column shard of N={Ntot} over {world} GPUs ({Nr} columns per GPU)"
        with_gather = None
        if gather is not None:
            with_gather = {"ms_per_step": round(gather["pipeline_ms"], 4),
                           "value": round(flops_all / (gather["pipeline_ms"] * 1e-3) / 1e9, 3),
                           "unit": "GFLOP/s",
                           "note": "compute + RCCL all-gather of Y into row-major [M, N_total], pipelined by "
                                   f"{gather['chunks']} M chunks (tsg_dist.GatherPipeline)",
                           "columns_match_compute_only": gather["columns_match"],
                           "bytes_received_per_gpu": gather["bytes_received_per_gpu"]}
        out = {
            "metric": "effective GFLOP/s + achieved HBM GB/s (% roofline), TCSC spGEMM M×K×N at s",
            "value": round(value, 3),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": mode,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (generateSparseMatrix law, seed_w=%d; X integer U[-512,512], seed_x=%d; b=2)"
                    % (a.seed_w, a.seed_x),
            "config": {"workload": workload, "M": M, "K": K, "N_per_gpu": Nr, "N_total": Ntot, "s": s,
                       "nnz_per_gpu": nnz, "parallelism": f"W columns x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": traffic,
                         "kernel": kname, "kernel_ms": round(kern_ms_max, 4),
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "kernel_gflops": round(adds / (kern_ms_max * 1e-3) / 1e9, 2),
                         "traffic_source": (os.path.relpath(PROFILE_PMC, REPO) if traffic is not None else None),
                         "binding": {"resource": "valu fp32 adds (DESIGN.md 4)", "adds_per_launch": adds,
                                     "achieved_Tadds": round(adds / (kern_ms_max * 1e-3) / 1e12, 2),
                                     "peak_Tadds": round(VALU_PEAK_TADDS, 2),
                                     "frac": round(adds / (kern_ms_max * 1e-3) / 1e12 / VALU_PEAK_TADDS, 4)}},
            "cpu_baseline": cpu,
            "stream_ms_per_step": round(stream_ms / a.steps, 4),
            "e2e_host_pointers": e2e,
            "allgather_ms": None if gather is None else round(gather["allgather_ms"], 3),
            "with_allgather": with_gather,
            "setup_s": round(setup_s, 2),
            "clock_warmup": {"seconds": round(clock_warmup_s, 3), "steps": n_clock},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
