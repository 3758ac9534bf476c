#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline: effective GFLOP/s (+ achieved HBM GB/s
vs roofline) of the TCSC ternary spGEMM Y = X*W + b on MI355X.

One step = one pass of the hot path over one batch: X [M,K] fp32 (resident in
HBM) -> Y [M,N] through the C-ABI (tcsc_hip_gemm_dev: X^T staging kernel +
the TCSC kernel).  Workload at N=1 = BASELINE.json configs[2]
(M=4096 K=4096 N=16384 s=4).

Multi-GPU (one process per GPU, RCCL): W's columns are sharded
(tsg_dist.py).  At world > 1 a step is configs[4]'s WHOLE work: every rank's
Y column block computed AND the RCCL all-gather of the blocks into the
row-major [M, N_total] result on every rank, pipelined by M chunks
(tsg_dist.GatherPipeline) -- `value` and `ms_per_step` time exactly that.
The compute-only step (no collective) is reported beside it as
`compute_only`, the gather alone as `allgather_ms` with its achieved
bandwidth per GPU (`allgather_gbps_per_gpu` = bytes received per GPU / time).
  * default (weak): every rank owns --N columns (N_total = N * P; P = 8 is
    configs[4], N = 131072); each rank draws only its own column block.
  * --strong: N_total = --N fixed, N/P columns per rank (same W for every P).

Launch: under torchrun (WORLD_SIZE set) this process is one rank, and
WORLD_SIZE must equal --gpus.  Without WORLD_SIZE and with --gpus N > 1 this
process is only the launcher: it starts N rank processes (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT) before anything touches the
GPU, forwards rank 0's JSON line, and exits non-zero if a rank fails, if the
world that ran differs from --gpus, or if the ranks are still running at the
--timeout deadline (then they are stopped by PID and the launcher names
them).  A rank whose LOCAL_RANK has no GPU fails (RCCL), except in the
one-GPU rehearsal TSG_BENCH_BACKEND=gloo, where ranks share the visible
devices.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strong] [--timeout S]
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
PROFILE_PMC = os.path.join(REPO, "profiles", "r06final_pmc_summary.json")
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
    ap.add_argument("--clock-warmup", type=float, default=1.0,
                    help="seconds of untimed steps before the warmup steps (GPU clock ramp; 0 = none)")
    ap.add_argument("--seed-w", type=int, default=42)
    ap.add_argument("--seed-x", type=int, default=12345)
    ap.add_argument("--cpu-rows", type=int, default=512,
                    help="rows of the bounded single-thread CPU-baseline samples (0 = skip the CPU legs)")
    ap.add_argument("--timeout", type=float, default=420.0,
                    help="launcher deadline in seconds (--gpus N > 1 without torchrun): ranks still running "
                         "then are stopped by PID and the launcher exits 124")
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
    omp_name = f"BaseTCSC_omp{threads}"
    for name, kern, th, rows in (("BaseTCSC", "BaseTCSC", 1, rows1),
                                 ("DoubleUnrolledTCSC_K4_M4", "DoubleUnrolledTCSC_K4_M4", 1, rows1),
                                 (omp_name, "BaseTCSC_omp", threads, M)):
        rows = min(rows, M)
        Xs = np.ascontiguousarray(Xh[:rows])
        sec, runs, cyc, Yc = O.perf_calibrated(kern, Xs, tc, bs, threads=th if kern.endswith("omp") else 0)
        same = bool(np.array_equal(Yc.view(np.uint32), Y_gpu[:rows].cpu().numpy().view(np.uint32)))
        legs.append({"kernel": name, "value": round(T.flops(rows, N, nnz) / sec / 1e9, 4), "unit": "GFLOP/s",
                     "cores": th, "rows": rows, "sec_per_call": round(sec, 4), "runs": runs,
                     "tsc_cycles_per_call": round(cyc), "flops_per_tsc_cycle": round(T.flops(rows, N, nnz) / cyc, 4),
                     "bit_identical_to_gpu_rows": same,
                     "source": {"BaseTCSC": "comp.h:25-69", "DoubleUnrolledTCSC_K4_M4": "comp.h:1227-1438",
                                omp_name: f"comp.h:25-69 + OpenMP over rows on {threads} threads (our "
                                          f"parallelisation; OMP_NUM_THREADS={host['omp_num_threads_env']}: "
                                          f"the box's CPU share, of {host['cpus_in_affinity']} CPUs in "
                                          f"affinity)"}[name]})
    base = legs[0]
    return {"value": base["value"], "unit": "GFLOP/s", "cores": 1, "kind": "port",
            "sample": (f"BaseTCSC restatement (oracle/tcsc_oracle.c, comp.h:25-69), first {base['rows']} of {M} rows, "
                       f"K={K} N={N} s={s}, gcc -O3 -fno-tree-vectorize, timed as perf.cpp:37-71 "
                       f"(rdtsc, calibrated to >= 1e8 cycles, {base['runs']} run(s) of {base['sec_per_call']} s); "
                       f"legs: 1-thread BaseTCSC, 1-thread DoubleUnrolledTCSC<4,4> (the reference's best), "
                       f"BaseTCSC + OpenMP on {threads} threads (the box's CPU share; "
                       f"{host['cpus_in_affinity']} CPUs in affinity) over all {M} rows"),
            "host": host, "legs": legs}


def launch_mode(gpus: int, env) -> str:
    """'rank': this process is one rank (torchrun, a launched rank, or N = 1);
    'launch': start `gpus` rank processes (no WORLD_SIZE and gpus > 1)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    return "rank" if "WORLD_SIZE" in env or gpus == 1 else "launch"


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a) -> int:
    """Start --gpus rank processes of this script (one per GPU) and wait for
    them.  Runs before any torch / HIP call in this process: the ranks are
    children (never an exec of this process).  Rank 0's stdout (the JSON
    line) is forwarded after checking its n_gpus; every other output goes to
    stderr.  If a rank fails, the others are terminated (by PID) and the
    failing exit code is returned.  If ranks are still running at the
    deadline (--timeout: e.g. one stuck in the RCCL rendezvous, neither
    exited nor failed), every running rank is terminated by PID, the
    launcher names them and returns 124."""
    import subprocess
    import threading
    n = a.gpus
    port = _free_port()
    dry = os.environ.get("TSG_BENCH_DRYRUN") == "1"
    procs, outs = [], [[] for _ in range(n)]
    t_launch = time.time()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        piped = r == 0 or dry
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if piped else sys.stderr, text=True))
    readers = []
    for r, p in enumerate(procs):
        if p.stdout is not None:
            t = threading.Thread(target=lambda p=p, o=outs[r]: o.extend(p.stdout), daemon=True)
            t.start()
            readers.append(t)

    def stop_running():
        # SIGTERM, then SIGKILL after 10 s, by PID (never by pattern)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + 10
        while time.time() < t_end and any(p.poll() is None for p in procs):
            time.sleep(0.1)
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()

    rc = 0
    while True:
        codes = [p.poll() for p in procs]  # every rank, every round (no short-circuit)
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            # a failed rank leaves the others waiting in the rendezvous or a
            # collective: stop them
            rc = bad[0]
            print(f"bench.py: a rank exited with {rc}; terminating the others", file=sys.stderr)
            stop_running()
            break
        if all(c is not None for c in codes):
            break
        if time.time() - t_launch > a.timeout:
            running = [r for r, c in enumerate(codes) if c is None]
            print(f"bench.py: deadline of {a.timeout:g} s passed with rank(s) {running} still running "
                  f"(pids {[procs[r].pid for r in running]}); terminating them", file=sys.stderr)
            stop_running()
            for t in readers:
                t.join(timeout=5)
            print(f"bench.py: no result: --gpus {n} timed out", file=sys.stderr)
            return 124
        time.sleep(0.2)
    for t in readers:
        t.join(timeout=10)
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    if dry:
        for r in range(n):
            sys.stdout.write("".join(outs[r]))
        return rc
    lines = [ln for ln in outs[0] if ln.strip()]
    for ln in lines[:-1]:
        sys.stderr.write(ln)
    if rc != 0:
        print(f"bench.py: rank failure (exit {rc}) with --gpus {n}", file=sys.stderr)
        return rc
    if not lines:
        print("bench.py: rank 0 printed no result line", file=sys.stderr)
        return 1
    try:
        ran = json.loads(lines[-1]).get("n_gpus")
    except ValueError:
        ran = None
    if ran != n:
        sys.stderr.write(lines[-1])
        print(f"bench.py: --gpus {n} but the run reported n_gpus={ran}", file=sys.stderr)
        return 1
    sys.stdout.write(lines[-1])
    sys.stdout.flush()
    return 0


def headline(world: int, steps: int, flops_all: int, compute_elapsed_max: float, pipe_elapsed_max=None):
    """(value GFLOP/s, ms_per_step) of the line.  At world > 1 a step is
    configs[4]'s whole work: the compute of every rank's column block AND the
    all-gather into row-major [M, N_total] (tsg_dist.GatherPipeline), timed
    over exactly `steps` steps, max over ranks; the compute-only step is a
    side figure.  At world == 1 there is no collective: the compute step."""
    if world > 1:
        if pipe_elapsed_max is None:
            raise ValueError("world > 1: the headline is the compute + all-gather step; it was not measured")
        el = pipe_elapsed_max
    else:
        el = compute_elapsed_max
    return flops_all * steps / el / 1e9, el / steps * 1e3


def build_line(a, *, world, mode, backend, M, K, Nr, Ntot, s, nnz, nnz_all, kname, compute_elapsed_max,
               kern_ms_max, gather=None, traffic=None, traffic_fs2=None, plan_asserted=False, cpu=None, e2e=None, stream_ms=None, setup_s=0.0,
               clock_warmup=(0.0, 0), kernel_timing=None) -> dict:
    """The JSON line rank 0 prints (bench.py contract), from the measured
    quantities (max over ranks).  Pure: tests/test_bench_launch.py checks it
    without a GPU."""
    flops_all = M * (nnz_all + Ntot)  # sum over ranks of T.flops(M, Nr, nnz_rank)
    value, ms_step = headline(world, a.steps, flops_all, compute_elapsed_max,
                              None if gather is None else gather["pipeline_elapsed_s"])
    alg_bytes = T.algorithmic_bytes(M, Nr, K, nnz)  # per launch, this rank
    adds = T.flops(M, Nr, nnz)                       # per launch: one IEEE add per (m, nonzero) + bias
    achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9
    binding_frac = round(adds / (kern_ms_max * 1e-3) / 1e12 / VALU_PEAK_TADDS, 4)
    if world == 1:
        workload = "BASELINE configs[2]" if (M, K, Nr, s) == (4096, 4096, 16384, 4) else "custom"
    elif mode == "weak":
        workload = (f"BASELINE configs[4]-style weak column shard + all-gather: {Nr} columns per GPU, "
                    f"N_total={Ntot}" + (" (= configs[4])" if (M, K, Ntot, s, world) == (4096, 4096, 131072, 4, 8)
                                         else ""))
    else:
        workload = f"strong column shard of N={Ntot} over {world} GPUs ({Nr} columns per GPU) + all-gather"
    compute_only = {"ms_per_step": round(compute_elapsed_max / a.steps * 1e3, 4),
                    "value": round(flops_all * a.steps / compute_elapsed_max / 1e9, 3), "unit": "GFLOP/s",
                    "note": "every rank's Y column block, no collective"}
    gather_info = None
    if gather is not None:
        coll = "RCCL" if backend == "nccl" else backend
        gather_info = {"ms_per_step": round(ms_step, 4), "value": round(value, 3), "unit": "GFLOP/s",
                       "note": f"the headline: compute + {coll} all-gather of Y into row-major [M, N_total], "
                               f"pipelined by {gather['chunks']} M chunks (tsg_dist.GatherPipeline)",
                       "columns_match_compute_only": gather["columns_match"],
                       "every_block_delivered": gather.get("blocks_match"),
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
                   "nnz_per_gpu": nnz, "parallelism": f"W columns x{world}"
                   + (" + all-gather of Y" if world > 1 else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                     "traffic": traffic,
                     "kernel": kname, "kernel_ms": round(kern_ms_max, 4), "kernel_timing": kernel_timing,
                     "algorithmic_bytes_per_launch": alg_bytes,
                     "kernel_gflops": round(adds / (kern_ms_max * 1e-3) / 1e9, 2),
                     "traffic_source": (os.path.relpath(PROFILE_PMC, REPO) + " (read bytes by request size "
                                        "TCC_EA0_RDREQ_{32,64,128}B + WRITE_SIZE"
                                        + ("; plan asserted)" if plan_asserted else ")")
                                        if traffic is not None else None),
                     "traffic_fetch_size_x2": traffic_fs2,
                     "binding": {"resource": "valu fp32 adds (DESIGN.md 4)", "adds_per_launch": adds,
                                 "achieved_Tadds": round(adds / (kern_ms_max * 1e-3) / 1e12, 2),
                                 "peak_Tadds": round(VALU_PEAK_TADDS, 2), "frac": binding_frac}},
        # the roof that binds this kernel, top level so a
        # parser that keeps only flat keys of `roofline` still sees it
        "binding_roof": {"resource": "valu fp32 adds", "frac": binding_frac, "kernel": kname,
                         "achieved_Tadds": round(adds / (kern_ms_max * 1e-3) / 1e12, 2),
                         "peak_Tadds": round(VALU_PEAK_TADDS, 2)},
        "cpu_baseline": cpu,
        "compute_only": compute_only if world > 1 else None,
        "stream_ms_per_step": None if stream_ms is None else round(stream_ms / a.steps, 4),
        "e2e_host_pointers": e2e,
        "allgather_ms": None if gather is None else round(gather["allgather_ms"], 3),
        "allgather_gbps_per_gpu": (None if gather is None else
                                   round(gather["bytes_received_per_gpu"] / (gather["allgather_ms"] * 1e-3) / 1e9, 2)),
        "with_allgather": gather_info,
        "setup_s": round(setup_s, 2),
        "clock_warmup": {"seconds": round(clock_warmup[0], 3), "steps": clock_warmup[1]},
    }
    return out


def main():
    a = parse()
    if launch_mode(a.gpus, os.environ) == "launch":
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        # a 1-GPU line under an N-GPU request is never reported
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if os.environ.get("TSG_BENCH_DRYRUN") == "1":  # launcher test (tests/test_bench_launch.py): no GPU
        if os.environ.get("TSG_BENCH_DRYRUN_FAIL_RANK") is not None:
            # a failing rank while the others wait (as in a rendezvous)
            if rank == int(os.environ["TSG_BENCH_DRYRUN_FAIL_RANK"]):
                sys.exit(3)
            time.sleep(600)
        if os.environ.get("TSG_BENCH_DRYRUN_HANG_RANK") is not None:
            # one rank never exits nor fails (stuck in a rendezvous); the others finish
            if rank == int(os.environ["TSG_BENCH_DRYRUN_HANG_RANK"]):
                time.sleep(600)
        print(json.dumps({"rank": rank, "world": world, "local_rank": local,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        return
    import torch
    import torch.distributed as dist

    backend = os.environ.get("TSG_BENCH_BACKEND", "nccl") if world > 1 else None
    ndev = torch.cuda.device_count()
    if local >= ndev:
        # one process per GPU; only the one-GPU rehearsal (gloo: RCCL refuses
        # two ranks on one device) shares the visible devices between ranks
        if backend != "gloo" or ndev == 0:
            print(f"bench.py: rank {rank} has LOCAL_RANK {local} but {ndev} GPU(s) are visible "
                  f"(--gpus {a.gpus}); TSG_BENCH_BACKEND=gloo rehearses several ranks per GPU",
                  file=sys.stderr)
            sys.exit(3)
        local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
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
    kname = h.call_kernel(M)  # the kernel THIS call launches (small M runs the ELL walks)
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
    barrier()
    torch.cuda.synchronize()
    # The timed steps run WITHOUT per-launch timing events: an event pair
    # around every launch leaves the GPU idle ~10 us per launch
    # (profiles/r05h_step_overhead.jsonl, rocprofv3 trace: 59.2-59.7 us kernels
    # back to back without, 58.6 us + 10.1 us gaps with, at configs[1]).  HIP
    # events on the kernel's stream (torch's current stream: gemm_torch
    # launches there) bracket the K steps; a step that is one launch (the
    # kernel reads X itself: tcsc_hip_call_launches) runs its kernels back to
    # back, so that stream time / K is the kernel's average launch duration.
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
    stream_ms = ev0.elapsed_time(ev1)
    step_launches = h.call_launches(X, M)
    # a second pass of K steps with an event pair around every launch of the
    # main kernel (tcsc_hip_set_timing): the kernel alone when the step also
    # stages X^T; reported beside (it includes ~3-5 us of the events' own gap)
    h.set_timing(True)
    h.kernel_time(reset=True)
    for _ in range(a.steps):
        h.gemm_torch(X, b, Y)
    torch.cuda.synchronize()
    pair_ms_total, launches = h.kernel_time(reset=True)
    h.set_timing(False)
    pair_ms = pair_ms_total / max(launches, 1)
    kern_ms_total = stream_ms if step_launches == 1 else pair_ms_total
    launches = a.steps if step_launches == 1 else launches

    # --- world > 1: configs[4]'s whole step = the compute of this rank's
    # column block AND the RCCL all-gather of every rank's block into the
    # row-major [M, N_total] Y (north_star's collective), pipelined by M
    # chunks.  This is the headline at world > 1: exactly a.steps steps,
    # barrier + synchronize on both sides, max over ranks.  The gather alone
    # is timed first (allgather_ms, its bandwidth per GPU).
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
        pipe_elapsed = time.perf_counter() - tp
        # the pipelined Y: this rank's columns equal its compute-only block,
        # and every other rank's columns carry that rank's block (a checksum
        # of each block, all-gathered, against the same checksum of Y_full)
        ok = torch.equal(Yfull[:, n0:n1].view(torch.int32), Y.view(torch.int32))
        mine = Y.view(torch.int32).to(torch.int64).sum().reshape(1)
        sums = torch.empty(world, dtype=torch.int64, device=dev)
        D._all_gather_into(sums, mine)
        got = torch.stack([Yfull[:, c0:c1].view(torch.int32).to(torch.int64).sum()
                           for c0, c1 in (D.column_shard(Ntot, world, r) for r in range(world))])
        blocks_ok = torch.equal(sums, got)
        tg = torch.tensor([ag_s, pipe_elapsed, 0.0 if ok else 1.0, 0.0 if blocks_ok else 1.0],
                          device=dev, dtype=torch.float64)
        dist.all_reduce(tg, op=dist.ReduceOp.MAX)
        gather = {"allgather_ms": float(tg[0]) * 1e3, "pipeline_elapsed_s": float(tg[1]),
                  "columns_match": float(tg[2]) == 0.0, "blocks_match": float(tg[3]) == 0.0,
                  "bytes_received_per_gpu": 4 * M * (Ntot - Nr), "chunks": len(pipe.ranges)}
        del pipe, Yfull

    tt = torch.tensor([elapsed, kern_ms_total / max(launches, 1), pair_ms], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed_max, kern_ms_max, pair_ms_max = float(tt[0]), float(tt[1]), float(tt[2])
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
        Yref = Y.cpu().numpy()

        def host_ms(chunks, reps=5):
            h.set_host_chunks(chunks)
            h(Xh, bh, Yh, M, Nr, K)
            ts = []
            for _ in range(reps):
                e0 = time.perf_counter()
                h(Xh, bh, Yh, M, Nr, K)
                ts.append((time.perf_counter() - e0) * 1e3)
            same = bool(np.array_equal(Yh.view(np.uint32), Yref.view(np.uint32)))
            return float(np.median(ts)), same

        serial_ms, serial_ok = host_ms(1)
        e_ms, e_ok = host_ms(0)  # the default: M-chunk pipeline
        with T.registered_host(Xh, Yh):  # the caller's buffers page-locked once (tcsc_hip_host_register)
            reg_ms, reg_ok = host_ms(0)
        rows = h.host_chunk_rows(M)
        e2e = {"ms": round(e_ms, 3), "gflops": round(T.flops(M, Nr, nnz) / (e_ms * 1e-3) / 1e9, 1),
               "chunk_rows": rows, "unpipelined_ms": round(serial_ms, 3),
               # what each chunk runs: the per-call plan of a call with `rows` rows
               "chunk_plan": {"kernel": h.call_kernel(rows), "width": h.jit_width(rows),
                              "waves": h.jit_waves(rows), "far": h.call_far(rows)},
               "registered_buffers_ms": round(reg_ms, 3),
               "bit_identical_to_device_call": e_ok and serial_ok and reg_ok, "timing": "median of 5 calls",
               "bytes_over_pcie": 4 * (M * K + Nr + M * Nr)}

    # --- CPU baseline (rank 0 at N=1 only): bounded samples of the same workload
    cpu = None
    if rank == 0 and world == 1 and a.cpu_rows > 0:
        cpu = cpu_baseline(X, csp, csn, rip, rin, K, Nr, s, Y, a.cpu_rows)

    if rank == 0:
        traffic = traffic_fs2 = None
        plan_asserted = False
        try:
            # HBM bytes per launch of THIS kernel on THIS workload, from the
            # committed rocprofv3 PMC passes (scripts/pmc_summary.py: FETCH_SIZE
            # and WRITE_SIZE with the gfx950 corrections of MI355X_MICROARCH.md)
            pm = json.load(open(PROFILE_PMC))
            plan = {k: list(v) if isinstance(v, tuple) else v for k, v in T.call_plan(K, Nr, nnz, M).items()}
            if (pm.get("workload") == f"{M}x{K}x{Nr}s{s}" and pm.get("kernel") == kname
                    and pm.get("plan", plan) == plan):  # (summaries before round 6 carry no plan)
                kp = pm.get("kernels", {}).get(kname, {})
                # read bytes by memory-side request size + WRITE_SIZE (VERDICT
                # r05: FETCH_SIZE x 2 overstated this kernel's reads by ~7%)
                traffic = kp.get("hbm_bytes_by_request_size", kp.get("hbm_bytes"))
                traffic_fs2 = kp.get("hbm_bytes")
                plan_asserted = "plan" in pm
        except Exception:
            pass
        out = build_line(a, world=world, mode=mode, backend=backend, M=M, K=K, Nr=Nr, Ntot=Ntot, s=s, nnz=nnz,
                         nnz_all=nnz_all, kname=kname, compute_elapsed_max=elapsed_max, kern_ms_max=kern_ms_max,
                         gather=gather, traffic=traffic, traffic_fs2=traffic_fs2,
                         plan_asserted=plan_asserted, cpu=cpu, e2e=e2e,
                         stream_ms=stream_ms, setup_s=setup_s, clock_warmup=(clock_warmup_s, n_clock),
                         kernel_timing={"launches_per_step": step_launches,
                                        "kernel_ms_source": ("HIP events on the kernel's stream over the timed "
                                                             "region / K (one launch per step, back to back)"
                                                             if step_launches == 1 else
                                                             "HIP event pair around every launch, second pass"),
                                        "event_pair_kernel_ms": round(pair_ms_max, 4)})
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
