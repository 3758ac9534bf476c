#!/usr/bin/env python3
"""GPU box: the step (staging + kernel) of one shape with the per-kernel HIP
timing events off and on -- what the timing itself adds to the step -- and
the step-minus-kernel remainder.  JSON lines.

    python scripts/step_overhead_ab.py [--M 4096 --K 4096 --N 16384 --s 4] [--tile-rows 0|64|128]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))
import tspgemm as T  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=4096)
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--N", type=int, default=16384)
ap.add_argument("--s", type=int, default=4)
ap.add_argument("--tile-rows", type=int, default=0)
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--small-m", type=int, default=0)
a = ap.parse_args()
import torch  # noqa: E402

h = T.TCSCDevice(*T.gen_tcsc(a.K, a.N, a.s, 42), a.K, a.N, device=0)
h.set_tile_rows(a.tile_rows)
h.set_small_m(a.small_m)
g = torch.Generator(device="cuda")
g.manual_seed(12345)
X = torch.randint(-512, 513, (a.M, a.K), generator=g, device="cuda", dtype=torch.int32).float()
b = torch.full((a.N,), 2.0, device="cuda")
Y = torch.empty((a.M, a.N), device="cuda")
t_end = time.perf_counter() + 0.3
while time.perf_counter() < t_end:  # clock warm-up
    h.gemm_torch(X, b, Y)
torch.cuda.synchronize()
out = {"M": a.M, "K": a.K, "N": a.N, "s": a.s, "kernel": h.call_kernel(a.M)}
for timing in (False, True, False, True):
    h.set_timing(timing)
    h.kernel_time(reset=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.reps):
        h.gemm_torch(X, b, Y)
    e1.record()
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / a.reps * 1e3
    out.setdefault("stream_ms_timing_on" if timing else "stream_ms_timing_off", []).append(
        round(e0.elapsed_time(e1) / a.reps, 5))
    ms, n = h.kernel_time(reset=True)
    out.setdefault("step_ms_timing_on" if timing else "step_ms_timing_off", []).append(round(step, 5))
    if timing:
        out.setdefault("kernel_ms", []).append(round(ms / max(n, 1), 5))
h.set_timing(False)
print(json.dumps(out), flush=True)
