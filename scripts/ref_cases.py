#!/usr/bin/env python3
"""GPU box: kernel time of the automatic path on the reference's own benchmark
cases (plots/run_benchmark.py:8-33: eight (M, K, N) shapes x s in {2, 4, 8,
16}, and with --sweep the one-dimension sweeps around 1024), each checked bit
for bit on sampled rows against the CPU oracle.  One JSON object per case:
the kernel the call runs, its time (HIP events, steady clock), GFLOP/s in the
reference's count (M * (nnz + N) adds, readme.md:84-85) and the fractions of
the VALU add peak and of the HBM roof on the algorithmic bytes.

    python scripts/ref_cases.py [--sweep] [--steps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ternary-spgemm_amd"), os.path.join(REPO, "oracle")]
import tspgemm as T  # noqa: E402
from tsg_report import CASES, SPARSITIES, cases_for  # noqa: E402

VALU_PEAK = 78.64e12  # fp32 adds/s: v_pk_add_f32, 256 CUs x 128 adds/clk x 2.4 GHz
HBM_PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sweep", action="store_true", help="also the M, K and N sweeps around 1024 (s = 4)")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch
    import oracle as O
    dev = torch.device("cuda", 0)
    todo = [(c, s) for c in CASES for s in SPARSITIES]
    if a.sweep:
        todo += [(c, 4) for v in ("M", "K", "N") for c in cases_for(v)]
    for (M, K, N), s in todo:
        arrs = T.gen_tcsc(K, N, s, 42)
        nnz = len(arrs[2]) + len(arrs[3])
        h = T.TCSCDevice(*arrs, K, N, device=0)
        g = torch.Generator(device=dev)
        g.manual_seed(12345)
        X = torch.randint(-512, 513, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.float32)
        b = torch.full((N,), 2.0, device=dev)
        Y = torch.empty((M, N), device=dev)
        h.reserve(M)
        import time
        t_end = time.perf_counter() + 0.2
        while time.perf_counter() < t_end:  # warmup incl. the GPU clock ramp
            for _ in range(4):
                h.gemm_torch(X, b, Y)
            torch.cuda.synchronize()
        # the call back to back without per-launch timing events (round 5:
        # an event pair idles the GPU ~10 us per launch): stream time per call
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            h.gemm_torch(X, b, Y)
        e1.record()
        torch.cuda.synchronize()
        step_ms = e0.elapsed_time(e1) / a.steps
        h.set_timing(True)
        h.kernel_time(reset=True)
        for _ in range(a.steps):
            h.gemm_torch(X, b, Y)
        torch.cuda.synchronize()
        ms, n = h.kernel_time(reset=True)
        ms /= max(n, 1)
        rows = np.unique(np.r_[0, M // 2, M - 1])
        ref = O.base_tcsc(np.ascontiguousarray(X[rows].cpu().numpy()), O.TCSC(*arrs, K, N),
                          np.full(N, 2.0, np.float32))
        ok = bool(np.array_equal(ref.view(np.uint32), Y[rows].cpu().numpy().view(np.uint32)))
        adds = T.flops(M, N, nnz)
        hbm = T.algorithmic_bytes(M, N, K, nnz)
        print(json.dumps({"M": M, "K": K, "N": N, "s": s, "kernel": h.call_kernel(M), "kernel_ms": round(ms, 4),
                          "step_ms": round(step_ms, 4), "launches": h.call_launches(X, M),
                          "gflops": round(adds / (ms * 1e-3) / 1e9, 1),
                          "valu_frac": round(adds / (ms * 1e-3) / VALU_PEAK, 4),
                          "hbm_frac": round(hbm / (ms * 1e-3) / HBM_PEAK, 4),
                          "bit_identical_rows": ok}), flush=True)
        h.close()
        del X, Y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
