#!/usr/bin/env python3
"""BASELINE configs[3]: M=4096 K=4096 N=16384, sparsity s in {2,4,8,16}, TCSC vs
"CSC + packed values" (readme.md:111) vs BlockedTCSC<B> (BlockedTCSC.h, B=512 as
main.cpp:7) as the registration format.  One GPU.

TCSC and CSC+packed register the same matrix (the packed one is converted on the
host, tsg_csc_packed_to_tcsc) and run the same generated code, so that
comparison is format bytes and registration time.  BlockedTCSC computes
BaseBlockedTCSC (its own accumulation order, comp.h:607-658) on the same
kernel with per-block sums.  Every line also checks 8 sampled rows bit for bit
against the CPU oracle of its order.
Writes one JSON object per s to stdout.

    python scripts/sweep.py [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ternary-spgemm_amd"), os.path.join(REPO, "oracle"), os.path.dirname(os.path.abspath(__file__))]
import tspgemm as T  # noqa: E402
from step_timing import time_calls  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--B", type=int, default=512, help="BlockedTCSC block size (main.cpp:7)")
    a = ap.parse_args()
    import torch
    import oracle as O
    dev = torch.device("cuda", 0)
    M, K, N = a.M, a.K, a.N
    g = torch.Generator(device=dev)
    g.manual_seed(12345)
    X = torch.randint(-512, 513, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.float32)
    b = torch.full((N,), 2.0, device=dev)
    Y = torch.empty((M, N), device=dev)
    Xs = X[:8].cpu().numpy()
    for s in (2, 4, 8, 16):
        arrs = T.gen_tcsc(K, N, s, 42)
        nnz = len(arrs[2]) + len(arrs[3])
        col_ptr, row_idx, packed = T.tcsc_to_csc_packed(*arrs, N)
        out = {"s": s, "M": M, "K": K, "N": N, "nnz": nnz,
               "tcsc_bytes": 4 * (2 * (N + 1) + nnz),
               "csc_packed_bytes": 4 * (N + 1) + 4 * len(row_idx) + len(packed)}
        blk = T.tcsc_to_blocked(*arrs, K, N, a.B)
        # what the device reads for each registration: CSC + packed values is an
        # input format only -- converted to TCSC on the host at registration and
        # compiled into the same code, so its time is TCSC's
        out["device_reads"] = {"tcsc": "TCSC (weight-compiled image)",
                               "csc_packed": "TCSC (converted at registration)",
                               "blocked": "BlockedTCSC (weight-compiled image with per-block sums)"}
        out["blocked_B"] = a.B
        out["blocked_bytes"] = 4 * (len(blk[0]) + len(blk[1]) + len(blk[2]) + len(blk[3]))
        for fmt in ("tcsc", "csc_packed", "blocked"):
            t0 = time.time()
            h = (T.TCSCDevice(*arrs, K, N, device=0) if fmt == "tcsc"
                 else T.TCSCDevice.from_csc_packed(col_ptr, row_idx, packed, K, N, device=0) if fmt == "csc_packed"
                 else T.TCSCDevice.from_blocked(*blk, K, N, a.B, device=0))
            out[f"{fmt}_register_s"] = round(time.time() - t0, 3)
            h.reserve(M)
            t = time_calls(h, X, b, Y, a.steps)
            # the kernel's duration: stream time per call when the call is one launch
            ms = t["step_ms"] if t["launches"] == 1 else t["event_pair_kernel_ms"]
            out[f"{fmt}_step_ms"] = round(t["step_ms"], 4)
            out[f"{fmt}_event_pair_kernel_ms"] = round(t["event_pair_kernel_ms"], 4)
            bb = np.full(N, 2.0, np.float32)
            ref = (O.base_blocked_tcsc(Xs, blk, bb, K, N, a.B) if fmt == "blocked"
                   else O.base_tcsc(Xs, O.TCSC(*arrs, K, N), bb))
            out[f"{fmt}_kernel_ms"] = round(ms, 4)
            out[f"{fmt}_bit_identical_rows"] = bool(np.array_equal(ref.view(np.uint32),
                                                                   Y[:8].cpu().numpy().view(np.uint32)))
            if fmt == "tcsc":
                out["kernel"] = h.call_kernel(M)
                out["gflops"] = round(T.flops(M, N, nnz) / (ms * 1e-3) / 1e9, 1)
                out["valu_frac"] = round(T.flops(M, N, nnz) / (ms * 1e-3) / 78.64e12, 4)
            h.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
