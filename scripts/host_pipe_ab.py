#!/usr/bin/env python3
"""GPU box: the host-pointer comp_func call (tcsc_hip_gemm, main.cpp:214-216) at
BASELINE configs[2] for several M-chunk counts of the pipeline (1 = one H2D,
one compute, one D2H), median of 7 calls each, every result checked bit for
bit against the device call.  JSON lines.   python scripts/host_pipe_ab.py"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))
import tspgemm as T  # noqa: E402


def main():
    import torch
    M, K, N, s = 4096, 4096, 16384, 4
    arrs = T.gen_tcsc(K, N, s, 42)
    h = T.TCSCDevice(*arrs, K, N, device=0)
    X = T.gen_x(M, K, 7)
    b = np.full(N, 2.0, np.float32)
    Yd = h.gemm_torch(torch.from_numpy(X).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
    Y = np.empty((M, N), np.float32)
    def run(tag, chunks):
        h.set_host_chunks(chunks)
        h(X, b, Y, M, N, K)
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            h(X, b, Y, M, N, K)
            ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"buffers": tag, "chunks": chunks or "auto", "chunk_rows": h.host_chunk_rows(M),
                          "ms_median": round(float(np.median(ts)), 3), "ms_min": round(min(ts), 3),
                          "bit_identical": bool(np.array_equal(Y.view(np.uint32), Yd.view(np.uint32)))}), flush=True)

    for chunks in (1, 4, 8, 12, 16, 0):
        run("pageable", chunks)
    with T.registered_host(X, Y):  # tcsc_hip_host_register: the caller's buffers page-locked once
        for chunks in (1, 16, 0):
            run("registered", chunks)


if __name__ == "__main__":
    main()
