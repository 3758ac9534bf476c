#!/usr/bin/env python3
"""Kernel time of the default (weight-compiled) path on BASELINE.json's configs
and on the small-M shapes of the reference's sweep (plots/run_benchmark.py:8-33),
one GPU, each checked bit for bit on sampled rows against the CPU oracle.
One JSON object per shape on stdout.

    python scripts/configs.py [--steps 10] [--all-widths]

--all-widths times every jit stream width (64/32/16/8) per shape, besides the
automatic pick, to check tsg_capi.cpp pick_jit_width.
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

SHAPES = [("configs[0]", 32, 1024, 4096, 4), ("configs[1]", 512, 4096, 4096, 4),
          ("configs[2]", 4096, 4096, 16384, 4),
          ("sweep M=1", 1, 4096, 16384, 4), ("sweep M=16", 16, 4096, 16384, 4),
          ("sweep M=64", 64, 4096, 16384, 4), ("sweep M=256", 256, 4096, 16384, 4),
          ("sweep M=1024", 1024, 4096, 16384, 4), ("run_benchmark (64000,16384,4096)", 8192, 16384, 4096, 4)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--all-widths", action="store_true")
    ap.add_argument("--only", default="", help="substring filter on shape names")
    ap.add_argument("--shape", action="append", default=[],
                    help="extra shape M,K,N,s (repeatable); with --shape only these run unless --only is given")
    a = ap.parse_args()
    shapes = list(SHAPES)
    if a.shape:
        extra = [("shape %s" % sh, *map(int, sh.split(","))) for sh in a.shape]
        shapes = extra + (shapes if a.only else [])
    import torch
    import oracle as O
    dev = torch.device("cuda", 0)
    for name, M, K, N, s in shapes:
      if a.only and a.only not in name:
          continue
      for width in ([0, 64, 32, 16, 8] if a.all_widths else [0]):
        arrs = T.gen_tcsc(K, N, s, 42)
        nnz = len(arrs[2]) + len(arrs[3])
        t0 = time.time()
        h = T.TCSCDevice(*arrs, K, N, device=0)
        if width:
            h.set_jit_width(width)
        jw = h.jit_width(M)
        reg_s = time.time() - t0
        g = torch.Generator(device=dev)
        g.manual_seed(12345)
        X = torch.randint(-512, 513, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.float32)
        b = torch.full((N,), 2.0, device=dev)
        Y = torch.empty((M, N), device=dev)
        h.reserve(M)
        t = time_calls(h, X, b, Y, a.steps)
        step_ms = t["step_ms"]
        # the kernel's duration: stream time per call when the call is one launch
        ms = step_ms if t["launches"] == 1 else t["event_pair_kernel_ms"]
        rows = min(M, 8)
        ref = O.base_tcsc(X[:rows].cpu().numpy(), O.TCSC(*arrs, K, N), np.full(N, 2.0, np.float32))
        ok = bool(np.array_equal(ref.view(np.uint32), Y[:rows].cpu().numpy().view(np.uint32)))
        adds = T.flops(M, N, nnz)
        print(json.dumps({"shape": name, "M": M, "K": K, "N": N, "s": s, "kernel": h.call_kernel(M),
                          "kernel_ms": round(ms, 4), "step_ms": round(step_ms, 4), "launches": t["launches"],
                          "event_pair_kernel_ms": round(t["event_pair_kernel_ms"], 4),
                          "gflops_kernel": round(adds / (ms * 1e-3) / 1e9, 1),
                          "valu_frac": round(adds / (ms * 1e-3) / 78.64e12, 4),
                          "jit_width": jw, "jit_waves": h.jit_waves(M), "width_pinned": bool(width),
                          "far_image": h.call_far(M),
                          # the call's own M tile (64 rows on the 64-row image, 128 on the 128-row one)
                          "workgroups": (-(-M // h.call_tile_rows(M)) * -(-N // (h.jit_waves(M) * max(jw, 1)))
                                         if h.call_tile_rows(M) else None),
                          "register_s": round(reg_s, 2),
                          "bit_identical_rows": ok}), flush=True)
        h.close()


if __name__ == "__main__":
    main()
