#!/usr/bin/env python3
"""GPU box: small-M kernel vs the weight-compiled kernel over M at a given
K, N, s (kernel time from the handle's HIP events, steady clock), JSON lines.

    python scripts/small_m_sweep.py [--K 4096 --N 16384 --s 4] [--M 1,2,4,...]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))
import tspgemm as T  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--N", type=int, default=16384)
ap.add_argument("--s", type=int, default=4)
ap.add_argument("--M", default="1,2,4,8,16,24,32,48,64,96,128,256,512")
ap.add_argument("--reps", type=int, default=30)
a = ap.parse_args()
import torch  # noqa: E402

arrs = T.gen_tcsc(a.K, a.N, a.s, 42)
nnz = len(arrs[2]) + len(arrs[3])
tcsc_bytes = 4 * (2 * (a.N + 1) + nnz)
h = T.TCSCDevice(*arrs, a.K, a.N, device=0)
b = torch.full((a.N,), 2.0, device="cuda")
for M in (int(v) for v in a.M.split(",")):
    X = torch.randint(-512, 513, (M, a.K), device="cuda", dtype=torch.int32).float()
    out = {"M": M, "K": a.K, "N": a.N, "s": a.s}
    Ys = {}
    for mode, name in ((2, "ell"), (1, "jit")):
        h.set_small_m(mode)
        h.reserve(M)
        Y = torch.empty((M, a.N), device="cuda")
        for _ in range(20):  # clock warm-up + warmup
            h.gemm_torch(X, b, Y)
        torch.cuda.synchronize()
        h.set_timing(True)
        h.kernel_time(reset=True)
        for _ in range(a.reps):
            h.gemm_torch(X, b, Y)
        ms, n = h.kernel_time(reset=True)
        h.set_timing(False)
        ms /= max(n, 1)
        Ys[name] = Y
        adds = M * (nnz + a.N)
        # bytes the launch moves at least: its device image once, X once, Y once
        img = h.call_image_bytes(M)
        moved = img + 4 * (M * a.K + M * a.N + a.N)
        out[name] = {"kernel_ms": round(ms, 5), "Tadds": round(adds / ms / 1e9, 3),
                     "valu_frac": round(adds / ms / 1e9 / 78.64, 4),
                     "tcsc_GBps": round(tcsc_bytes / ms / 1e6, 1),
                     "hbm_frac_on_tcsc_bytes": round(tcsc_bytes / ms / 1e6 / 8000.0, 4),
                     "image_bytes": img, "bytes_moved_min": moved,
                     "hbm_frac_on_bytes_moved": round(moved / ms / 1e6 / 8000.0, 4)}
    out["bit_identical"] = bool(torch.equal(Ys["ell"].view(torch.int32), Ys["jit"].view(torch.int32)))
    h.set_small_m(0)
    out["auto"] = h.call_kernel(M)
    print(json.dumps(out), flush=True)
