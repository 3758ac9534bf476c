#!/usr/bin/env python3
"""Diagnostic (not product): one config-3 call with TSG_STAMPS=1 -- per-wave
cycles spent walking vs waiting at step barriers (printed by the library), plus
the plain event time of the same launch.  Usage: TSG_KERNEL=rx python scripts/diag_stamps.py"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))
import torch
import tspgemm as T
M, K, N, s = 4096, 4096, 16384, 4
csp, csn, rip, rin = T.gen_tcsc(K, N, s, 42)
h = T.TCSCDevice(csp, csn, rip, rin, K, N, device=0)
X = torch.randint(-512, 513, (M, K), device="cuda", dtype=torch.int32).float()
b = torch.full((N,), 2.0, device="cuda")
Y = torch.empty((M, N), device="cuda")
h.reserve(M)
for _ in range(3):
    h.gemm_torch(X, b, Y)
torch.cuda.synchronize()
h.set_timing(True); h.kernel_time(reset=True)
for _ in range(10):
    h.gemm_torch(X, b, Y)
torch.cuda.synchronize()
ms, n = h.kernel_time(reset=True)
print(f"kernel ms {ms / max(n, 1):.4f}", flush=True)
h.set_timing(False)
os.environ["TSG_STAMPS"] = "1"
h.gemm_torch(X, b, Y)
torch.cuda.synchronize()
