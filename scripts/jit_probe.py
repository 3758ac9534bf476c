#!/usr/bin/env python3
"""GPU probe of the weight-compiled kernel (TSG_KERNEL=jit): small shapes
through the C-ABI, bitwise against the oracle.  Diagnostic script."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ternary-spgemm_amd"), os.path.join(REPO, "oracle")]
os.environ["TSG_KERNEL"] = "jit"
import numpy as np
import torch
import tspgemm as T
import oracle as O
torch.cuda.set_device(0)
for (M, K, N, s) in [(64, 130, 300, 4), (300, 700, 513, 2), (1, 1, 1, 1)]:
    W = O.gen_ternary(K, N, s, 5)
    t = O.tcsc_encode(W)
    h = T.TCSCDevice(*t.arrays, K, N, device=0)
    print("created", (M, K, N, s), h.info(), flush=True)
    b = np.linspace(-3, 3, N).astype(np.float32)
    for X in (O.init_x_int(M, K, 1), O.init_x_frac(M, K, 2)):
        Y = h.gemm_torch(torch.from_numpy(X).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
        ref = O.base_tcsc(X, t, b)
        ok = np.array_equal(Y.view(np.uint32), ref.view(np.uint32))
        print("  bitwise equal:", ok, "max abs diff", float(np.abs(Y - ref).max()), flush=True)
        assert ok
    h.close()
print("jit probe ok")
