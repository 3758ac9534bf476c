#!/usr/bin/env python3
"""GPU box: the 64-row image (tsg_jit64_kernel) against the 128-row image and
the small-M walk over M at one K, N, s -- kernel time (HIP events on the
call's stream, steady clock) and the step (X^T staging + kernel), every
result bit-identical across the kernels.  JSON lines.

    python scripts/rows64_ab.py [--K 4096 --N 16384 --s 4] [--M 1,16,32,64,...]
        [--widths 0,16,8]   (0 = the automatic shape; others pin the width:
                             8 waves, or 4 with TSG_JIT_WAVES=4 in the env)
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
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--N", type=int, default=16384)
ap.add_argument("--s", type=int, default=4)
ap.add_argument("--M", default="1,8,16,32,48,64,96,128,192,256,512")
ap.add_argument("--widths", default="0")
ap.add_argument("--modes", default="ell,jit128,jit64")
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--xint", action="store_true", help="X integer U[-512, 512] (bench.py's X) instead of order-sensitive")
a = ap.parse_args()
import torch  # noqa: E402

step_timed = None

arrs = T.gen_tcsc(a.K, a.N, a.s, 42)
nnz = len(arrs[2]) + len(arrs[3])
h = T.TCSCDevice(*arrs, a.K, a.N, device=0)
b = torch.full((a.N,), 2.0, device="cuda")
VALU = 128 * 256 * 2.4e9 / 1e12  # T adds/s, v_pk_add_f32 (the VOP2 add issues at half that)


def timed(M, X, Y):
    """kernel ms (HIP events around every launch) and step ms (back-to-back
    calls with the per-kernel events OFF: the events themselves add ~8-10 us
    between launches, profiles/r05g_event_overhead.jsonl)"""
    t_end = time.perf_counter() + 0.3  # clock warm-up (time-based: 20 calls left the first mode of a process
    while time.perf_counter() < t_end:  # 3-10% slow, profiles/r05z_r64_shapes_ab.jsonl)
        for _ in range(4):
            h.gemm_torch(X, b, Y)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        h.gemm_torch(X, b, Y)
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / a.reps * 1e3
    h.set_timing(True)
    h.kernel_time(reset=True)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        h.gemm_torch(X, b, Y)
    torch.cuda.synchronize()
    global step_timed
    step_timed = (time.perf_counter() - t0) / a.reps * 1e3
    ms, n = h.kernel_time(reset=True)
    h.set_timing(False)
    return ms / max(n, 1), step


for M in (int(v) for v in a.M.split(",")):
    g = torch.Generator(device="cuda")
    g.manual_seed(12345)
    if a.xint:  # bench.py's X: small integers (exact partial sums, few toggling bits)
        X = torch.randint(-512, 513, (M, a.K), generator=g, device="cuda", dtype=torch.int32).float()
    else:  # order-sensitive X: mantissas over an exponent spread (every partial sum rounds)
        X = (torch.randint(-(1 << 23), 1 << 23, (M, a.K), generator=g, device="cuda", dtype=torch.int32).float()
             * torch.exp2(-torch.randint(0, 24, (M, a.K), generator=g, device="cuda").float()))
    out = {"M": M, "K": a.K, "N": a.N, "s": a.s, "x": "int" if a.xint else "frac", "waves_env": os.environ.get("TSG_JIT_WAVES"),
           "xdirect_env": os.environ.get("TSG_JIT_XDIRECT"), "qblock_env": os.environ.get("TSG_JIT_QBLOCK")}
    ref = None
    for mode in a.modes.split(","):
        for w in ([0] if mode == "ell" else [int(x) for x in a.widths.split(",")]):
            h.set_small_m(2 if mode == "ell" else 1)
            h.set_tile_rows({"ell": 0, "jit128": 128, "jit64": 64}[mode])
            h.set_jit_width(w)
            h.reserve(M)
            Y = torch.empty((M, a.N), device="cuda")
            ms, step = timed(M, X, Y)
            adds = M * (nnz + a.N)
            key = mode + ("" if not w else f"_w{w}")
            out[key] = {"kernel": h.call_kernel(M), "kernel_ms": round(ms, 5), "step_ms": round(step, 5),
                        "step_with_events_ms": round(step_timed, 5),
                        "width": h.jit_width(M), "waves": h.jit_waves(M), "image_bytes": h.call_image_bytes(M),
                        "valu_frac_pk": round(adds / ms / 1e9 / VALU, 4)}
            if ref is None:
                ref = Y.clone()
            out[key]["bit_identical"] = bool(torch.equal(Y.view(torch.int32), ref.view(torch.int32)))
    h.set_small_m(0)
    h.set_tile_rows(0)
    h.set_jit_width(0)
    out["auto"] = h.call_kernel(M)
    print(json.dumps(out), flush=True)
