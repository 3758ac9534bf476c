#!/usr/bin/env python3
"""GPU box, one GPU: what configs[4] and the strong split should measure
(VERDICT r05 "next" 2).  One JSON line per item on stdout:

* ``compute``: the per-rank compute of the 1/2/4/8-GPU column shards, timed
  as the pipeline runs them (tsg_dist.GatherPipeline: 4 M chunks of 1024
  rows, back to back on one stream) and as one full-M call:
  - weak: rank 0's block of a weak-scaled W = configs[2] exactly (every rank's
    block has the same shape and nonzero count, block_seed(seed, r));
  - strong: rank 0's N/P columns of the N = 16384 W (ShardedTCSC.draw strong),
    P = 1, 2, 4, 8 -> (4096, 4096, 16384 / 8192 / 4096 / 2048).
* ``reorder``: the pipeline's reorder of one gathered chunk at configs[4]
  size ([8, 1024, 16384] rank-major -> Y[1024, 131072], tsg_dist._reorder)
  alone, and on a side stream beside a running chunk kernel (as the pipeline
  issues it); the strong P = 8 chunk ([8, 1024, 2048]) as well.

Times are HIP events on the stream the work runs on, after a clock warm-up,
median of `--reps` repetitions.

    python scripts/scale_proxy.py [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))
import tspgemm as T  # noqa: E402
import tsg_dist as D  # noqa: E402

M, K, S, NW = 4096, 4096, 4, 16384
CHUNKS = 4


def ev_ms(fn, stream, reps):
    import torch
    out = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    return statistics.median(out), min(out), max(out)


def warm(fn, seconds=0.3):
    import torch
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        fn()
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(12345)
    X = torch.randint(-512, 513, (M, K), generator=g, device=dev, dtype=torch.int32).float()
    main_s = torch.cuda.current_stream(dev)
    ranges = D.m_chunks(M, CHUNKS)
    shards = [("weak", 8, D.ShardedTCSC.draw(K, NW * 8, S, 42, 0, 8, "weak"), NW)]
    for P in (1, 2, 4, 8):
        shards.append(("strong", P, D.ShardedTCSC.draw(K, NW, S, 42, 0, P, "strong"), NW // P))
    kept = None
    for mode, P, arrs, w in shards:
        h = T.TCSCDevice(*arrs, K, w, device=0)
        h.reserve(M)
        b = torch.full((w,), 2.0, device=dev)
        Yc = [torch.empty((r1 - r0, w), device=dev) for r0, r1 in ranges]
        Yf = torch.empty((M, w), device=dev)

        def chunks():
            for (r0, r1), y in zip(ranges, Yc):
                h.gemm_torch(X[r0:r1], b, y)

        def full():
            h.gemm_torch(X, b, Yf)
        warm(chunks)
        c_med, c_lo, c_hi = ev_ms(chunks, main_s, a.reps)
        f_med, f_lo, f_hi = ev_ms(full, main_s, a.reps)
        ok = all(torch.equal(Yf[r0:r1].view(torch.int32), y.view(torch.int32)) for (r0, r1), y in zip(ranges, Yc))
        nnz = len(arrs[2]) + len(arrs[3])
        adds = T.flops(M, w, nnz)
        print(json.dumps({"item": "compute", "mode": mode, "P": P, "shape": [M, K, w], "s": S, "nnz": nnz,
                          "kernel": h.call_kernel(M), "chunk_kernel": h.call_kernel(ranges[0][1] - ranges[0][0]),
                          "chunks": len(ranges), "chunked_ms": round(c_med, 4), "chunked_ms_range": [round(c_lo, 4), round(c_hi, 4)],
                          "full_ms": round(f_med, 4), "full_ms_range": [round(f_lo, 4), round(f_hi, 4)],
                          "chunked_valu_frac": round(adds / (c_med * 1e-3) / 78.64e12, 4),
                          "chunks_equal_full_call": bool(ok)}), flush=True)
        if mode == "weak":
            kept = (h, b, Yc)
        else:
            h.close()

    # the reorder of one gathered chunk, alone and beside a chunk kernel
    h, b, Yc = kept
    side = torch.cuda.Stream(device=dev)
    for P, w in ((8, NW), (8, NW // 8)):
        Mc = ranges[0][1] - ranges[0][0]
        G = torch.randn((P * Mc, w), device=dev)
        Yfull = torch.empty((Mc, P * w), device=dev)
        widths = [w] * P

        def reorder():
            D._reorder(G.view(P, Mc, w), Yfull, widths)
        warm(reorder, 0.1)
        r_med, r_lo, r_hi = ev_ms(reorder, main_s, a.reps)
        moved = 2 * G.numel() * 4
        ok = torch.equal(Yfull.view(Mc, P, w), G.view(P, Mc, w).transpose(0, 1))
        line = {"item": "reorder", "P": P, "gathered": [P, Mc, w], "bytes_moved": moved, "alone_ms": round(r_med, 4),
                "alone_ms_range": [round(r_lo, 4), round(r_hi, 4)], "alone_gbps": round(moved / (r_med * 1e-3) / 1e9, 1),
                "row_major_ok": bool(ok)}
        if w == NW:
            # beside a chunk kernel: kernel on the main stream, reorder on the side
            k_only = ev_ms(lambda: h.gemm_torch(X[:Mc], b, Yc[0]), main_s, a.reps)[0]

            def both():
                side.wait_stream(main_s)
                h.gemm_torch(X[:Mc], b, Yc[0])
                with torch.cuda.stream(side):
                    reorder()
                main_s.wait_stream(side)
            warm(both, 0.1)
            bo = ev_ms(both, main_s, a.reps)[0]
            line.update({"chunk_kernel_alone_ms": round(k_only, 4), "kernel_plus_reorder_side_stream_ms": round(bo, 4),
                         "added_by_reorder_ms": round(bo - k_only, 4)})
        print(json.dumps(line), flush=True)
        del G, Yfull
    h.close()


if __name__ == "__main__":
    main()
