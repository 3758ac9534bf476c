"""World-size-2 (and 3) column sharding on CPU with the gloo backend.

Each rank slices its W columns with the product's tsg_tcsc_slice (or draws
them with tsg_gen_tcsc), computes its Y block with the CPU oracle standing in
for the GPU kernel, and the blocks are all-gathered by
tsg_dist.allgather_columns or by the M-chunked tsg_dist.GatherPipeline (the
path bench.py times for world > 1).  The gathered Y must equal the unsharded
oracle bit for bit: this covers the shard arithmetic, the rebasing, the chunk
ranges and the gather layout of the multi-GPU path (the GPU kernel itself is
covered by -m gpu).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, K, N, s, seed, M, use_gen, q):
    import sys
    sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "ternary-spgemm_amd")]
    import oracle as O
    import tspgemm as T
    import tsg_dist as D

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n0, n1 = D.column_shard(N, world, rank)
        if use_gen:
            sl = T.gen_tcsc(K, N, s, seed, n0, n1)
        else:
            full = O.tcsc_encode(O.gen_ternary(K, N, s, seed))
            sl = T.tcsc_slice(*full.arrays, N, n0, n1)
        X = O.init_x_frac(M, K, 99)
        b = (np.arange(N, dtype=np.float32) * 0.25 - 3).astype(np.float32)
        tl = O.TCSC(*sl, K, n1 - n0)
        bl = np.ascontiguousarray(b[n0:n1])
        Yl = O.base_tcsc(X, tl, bl)
        Y = D.allgather_columns(torch.from_numpy(Yl), N, world)
        # the chunked pipeline (compute chunk i+1 while chunk i is gathered), twice
        # through the same buffers, 3 chunks of 128-row multiples + a ragged tail
        pipe = D.GatherPipeline(M, N, world, chunks=3)

        def compute(r0, r1, Yc):
            Yc.copy_(torch.from_numpy(O.base_tcsc(np.ascontiguousarray(X[r0:r1]), tl, bl)))

        Yp = torch.full((M, N), float("nan"))
        for _ in range(2):
            pipe.run(compute, Yp, n1 - n0)
        if rank == 0:
            ref = O.base_tcsc(X, O.tcsc_encode(O.gen_ternary(K, N, s, seed)), b)
            q.put(bool(np.array_equal(Y.numpy().view(np.uint32), ref.view(np.uint32))) and
                  bool(np.array_equal(Yp.numpy().view(np.uint32), ref.view(np.uint32))) and
                  1 <= len(pipe.ranges) <= 3)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,M,use_gen", [(2, 300, 9, False), (2, 37, 300, True), (3, 64, 400, False)])
def test_column_shard_allgather_gloo(world, N, M, use_gen):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 200, N, 4, 5, M, use_gen, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_column_shard_arithmetic():
    import tsg_dist as D
    for N in (1, 7, 16384, 131072, 100003):
        for world in (1, 2, 3, 8):
            ranges = [D.column_shard(N, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == N
            assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
            w = D.shard_widths(N, world)
            assert max(w) - min(w) <= 1


def test_m_chunks():
    import tsg_dist as D
    for M in (1, 127, 128, 129, 300, 4096, 4097):
        for c in (1, 2, 3, 4, 8):
            r = D.m_chunks(M, c)
            assert r[0][0] == 0 and r[-1][1] == M
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert all(a0 % 128 == 0 for a0, _ in r) and len(r) <= c


def test_synthetic_w_modes():
    """strong: the same W for every world size (slices concatenate to the
    unsharded draw); weak: rank 0's block is the single-GPU W, and each rank
    draws only its own block (block j from block_seed(seed, j))."""
    import tspgemm as T
    import tsg_dist as D
    K, N, s, seed = 300, 96, 4, 11
    full = T.gen_tcsc(K, N, s, seed)
    for world in (2, 3, 4):
        parts = [D.ShardedTCSC.draw(K, N, s, seed, r, world, "strong") for r in range(world)]
        rip = np.concatenate([p[2] for p in parts])
        rin = np.concatenate([p[3] for p in parts])
        assert np.array_equal(rip, full[2]) and np.array_equal(rin, full[3])
        csp = np.concatenate([parts[0][0]] + [p[0][1:] + sum(len(q[2]) for q in parts[:i])
                                               for i, p in enumerate(parts) if i])
        assert np.array_equal(csp, full[0])
    Nr = 48
    w0 = D.ShardedTCSC.draw(K, Nr * 4, s, seed, 0, 4, "weak")
    assert all(np.array_equal(a, b) for a, b in zip(w0, T.gen_tcsc(K, Nr, s, seed)))
    w3 = D.ShardedTCSC.draw(K, Nr * 4, s, seed, 3, 4, "weak")
    assert all(np.array_equal(a, b) for a, b in zip(w3, T.gen_tcsc(K, Nr, s, D.block_seed(seed, 3))))
    # the generateSparseMatrix law per block: exactly Nr/s nonzeros in every row
    W = np.zeros((K, Nr), np.int32)
    for n in range(Nr):
        W[w3[2][w3[0][n]:w3[0][n + 1]], n] = 1
        W[w3[3][w3[1][n]:w3[1][n + 1]], n] = -1
    assert (np.count_nonzero(W, axis=1) == Nr // s).all()
    with pytest.raises(ValueError):
        D.ShardedTCSC.draw(K, 97, s, seed, 0, 2, "weak")
