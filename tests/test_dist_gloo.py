"""World-size-2 (and 3) column sharding on CPU with the gloo backend.

Each rank slices its W columns with the product's tsg_tcsc_slice (or draws
them with tsg_gen_tcsc), computes its Y block with the CPU oracle standing in
for the GPU kernel, and the blocks are all-gathered by
tsg_dist.allgather_columns.  The gathered Y must equal the unsharded oracle
bit for bit: this covers the shard arithmetic, the rebasing and the gather
layout of the multi-GPU path (the GPU kernel itself is covered by -m gpu).
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
        Yl = O.base_tcsc(X, O.TCSC(*sl, K, n1 - n0), np.ascontiguousarray(b[n0:n1]))
        Y = D.allgather_columns(torch.from_numpy(Yl), N, world)
        if rank == 0:
            ref = O.base_tcsc(X, O.tcsc_encode(O.gen_ternary(K, N, s, seed)), b)
            q.put(bool(np.array_equal(Y.numpy().view(np.uint32), ref.view(np.uint32))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,use_gen", [(2, 300, False), (2, 37, True), (3, 64, False)])
def test_column_shard_allgather_gloo(world, N, use_gen):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 200, N, 4, 5, 9, use_gen, q))
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
