"""The multi-GPU gather path with the HIP kernel on the GPU (SURVEY.md 8e,
VERDICT r02 "next" 2).

* RCCL: a world-1 "nccl" process group on cuda:0 (one process, HashStore).
  tsg_dist.GatherPipeline runs the HIP kernel per M chunk (chunks=3, a ragged
  tail) and issues each chunk's all_gather_into_tensor asynchronously on
  device tensors, with the work.wait() ordering against the next chunk's
  kernel and the reorder into row-major Y -- the same calls bench.py makes at
  world > 1.  Checked bitwise against the one-shot allgather_columns, a
  single full call and the oracle, under the weight-compiled and the
  automatic kernel choice.
* Uneven shards (w_local < the widest shard) need two ranks, and RCCL
  refuses two ranks on one device: two processes on cuda:0 over gloo (device
  tensors staged through host memory) run the same pipeline with the HIP
  kernel on an odd N, and the gathered Y must equal the unsharded call.
"""
import os
import socket

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.cpu().numpy().view(np.uint32)


def test_rccl_gather_pipeline_world1(tsg, oracle_mod):
    import torch
    import torch.distributed as dist
    import tsg_dist as D
    O = oracle_mod
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    assert not dist.is_initialized()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        K, N, M = 1000, 777, 300
        t = O.tcsc_encode(O.gen_ternary(K, N, 4, 31))
        h = tsg.TCSCDevice(*t.arrays, K, N, device=0)
        Xn = O.init_x_frac(M, K, 32)
        bn = np.linspace(-2, 2, N).astype(np.float32)
        X, b = torch.from_numpy(Xn).to(dev), torch.from_numpy(bn).to(dev)
        ref = O.base_tcsc(Xn, t, bn).view(np.uint32)
        for mode in (1, 0):  # weight-compiled kernel forced, then the automatic choice per chunk
            h.set_small_m(mode)
            Y1 = h.gemm_torch(X, b)
            Yg = D.allgather_columns(Y1, N, 1)
            pipe = D.GatherPipeline(M, N, 1, chunks=3, device=dev)
            assert [r1 - r0 for r0, r1 in pipe.ranges] == [128, 128, 44]
            Xc = {(r0, r1): X[r0:r1] for r0, r1 in pipe.ranges}
            Yp = torch.full((M, N), float("nan"), device=dev)
            for _ in range(2):  # twice through the same buffers
                pipe.run(lambda r0, r1, Yc: h.gemm_torch(Xc[(r0, r1)], b, Yc), Yp, N)
            torch.cuda.synchronize()
            assert np.array_equal(_bits(Y1), ref), h.call_kernel(M)
            assert torch.equal(Yg.view(torch.int32), Y1.view(torch.int32))
            assert torch.equal(Yp.view(torch.int32), Y1.view(torch.int32))
        h.close()
    finally:
        dist.destroy_process_group()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, K, N, M, q):
    import sys
    sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "ternary-spgemm_amd")]
    import torch
    import torch.distributed as dist
    import oracle as O
    import tspgemm as T
    import tsg_dist as D

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = O.tcsc_encode(O.gen_ternary(K, N, 4, 41))
        sh = D.ShardedTCSC.from_tcsc(*t.arrays, K, N, rank, world, device=0)
        Xn = O.init_x_frac(M, K, 42)
        bn = np.linspace(-1, 3, N).astype(np.float32)
        X, b = torch.from_numpy(Xn).to(dev), torch.from_numpy(bn).to(dev)
        w_local = sh.n1 - sh.n0
        pipe = D.GatherPipeline(M, N, world, chunks=3, device=dev)
        Xc = {(r0, r1): X[r0:r1] for r0, r1 in pipe.ranges}
        Yp = torch.full((M, N), float("nan"), device=dev)
        for _ in range(2):
            pipe.run(lambda r0, r1, Yc: sh.forward(Xc[(r0, r1)], b, Yc), Yp, w_local)
        torch.cuda.synchronize()
        if rank == 0:
            full = T.TCSCDevice(*t.arrays, K, N, device=0)
            Yf = full.gemm_torch(X, b)
            ref = O.base_tcsc(Xn, t, bn).view(np.uint32)
            q.put((w_local, pipe.wmax,
                   bool(torch.equal(Yp.view(torch.int32), Yf.view(torch.int32))),
                   bool(np.array_equal(Yf.cpu().numpy().view(np.uint32), ref))))
            full.close()
        sh.local.close()
    finally:
        dist.destroy_process_group()


def test_gather_pipeline_uneven_shards_two_ranks_one_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    K, N, M = 900, 1001, 300  # N odd: widths 501 / 500
    procs = [ctx.Process(target=_rank, args=(r, 2, port, K, N, M, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    w_local, wmax, pipe_ok, ref_ok = q.get(timeout=5)
    assert (w_local, wmax) == (501, 501)
    assert pipe_ok and ref_ok
