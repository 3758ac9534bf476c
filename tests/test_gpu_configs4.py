"""BASELINE configs[4] on one GPU, shard by shard.

configs[4] is M=4096 K=4096 N=131072 s=4 with W's columns sharded over 8
GPUs and the Y column blocks all-gathered (RCCL over xGMI).  The driver's
8-GPU run is the only place the eight ranks run side by side; this test runs
the SAME eight rank workloads one after the other on cuda:0, through the
code the ranks run:

  * tsg_dist.ShardedTCSC.draw(K, 131072, 4, 42, r, 8, "weak") -- rank r's
    column block, drawn from block_seed(42, r) with the generateSparseMatrix
    law (sparseUtils.h:52-87); rank 0's block is the single-GPU W;
  * TCSCDevice + gemm_torch at M=4096 (the automatic kernel choice), every
    element of Y_r checked against a dense fp32 GEMM of X and the +-1 block
    (integer X: every partial sum is exact, so any order gives the same bits;
    main.cpp:206-227's own argument);
  * tsg_dist._reorder of the eight [M, 16384] blocks, stacked as the
    all-gather delivers them ([P, M, w], rank-major), into the row-major
    [4096, 131072] Y -- every column block compared with its rank's Y_r.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M, K, NTOT, S, P, SEED = 4096, 4096, 131072, 4, 8, 42


def _dense_w(csp, csn, rip, rin, K, N, dev):
    import torch
    W = torch.zeros((K, N), dtype=torch.float32, device=dev)
    cols_p = np.repeat(np.arange(N), np.diff(csp))
    cols_n = np.repeat(np.arange(N), np.diff(csn))
    W[torch.from_numpy(rip.astype(np.int64)).to(dev), torch.from_numpy(cols_p).to(dev)] = 1.0
    W[torch.from_numpy(rin.astype(np.int64)).to(dev), torch.from_numpy(cols_n).to(dev)] = -1.0
    return W


@pytest.mark.timeout(900)
def test_configs4_shards_on_one_gpu(tsg):
    import torch
    import tsg_dist as D
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    w = NTOT // P
    assert D.shard_widths(NTOT, P) == [w] * P
    g = torch.Generator(device=dev)
    g.manual_seed(12345)
    X = torch.randint(-512, 513, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.float32)
    b_full = (torch.arange(NTOT, device=dev, dtype=torch.float32) % 7) - 3.0
    G = torch.empty((P, M, w), dtype=torch.float32, device=dev)  # what the all-gather delivers
    nnz_total = 0
    digests = set()
    for r in range(P):
        csp, csn, rip, rin = D.ShardedTCSC.draw(K, NTOT, S, SEED, r, P, "weak")
        assert len(csp) == w + 1 and int(csp[-1]) == len(rip) and int(csn[-1]) == len(rin)
        tsg.validate(csp, csn, rip, rin, K, w)
        if r == 0:  # rank 0's block is exactly the single-GPU workload (bench.py configs[2])
            ref0 = tsg.gen_tcsc(K, w, S, SEED)
            assert all(np.array_equal(a, b) for a, b in zip((csp, csn, rip, rin), ref0))
        digests.add(hash(rip[:4096].tobytes()))
        nnz_total += len(rip) + len(rin)
        sh = D.ShardedTCSC((csp, csn, rip, rin), K, NTOT, r, P, device=0, already_sliced=True)
        assert (sh.n0, sh.n1) == (r * w, (r + 1) * w)
        Yr = sh.forward(X, b_full)
        kernel = sh.local.call_kernel(M)
        W = _dense_w(csp, csn, rip, rin, K, w, dev)
        ref = torch.matmul(X, W) + b_full[sh.n0:sh.n1]
        del W
        torch.cuda.synchronize()
        same = torch.equal(Yr.view(torch.int32), ref.view(torch.int32))
        bad = 0 if same else int((Yr.view(torch.int32) != ref.view(torch.int32)).sum())
        assert same, f"rank {r}: {bad} of {M * w} elements differ ({kernel})"
        G[r].copy_(Yr)
        sh.local.close()
        del Yr, ref
    assert len(digests) == P, "every rank draws its own block"
    # configs[4]'s nonzeros: N_total / s per row of W, drawn block by block
    assert nnz_total == K * NTOT // S
    Yfull = torch.empty((M, NTOT), dtype=torch.float32, device=dev)
    D._reorder(G, Yfull, D.shard_widths(NTOT, P))
    torch.cuda.synchronize()
    for r in range(P):
        assert torch.equal(Yfull[:, r * w:(r + 1) * w].view(torch.int32), G[r].view(torch.int32)), f"block {r}"


def _oracle_threads():
    import os
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, min(16, n or len(os.sched_getaffinity(0))))


@pytest.mark.timeout(900)
def test_configs4_shards_fractional_x(tsg, oracle_mod):
    """The eight configs[4] rank workloads with ORDER-SENSITIVE X (24-bit
    mantissas over a 2^-23..2^0 exponent spread: every partial sum rounds),
    EVERY element of every shard compared bitwise with the BaseTCSC
    restatement (oracle/tcsc_oracle.c, comp.h:37-63) run over all 4096 rows
    with OpenMP: the shards are other W matrices than configs[2]'s, so their
    accumulation order is pinned here, not only by the integer-X test above
    (where any order gives the same bits)."""
    import torch
    import tsg_dist as D
    O = oracle_mod
    w = NTOT // P
    X = O.init_x_frac(M, K, 77)
    Xd = torch.from_numpy(X).cuda()
    b_full = ((np.arange(NTOT, dtype=np.float32) % 13) - 6) * np.float32(0.37)
    th = _oracle_threads()
    for r in range(P):
        csp, csn, rip, rin = D.ShardedTCSC.draw(K, NTOT, S, SEED, r, P, "weak")
        sh = D.ShardedTCSC((csp, csn, rip, rin), K, NTOT, r, P, device=0, already_sliced=True)
        b = np.ascontiguousarray(b_full[sh.n0:sh.n1])
        Yr = sh.forward(Xd, torch.from_numpy(b_full).cuda()).cpu().numpy()
        kernel = sh.local.call_kernel(M)
        sh.local.close()
        ref = O.base_tcsc(X, O.TCSC(csp, csn, rip, rin, K, w), b, threads=th)
        diff = Yr.view(np.uint32) != ref.view(np.uint32)
        assert not diff.any(), f"rank {r}: {int(diff.sum())} of {M * w} elements differ ({kernel})"
