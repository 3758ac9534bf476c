"""Device-pointer API contract on the GPU (include/ternary_spgemm.h,
tcsc_hip_gemm_dev): several streams / threads on one handle, graph capture
after tcsc_hip_reserve, and the argument checks of the Python mirror."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.cpu().numpy().view(np.uint32)


def test_two_streams_one_handle(tsg, oracle_mod):
    """Calls on two streams with different X, issued back to back without a
    host sync: each call's X^T staging must wait for the other stream's kernel
    (shared work buffer), so both results stay bit-exact."""
    import torch
    O = oracle_mod
    K, N, M = 2048, 4096, 1024
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 21))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.reserve(M)
    b = torch.from_numpy(np.linspace(-1, 1, N).astype(np.float32)).cuda()
    X1n, X2n = O.init_x_frac(M, K, 1), O.init_x_frac(M, K, 2)
    X1, X2 = torch.from_numpy(X1n).cuda(), torch.from_numpy(X2n).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for _ in range(4):
        with torch.cuda.stream(s1):
            Y1 = h.gemm_torch(X1, b)
        with torch.cuda.stream(s2):
            Y2 = h.gemm_torch(X2, b)
        outs.append((Y1, Y2))
    torch.cuda.synchronize()
    rows = np.r_[0:64, M - 64:M]
    bn = b.cpu().numpy()
    r1 = O.base_tcsc(np.ascontiguousarray(X1n[rows]), t, bn)
    r2 = O.base_tcsc(np.ascontiguousarray(X2n[rows]), t, bn)
    for Y1, Y2 in outs:
        assert np.array_equal(_bits(Y1)[rows], r1.view(np.uint32))
        assert np.array_equal(_bits(Y2)[rows], r2.view(np.uint32))
        assert torch.equal(Y1.view(torch.int32), outs[0][0].view(torch.int32))
        assert torch.equal(Y2.view(torch.int32), outs[0][1].view(torch.int32))
    h.close()


def test_threads_one_handle(tsg, oracle_mod):
    """Two host threads, each on its own stream, share one handle."""
    import torch
    O = oracle_mod
    K, N, M = 1000, 1500, 300
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 22))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    b = torch.full((N,), 2.0, device="cuda")
    Xs = [O.init_x_frac(M, K, 10 + i) for i in range(2)]
    res = [None, None]

    def work(i):
        torch.cuda.set_device(0)
        s = torch.cuda.Stream()
        X = torch.from_numpy(Xs[i]).cuda()
        with torch.cuda.stream(s):
            for _ in range(5):
                Y = h.gemm_torch(X, b)
        s.synchronize()
        res[i] = Y.cpu().numpy()

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    bn = np.full(N, 2.0, np.float32)
    for i in range(2):
        assert np.array_equal(res[i].view(np.uint32), O.base_tcsc(Xs[i], t, bn).view(np.uint32))
    h.close()


def test_threads_host_pointer_calls(tsg, oracle_mod):
    """Two host threads call the synchronous host-pointer comp_func
    (tcsc_hip_gemm, main.cpp:214-216) on one handle with different X and M:
    the handle's staging buffers serve one call at a time."""
    O = oracle_mod
    K, N = 700, 900
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 23))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    bn = np.full(N, 2.0, np.float32)
    Ms = (257, 33)  # different M: the staging buffers grow while the other thread runs
    Xs = [O.init_x_frac(Ms[i], K, 40 + i) for i in range(2)]
    res, err = [None, None], []

    def work(i):
        try:
            Y = np.empty((Ms[i], N), np.float32)
            for _ in range(6):
                h(Xs[i], bn, Y, Ms[i], N, K)
            res[i] = Y.copy()
        except Exception as e:  # surfaced below
            err.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not err, err
    for i in range(2):
        assert np.array_equal(res[i].view(np.uint32), O.base_tcsc(Xs[i], t, bn).view(np.uint32))
    h.close()


@pytest.mark.parametrize("chunks", [3, 5, 16])
def test_host_pointer_pipeline_chunks(tsg, oracle_mod, chunks):
    """The host-pointer call pipelined by M chunks (H2D / compute / D2H on three
    streams + a helper thread) with M not divisible by the chunk: comp_func and
    the PReLU twin stay bit-exact, and the handle can switch back to one
    unchunked call."""
    O = oracle_mod
    K, N, M = 800, 1300, 1000
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 26))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.set_host_chunks(chunks)
    rows = h.host_chunk_rows(M)
    assert rows % 128 == 0 and rows < M and M % rows != 0
    X = O.init_x_frac(M, K, 27)
    bn = np.linspace(-3, 3, N).astype(np.float32)
    al = np.linspace(0.1, 0.5, N).astype(np.float32)
    for _ in range(2):
        Y = h.gemm(X, bn)
        assert np.array_equal(Y.view(np.uint32), O.base_tcsc(X, t, bn).view(np.uint32))
    Yp = h.gemm_prelu(X, bn, al)
    assert np.array_equal(Yp.view(np.uint32), O.base_tcsc_prelu(X, t, bn, al).view(np.uint32))
    h.set_host_chunks(1)
    assert h.host_chunk_rows(M) == M
    assert np.array_equal(h.gemm(X, bn).view(np.uint32), Y.view(np.uint32))
    h.close()


def test_host_pointer_registered_buffers(tsg, oracle_mod):
    """Caller buffers page-locked once (tcsc_hip_host_register) for repeated
    host-pointer calls: same bits as pageable buffers, pipelined or not."""
    O = oracle_mod
    K, N, M = 900, 1100, 700
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 28))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    X = O.init_x_frac(M, K, 29)
    bn = np.linspace(-1, 1, N).astype(np.float32)
    Y = np.empty((M, N), np.float32)
    ref = O.base_tcsc(X, t, bn).view(np.uint32)
    with tsg.registered_host(X, Y):
        for chunks in (0, 1, 5):
            h.set_host_chunks(chunks)
            Y[:] = np.nan
            h(X, bn, Y, M, N, K)
            assert np.array_equal(Y.view(np.uint32), ref)
    h(X, bn, Y, M, N, K)  # unregistered again
    assert np.array_equal(Y.view(np.uint32), ref)
    h.close()


@pytest.mark.parametrize("M", [4096, 96])
def test_graph_capture_after_reserve(tsg, oracle_mod, M):
    """tcsc_hip_reserve(max_M) prepares every width a call with M <= max_M runs;
    the call is then captured into a HIP graph (no allocation, compile or sync
    inside) and each replay recomputes Y from the current X."""
    import torch
    O = oracle_mod
    K, N = 1024, 2048
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 23))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.reserve(4096)
    b = torch.full((N,), 2.0, device="cuda")
    Xs = torch.zeros((M, K), device="cuda")
    Ys = torch.empty((M, N), device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside capture
        h.gemm_torch(Xs, b, Ys)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        h.gemm_torch(Xs, b, Ys)
    bn = np.full(N, 2.0, np.float32)
    for seed in (1, 2):
        Xn = O.init_x_frac(M, K, seed)
        Xs.copy_(torch.from_numpy(Xn).cuda())
        g.replay()
        torch.cuda.synchronize()
        rows = np.r_[0:16, M - 16:M]
        ref = O.base_tcsc(np.ascontiguousarray(Xn[rows]), t, bn)
        assert np.array_equal(_bits(Ys)[rows], ref.view(np.uint32)), seed
    h.close()


def test_capture_keeps_uncaptured_ordering(tsg, oracle_mod):
    """An uncaptured call A on s3 is still reading the shared X^T buffer when a
    call is captured on s1; a later uncaptured call C on s2 must still wait
    for A before its staging overwrites X^T (the capture does not reset what
    uncaptured calls wait for).  A's and C's results stay bit-exact."""
    import torch
    O = oracle_mod
    K, N, M = 4096, 8192, 4096
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 25))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.reserve(M)
    bn = np.linspace(-1, 1, N).astype(np.float32)
    b = torch.from_numpy(bn).cuda()
    XAn, XCn = O.init_x_frac(M, K, 5), O.init_x_frac(M, K, 6)
    XA, XC = torch.from_numpy(XAn).cuda(), torch.from_numpy(XCn).cuda()
    Xg, Yg = torch.zeros((M, K), device="cuda"), torch.empty((M, N), device="cuda")
    YA, YC = torch.empty((M, N), device="cuda"), torch.empty((M, N), device="cuda")
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s1):  # warm-up outside capture
        h.gemm_torch(Xg, b, Yg)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s3):
        h.gemm_torch(XA, b, YA)          # A: uncaptured, still running below
    with torch.cuda.stream(s1):
        g.capture_begin()                # (no device sync, unlike torch.cuda.graph)
        h.gemm_torch(Xg, b, Yg)
        g.capture_end()
    with torch.cuda.stream(s2):
        h.gemm_torch(XC, b, YC)          # C: must wait for A's kernel
    torch.cuda.synchronize()
    rows = np.r_[0:32, M // 2:M // 2 + 32, M - 32:M]
    for X, Y in ((XAn, YA), (XCn, YC)):
        ref = O.base_tcsc(np.ascontiguousarray(X[rows]), t, bn)
        assert np.array_equal(_bits(Y)[rows], ref.view(np.uint32))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(Yg, torch.zeros_like(Yg) + b)
    h.close()


def test_capture_without_reserve_fails_loudly(tsg, oracle_mod):
    """A call that would have to grow the work buffer inside a capture is refused
    with TSG_ERR_ARG (and a hint), instead of breaking the capture."""
    import torch
    O = oracle_mod
    K, N = 500, 300
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 24))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    b = torch.full((N,), 2.0, device="cuda")
    X = torch.zeros((2000, K), device="cuda")
    g = torch.cuda.CUDAGraph()
    with pytest.raises(tsg.TSGError, match="tcsc_hip_reserve"):
        with torch.cuda.graph(g):
            h.gemm_torch(X, b)
    torch.cuda.synchronize()
    h.close()


def test_torch_argument_checks(tsg, oracle_mod):
    """gemm_torch refuses tensors the raw-pointer C-ABI would misread."""
    import torch
    O = oracle_mod
    K, N, M = 64, 48, 8
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 25))
    h = tsg.TCSCDevice(*t.arrays, K, N)
    X = torch.zeros((M, K), device="cuda")
    b = torch.zeros(N, device="cuda")
    Ybig = torch.zeros((M, 2 * N), device="cuda")
    bad = [
        dict(X=torch.zeros((M, K - 1), device="cuda"), b=b),            # narrow X
        dict(X=X, b=torch.zeros(N - 1, device="cuda")),                 # short b
        dict(X=X, b=b, Y=Ybig[:, :N]),                                   # non-contiguous Y
        dict(X=X, b=b, Y=torch.zeros((M, N + 1), device="cuda")),       # wrong Y shape
        dict(X=X.double(), b=b),                                         # dtype
        dict(X=X, b=b.cpu()),                                            # device
        dict(X=X, b=b, alpha=torch.zeros(N - 2, device="cuda")),        # short alpha
    ]
    for kw in bad:
        with pytest.raises(tsg.TSGError):
            h.gemm_torch(**kw)
    with pytest.raises(tsg.TSGError):
        h(np.zeros((M, K - 1), np.float32), np.zeros(N, np.float32), np.zeros((M, N), np.float32), M, N, K)
    with pytest.raises(tsg.TSGError):
        h(np.zeros((M, K), np.float32), np.zeros(N - 1, np.float32), np.zeros((M, N), np.float32), M, N, K)
    # Y with a storage offset that breaks 16-byte alignment still gets correct
    # values (the kernel's float4 stores check the pointer)
    Yo = torch.zeros(M * N + 1, device="cuda")[1:].view(M, N)
    Xn = O.init_x_frac(M, K, 3)
    h.gemm_torch(torch.from_numpy(Xn).cuda(), b, Y=Yo)
    torch.cuda.synchronize()
    assert np.array_equal(_bits(Yo), O.base_tcsc(Xn, t, np.zeros(N, np.float32)).view(np.uint32))
    h.close()
