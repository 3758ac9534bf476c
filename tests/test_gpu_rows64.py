"""The 64-row image of the weight-compiled kernel (tsg_jit64_kernel; one M row
per lane, 64-row M tiles, every nonzero one VOP2 v_add_f32 / v_sub_f32, X^T in
the k-quad layout; tsg_internal.h) on the GPU through the
C-ABI: forced onto every call (tcsc_hip_set_tile_rows(h, 64), small-M walks
off) over the edge shapes, every stream shape, ragged M / K (64-row tiles,
192-row chunks), PReLU, special values, graph capture after reserve, and
every element at configs[2]'s K and N -- bit for bit against the BaseTCSC
oracle (comp.h:25-69)."""
import numpy as np
import pytest

from test_gpu_parity import EDGE, _bits_eq

pytestmark = pytest.mark.gpu


def _handle(tsg, t, K, N, width=0):
    h = tsg.TCSCDevice(*t.arrays, K, N)
    h.set_small_m(1)
    h.set_tile_rows(64)
    if width:
        h.set_jit_width(width)
    return h


@pytest.mark.parametrize("M,K,N,s", EDGE)
def test_edges_rows64(tsg, oracle_mod, M, K, N, s):
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, s, M * 7 + K))
    h = _handle(tsg, t, K, N)
    assert h.call_kernel(M) == "tsg_jit64_kernel" and h.call_tile_rows(M) == 64
    b = (np.arange(N, dtype=np.float32) - N / 2) * 0.37
    alpha = np.linspace(-0.5, 0.5, N).astype(np.float32)
    for X in (O.init_x_int(M, K, 5), O.init_x_frac(M, K, 6)):
        assert _bits_eq(h.gemm(X, b), O.base_tcsc(X, t, b)), (M, K, N, s)
        assert _bits_eq(h.gemm_prelu(X, b, alpha), O.base_tcsc_prelu(X, t, b, alpha))
    h.close()


@pytest.mark.parametrize("width", [128, 64, 32, 16, 8])
@pytest.mark.parametrize("M,K", [(1, 191), (63, 192), (64, 193), (65, 385), (130, 1000), (37, 4096)])
def test_rows64_widths_and_tiles(tsg, oracle_mod, width, M, K):
    """Every stream width (8 waves when pinned; 128 columns per wave only
    here), M across 64-row tiles and K across 192-row chunks."""
    O = oracle_mod
    N = 700
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, width + M + K))
    h = _handle(tsg, t, K, N, width)
    assert h.jit_width(M) == width
    b = np.linspace(-3, 3, N).astype(np.float32)
    X = O.init_x_frac(M, K, M + 3)
    assert _bits_eq(h.gemm(X, b), O.base_tcsc(X, t, b)), (width, M, K)
    h.close()


@pytest.mark.parametrize("M,N", [(64, 16384), (40, 4096), (200, 4096), (512, 4096)])
def test_rows64_automatic_shapes(tsg, oracle_mod, M, N):
    """The automatic stream shape of the 64-row image (4-wave workgroups at
    small M) against the oracle, sampled rows at K = 4096."""
    O = oracle_mod
    K = 4096
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, M + N))
    h = _handle(tsg, t, K, N)
    b = np.linspace(-1, 1, N).astype(np.float32)
    X = O.init_x_frac(M, K, 9)
    Y = h.gemm(X, b)
    rows = np.unique(np.linspace(0, M - 1, 9).astype(int))
    assert _bits_eq(Y[rows], O.base_tcsc(X[rows], t, b)), (M, N, h.jit_width(M), h.jit_waves(M))
    h.close()


def test_rows64_special_values(tsg, oracle_mod):
    from test_gpu_special import _same, _special_b, _special_x
    O = oracle_mod
    K, N = 700, 300
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 31))
    h = _handle(tsg, t, K, N)
    alpha = np.linspace(-0.5, 0.5, N).astype(np.float32)
    for M, kind in ((3, "mixed"), (64, "subnormal"), (70, "nan"), (7, "zeros")):
        X = _special_x(M, K, M, kind)
        b = _special_b(N, M + 1)
        _same(h.gemm(X, b), O.base_tcsc(X, t, b))
        _same(h.gemm_prelu(X, b, alpha), O.base_tcsc_prelu(X, t, b, alpha))
    h.close()


def test_rows64_capture_after_reserve(tsg, oracle_mod):
    """tcsc_hip_reserve prepares the 64-row images too: a captured call
    allocates and compiles nothing and replays bit-exact."""
    import torch
    O = oracle_mod
    K, N, M = 1000, 2048, 64
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, 5))
    h = _handle(tsg, t, K, N)
    h.reserve(M)
    X = torch.from_numpy(O.init_x_frac(M, K, 2)).cuda()
    b = torch.linspace(-1, 1, N).cuda()
    Y = torch.empty((M, N), device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        h.gemm_torch(X, b, Y)  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            h.gemm_torch(X, b, Y)
    Y.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert _bits_eq(Y.cpu().numpy(), O.base_tcsc(X.cpu().numpy(), t, b.cpu().numpy()))
    h.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("M", [64, 32, 1])
def test_rows64_full_y_configs2_kn(tsg, oracle_mod, M):
    """Every element at configs[2]'s K = 4096, N = 16384 with order-sensitive X
    (the shapes the 64-row image is for)."""
    import os
    O = oracle_mod
    K, N = 4096, 16384
    csp, csn, rip, rin = tsg.gen_tcsc(K, N, 4, 42)
    t = O.TCSC(csp, csn, rip, rin, K, N)
    h = _handle(tsg, t, K, N)
    X = O.init_x_frac(M, K, 77)
    b = (np.arange(N, dtype=np.float32) % 13 - 6) * np.float32(0.37)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or len(os.sched_getaffinity(0)))))
    assert _bits_eq(h.gemm(X, b), O.base_tcsc(X, t, b, threads=threads))
    h.close()


@pytest.mark.parametrize("qblock", ["rows", "16", "8"])
@pytest.mark.parametrize("M,K", [(1, 1024), (64, 4096), (130, 1000), (37, 192 * 3), (70, 208), (70, 196),
                                 (70, 188), (70, 376), (64, 189), (5, 190), (130, 4100)])
def test_rows64_direct_x_and_staged(tsg, oracle_mod, monkeypatch, M, K, qblock):
    """The 64-row image stages its DMA pieces straight from row-major X
    (TSG_JIT_XDIRECT=1; automatic for the row layout, tsg_internal.h
    kJit64RowFlag) when the rows are 16-B aligned and K allows it (row layout:
    K >= 188 and K % 4 == 0, the last chunk starting at K - 188; blocked
    layout: no piece straddles K), and through the staged copy otherwise
    (TSG_JIT_XDIRECT=0, or X at a 4-byte offset).  The row layout and both
    piece shapes of the blocked layout (TSG_JIT_QBLOCK: 16 rows x 4 quads, 8 x
    8).  Bit-exact against the oracle (rows past M read row M-1 and are
    dropped; blocked pieces past K are never staged)."""
    import torch
    if qblock == "rows":
        monkeypatch.delenv("TSG_JIT_QBLOCK", raising=False)
    else:
        monkeypatch.setenv("TSG_JIT_QBLOCK", qblock)
    O = oracle_mod
    N = 333
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, M + K))
    h = _handle(tsg, t, K, N)
    Xh = O.init_x_frac(M, K, 21)
    b = torch.linspace(-2, 2, N).cuda()
    ref = O.base_tcsc(Xh, t, b.cpu().numpy())
    buf = torch.empty(M * K + 4, device="cuda")
    for direct in ("1", "0"):
        monkeypatch.setenv("TSG_JIT_XDIRECT", direct)
        for shift in (0, 1):  # 0: 16-B aligned (direct when K allows); 1: 4-byte offset (staged)
            X = buf[shift:shift + M * K].view(M, K)
            X.copy_(torch.from_numpy(Xh))
            if qblock == "rows":  # tcsc_hip_call_launches: 1 when the kernel reads X itself
                direct_ok = direct == "1" and shift == 0 and K >= 188 and K % 4 == 0
                assert h.call_launches(X, M) == (1 if direct_ok else 2), (M, K, direct, shift)
            Y = h.gemm_torch(X, b)
            torch.cuda.synchronize()
            assert _bits_eq(Y.cpu().numpy(), ref), (M, K, shift, direct, qblock)
    h.close()


@pytest.mark.parametrize("M,K,N", [(64, 4096, 16384), (37, 1000, 4096), (1, 777, 2048), (130, 1000, 2048),
                                   (64, 96, 1500), (70, 97, 3000)])
def test_rows64_half_ring(tsg, oracle_mod, monkeypatch, M, K, N):
    """The half ring (TSG_JIT_HALF=1: the 4-wave shapes run 96-row chunks in a
    72-KiB ring, two workgroups per CU; tsg_internal.h kJit64HalfChunk),
    staged and direct X, bit for bit against the oracle."""
    import torch
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, M + K + N))
    b = np.linspace(-2, 2, N).astype(np.float32)
    Xh = O.init_x_frac(M, K, 23)
    ref = O.base_tcsc(Xh, t, b)
    monkeypatch.setenv("TSG_JIT_HALF", "1")
    h = _handle(tsg, t, K, N)
    assert h.jit_waves(M) == 4, (M, K, N, h.jit_width(M))  # these shapes pick 4-wave workgroups
    X = torch.from_numpy(Xh).cuda()
    bt = torch.from_numpy(b).cuda()
    for direct in ("0", "1"):
        monkeypatch.setenv("TSG_JIT_XDIRECT", direct)
        Y = h.gemm_torch(X, bt)
        torch.cuda.synchronize()
        assert _bits_eq(Y.cpu().numpy(), ref), (M, K, N, direct, h.jit_width(M), h.jit_waves(M))
    h.close()


@pytest.mark.parametrize("M,K,N", [(64, 4096, 16384), (37, 1000, 4096), (1, 777, 2048), (130, 1000, 2048),
                                   (64, 96, 1500), (70, 97, 3000), (1024, 4096, 1024)])
def test_rows64_wave_pairs(tsg, oracle_mod, monkeypatch, M, K, N):
    """Wave pairs (TSG_JIT_PAIR=1: the 4-wave streams run by 8-wave
    workgroups, waves w and w + 4 on one half of the rows each, exec-masked;
    tsg_jit_kernel.hip): staged and direct X, with PReLU, bit for bit against
    the oracle -- every row is stored by exactly one wave of its pair and
    every DMA piece is staged by the two halves together."""
    import torch
    O = oracle_mod
    t = O.tcsc_encode(O.gen_ternary(K, N, 4, M + K + N + 5))
    b = np.linspace(-2, 2, N).astype(np.float32)
    alpha = np.linspace(0.05, 0.3, N).astype(np.float32)
    Xh = O.init_x_frac(M, K, 29)
    ref = O.base_tcsc(Xh, t, b)
    ref_p = O.base_tcsc_prelu(Xh, t, b, alpha)
    monkeypatch.setenv("TSG_JIT_PAIR", "1")
    h = _handle(tsg, t, K, N)
    assert h.jit_waves(M) == 4, (M, K, N, h.jit_width(M))  # these shapes pick 4-wave streams
    X = torch.from_numpy(Xh).cuda()
    bt = torch.from_numpy(b).cuda()
    at = torch.from_numpy(alpha).cuda()
    for direct in ("0", "1"):
        monkeypatch.setenv("TSG_JIT_XDIRECT", direct)
        Y = h.gemm_torch(X, bt)
        Yp = h.gemm_torch(X, bt, alpha=at)
        torch.cuda.synchronize()
        assert _bits_eq(Y.cpu().numpy(), ref), (M, K, N, direct, h.jit_width(M))
        assert _bits_eq(Yp.cpu().numpy(), ref_p), (M, K, N, direct, h.jit_width(M))
    h.close()
