"""The four kernels on one small handle, as the round-end smoke check runs
them (M = 600 pinned to the 128-row image, M = 96 on the 64-row image, M = 5
on the walk, M = 1 on the producer/consumer walk), each bit for bit against
the BaseTCSC oracle (comp.h:25-69) with integer and order-sensitive X.  Since
round 5 registration compiles the 64-row image, so the 128-row one is built
by the pinned call itself."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_four_kernels_on_one_handle(tsg, oracle_mod):
    import torch
    O = oracle_mod
    K, N, s = 700, 300, 4
    t = O.tcsc_encode(O.gen_ternary(K, N, s, 1234))
    h = tsg.TCSCDevice(*t.arrays, K, N, device=0)
    info = h.info()  # the registration image: the 64-row image's 128 x 8
    assert (info["tile_rows"], info["tile_cols"], info["chunk_rows"]) == (64, 1024, 188)
    b = np.linspace(-3, 3, N).astype(np.float32)
    ran = []
    for M in (600, 96, 5, 1):
        h.set_small_m(1 if M >= 96 else 0)
        h.set_tile_rows(128 if M == 600 else 0)
        for X in (O.init_x_int(M, K, 1), O.init_x_frac(M, K, 2)):
            Y = h.gemm_torch(torch.from_numpy(X).cuda(), torch.from_numpy(b).cuda()).cpu().numpy()
            assert np.array_equal(Y.view(np.uint32), O.base_tcsc(X, t, b).view(np.uint32)), h.call_kernel(M)
        ran.append(h.call_kernel(M))
    assert ran == ["tsg_jit_kernel", "tsg_jit64_kernel", "tsg_tcsc_ell_kernel", "tsg_tcsc_ell_pc_kernel"], ran
    h.close()
