"""The reference's own benchmark case list (plots/run_benchmark.py:8-33 via
tsg_report.CASES: eight (M, K, N) from GEMV-like M = 1 to M = 64000) through
the automatic kernel choice, at its default sparsity s = 4 and at s = 16, with
order-sensitive X (integer mantissas scaled by 2^-23 ... 2^0, generated on the
GPU): sampled rows (first, middle, last) bit for bit against the BaseTCSC
restatement (comp.h:37-63 order).  Covers the jit kernel at 8 and 4 waves, the
small-M walks and the starved-jit ELL pick on the shapes the reference
itself benchmarks."""
import numpy as np
import pytest

from tsg_report import CASES

pytestmark = pytest.mark.gpu


def _frac_x(M, K, seed, dev):
    import torch
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    mant = torch.randint(-(1 << 23), 1 << 23, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.float32)
    exp = torch.randint(-46, -22, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.float32)
    return mant * torch.pow(2.0, exp)  # |x| in [2^-46, 2^0): partial sums round


@pytest.mark.parametrize("s", [4, 16])
@pytest.mark.parametrize("M,K,N", CASES)
def test_reference_case_list(tsg, oracle_mod, M, K, N, s):
    import torch
    O = oracle_mod
    dev = torch.device("cuda", 0)
    arrs = tsg.gen_tcsc(K, N, s, 42)
    h = tsg.TCSCDevice(*arrs, K, N, device=0)
    X = _frac_x(M, K, 1000 + M + K + N + s, dev)
    b = torch.linspace(-3.0, 3.0, N, device=dev)
    Y = h.gemm_torch(X, b)
    torch.cuda.synchronize()
    rows = np.unique(np.r_[0, M // 2, M - 1])
    ref = O.base_tcsc(np.ascontiguousarray(X[rows].cpu().numpy()), O.TCSC(*arrs, K, N), b.cpu().numpy())
    got = Y[rows].cpu().numpy()
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32)), (M, K, N, s, h.call_kernel(M))
    h.close()
    del X, Y
    torch.cuda.empty_cache()
