import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "oracle"), os.path.join(REPO, "ternary-spgemm_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running CPU case")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build(ref=False) if not os.path.exists(os.path.join(REPO, "oracle", "liboracle.so")) else None
    return oracle


@pytest.fixture(scope="session")
def tsg():
    import tspgemm
    if not os.path.exists(tspgemm.LIB_PATH):
        tspgemm.build()
    return tspgemm
