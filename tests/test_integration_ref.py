"""The drop-in compiled against the reference's own headers (CPU).

oracle/plugin_ref_check.cpp includes cpp_impl/common.h,
data_structures/DataStructureInterface.hpp and sparseUtils.h where they lie
under /root/reference, builds include/tcsc_hip_plugin.hpp with
TSG_WITH_REFERENCE_DSI (HipTCSC derives from DataStructureInterface) and
registers it exactly as INTEGRATION.md section 2 shows.  Compiling and linking
it is the check that the C-ABI, the plugin and the reference's interfaces
agree; tests/test_gpu_parity.py::test_plugin_against_reference_headers runs it
on the GPU (the reference's generator, TCSC / BlockedTCSC<512> ctors, GEMM and
compare_results around our kernel).
"""
import os
import subprocess

import pytest

from conftest import REPO

REF = os.environ.get("REF", "/root/reference")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "cpp_impl")), reason="reference sources not mounted")
def test_plugin_builds_against_reference_headers():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "refplugin"], check=True)
    exe = os.path.join(REPO, "oracle", "_ref", "plugin_ref_check")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env={**os.environ, "HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "built and linked against the reference headers" in r.stdout or "passed!" in r.stdout
