"""The reference's benchmark report, parsed and collected.

The reference's harness (plots/run_benchmark.py:44-117) runs its binary per
(M, K, N, s), scrapes stdout and saves one JSON list for the plotting scripts.
bin/sparseGEMM_hip.out prints the same report lines (host/sparseGEMM_hip.cpp,
the format of cpp_impl/main.cpp:259-271), so:

* ``parse_report`` reads a report the way run_benchmark.py:63-77 does: per
  function "Running: <name>" followed by "Performance: <flops/cycle>",
  "Total Input Size: <bytes>" and "Operational Intensity: <flops/byte>", ANSI
  colour codes stripped from the name; "Test case <name> passed|failed!" lines
  give the correctness status;
* ``run_benchmark`` sweeps the same test-case lists and writes the same JSON
  schema ({"test_case": {M, K, N}, "results": {"<name> (Sparsity 1/<s>)":
  {"total_input_size": ..., "operational_intensity": ...,
  "performance": ...}}}), so the reference's plot_*.py can chart GPU runs.

    python -m tsg_report [--save] [--output F] [--varyonly M|K|N] [--sparsityonly s] [--quick]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
from typing import Dict, List, Optional, Tuple

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(PKG_DIR, "bin", "sparseGEMM_hip.out")

_ANSI = re.compile(r"\x1b\[[0-9;]*m")
_NUM = r"([0-9.eE+-]+)"
_BLOCK = re.compile(r"Running:\s*(.*?)\s*\n.*?Performance:\s*" + _NUM + r".*?Total Input Size:\s*" + _NUM +
                    r".*?Operational Intensity:\s*" + _NUM, re.S)
_TEST = re.compile(r"Test case (.*?) (passed|failed)!")

# run_benchmark.py:8-33: the default (M, K, N) list, the one-dimension sweeps
# around 1024, and the sparsities
CASES = [(1, 512, 2048), (16, 1024, 4096), (64, 2048, 8192), (256, 4096, 16384), (1000, 2048, 512),
         (4000, 4096, 1024), (16000, 8192, 2048), (64000, 16384, 4096)]
SWEEP = {"M": [1, 16, 64, 256, 1000, 4000, 16000, 64000], "K": [512, 1024, 2048, 4096, 8192, 16384],
         "N": [512, 1024, 2048, 4096, 8192, 16384]}
SPARSITIES = [2, 4, 8, 16]


def parse_report(stdout: str) -> Tuple[List[Tuple[str, float, int, float]], Dict[str, str]]:
    """[(name, flops/cycle, total input bytes, flops/byte)], {name: passed|failed}."""
    rows = [(_ANSI.sub("", name).strip(), float(p), int(float(size)), float(oi))
            for name, p, size, oi in _BLOCK.findall(stdout)]
    status = {_ANSI.sub("", name).strip(): st for name, st in _TEST.findall(stdout)}
    return rows, status


def cases_for(varyonly: Optional[str] = None) -> List[Tuple[int, int, int]]:
    if varyonly is None:
        return list(CASES)
    d = 1024
    return [(v if varyonly == "M" else d, v if varyonly == "K" else d, v if varyonly == "N" else d)
            for v in SWEEP[varyonly]]


def run_case(M: int, K: int, N: int, s: int, driver: str = DRIVER, correctness: bool = False,
             timeout: Optional[float] = None) -> subprocess.CompletedProcess:
    cmd = [driver, "-M", str(M), "-K", str(K), "-N", str(N), "-s", str(s)]
    if correctness:
        cmd.append("-correctness")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)


def run_benchmark(cases, sparsities, varyonly: Optional[str] = None, driver: str = DRIVER,
                  log=print) -> List[dict]:
    out = []
    for M, K, N in cases:
        entry = {"test_case": {"M": M, "K": K, "N": N}, "results": {}}
        log(f"--- Running test case: M={M}, K={K}, N={N} ---")
        for s in sparsities:
            p = run_case(M, K, N, s, driver)
            if p.returncode != 0:
                log(f"  ERROR: M={M}, K={K}, N={N}, s={s}: exit {p.returncode}\n{p.stderr}")
                continue
            rows, status = parse_report(p.stdout)
            if not rows:
                log(f"  No performance results found for sparsity 1/{s}.")
            for name, perf, size, oi in rows:
                # the size is stored under "total_input_size" always; with
                # --varyonly it is the varied dimension (run_benchmark.py:86-101)
                val = {"M": M, "K": K, "N": N}.get(varyonly, size)
                entry["results"][f"{name} (Sparsity 1/{s})"] = {"total_input_size": val,
                                                                "operational_intensity": oi, "performance": perf}
                log(f"  {name} (Sparsity 1/{s}): total_input_size={val}, {perf} flops/cycle, {oi} flops/Byte")
                if status.get(name) == "failed":
                    log(f"    WARNING: {name} failed correctness check!")
        out.append(entry)
    return out


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="run_benchmark.py-compatible sweep of the MI355X driver")
    ap.add_argument("-s", "--save", action="store_true")
    ap.add_argument("--output", default="benchmark_results.json")
    ap.add_argument("--varyonly", choices=["M", "K", "N"])
    ap.add_argument("--sparsityonly", type=int)
    ap.add_argument("--quick", action="store_true", help="the first three default cases only")
    ap.add_argument("--driver", default=DRIVER)
    a = ap.parse_args(argv)
    cases = cases_for(a.varyonly)
    if a.quick:
        cases = cases[:3]
    sp = [a.sparsityonly] if a.sparsityonly is not None else SPARSITIES
    res = run_benchmark(cases, sp, a.varyonly, a.driver)
    if a.save:
        with open(a.output, "w") as f:
            json.dump(res, f, indent=4)
        print(f"\nAll benchmark results saved to {a.output}")


if __name__ == "__main__":
    main()
