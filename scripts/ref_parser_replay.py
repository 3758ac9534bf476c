#!/usr/bin/env python3
"""Build container only (reads /root/reference): replay the driver reports
captured on the GPU box (tests/golden/f4_reports.json, written by
scripts/capture_reports.py) through the REFERENCE's own scraper,
plots/run_benchmark.py:run_and_parse_benchmark (its regexes and JSON schema,
:63-107), with its subprocess.run stubbed to hand back the captured stdout of
each (M, K, N, s) it asks for.  The JSON it saves is committed as
tests/golden/f4_ref_parsed.json; tests/test_report.py checks that
tsg_report.run_benchmark writes the same JSON from the same stdout.  The
reference's Python never travels: only its output (data) is committed.

    python scripts/ref_parser_replay.py [--reports tests/golden/f4_reports.json]
                                        [--out tests/golden/f4_ref_parsed.json]
"""
import argparse
import importlib.util
import io
import json
import os
import subprocess
import sys
from contextlib import redirect_stdout

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/plots/run_benchmark.py"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reports", default=os.path.join(REPO, "tests", "golden", "f4_reports.json"))
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "f4_ref_parsed.json"))
    a = ap.parse_args()
    reports = json.load(open(a.reports))["reports"]
    spec = importlib.util.spec_from_file_location("ref_run_benchmark", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    asked = []

    def fake_run(command, capture_output=True, text=True, check=False, **kw):
        # command = ["sudo", "./SparseGEMM.out", "-M", m, "-K", k, "-N", n, "-s", s] (run_benchmark.py:36-59)
        args = dict(zip(command[2::2], command[3::2]))
        key = ",".join(args[f] for f in ("-M", "-K", "-N", "-s"))
        asked.append(key)
        rep = reports[key]
        return subprocess.CompletedProcess(command, rep["returncode"], rep["stdout"], "")

    mod.subprocess.run = fake_run
    log = io.StringIO()
    with redirect_stdout(log):
        mod.run_and_parse_benchmark(save_results=True, outname=a.out)
    missing = sorted(set(reports) - set(asked))
    print(f"replayed {len(asked)} reports through {REF}; written {a.out}"
          + (f"; not asked for: {missing}" if missing else ""))
    sys.stdout.write(log.getvalue()[-600:])


if __name__ == "__main__":
    main()
