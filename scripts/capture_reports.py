#!/usr/bin/env python3
"""GPU box: capture bin/sparseGEMM_hip.out's stdout over the reference's own
sweep (plots/run_benchmark.py:8-33 default case list x s in {2, 4, 8, 16}),
plus configs[0] with -correctness, into one JSON file {"M,K,N,s": stdout}.
The file becomes tests/golden/f4_reports.json; the build container replays it
through the reference's parser (scripts/ref_parser_replay.py) and through
tsg_report (tests/test_report.py).

    python scripts/capture_reports.py OUT.json [--timeout 240]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ternary-spgemm_amd"))
import tsg_report as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--timeout", type=float, default=240)
    a = ap.parse_args()
    res = {"driver": "ternary-spgemm_amd/bin/sparseGEMM_hip.out", "reports": {}, "correctness": {}}
    p = R.run_case(32, 1024, 4096, 4, correctness=True, timeout=a.timeout)
    res["correctness"]["32,1024,4096,4"] = {"returncode": p.returncode, "stdout": p.stdout}
    print("configs[0] -correctness rc", p.returncode, flush=True)
    for M, K, N in R.CASES:
        for s in R.SPARSITIES:
            t0 = time.time()
            p = R.run_case(M, K, N, s, timeout=a.timeout)
            res["reports"][f"{M},{K},{N},{s}"] = {"returncode": p.returncode, "stdout": p.stdout}
            print(f"{M},{K},{N},{s} rc {p.returncode} {time.time() - t0:.1f} s", flush=True)
            if p.returncode != 0:
                print(p.stderr[-2000:], flush=True)
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
    bad = [k for k, v in res["reports"].items() if v["returncode"] != 0]
    sys.exit(1 if bad or res["correctness"]["32,1024,4096,4"]["returncode"] != 0 else 0)


if __name__ == "__main__":
    main()
