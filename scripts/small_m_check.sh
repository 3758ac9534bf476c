#!/bin/bash
# GPU box: small-M kernel parity tests, then the M sweep against the jit kernel.
set -o pipefail
TAG=${1:-x}; shift || true
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_small_m.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_small.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest_small.log; [ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_pytest_small.log; exit $rc; }
timeout -k 10 300 python scripts/small_m_sweep.py "$@" > gpurun_out/${TAG}_small_m.jsonl 2>&1 || { tail -5 gpurun_out/${TAG}_small_m.jsonl; exit 1; }
python3 - gpurun_out/${TAG}_small_m.jsonl <<'P'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["M"], "ell", d["ell"]["kernel_ms"], "hbm", d["ell"]["hbm_frac_on_tcsc_bytes"], "valu", d["ell"]["valu_frac"],
              "| jit", d["jit"]["kernel_ms"], d["bit_identical"], d["auto"])
P
