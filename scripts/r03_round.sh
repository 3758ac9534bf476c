#!/bin/bash
# GPU box, round 3: full GPU suite, the default bench line, the host-pointer
# pipeline chunk A/B, the reference's own case list with the sweeps, DMA spread
# A/B at the sparse end under the current map rule.  Stops at the first failure.
# Usage: scripts/r03_round.sh <tag> [skip-suite]
set -o pipefail
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "$2" != skip-suite ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "gpu suite rc=$rc: $(tail -1 gpurun_out/pytest_$TAG.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_$TAG.log; exit $rc; }
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.jsonl 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
python - gpurun_out/bench_$TAG.jsonl <<'P'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "kernel_ms", d["roofline"]["kernel_ms"], "valu", d["roofline"]["binding"]["frac"])
print("e2e", d["e2e_host_pointers"])
P
timeout -k 10 170 python scripts/host_pipe_ab.py > gpurun_out/host_pipe_$TAG.jsonl 2>&1
rc=$?; echo "host pipe A/B rc=$rc"; cat gpurun_out/host_pipe_$TAG.jsonl | grep chunks; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/ref_cases.py --sweep > gpurun_out/ref_cases_$TAG.jsonl 2> gpurun_out/ref_cases_$TAG.err
rc=$?; echo "ref cases rc=$rc ($(wc -l < gpurun_out/ref_cases_$TAG.jsonl) cases)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ref_cases_$TAG.err; exit $rc; }
: > gpurun_out/spread_$TAG.txt
for rep in 1 2; do
  for v in 0.5,1 0.75,1 1.0,1; do
    TSG_JIT_DMA=$v timeout -k 10 170 python scripts/configs.py --shape 4096,4096,16384,16 --shape 4096,4096,16384,8 --shape 4096,4096,16384,4 --shape 512,4096,4096,4 --steps 20 2>/dev/null | sed "s/^/dma=$v rep=$rep /" >> gpurun_out/spread_$TAG.txt || { echo "spread $v failed"; exit 1; }
  done
  echo "spread rep $rep done"
done
