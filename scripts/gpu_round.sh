#!/bin/bash
# GPU box: micro-benchmarks (optional), parity tests per kernel variant, bench per variant.
# Usage: scripts/gpu_round.sh <tag> "<micro bins>" <variant>...
#   variant: "default" or a TSG_KERNEL value, optionally @<lib dir> (TSG_LIB variant build);
#   a leading "+" skips the parity tests for that variant.  Every GPU step has its own time limit.
set -o pipefail
TAG=${1:-x}; MICROS=${2:-}; shift 2 || true
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in $MICROS; do
  timeout -k 10 120 ./scripts/$m > gpurun_out/${m%.bin}_$TAG.log 2>&1 || { echo "micro $m failed rc=$?"; cat gpurun_out/${m%.bin}_$TAG.log | tail -5; exit 1; }
  cat gpurun_out/${m%.bin}_$TAG.log
done
for v in "$@"; do
  # v = <TSG_KERNEL or default>[@<lib dir under ternary-spgemm_amd>]
  unset TSG_KERNEL TSG_LIB
  skip=0; [ "${v:0:1}" = "+" ] && { skip=1; v=${v:1}; }
  k=${v%@*}; [ "$k" = default ] || export TSG_KERNEL=$k
  [ "$v" = "${v#*@}" ] || export TSG_LIB=ternary-spgemm_amd/${v#*@}/libternary_spgemm.so
  if [ $skip = 0 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc: $(tail -1 gpurun_out/pytest_${TAG}_$v.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_${TAG}_$v.log; exit $rc; }
  fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-rows 0 > gpurun_out/bench_${TAG}_$v.log 2>&1
  rc=$?; echo "bench $v rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_${TAG}_$v.log; exit $rc; }
  python - gpurun_out/bench_${TAG}_$v.log <<'P'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "GFLOP/s", round(d["value"],1), "kernel_ms", d["roofline"].get("kernel_ms"), "ms/step", d["ms_per_step"])
P
done
