#!/bin/bash
# GPU box: parity tests on the default kernel, then bench A/B over TSG_KERNEL
# variants.  Usage: scripts/ab_bench.sh <tag> <variant>...
# variant: "default" (TSG_KERNEL unset), a TSG_KERNEL value, or lib:<dir>
# (TSG_LIB=ternary-spgemm_amd/<dir>/libternary_spgemm.so, a variant build).
TAG=${1:-x}; shift || true
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  unset TSG_KERNEL TSG_LIB
  case "$v" in
    default) ;;
    lib:*) export TSG_LIB=ternary-spgemm_amd/${v#lib:}/libternary_spgemm.so ;;
    *) export TSG_KERNEL=$v ;;
  esac
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-rows 0 > gpurun_out/bench_${TAG}_${v//[:\/]/_}.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python - gpurun_out/bench_${TAG}_${v//[:\/]/_}.log <<'P'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "value", round(d["value"],1), "kernel_ms", d["roofline"].get("kernel_ms"), "lds_frac", d["roofline"]["lds"]["frac"])
P
done
