#!/bin/bash
# GPU box: parity tests then a short bench.  Usage: scripts/gpu_check.sh <tag> [bench args]
TAG=${1:-x}; shift || true
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-rows 0 "$@" > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
exit $rc
