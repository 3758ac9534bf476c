#!/bin/bash
# GPU box: parity tests, the default bench line (with the CPU baseline), then a
# rocprofv3 kernel-trace/stats pass and PMC passes, summarised into gpurun_out/.
# Usage: scripts/round_check.sh <tag>
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_$TAG.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_$TAG.log; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.jsonl 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
tail -1 gpurun_out/bench_$TAG.jsonl | cut -c1-400
bash scripts/profile_gpu.sh $TAG || exit $?
python3 scripts/make_profile_summary.py gpurun_out/prof_$TAG gpurun_out/summary_$TAG 4096 4096 16384 4 > /dev/null && echo summary ok
