#!/bin/bash
# GPU box, round 4: configs[4] shard by shard, fractional-X full-Y, the
# reference's own correctness loop at configs[0]/[1], then the 8-rank gloo
# launcher rehearsal of configs[4].  Usage: scripts/r04_check.sh <tag> [tests...]
set -o pipefail
TAG=${1:-r04a}
shift
TESTS=${*:-tests/test_gpu_configs4.py tests/test_gpu_full_y.py tests/test_gpu_parity.py::test_plugin_against_reference_headers}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/pytest_$TAG.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_$TAG.log; exit $rc; }
TSG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 8 --M 512 --steps 3 > gpurun_out/bench_gloo8_$TAG.jsonl 2> gpurun_out/bench_gloo8_$TAG.err
rc=$?; echo "gloo8 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_gloo8_$TAG.err; exit $rc; }
tail -1 gpurun_out/bench_gloo8_$TAG.jsonl | cut -c1-600
