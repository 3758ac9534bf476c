#!/bin/bash
# GPU box: a batch of GPU tests (TESTS="..." pytest arguments; default: the
# files round 5 touched -- the image fallback, the reference's perf_test loop
# around the HIP comp_funcs, configs[4] shards with fractional X, the RCCL
# pipeline), smoke(), the default bench line and the 8-rank gloo rehearsal of
# the world > 1 line (compute + all-gather).
#   [TESTS="tests/x.py -k y"] bash scripts/check.sh <tag>
set -o pipefail
TAG=${1:-r05a}
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/ref_perf_$TAG.txt
TSG_REF_PERF_OUT=gpurun_out/ref_perf_$TAG.txt timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread \
    ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_configs4.py tests/test_gpu_dist.py} > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_$TAG.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_$TAG.log | head -20; tail -30 gpurun_out/pytest_$TAG.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/smoke_$TAG.log; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.jsonl 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
tail -1 gpurun_out/bench_$TAG.jsonl | cut -c1-300
TSG_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 8 --M 512 --steps 3 --timeout 350 \
    > gpurun_out/bench_gloo8_$TAG.jsonl 2> gpurun_out/bench_gloo8_$TAG.err
rc=$?; echo "gloo8 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_gloo8_$TAG.err; exit $rc; }
tail -1 gpurun_out/bench_gloo8_$TAG.jsonl | cut -c1-300
