#!/bin/bash
# GPU box, round 6's final evidence, part 1: the GPU suite, smoke(), the
# default bench line, rocprofv3 --kernel-trace --stats of the exact default
# bench command and separate PMC passes of it (scripts/profile_gpu.sh),
# summarised with the call plan (scripts/make_profile_summary.py).
#   bash scripts/final6.sh <tag>
set -o pipefail
TAG=${1:?tag}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "gpu suite rc=$rc: $(tail -1 gpurun_out/pytest_$TAG.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_$TAG.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/smoke_$TAG.log; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.jsonl 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
tail -1 gpurun_out/bench_$TAG.jsonl | cut -c1-300
bash scripts/profile_gpu.sh $TAG || exit $?
python3 scripts/make_profile_summary.py gpurun_out/prof_$TAG gpurun_out/summary_$TAG 4096 4096 16384 4 > /dev/null && echo summary ok
