#!/bin/bash
# GPU box, round 3: the new multi-GPU / host-pipeline tests first, the whole GPU
# suite, the default bench line, then the launcher checks (a 2-rank gloo
# rehearsal on one GPU must print n_gpus 2; --gpus 2 over RCCL on a 1-GPU box
# must fail loudly).  Every GPU step has its own time limit; stops at the first
# failure.  Usage: scripts/r03_check.sh <tag> [quick]
set -o pipefail
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_dist.py tests/test_gpu_streams.py > gpurun_out/pytest_new_$TAG.log 2>&1
rc=$?; echo "new tests rc=$rc: $(tail -1 gpurun_out/pytest_new_$TAG.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_new_$TAG.log; exit $rc; }
if [ "$2" != quick ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "gpu suite rc=$rc: $(tail -1 gpurun_out/pytest_$TAG.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_$TAG.log; exit $rc; }
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.jsonl 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$TAG.err; exit $rc; }
tail -1 gpurun_out/bench_$TAG.jsonl | cut -c1-300
python - gpurun_out/bench_$TAG.jsonl <<'P'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("e2e_host_pointers", d["e2e_host_pointers"])
P
TSG_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --cpu-rows 0 > gpurun_out/bench_gloo2_$TAG.jsonl 2> gpurun_out/bench_gloo2_$TAG.err
rc=$?; echo "gloo 2-rank rehearsal rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_gloo2_$TAG.err; exit $rc; }
python - gpurun_out/bench_gloo2_$TAG.jsonl <<'P'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("n_gpus", d["n_gpus"], "allgather_ms", d["allgather_ms"], "with_allgather", d["with_allgather"])
assert d["n_gpus"] == 2 and d["allgather_ms"] is not None
P
[ $? -eq 0 ] || exit 1
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --cpu-rows 0 > gpurun_out/bench_rccl2_$TAG.jsonl 2> gpurun_out/bench_rccl2_$TAG.err
rc=$?; echo "--gpus 2 over RCCL on this box rc=$rc (expected non-zero on a 1-GPU box)"; tail -3 gpurun_out/bench_rccl2_$TAG.err
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 1
[ -s gpurun_out/bench_rccl2_$TAG.jsonl ] && { echo "unexpected result line"; exit 1; }
exit 0
