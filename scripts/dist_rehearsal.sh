#!/bin/bash
# GPU box (1 GPU): rehearses bench.py's multi-rank path -- per-rank column
# draws, barrier + max-over-ranks timing, nnz all-reduce, the all-gather of
# the Y blocks (alone and pipelined with the compute by M chunks), the JSON
# line -- with 2 ranks on cuda:0 over gloo (RCCL refuses two ranks on one
# device; gloo stages the device tensors through host memory), in weak and in
# strong mode.  The driver's real N-GPU runs use RCCL, one rank per GPU.
# NPROC=4 (default 2) rehearses 4 ranks; MODES="weak" limits the modes.
set -o pipefail
export TMPDIR=/tmp TSG_BENCH_BACKEND=gloo
mkdir -p gpurun_out
NPROC=${NPROC:-2}
for mode in ${MODES:-weak strong}; do
  extra=""; [ $mode = strong ] && extra="--strong"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NPROC --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus $NPROC --steps 5 --warmup 2 $extra > gpurun_out/dist_rehearsal_${mode}_$NPROC.log 2>&1
  rc=$?; echo "rehearsal $mode rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/dist_rehearsal_${mode}_$NPROC.log; exit $rc; }
  python3 - gpurun_out/dist_rehearsal_${mode}_$NPROC.log <<'P'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[1], "scaling", d["scaling"], "value", d["value"], "allgather_ms", d["allgather_ms"],
      "with_allgather", d["with_allgather"], "workload", d["config"]["workload"])
assert d["allgather_ms"] is not None and d["with_allgather"]["columns_match_compute_only"]
P
done
