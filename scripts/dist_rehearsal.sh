#!/bin/bash
# GPU box (1 GPU): rehearses bench.py's multi-rank path -- column shards,
# barrier + max-over-ranks timing, nnz all-reduce, the JSON line -- with 2
# ranks on cuda:0 over gloo (RCCL refuses two ranks on one device).  The
# driver's real N-GPU runs use RCCL, one rank per GPU.
set -o pipefail
export TMPDIR=/tmp TSG_BENCH_BACKEND=gloo
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist_rehearsal.log 2>&1
rc=$?; echo "rehearsal rc=$rc"; tail -3 gpurun_out/dist_rehearsal.log; exit $rc
