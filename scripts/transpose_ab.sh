#!/bin/bash
# GPU box: the k-pair X^T staging kernels A/B (LDS-free register transpose, the
# default, vs TSG_TRANSPOSE=lds): bench step time interleaved, then the
# rocprofv3 kernel-trace stats of each.  Usage: transpose_ab.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
OUT=gpurun_out/transpose_ab_$TAG.txt; mkdir -p gpurun_out; : > $OUT
for rep in 1 2 3; do
  for v in default lds; do
    unset TSG_TRANSPOSE; [ $v = default ] || export TSG_TRANSPOSE=$v
    timeout -k 10 120 python bench.py --steps 40 --cpu-rows 0 > /tmp/tab.log 2>&1 || { echo "$v failed"; tail -3 /tmp/tab.log; exit 1; }
    python3 - $rep $v >> $OUT <<'P'
import json, sys
d = json.loads([l for l in open("/tmp/tab.log") if l.startswith("{")][-1])
print(sys.argv[1], sys.argv[2], "ms_per_step", d["ms_per_step"], "kernel_ms", d["roofline"]["kernel_ms"], "GFLOP/s", d["value"])
P
  done
done
cat $OUT
for v in default lds; do
  unset TSG_TRANSPOSE; [ $v = default ] || export TSG_TRANSPOSE=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tprof_${TAG}_$v -o run -- \
      python3 bench.py --steps 40 --cpu-rows 0 > gpurun_out/tprof_${TAG}_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
  grep -h transpose gpurun_out/tprof_${TAG}_$v/*/run_kernel_stats.csv gpurun_out/tprof_${TAG}_$v/run_kernel_stats.csv 2>/dev/null | cut -c1-160
done
