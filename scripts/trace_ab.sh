#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of the default bench command under
# environment variants, alternating (the average over ~259 launches is the
# comparison).  Usage: trace_ab.sh <out> <reps> <variant>...   (variant:
# "default" or VAR=value[,VAR=value])
set -o pipefail
export TMPDIR=/tmp
OUT=$1; REPS=$2; shift 2
mkdir -p gpurun_out; : > "$OUT"
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    envs=(); [ "$v" = default ] || IFS=',' read -ra envs <<< "$v"
    d=gpurun_out/tab_${rep}_${v//[=,]/_}
    env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
        python3 bench.py --cpu-rows 0 > $d.log 2>&1 || { echo "$v failed"; tail -3 $d.log; exit 1; }
    avg=$(grep -h '"tsg_jit_kernel"' $(find $d -name 'run_kernel_stats.csv') | cut -d, -f4)
    step=$(grep '^{' $d.log | tail -1 | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "$rep $v jit_avg_ns $avg ms_per_step $step" | tee -a "$OUT"
  done
done
