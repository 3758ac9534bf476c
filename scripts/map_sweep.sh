#!/bin/bash
# GPU box: jit kernel time over M for library variants (tile-mapping knobs built
# into ternary-spgemm_amd/<dir>), interleaved.  Usage: map_sweep.sh <tag> "<Ms>" <dir|default>...
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; MS=$2; shift 2
OUT=gpurun_out/map_sweep_$TAG.txt; : > $OUT
for M in $MS; do
  for v in "$@"; do
    unset TSG_LIB; [ "$v" = default ] || export TSG_LIB=ternary-spgemm_amd/$v/libternary_spgemm.so
    timeout -k 10 120 python bench.py --M $M --steps 20 --warmup 3 --cpu-rows 0 > /tmp/ms.log 2>&1 || { echo "$v M=$M failed"; tail -3 /tmp/ms.log; exit 1; }
    python3 - $M $v >> $OUT <<'P'
import json, sys
d = json.loads([l for l in open("/tmp/ms.log") if l.startswith("{")][-1])
print("M", sys.argv[1], sys.argv[2], "kernel_ms", d["roofline"]["kernel_ms"], "valu", d["roofline"]["binding"]["frac"])
P
    tail -1 $OUT
  done
done
