#!/bin/bash
# GPU box: jit tile-mapping variants through bench.py on several (M, K, N),
# interleaved.  variant: "default", a library dir under ternary-spgemm_amd
# (TSG_LIB), or VAR=value[,VAR=value] (e.g. TSG_JIT_GN=2,TSG_JIT_GM=16).
# Usage: map_bench_ab.sh <out> "<M,K,N> ..." <variant>...
set -o pipefail
export TMPDIR=/tmp
OUT=$1; SHAPES=$2; shift 2
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2 3; do
  for sh in $SHAPES; do
    IFS=, read -r M K N <<< "$sh"
    for v in "$@"; do
      envs=()
      if [ "$v" != default ]; then
        if [[ "$v" == *=* ]]; then IFS=',' read -ra envs <<< "$v"; else envs=("TSG_LIB=ternary-spgemm_amd/$v/libternary_spgemm.so"); fi
      fi
      env "${envs[@]}" timeout -k 10 200 python bench.py --M $M --K $K --N $N --steps 10 --warmup 2 --cpu-rows 0 > /tmp/mb.log 2>&1 || { echo "$v $sh failed"; tail -3 /tmp/mb.log; exit 1; }
      python3 - $rep $v $sh >> "$OUT" <<'P'
import json, sys
d = json.loads([l for l in open("/tmp/mb.log") if l.startswith("{")][-1])
print(sys.argv[1], sys.argv[2], sys.argv[3], "kernel_ms", d["roofline"]["kernel_ms"], "valu", d["roofline"]["binding"]["frac"], "ms_step", d["ms_per_step"])
P
    done
  done
  echo "rep $rep done"
done
