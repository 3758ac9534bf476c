#!/bin/bash
# GPU box: kernel-time A/B of library builds or environment knobs on the shapes
# of scripts/configs.py, two interleaved repeats.
#   variant: "default", a library dir under ternary-spgemm_amd (TSG_LIB), or
#   VAR=value[,VAR=value] (environment knobs, e.g. TSG_JIT_HELPERS=0)
# Usage: map_mid_ab.sh <out> "<shape filters, '_' for ' '>" <variant>...
set -o pipefail
export TMPDIR=/tmp
OUT=$1; SHAPES=$2; shift 2
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for sh in $SHAPES; do
    for v in "$@"; do
      envs=()
      if [ "$v" != default ]; then
        if [[ "$v" == *=* ]]; then IFS=',' read -ra envs <<< "$v"; else envs=("TSG_LIB=ternary-spgemm_amd/$v/libternary_spgemm.so"); fi
      fi
      line=$(env "${envs[@]}" timeout -k 10 150 python scripts/configs.py --only "${sh//_/ }" --steps 20 2>/dev/null | tail -1) || { echo "$v $sh failed"; exit 1; }
      echo "$rep $v $line" >> "$OUT"
    done
  done
  echo "rep $rep done"
done
