#!/bin/bash
# GPU box: jit tile-mapping variants (TSG_JIT_GN / TSG_JIT_GM built into
# ternary-spgemm_amd/<dir>) on mid-M shapes, two interleaved repeats.
# Usage: map_mid_ab.sh <out> "<shape filters>" <dir|default>...
set -o pipefail
export TMPDIR=/tmp
OUT=$1; SHAPES=$2; shift 2
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for rep in 1 2; do
  for sh in $SHAPES; do
    for v in "$@"; do
      unset TSG_LIB; [ "$v" = default ] || export TSG_LIB=ternary-spgemm_amd/$v/libternary_spgemm.so
      line=$(timeout -k 10 150 python scripts/configs.py --only "${sh//_/ }" --steps 20 2>/dev/null | tail -1) || { echo "$v $sh failed"; exit 1; }
      echo "$rep $v $line" >> "$OUT"
    done
  done
  echo "rep $rep done"
done
