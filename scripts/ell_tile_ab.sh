#!/bin/bash
# GPU box: small-M kernel tile (TSG_ELL_VARIANT: 2 = 8-row, 3 = 16-row, 4 =
# 32-row M tiles; larger tiles re-read the index image fewer times but need
# K in several LDS chunks) and lanes per column (TSG_ELL_LG) at M = 16..64,
# configs[2]'s K, N.  JSON lines of scripts/small_m_sweep.py (ell = forced
# small-M kernel, jit = weight-compiled), bit-identical between the two.
# Usage: scripts/ell_tile_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/ell_tile_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for v in "" "TSG_ELL_VARIANT=2" "TSG_ELL_VARIANT=3" "TSG_ELL_VARIANT=4" "TSG_ELL_VARIANT=3 TSG_ELL_LG=16" "TSG_ELL_VARIANT=4 TSG_ELL_LG=16" "TSG_ELL_VARIANT=2 TSG_ELL_LG=8" "TSG_ELL_VARIANT=2 TSG_ELL_LG=2"; do
  env $v timeout -k 10 170 python scripts/small_m_sweep.py --M 16,32,48,64 --reps 20 2>/dev/null | sed "s/^/[$v] /" >> "$OUT" || { echo "variant [$v] failed"; exit 1; }
  echo "variant [$v] done"
done
