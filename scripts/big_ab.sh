#!/bin/bash
# GPU box: the reference's largest case (64000, 16384, 4096) under tile-map,
# code-touch, DMA cache-policy and DMA-issue variants (kernel ms, configs.py;
# results checked bit for bit on sampled rows).  Round 3: the no-DMA diagnostic
# runs this shape at 0.77 of the VALU peak against 0.54 with the DMA
# (profiles/r03_big_diag.txt), so the variants target the X^T staging.
# Usage: scripts/big_ab.sh <out> [shapes...]
set -o pipefail
OUT=${1:-gpurun_out/big_ab.txt}; shift
SHAPES=${*:-64000,16384,4096,4 64000,16384,4096,8}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
VARS=${BIG_AB_VARS:-"default TSG_JIT_TOUCH=1,0 TSG_JIT_TOUCH=1,0:TSG_JIT_CP=20000,0 TSG_JIT_GN=2:TSG_JIT_GM=16 TSG_JIT_GN=2:TSG_JIT_GM=16:TSG_JIT_TOUCH=1,0 TSG_JIT_GN=8:TSG_JIT_GM=4 TSG_JIT_GN=4:TSG_JIT_GM=8:TSG_JIT_TOUCH=1,0 TSG_JIT_DMA=0,1,1 TSG_JIT_DMA=0.5,1,2:TSG_JIT_TOUCH=1,0"}
args=""; for sh in $SHAPES; do args="$args --shape $sh"; done
for v in $VARS; do
  envs=""; [ "$v" = default ] || envs="${v//:/ }"
  env $envs timeout -k 10 200 python scripts/configs.py $args --steps 3 2>/dev/null | sed "s/^/[$v] /" >> "$OUT"
  rc=$?; [ $rc -eq 0 ] || { echo "variant $v failed rc=$rc"; exit $rc; }
  echo "variant $v done: $(tail -n $(echo $SHAPES | wc -w) "$OUT" | grep -o '"kernel_ms": [0-9.]*' | tr '\n' ' ')"
done
