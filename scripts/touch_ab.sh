#!/bin/bash
# GPU box: code-touch thinning (TSG_JIT_TMASK: only M tiles with (mt & mask) == 0
# spread their touches over the stream's lines; the others load one line),
# no touches (TSG_JIT_TOUCH=1,0) and nt DMA (TSG_JIT_CP=20000,0): kernel ms
# (configs.py, bit-checked rows) on the BASELINE configs, the sparse end, and the
# long-K reference shapes; two interleaved repetitions.
# Usage: scripts/touch_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/touch_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
MID="--shape 4096,4096,16384,4 --shape 512,4096,4096,4 --shape 4096,4096,16384,16 --shape 4096,4096,16384,8 --shape 16000,8192,2048,4 --shape 8192,16384,4096,4"
for rep in 1 2; do
  for v in default TSG_JIT_TMASK=1 TSG_JIT_TMASK=3 TSG_JIT_TMASK=7 TSG_JIT_TMASK=31 TSG_JIT_TOUCH=1,0; do
    envs=""; [ "$v" = default ] || envs="${v//:/ }"
    env $envs timeout -k 10 200 python scripts/configs.py $MID --steps 10 2>/dev/null | sed "s/^/[$v] rep=$rep /" >> "$OUT"
    rc=$?; [ $rc -eq 0 ] || { echo "variant $v failed rc=$rc"; exit $rc; }
    echo "rep $rep $v: $(tail -n 6 "$OUT" | grep -o '"kernel_ms": [0-9.]*' | cut -d' ' -f2 | tr '\n' ' ')"
  done
done
for v in default TSG_JIT_TMASK=7 TSG_JIT_TMASK=31 TSG_JIT_TMASK=7:TSG_JIT_CP=20000,0 TSG_JIT_TOUCH=1,0:TSG_JIT_CP=20000,0; do
  envs=""; [ "$v" = default ] || envs="${v//:/ }"
  env $envs timeout -k 10 200 python scripts/configs.py --shape 64000,16384,4096,4 --steps 3 2>/dev/null | sed "s/^/[$v] big /" >> "$OUT"
  rc=$?; [ $rc -eq 0 ] || { echo "big variant $v failed rc=$rc"; exit $rc; }
  echo "big $v: $(tail -n 1 "$OUT" | grep -o '"kernel_ms": [0-9.]*')"
done
