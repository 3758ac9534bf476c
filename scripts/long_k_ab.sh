#!/bin/bash
# GPU box: (1) code image without code touches and with non-temporal X^T DMA
# (TSG_JIT_TOUCH=1,0 TSG_JIT_CP=20000,0) on the long-K shapes whose calls run
# the 64-wide image; (2) code-touch thinning (TSG_JIT_TMASK) on the mid-M shapes
# that run the narrow 4-wave images.  Kernel ms (configs.py, bit-checked
# rows), two interleaved repetitions.  Usage: scripts/long_k_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/long_k_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
run() {  # tag envs shapes...
  local tag=$1 envs=$2; shift 2
  [ "$envs" = default ] && envs=""
  local args=""; for sh in "$@"; do args="$args --shape $sh"; done
  env $envs timeout -k 10 200 python scripts/configs.py $args --steps ${STEPS:-10} 2>/dev/null | sed "s/^/[$tag] /" >> "$OUT"
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag failed rc=$rc"; exit $rc; }
  echo "$tag: $(tail -n $# "$OUT" | grep -o '"kernel_ms": [0-9.]*' | cut -d' ' -f2 | tr '\n' ' ')"
}
for rep in 1 2; do
  for v in default TSG_JIT_TOUCH=1,0:TSG_JIT_CP=20000,0; do
    STEPS=3 run "$v rep=$rep" "${v//:/ }" 64000,16384,4096,2 64000,16384,4096,4
    STEPS=5 run "$v rep=$rep" "${v//:/ }" 8192,16384,4096,4 4096,16384,4096,4 16000,16384,4096,4 4096,16384,16384,4 16000,8192,2048,4 16000,8192,4096,4
  done
  for v in default TSG_JIT_TMASK=1 TSG_JIT_TMASK=3; do
    run "$v rep=$rep" "${v/default/}" 512,4096,4096,4 256,4096,16384,4 4000,4096,1024,4 1024,4096,1024,4 1024,16384,1024,4 256,16384,16384,4
  done
done
