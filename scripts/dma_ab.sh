#!/bin/bash
# GPU box: kernel time of the weight-compiled kernel under LDS-DMA issue variants
# (TSG_JIT_DMA="spread,m0k", tsg_jit.cpp) on the BASELINE shapes and the sparse
# end; 2 alternating reps; parity of the default first.
# Usage: scripts/dma_ab.sh <out> [variants...]
set -o pipefail
OUT=${1:-gpurun_out/dma_ab.txt}; shift
VARS=${@:-"0,0 0,1 0.5,1 0.75,1 0.33,1"}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dma_ab_parity.log 2>&1
rc=$?; echo "parity rc=$rc: $(tail -1 gpurun_out/dma_ab_parity.log)"; [ $rc -eq 0 ] || { tail -20 gpurun_out/dma_ab_parity.log; exit $rc; }
SH="--shape 512,4096,4096,4 --shape 4096,4096,16384,4 --shape 4096,4096,16384,16 --shape 4096,4096,16384,8 --shape 256,4096,16384,4 --shape 1024,4096,16384,4"
for rep in 1 2; do
  for v in $VARS; do
    TSG_JIT_DMA=$v timeout -k 10 170 python scripts/configs.py $SH --steps 20 2>/dev/null | sed "s/^/dma=$v rep=$rep /" >> "$OUT" || { echo "variant $v failed"; exit 1; }
    echo "rep $rep dma=$v done"
  done
done
