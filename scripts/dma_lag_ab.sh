#!/bin/bash
# GPU box: LDS-DMA spread x lag (TSG_JIT_DMA="spread,m0k,lag", tsg_jit.cpp) on
# MALL-resident and far-memory X^T shapes; GPU parity of lag 2 first.
# Usage: scripts/dma_lag_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/dma_lag_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
TSG_JIT_DMA=0.5,1,2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dma_lag_parity.log 2>&1
rc=$?; echo "lag-2 parity rc=$rc: $(tail -1 gpurun_out/dma_lag_parity.log)"; [ $rc -eq 0 ] || { tail -20 gpurun_out/dma_lag_parity.log; exit $rc; }
VARS="0.5,1,1 0,1,1 0.5,1,2 0,1,2"
for rep in 1 2; do
  for v in $VARS; do
    TSG_JIT_DMA=$v timeout -k 10 170 python scripts/configs.py --shape 4096,4096,16384,4 --shape 4096,4096,16384,8 --shape 4096,4096,16384,16 --shape 512,4096,4096,4 --shape 16000,8192,2048,8 --shape 16000,8192,2048,4 --shape 1024,16384,1024,4 --shape 256,4096,16384,16 --steps 20 2>/dev/null | sed "s/^/dma=$v rep=$rep /" >> "$OUT" || { echo "variant $v failed"; exit 1; }
    echo "rep $rep dma=$v done"
  done
done
for v in $VARS; do
  TSG_JIT_DMA=$v timeout -k 10 170 python scripts/configs.py --shape 64000,16384,4096,4 --shape 64000,16384,4096,8 --steps 3 2>/dev/null | sed "s/^/dma=$v rep=1 /" >> "$OUT" || { echo "big variant $v failed"; exit 1; }
  echo "big dma=$v done"
done
