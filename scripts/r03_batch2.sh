#!/bin/bash
# GPU box: (1) DMA spread 0 vs 0.5 on shapes whose X^T does not fit the
# Infinity Cache or that regressed in r03b; (2) small-M tile A/B; (3) PMC of
# the reference's largest shape.  Usage: scripts/r03_batch2.sh <tag>
set -o pipefail
TAG=${1:-r03c}
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/spread_hbm_$TAG.txt
for rep in 1 2; do
  for v in 0,1 0.5,1 0.25,1; do
    TSG_JIT_DMA=$v timeout -k 10 170 python scripts/configs.py --shape 16000,8192,2048,8 --shape 16000,8192,2048,16 --shape 16000,8192,2048,4 --shape 1024,4096,1024,4 --shape 1024,16384,1024,4 --shape 256,4096,16384,16 --steps 20 2>/dev/null | sed "s/^/dma=$v rep=$rep /" >> gpurun_out/spread_hbm_$TAG.txt || { echo "spread $v failed"; exit 1; }
  done
  echo "spread rep $rep done"
done
for v in 0,1 0.5,1; do
  TSG_JIT_DMA=$v timeout -k 10 170 python scripts/configs.py --shape 64000,16384,4096,8 --shape 64000,16384,4096,4 --steps 4 2>/dev/null | sed "s/^/dma=$v rep=1 /" >> gpurun_out/spread_hbm_$TAG.txt || { echo "big spread $v failed"; exit 1; }
done
echo "big spread done"
bash scripts/ell_tile_ab.sh gpurun_out/ell_tile_ab_$TAG.txt || exit 1
bash scripts/big_pmc.sh big_$TAG 64000,16384,4096,4 || exit 1
