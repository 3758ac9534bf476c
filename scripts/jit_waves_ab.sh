#!/bin/bash
# GPU box: 4-wave workgroups for the narrow jit widths (TSG_JIT_WAVES=4) vs the
# 8-wave default: parity suite with the 4-wave variants, then every width on
# mid-M shapes (scripts/configs.py --all-widths).
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
TSG_JIT_WAVES=4 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_4w.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_4w.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_4w.log
out=gpurun_out/${TAG}_waves_ab.txt
: > $out
for w in 8 4; do
  for sh in "configs[1]" "sweep M=256" "sweep M=1024"; do
    echo "# waves=$w $sh" >> $out
    TSG_JIT_WAVES=$w timeout -k 10 200 python scripts/configs.py --only "$sh" --all-widths >> $out 2>&1 || exit 1
  done
done
