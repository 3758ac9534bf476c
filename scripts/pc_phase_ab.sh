#!/bin/bash
# GPU box: the M = 1 producer/consumer walk's phase length (TSG_ELL_PC_E = 16,
# 32, 64 entries of every chain per barrier): small-M parity tests per E, then
# kernel time at M = 1 and 2 on three K x N shapes, interleaved.  (K = 34812 and
# 34816 are deselected: their kernel choice, pinned by the test, depends on the ring size.)
# Usage: pc_phase_ab.sh <out>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pc_phase_ab.txt}
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
for E in 16 64; do
  TSG_ELL_PC_E=$E timeout -k 10 200 python -u -m pytest tests/test_gpu_small_m.py -x -q -k "not 3481" --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_pc$E.log 2>&1 || { echo "E=$E tests failed"; tail -20 gpurun_out/pytest_pc$E.log; exit 1; }
  echo "E=$E $(tail -1 gpurun_out/pytest_pc$E.log)"
done
for rep in 1 2; do
  for shape in "4096 16384" "4096 4096" "16384 16384"; do
    set -- $shape
    for E in 32 16 64; do
      line=$(TSG_ELL_PC_E=$E timeout -k 10 120 python scripts/small_m_sweep.py --K $1 --N $2 --M 1,2 2>/dev/null | tr '\n' ' ') || { echo "E=$E $shape failed"; exit 1; }
      echo "$rep E=$E K=$1 N=$2 $line" >> "$OUT"
    done
  done
  echo "rep $rep done"
done
