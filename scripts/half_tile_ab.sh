#!/bin/bash
# GPU box: M <= 64 on the weight-compiled kernel -- the half (64-row) tile vs
# the 128-row tile (TSG_JIT_HALF=0) vs the small-M walk, at configs[2]'s K, N
# and smaller N (scripts/small_m_sweep.py JSON lines: ell = small-M walk, jit =
# weight-compiled, bit-identical between them); GPU parity of the half tile
# first.  Usage: scripts/half_tile_ab.sh <out>
set -o pipefail
OUT=${1:-gpurun_out/half_tile_ab.txt}
export TMPDIR=/tmp
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_small_m.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/half_parity.log 2>&1
rc=$?; echo "parity rc=$rc: $(tail -1 gpurun_out/half_parity.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/half_parity.log; exit $rc; }
for half in 1 0; do
  for shape in "--K 4096 --N 16384" "--K 4096 --N 4096" "--K 16384 --N 16384" "--K 1024 --N 4096"; do
    TSG_JIT_HALF=$half timeout -k 10 170 python scripts/small_m_sweep.py $shape --M 8,16,24,32,40,48,56,64,96 --reps 20 2>/dev/null | sed "s/^/half=$half /" >> "$OUT" || { echo "half=$half $shape failed"; exit 1; }
    echo "half=$half $shape done"
  done
done
