#!/bin/bash
# GPU box: small-M parity (bitwise) with the current library, then the M = 1/2/4
# sweep on four K x N shapes, current vs a previous build (ternary-spgemm_amd/lib_old,
# TSG_LIB), interleaved.  Usage: pc_pipe_ab.sh <out>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pc_pipe_ab.txt}
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_small_m.py tests/test_gpu_special.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_pcpipe.log 2>&1 || { tail -25 gpurun_out/pytest_pcpipe.log; exit 1; }
tail -1 gpurun_out/pytest_pcpipe.log
for rep in 1 2; do
  for shape in "4096 16384" "4096 4096" "16384 16384" "1024 4096"; do
    set -- $shape
    for v in new old; do
      if [ $v = old ]; then export TSG_LIB=ternary-spgemm_amd/lib_old/libternary_spgemm.so; else unset TSG_LIB; fi
      timeout -k 10 120 python scripts/small_m_sweep.py --K $1 --N $2 --M 1,2,4 2>/dev/null | sed "s/^/$rep $v /" >> "$OUT" || { echo "$v $shape failed"; exit 1; }
    done
  done
  echo "rep $rep done"
done
