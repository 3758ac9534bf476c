#!/bin/bash
# GPU box: small-M walk (forced) vs the jit kernel on the reference cases
# where the jit kernel has few column tiles (plots/run_benchmark.py:8-33).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${1:-x}_ell_vs_jit_ref.jsonl
: > $out
run() { timeout -k 10 200 python scripts/small_m_sweep.py --K $1 --N $2 --s $3 --M $4 >> $out 2>&1 || exit 1; }
run 2048 512 4 128,256,512,1000
run 1024 1024 4 128,256,1024
run 4096 1024 4 256,1000,4000
run 4096 16384 4 96,128,256
run 2048 8192 4 64,128
run 16384 1024 4 128,1024
