set -o pipefail
mkdir -p gpurun_out
bash scripts/jit_ab.sh lib:24,24,0 lib_g2:12,12,0 > gpurun_out/ab_halfreads.txt 2>&1 &&
TSG_JIT_DIAG=halfreads bash scripts/jit_ab.sh lib:24,24,0 lib_g2:12,12,0 >> gpurun_out/ab_halfreads.txt 2>&1 &&
timeout -k 10 300 python scripts/sweep.py --steps 10 > gpurun_out/sweep_blocked.jsonl 2> gpurun_out/sweep_blocked.err &&
timeout -k 10 300 python bench.py > gpurun_out/bench_e2e.jsonl 2> gpurun_out/bench_e2e.err
