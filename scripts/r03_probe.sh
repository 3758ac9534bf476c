#!/bin/bash
# TSG_JIT_DIAG code variants exist only in the diagnostic build (make -C ternary-spgemm_amd diag)
export TSG_LIB=${TSG_LIB:-ternary-spgemm_amd/lib/libternary_spgemm_diag.so}
# GPU box, round 3 probe: LDS-DMA offset semantics micro-test, the launcher's
# RCCL failure path on a 1-GPU box, kernel-time diagnostics (TSG_JIT_DIAG code
# variants, results WRONG) at the sparse end (configs[3] s=16, s=8) and at
# configs[1], then PMC passes of the s=16 bench workload.
# Usage: scripts/r03_probe.sh <tag>
set -o pipefail
TAG=${1:-r03p}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/glds_offset_micro.bin > gpurun_out/glds_offset_$TAG.txt 2>&1
rc=$?; cat gpurun_out/glds_offset_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --gpus 2 --steps 2 --cpu-rows 0 > gpurun_out/bench_rccl2_$TAG.jsonl 2> gpurun_out/bench_rccl2_$TAG.err
rc=$?; echo "--gpus 2 over RCCL on this 1-GPU box rc=$rc (expected 3)"; tail -2 gpurun_out/bench_rccl2_$TAG.err
{ [ $rc -eq 124 ] || [ $rc -eq 137 ]; } && exit 1
OUT=gpurun_out/diag_$TAG.txt; : > $OUT
export TSG_KERNEL=jit
for d in "" nobar nodma notouch nolgkm noreads nobar,nodma; do
  for sh in "4096,4096,16384,16" "4096,4096,16384,8" "512,4096,4096,4"; do
    line=$(TSG_JIT_DIAG=$d timeout -k 10 150 python scripts/configs.py --shape $sh --steps 10 2>/dev/null | tail -1) || { echo "diag=[$d] $sh failed"; exit 1; }
    echo "diag=[$d] $line" >> $OUT
  done
  echo "diag=[$d] done"
done
unset TSG_KERNEL
PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT;\
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE;\
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE;\
SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE;\
FETCH_SIZE;WRITE_SIZE" NO_TRACE=1 bash scripts/profile_gpu.sh s16_$TAG --s 16 || exit $?
python3 scripts/pmc_summary.py gpurun_out/prof_s16_$TAG > gpurun_out/prof_s16_$TAG/summary.json && echo summary ok
