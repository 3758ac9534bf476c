#!/bin/bash
# Runs on the GPU box (via gpurun): kernel-trace stats + PMC passes of bench.py.
# Usage: [PMC_SETS="A B;C D"] [NO_TRACE=1] [NO_PMC=1] scripts/profile_gpu.sh <tag> [bench args...]
# Each ';'-separated set is one rocprofv3 --pmc pass (kernel-trace only, never
# combined with sys/runtime traces).
set -u
TAG=${1:-r01}; shift || true
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
DEFAULT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVE_CYCLES;SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS;FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE GRBM_COUNT;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES"
IFS=';' read -ra SETS <<< "${PMC_SETS:-$DEFAULT}"
if [ -z "${NO_TRACE:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
      python3 bench.py --steps 20 --warmup 3 --cpu-rows 0 "$@" > $OUT/trace_bench.log 2>&1 || { echo "trace failed rc=$?"; exit 1; }
fi
[ -n "${NO_PMC:-}" ] && { echo profile done; exit 0; }
i=0
for CTR in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-rows 0 "$@" > $OUT/pmc${i}_bench.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i ($CTR) failed rc=$rc"; [ $rc -ge 124 ] && exit $rc; fi
done
echo profile done
