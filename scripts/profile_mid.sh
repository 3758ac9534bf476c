#!/bin/bash
# GPU box: PMC passes of the configs[1] shape (M = 512, jit width 8) through
# scripts/configs.py, one rocprofv3 --pmc pass per counter set (kernel trace
# never combined), to see what bounds the narrow-width kernel.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/prof_mid_$TAG
mkdir -p $OUT
SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE;\
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE;\
SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH GRBM_GUI_ACTIVE"
IFS=';' read -ra S <<< "$SETS"
i=0
for CTR in "${S[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 scripts/configs.py --only "configs[1]" --steps 2 > $OUT/pmc${i}.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc ($CTR)"
  if [ $rc -ne 0 ]; then tail -3 $OUT/pmc${i}.log; [ $rc -ge 124 ] && exit $rc; fi
done
python3 scripts/pmc_summary.py $OUT > $OUT/summary.json && echo summary ok
