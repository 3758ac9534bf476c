#!/bin/bash
# GPU box: PMC passes over the M = 1 producer/consumer walk (K = 4096,
# N = 16384), one counter set per rocprofv3 run (kernel-trace only).
# Usage: pc_pmc.sh <out dir>
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pc_pmc}
mkdir -p $OUT
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
      "FETCH_SIZE"
      "SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_IFETCH")
i=0
for CTR in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 scripts/small_m_sweep.py --K 4096 --N 16384 --M 1 --reps 5 > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc ($CTR)"
  [ $rc -ne 0 ] && { tail -3 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit $rc; }
done
python3 - $OUT <<'P'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ell_pc_kernel" in r["Kernel_Name"]:
            agg[(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(list)
for (c, d), v in agg.items():
    per[c].append(sum(v))
for c in sorted(per):
    vals = per[c]
    print(c, round(sum(vals) / len(vals), 1), "over", len(vals), "dispatches")
P
