#!/bin/bash
# GPU box: rocprofv3 counters of the small-M kernel at a few M (separate passes).
export TMPDIR=/tmp
OUT=gpurun_out/pmc_small_${1:-x}
mkdir -p $OUT
i=0
for CTR in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/p$i -o run -- \
      python3 scripts/small_m_sweep.py --M ${SMALL_M_LIST:-16,64} --reps 3 > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
python3 - $OUT <<'P'
import csv, glob, sys, collections
tot = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ell" in r["Kernel_Name"]:
            tot[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in tot.items():
    print(k)
    for c, xs in sorted(v.items()):
        print("   ", c, [round(x) for x in xs[:8]])
P
