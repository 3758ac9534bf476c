#!/bin/bash
# GPU box: rocprofv3 counters (separate passes, kernel-trace only) of one
# scripts/rows64_ab.py run; per-dispatch means per kernel in
# gpurun_out/pmc_<tag>/summary.json.
#   bash scripts/pmc_shape.sh <tag> <rows64_ab.py arguments>
# e.g. the sparse end: pmc_shape.sh s16 --xint --modes jit64 --s 16 --M 4096 --reps 3
#      small M:        pmc_shape.sh m64 --M 64 --reps 5
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for CTR in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ${PMC_EXTRA:+"$PMC_EXTRA"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTR --output-format csv -d $OUT/pmc$i -o run -- \
      python3 scripts/rows64_ab.py "$@" > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit $rc; fi
done
python3 - $OUT "$*" <<'P'
import csv, glob, json, os, sys, collections
d, args = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "tsg" not in k or "probe" in k:
            continue
        acc[k][(r["Counter_Name"], r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
out = {"args": args, "note": "per-dispatch means; FETCH_SIZE x2 (gfx950 correction, MI355X_MICROARCH.md); "
                             "SQ_*CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* in quad-cycles"}
for k, v in acc.items():
    per = collections.defaultdict(list)
    for (c, _), xs in v.items():
        per[c].append(sum(xs))  # sum over XCD/instance rows of one dispatch
    m = {c: sum(xs) / len(xs) for c, xs in per.items()}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
    o = {"counters": m}
    if "SQ_IFETCH" in m:
        o["ifetch_bytes"] = 32 * m["SQ_IFETCH"]
    if cyc and "SQC_ICACHE_BUSY_CYCLES" in m:
        o["sqc_icache_busy_frac"] = m["SQC_ICACHE_BUSY_CYCLES"] / (128 * cyc)
    if "FETCH_SIZE" in m:
        o["hbm_read_bytes"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        o["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                o[c.lower() + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
    out[k] = o
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
for k in out:
    if isinstance(out[k], dict):
        print(k, {x: (round(y) if isinstance(y, float) and y > 10 else round(y, 4) if isinstance(y, float) else y)
                  for x, y in out[k].items() if x != "counters"})
P
