#!/bin/bash
# GPU box: the producer/consumer small-M walk (tsg_tcsc_ell_pc_kernel, M <= 4)
# against the plain one (TSG_ELL_PC=0), on configs[2]'s and configs[0]'s K, N.
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
out=gpurun_out/${TAG}_ell_pc.txt
: > $out
for pc in 1 0; do
  for shape in "--K 4096 --N 16384" "--K 1024 --N 4096" "--K 4096 --N 4096" "--K 16384 --N 16384"; do
    echo "# TSG_ELL_PC=$pc $shape" >> $out
    TSG_ELL_PC=$pc timeout -k 10 240 python scripts/small_m_sweep.py $shape --M 1,2,3,4 >> $out 2>&1 || { tail -5 $out; exit 1; }
  done
done
python3 - $out <<'P'
import json, sys
tag = ""
for l in open(sys.argv[1]):
    if l.startswith("#"):
        tag = l[1:].strip()
    elif l.startswith("{"):
        d = json.loads(l)
        print(tag, "M", d["M"], "ell", d["ell"]["kernel_ms"], "hbm", d["ell"]["hbm_frac_on_tcsc_bytes"],
              "| jit", d["jit"]["kernel_ms"], d["bit_identical"], d["auto"])
P
