#!/bin/bash
# GPU box: small-M kernel by M tile (TSG_ELL_VARIANT) and lanes per column
# (TSG_ELL_LG) -- diagnostic overrides of the automatic choices; the image
# depends on the M tile only -- on configs[2]'s K, N.  bit_identical compares
# the full Y against the jit kernel.
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
out=gpurun_out/${TAG}_ell_lg.txt
: > $out
run() {  # variant LG M-list
  echo "# TSG_ELL_VARIANT=$1 TSG_ELL_LG=$2" >> $out
  TSG_ELL_VARIANT=$1 TSG_ELL_LG=$2 timeout -k 10 240 python scripts/small_m_sweep.py --M $3 >> $out 2>&1 || { tail -5 $out; exit 1; }
}
echo "# default K=4096 N=16384" >> $out
timeout -k 10 240 python scripts/small_m_sweep.py --M 1,2,4,8,12,16,24,32,48,64,96,128 >> $out 2>&1 || { tail -5 $out; exit 1; }
echo "# default K=1024 N=4096 (configs[0] shape)" >> $out
timeout -k 10 240 python scripts/small_m_sweep.py --K 1024 --N 4096 --M 1,4,8,16,24,32,48,64 >> $out 2>&1 || { tail -5 $out; exit 1; }
echo "# TSG_ELL_VARIANT=2 K=1024 N=4096" >> $out
TSG_ELL_VARIANT=2 timeout -k 10 240 python scripts/small_m_sweep.py --K 1024 --N 4096 --M 16,32,64 >> $out 2>&1 || { tail -5 $out; exit 1; }
echo "# TSG_ELL_VARIANT=1 K=4096 N=16384" >> $out
TSG_ELL_VARIANT=1 timeout -k 10 240 python scripts/small_m_sweep.py --M 8,16 >> $out 2>&1 || { tail -5 $out; exit 1; }
python3 - $out <<'P'
import json, sys
tag = "default"
for l in open(sys.argv[1]):
    if l.startswith("#"):
        tag = l[1:].strip()
    elif l.startswith("{"):
        d = json.loads(l)
        print(tag, "M", d["M"], "ell", d["ell"]["kernel_ms"], "hbm", d["ell"]["hbm_frac_on_tcsc_bytes"],
              "| jit", d["jit"]["kernel_ms"], d["bit_identical"])
P
