#!/bin/bash
# TSG_JIT_DIAG code variants exist only in the diagnostic build (make -C ternary-spgemm_amd diag)
export TSG_LIB=${TSG_LIB:-ternary-spgemm_amd/lib/libternary_spgemm_diag.so}
for d in none samecode samewave pairwave samecode,samewave; do
  echo "diag=$d $(TSG_JIT_DIAG=$d timeout -k 10 120 python scripts/diag_stamps.py 2>/dev/null | grep 'kernel ms')" || exit 1
done
