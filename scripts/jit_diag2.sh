#!/bin/bash
# TSG_JIT_DIAG code variants exist only in the diagnostic build (make -C ternary-spgemm_amd diag)
export TSG_LIB=${TSG_LIB:-ternary-spgemm_amd/lib/libternary_spgemm_diag.so}
# GPU box: kernel time vs code placement / prefetch (diagnostic).
run() { echo "$1 $(env $1 timeout -k 10 120 python scripts/diag_stamps.py 2>/dev/null | grep 'kernel ms')" || exit 1; }
run "TSG_JIT_DIAG=none"
run "TSG_JIT_DIAG=samecode"
run "TSG_JIT_DIAG=samecode,notouch"
run "TSG_JIT_TOUCH=1,4"
run "TSG_JIT_TOUCH=2,4"
run "TSG_JIT_TOUCH=4,4"
run "TSG_JIT_TOUCH=1,8"
run "TSG_JIT_DIAG=nobar,nodma,noreads,nolgkm,samecode"
