#!/bin/bash
for d in none samecode samewave pairwave samecode,samewave; do
  echo "diag=$d $(TSG_JIT_DIAG=$d timeout -k 10 120 python scripts/diag_stamps.py 2>/dev/null | grep 'kernel ms')" || exit 1
done
