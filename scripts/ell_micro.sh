#!/bin/bash
# GPU box: the small-M walk micro-benchmark (scripts/ell_micro.hip, built on
# the CPU into ternary-spgemm_amd/build/ell_micro).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ternary-spgemm_amd/build/ell_micro > gpurun_out/ell_micro.txt 2>&1
