#!/bin/bash
# regression check: this tree's libdmc.so vs the previous commit's (probe_lib/libdmc_prev.so) on one box
set -e -o pipefail
export TMPDIR=/tmp
bash scripts/ab_bench.sh gpurun_out/prev "DMC_LIB=$PWD/probe_lib/libdmc_prev.so" "DMC_X=0" "DMC_LIB=$PWD/probe_lib/libdmc_prev.so" "DMC_X=0"
