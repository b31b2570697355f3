#!/bin/bash
# kernel-trace of a short train bench under a given build (DMC_LIB), pack / total rows
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --no-sample --no-cpu --no-cfg --no-extra --no-dit --no-roofline --steps 5 --warmup 2 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
grep -h "${PAT:-pack_tiles\|adamw\|conv_wgrad_kernel}" $(find $O/kt -name "*kernel_stats.csv") | cut -d, -f1-4
