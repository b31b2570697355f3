#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5dp3}
mkdir -p $O
A="--no-sample --no-extra --no-dit --no-cpu --no-roofline --steps 8 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 bench.py --dist-one-rank $A > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
find $O/kt -name "*kernel_trace.csv" | head -2
