#!/bin/bash
# kernel trace of the graphed CIFAR train step (8 timed steps) + per-family time per step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5step}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- \
  python3 bench.py --steps 8 --warmup 3 --no-sample --no-cpu --no-cfg --no-extra --no-dit --no-roofline \
  > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -2 $O/bench.log
python3 scripts/step_families.py $(find $O/kt -name "*kernel_trace.csv" | head -1) 8 | tee $O/families.txt | head -40
