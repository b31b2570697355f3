#!/bin/bash
# kernel-trace stats of the graphed train step (bench.py, train only), optional env settings as arguments
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6tt}; shift
mkdir -p $O
env "$@" timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trn -o trn --output-format csv -- python3 bench.py --no-sample --no-cpu --no-cfg --no-extra --no-dit --no-roofline --steps 8 > $O/trn.log 2>&1 || { tail $O/trn.log; exit 1; }
f=$(find $O -name "trn_kernel_trace.csv" | head -1)
python3 scripts/step_families.py $f 8 > $O/families.txt && head -40 $O/families.txt
