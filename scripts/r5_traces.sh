#!/bin/bash
# kernel-trace summaries of the DDIM-50 loop and the graphed train step (the final tree's sampling / train profiles)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5tr}
mkdir -p $O
S=(python3 bench.py --no-train --no-cpu --no-cfg --no-extra --no-dit --no-roofline)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/smp -o smp --output-format csv -- "${S[@]}" > $O/smp.log 2>&1 || { tail $O/smp.log; exit 1; }
T=(python3 bench.py --no-sample --no-cpu --no-cfg --no-extra --no-dit --no-roofline)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trn -o trn --output-format csv -- "${T[@]}" > $O/trn.log 2>&1 || { tail $O/trn.log; exit 1; }
find $O -name "*kernel_stats.csv" -o -name "*kernel_trace.csv" | sort
