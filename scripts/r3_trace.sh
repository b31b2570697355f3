#!/bin/bash
# training-step kernel trace of the current tree (per-kernel us/step summary)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3t}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/proft -o proft --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline > $O/proft.json 2> $O/proft.err \
  || { tail -30 $O/proft.err; exit 1; }
python3 scripts/trace_summary.py "$(find $O/proft -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 70 > $O/train_summary.txt
head -3 $O/train_summary.txt
