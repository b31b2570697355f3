#!/bin/bash
# kernel traces of the train line under probe variants: PROBES="a b"
set -e -o pipefail
O=gpurun_out/pp; mkdir -p $O
for w in ${PROBES}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$w -o $w --output-format csv -- python3 scripts/probe_skip.py $w --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline > /dev/null 2>&1
  python3 scripts/step_families.py "$(find $O/$w -name '*kernel_trace.csv' | head -1)" 9 > $O/fam_$w.txt
  head -25 $O/fam_$w.txt
done
