#!/bin/bash
# kernel trace of the 4x4 / 8x8 convs: split-K (default) vs the small-map kernel (DMC_SMALL_MASK=15)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/${1:-r4probe2}
mkdir -p $O
for m in 1 15; do
  for sh in r256_4 r512_4 r256_8; do
    DMC_SMALL_MASK=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k_${m}_$sh -o run -- \
      python3 -u scripts/conv_probe.py --shape $sh --iters 30 >> $O/probe2.txt 2>&1 || exit 1
  done
done
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-8 $f | head -6; done > $O/stats.txt
cat $O/stats.txt
