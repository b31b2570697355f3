#!/bin/bash
# small-map conv latency: back-to-back launches, one launch at a time with caches kept, and with L2 / MALL evicted
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4probe}
mkdir -p $O
for sh in r256_4 r512_4 d512_4 r256_8 r512_8 d512_8; do
  for mode in "" "--cold hot1" "--cold cold"; do
    timeout -k 10 120 python -u scripts/conv_probe.py --shape $sh --iters 30 $mode >> $O/probe.txt 2>&1 || exit 1
  done
done
cat $O/probe.txt
