#!/bin/bash
# split-K target sweep on the small-map convs (kernel trace: conv + split-K epilogue per launch)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4probe3}
mkdir -p $O
for t in 240 128 64 32; do
  for sh in r256_4 r512_4 d512_4 r512_8; do
    echo "DMC_SK_TARGET=$t" >> $O/probe3.txt
    DMC_SK_TARGET=$t timeout -k 10 120 python3 -u scripts/conv_probe.py --shape $sh --iters 50 2>/dev/null | grep " us" >> $O/probe3.txt || exit 1
  done
done
cat $O/probe3.txt
