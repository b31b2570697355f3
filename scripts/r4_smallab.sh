#!/bin/bash
# small-map kernel per-shape A/B: conv probes (small vs split-K) incl. the dgrad shapes, then the bench per mask
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4sab}
mkdir -p $O
for sh in r256_8 d512_8 r256_4 d512_4; do
  timeout -k 10 120 python -u scripts/conv_probe.py --shape $sh --epi full 2>/dev/null | grep -v amdgpu || exit 1
  DMC_NO_SMALL=1 timeout -k 10 120 python -u scripts/conv_probe.py --shape $sh --epi full 2>/dev/null | sed 's/^/  splitK /' | grep -v amdgpu || exit 1
done
REPS=2 bash scripts/ab.sh $O "DMC_SMALL_MASK=15" "DMC_SMALL_MASK=0" "DMC_SMALL_MASK=1" "DMC_SMALL_MASK=2" "DMC_SMALL_MASK=4" "DMC_SMALL_MASK=8"
