#!/bin/bash
# Small-map conv A/B (8x8 / 4x4 UNet levels): parity of the chosen tiles, then scripts/conv_probe.py per setting.
#   scripts/small_ab.sh OUTDIR "ENV=a" "ENV=b" ...
set -e -o pipefail
export TMPDIR=/tmp
O=$1; shift
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "conv_forward or groupnorm_partials or dgrad" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
for rep in 1 2; do
  for cfg in "$@"; do
    for s in ${SHAPES:-r256_8 r512_8 r256_4 r512_4 p1_8}; do
      env $cfg timeout -k 10 60 python -u scripts/conv_probe.py --shape $s 2>/dev/null | sed "s/^/$cfg  /" >> "$O/probe.txt"
    done
  done
done
cat "$O/probe.txt"
