#!/bin/bash
# small-map conv shapes under the available kernel choices (per-launch timing, conv_probe)
set -o pipefail
O=gpurun_out/${1:-r5small}
mkdir -p $O
for cfg in "" "DMC_SMALL_MASK=0" "DMC_SMALL_MASK=15" "DMC_SK_TARGET=1 DMC_SMALL_MASK=0"; do
  echo "== ${cfg:-default}"
  for sh in r256_8 r512_8 d512_8 r256_4 r512_4 d512_4; do
    env $cfg timeout -k 10 60 python3 scripts/conv_probe.py --shape $sh --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done | tee $O/small.txt
