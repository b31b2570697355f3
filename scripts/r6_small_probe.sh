#!/bin/bash
# small-map conv plans: default (split-K / small kernel) vs the whole-image kernel (DMC_IMG_MASK; BN auto / 16 / 32)
set -o pipefail
O=gpurun_out/${1:-r6sp}; mkdir -p $O
for cfg in "DMC_X=0" "DMC_IMG_MASK=15" "DMC_IMG_MASK=15 DMC_IMG_BN=16" "DMC_IMG_MASK=15 DMC_IMG_BN=32"; do
  echo "## $cfg"
  for s in r256_4 r512_4 d512_4 r256_8 r512_8 d512_8; do
    env $cfg timeout -k 10 60 python -u scripts/conv_probe.py --shape $s --epi full --iters 50 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
