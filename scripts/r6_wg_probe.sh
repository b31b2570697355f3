#!/bin/bash
# 4x4 weight gradients: pipelined slab kernel + reduce vs the whole-image kernel (DMC_WG_IMG4)
set -o pipefail
for only in pipe img4; do
  for sh in "4 256-256" "4 512-256"; do
    timeout -k 10 120 python -u scripts/wgrad_probe2.py --only $only --shape "$sh" --iters 40 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
