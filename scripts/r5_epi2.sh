#!/bin/bash
set -o pipefail
for sh in r128_32 r256_16; do
  for e in bias temb gn full; do
    for r in 3 0; do
      DMC_REG_EPI=$r timeout -k 10 60 python3 scripts/conv_probe.py --shape $sh --iters 40 --epi $e 2>&1 | grep -v amdgpu.ids | sed "s/^/reg$r $e /" || exit 1
    done
  done
done | tee gpurun_out/epi2.txt
