#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5small3}
mkdir -p $O
for lib in libdmc.so libdmc_sa1.so libdmc_sa2.so libdmc_sa4.so libdmc_sa7.so; do
  echo "== $lib"
  for sh in r256_8 r256_4; do
    DMC_LIB=diffusion_models_collection_amd/$lib DMC_SMALL_MASK=15 timeout -k 10 60 python3 scripts/conv_probe.py --shape $sh --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
done | tee $O/small.txt
