#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5habl}
mkdir -p $O
for lib in libdmc.so libdmc_ha1.so libdmc_ha2.so libdmc_ha4.so libdmc_ha8.so libdmc_ha15.so; do
  echo "== $lib"
  for sh in r128_32 r256_16; do
    DMC_LIB=diffusion_models_collection_amd/$lib timeout -k 10 60 python3 scripts/conv_probe.py --shape $sh --iters 30 --epi full 2>&1 | grep -v amdgpu.ids || exit 1
  done
done | tee $O/habl.txt
