#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5small4}
mkdir -p $O
for lib in libdmc.so libdmc_mt4.so; do
  for m in 1 3 15; do
  echo "== $lib SMALL_MASK=$m"
  for sh in r256_8 d512_8; do
    DMC_LIB=diffusion_models_collection_amd/$lib DMC_SMALL_MASK=$m timeout -k 10 60 python3 scripts/conv_probe.py --shape $sh --iters 20 2>&1 | grep -v amdgpu.ids || exit 1
  done
  done
done | tee $O/small.txt
REPS=1 bash scripts/ab.sh $O "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc.so" "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc_mt4.so" "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc_mt4.so DMC_SMALL_MASK=3"
