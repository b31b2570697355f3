#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5nt}
mkdir -p $O
for lib in libdmc.so libdmc_nt.so; do
  echo "== $lib"
  for sh in r128_32 r256_16; do
    for e in full bias; do
      DMC_LIB=diffusion_models_collection_amd/$lib timeout -k 10 60 python3 scripts/conv_probe.py --shape $sh --iters 30 --epi $e 2>&1 | grep -v amdgpu.ids | sed "s/^/$e /" || exit 1
    done
  done
done | tee $O/nt.txt
REPS=1 bash scripts/ab.sh $O "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc.so" "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc_nt.so"
