#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5epi}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "conv or halo or epilogue or gemm1x1" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in libdmc.so libdmc_prev.so; do
  echo "== $lib"
  for sh in r128_32 r256_16 qkv_16 p1_16; do
    for e in full bias; do
      DMC_LIB=diffusion_models_collection_amd/$lib timeout -k 10 60 python3 scripts/conv_probe.py --shape $sh --iters 30 --epi $e 2>&1 | grep -v amdgpu.ids | sed "s/^/$e /" || exit 1
    done
  done
done | tee $O/epi.txt
REPS=2 bash scripts/ab.sh $O "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc.so" "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc_prev.so"
