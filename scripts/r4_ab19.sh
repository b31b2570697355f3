#!/bin/bash
# same-box regression check of this tree's library (two-base halo fragment in the default weight-gradient kernel)
# against the previous commit's build (libdmc_prev.so); halo / wgrad parity first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab19}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "halo_kernel or wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BENCH_ARGS="--no-extra --no-dit --no-cpu --no-roofline --no-sample" REPS=3 bash scripts/ab.sh $O \
  "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc.so" "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc_prev.so"
