#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5w1}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 scripts/gemm_wgrad_probe.py --iters 20 2>&1 | grep -v amdgpu.ids | sed 's/| mm.*//' | tee $O/w1.txt
REPS=2 bash scripts/ab.sh $O "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc.so" "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc_prev.so"
