#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5w4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "wgrad" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for L in libdmc.so libdmc_prev.so; do
  echo "== $L"; DMC_LIB=diffusion_models_collection_amd/$L timeout -k 10 120 python3 scripts/wgrad_probe2.py --only pipe --iters 20 2>&1 | grep -E "^4 |^8 |per train" | cut -c1-70 || exit 1
done | tee $O/probe.txt
REPS=2 bash scripts/ab.sh $O "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc.so" "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc_prev.so"
