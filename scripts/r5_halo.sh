#!/bin/bash
# wgrad tests, then the pipelined-wgrad per-shape timing of this build against libdmc_prev.so (the previous commit)
set -o pipefail
O=gpurun_out/${1:-r5halo}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for L in libdmc.so libdmc_prev.so libdmc.so libdmc_prev.so; do
  echo "== $L"
  DMC_LIB=diffusion_models_collection_amd/$L timeout -k 10 120 python3 scripts/wgrad_probe2.py --only pipe --iters 20 2>&1 | grep -v amdgpu.ids | grep -E "per train|^32 128|^16 256|^8 256|^4 256" | cut -c1-60 || exit 1
done | tee $O/probe.txt
