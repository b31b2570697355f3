#!/bin/bash
# wgrad tests, then the per-family step profile
set -o pipefail
O=${1:-r5red}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "wgrad or halo_kernel or dgrad" > gpurun_out/$O/tests.log 2>&1 || { tail -40 gpurun_out/$O/tests.log; exit 1; }
tail -1 gpurun_out/$O/tests.log
bash scripts/r5_step.sh $O/step
