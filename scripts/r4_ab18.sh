#!/bin/bash
# 4x4 weight gradients on the halo kernel (DMC_WG_HALO9) vs the register-staged kernel; parity first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab18}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "halo_kernel or wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BENCH_ARGS="--no-extra --no-dit --no-cpu --no-roofline --no-sample" REPS=3 bash scripts/ab.sh $O "DMC_WG_HALO9=0" "DMC_WG_HALO9=1"
