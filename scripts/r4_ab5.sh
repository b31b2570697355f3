#!/bin/bash
# split-K small-map convs on the 2-stage ring (two blocks per CU), and the one-pass GroupNorm backward limited to
# HW <= 256: parity tests, then the same-box A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab5}
mkdir -p $O
DMC_SK_2B=1 DMC_SK_TARGET=480 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_protocol.py -k "conv or b128_rows" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_GEMM1X1=2" "DMC_SK_2B=1 DMC_SK_TARGET=480" "DMC_SK_2B=1" "DMC_GN_BWD_FUSED_MAXHW=256"
