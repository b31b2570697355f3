#!/bin/bash
# one-pass GroupNorm backward on 512-thread blocks (two per CU): parity tests, then the same-box A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab7}
mkdir -p $O
DMC_GN_BWD_NT=512 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_protocol.py -k "fused_one_pass or one_block_per_sample or stats_and_backward or b128_rows" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_GN_BWD_NT=512" "DMC_GN_BWD_NT=1024"
