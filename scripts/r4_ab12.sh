#!/bin/bash
# weight gradients of the small (<= 8x8 / <= 16x16) maps on a side stream vs none; the tests of the executor first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab12}
mkdir -p $O
DMC_SIDE_STREAM=1 DMC_SIDE_MAXHW=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_model.py > $O/tests_side.log 2>&1 || { tail -30 $O/tests_side.log; exit 1; }
tail -1 $O/tests_side.log
REPS=2 bash scripts/ab.sh $O "DMC_SIDE_STREAM=0" "DMC_SIDE_STREAM=1 DMC_SIDE_MAXHW=64" "DMC_SIDE_STREAM=1 DMC_SIDE_MAXHW=256"
