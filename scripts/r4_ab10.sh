#!/bin/bash
# register epilogue only where the tile emits GroupNorm partials (DMC_REG_EPI=1) vs everywhere (2) vs never (0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab10}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_protocol.py -k "deferred or conv_epilogue or halo or b128_rows" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_REG_EPI=1" "DMC_REG_EPI=2" "DMC_REG_EPI=0"
