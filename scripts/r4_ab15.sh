#!/bin/bash
# GroupNorm backward with two samples per block (512-thread blocks) vs one (1024 / 512 threads)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab15}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "gn_bwd or groupnorm_backward" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_GN_BWD_IPB=1" "DMC_GN_BWD_IPB=2" "DMC_GN_BWD_NT=512"
