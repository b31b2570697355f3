#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5gn3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py \
  -k "groupnorm or gn_ or train" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_GN_BWD_IPB2=1" "DMC_GN_BWD_IPB2=0"
