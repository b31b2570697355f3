#!/bin/bash
# wgrad kernel tests, then same-box bench A/B (this tree vs DMC_WG_FLUSH_EVERY=0) and the step profile
set -o pipefail
O=gpurun_out/${1:-r5chk2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=1 bash scripts/ab.sh $O "DMC_WG_FLUSH_EVERY=3" "DMC_WG_FLUSH_EVERY=0" || exit 1
bash scripts/r5_step.sh ${1:-r5chk2}/step
