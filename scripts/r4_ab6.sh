#!/bin/bash
# GroupNorm finalize folded into the apply (v2: partials loaded ahead of the rows, every group combined at once):
# bitwise tests, then the same-box A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab6}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_model.py -k "apply_fin or finalize_in_apply" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_GN_APPLY_FIN=1" "DMC_GN_APPLY_FIN=0"
