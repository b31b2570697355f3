#!/bin/bash
# full -m gpu suite, then same-box A/B of the deferred weight-gradient reductions (DMC_WG_DEFER=1 vs 0), then the step profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5def}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_WG_DEFER=1" "DMC_WG_DEFER=0" || exit 1
bash scripts/r5_step.sh ${1:-r5def}/step
