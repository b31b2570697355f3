#!/bin/bash
# the one-pass GroupNorm backward (v2) and the weight-gradient slab cap: parity tests, then the same-box A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab2}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_protocol.py -k "fused_one_pass or one_block_per_sample or stats_and_backward or wgrad or b128_rows" \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
REPS=2 bash scripts/ab.sh $O "DMC_WG_SLAB_RATIO=4" "DMC_WG_SLAB_RATIO=0" "DMC_WG_SLAB_RATIO=2" "DMC_WG_SLAB_RATIO=8" "DMC_GLDS_2B=1" \
  "DMC_GN_BWD_FUSED=0"
bash scripts/r4_pmc_glds.sh r4ab2_pmc
