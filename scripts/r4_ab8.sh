#!/bin/bash
# the halo conv's epilogue from the accumulators (DMC_REG_EPI) and the deferred GroupNorm-backward column sums
# (DMC_GN_DEFER): parity tests, kernel-trace probes, then the same-box A/B (incl. the previous commit's library)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab8}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_protocol.py tests/test_gpu_model.py -k "halo or groupnorm or epilogue or b128_rows or sampling_graph or bitwise or graphed or train_step" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt1 -o kt --output-format csv -- python3 scripts/conv_probe.py --shape r128_32 --iters 20 --epi full > $O/kt1.log 2>&1 || exit 1
DMC_REG_EPI=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt0 -o kt --output-format csv -- python3 scripts/conv_probe.py --shape r128_32 --iters 20 --epi full > $O/kt0.log 2>&1 || exit 1
REPS=2 bash scripts/ab.sh $O "DMC_REG_EPI=1" "DMC_REG_EPI=0" "DMC_GN_DEFER=0"
