#!/bin/bash
# which of the PRO_PART parity checks fails: the kernel-level prologue test, and the model test with / without it
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4dbg}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "halo_gn_silu_prologue" > $O/k.log 2>&1; tail -3 $O/k.log; grep -E "^E .*(assert|Error)" $O/k.log | head -5
DMC_PRO_PART=0 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_model.py \
  -k "halo_prologue_bitwise" > $O/m0.log 2>&1; tail -1 $O/m0.log
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_model.py \
  -k "halo_prologue_bitwise" > $O/m1.log 2>&1; tail -1 $O/m1.log
exit 0
