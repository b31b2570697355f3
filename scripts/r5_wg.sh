#!/bin/bash
# round-5 weight-gradient check: the wgrad kernel tests, then the per-shape timing of the pipelined kernel
# (DMC_WG_PIPE=1, default) against the round-4 halo kernel (DMC_WG_PIPE=0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5wg}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "wgrad or halo_kernel or dgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u scripts/wgrad_probe2.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
