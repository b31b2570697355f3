#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r5red3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "wgrad" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 scripts/wgrad_reduce_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/red.txt
