#!/bin/bash
# round 3 session b: GroupNorm statistics folded into the consumers (DMC_GN_LAZY), parity + A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k "halo or gn_ or groupnorm" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -1 $O/kern.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_protocol.py -x -q -s --timeout 300 --timeout-method thread -m gpu > $O/model.log 2>&1 || { grep -E "passed|failed|Error" $O/model.log | tail -5; tail -40 $O/model.log; exit 1; }
grep -E "passed|failed|DDIM-50|1000 steps" $O/model.log | tail -6
bash scripts/ab.sh $O/ab "DMC_GN_LAZY=0" "DMC_GN_LAZY=1" "DMC_GN_LAZY=0" "DMC_GN_LAZY=1" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_dit.py tests/test_gpu_dit_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/rest.log 2>&1 || { tail -30 $O/rest.log; exit 1; }
tail -1 $O/rest.log
