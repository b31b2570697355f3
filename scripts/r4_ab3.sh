#!/bin/bash
# the persistent 1x1 GEMM: bitwise test, probe timings (kernel trace) on/off, then the same-box A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab3}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_protocol.py -k "gemm1x1 or b128_rows" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for on in 1 0; do
  for sh in qkv_16 qkv_8 p1_16; do
    DMC_GEMM1X1=$on timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt${on}_$sh -o kt --output-format csv -- python3 scripts/conv_probe.py --shape $sh --iters 20 > $O/kt${on}_$sh.log 2>&1 || exit 1
  done
done
REPS=2 bash scripts/ab.sh $O "DMC_GEMM1X1=1" "DMC_GEMM1X1=0"
