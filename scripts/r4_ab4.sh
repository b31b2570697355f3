#!/bin/bash
# persistent 1x1 GEMM: 4-slot one-block-per-CU (1) vs 2-slot two-blocks-per-CU (2) vs the per-tile kernel (0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab4}
mkdir -p $O
DMC_GEMM1X1=2 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "gemm1x1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for sh in qkv_16 qkv_8 p1_16; do
  DMC_GEMM1X1=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt2_$sh -o kt --output-format csv -- python3 scripts/conv_probe.py --shape $sh --iters 20 > $O/kt2_$sh.log 2>&1 || exit 1
done
REPS=2 bash scripts/ab.sh $O "DMC_GEMM1X1=1" "DMC_GEMM1X1=2" "DMC_GEMM1X1=0"
