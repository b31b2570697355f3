#!/bin/bash
# register epilogue v2 (16-byte stores / residual loads by lane-pair exchange; also in the LDS-DMA GEMM kernel):
# parity tests, kernel-trace probes, same-box A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab9}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_protocol.py tests/test_gpu_model.py -k "conv or halo or groupnorm or epilogue or b128_rows or bitwise or graphed or train_step or unet" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for on in 1 0; do
  for sh in r128_32 r256_16 p1_16; do
    DMC_REG_EPI=$on timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt${on}_$sh -o kt --output-format csv -- python3 scripts/conv_probe.py --shape $sh --iters 20 --epi full > $O/kt${on}_$sh.log 2>&1 || exit 1
  done
done
REPS=2 bash scripts/ab.sh $O "DMC_REG_EPI=1" "DMC_REG_EPI=0"
