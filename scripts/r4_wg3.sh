#!/bin/bash
# one-block-per-CU halo wgrad (wgrad3x3_halo3_kernel): parity, probe A/B, bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4w}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_model.py -k "halo_kernel or dgrad_wgrad or bench_size or train_step_grads or big_unet" > $O/gpu.log 2>&1
rc=$?; tail -3 $O/gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error|assert" $O/gpu.log | head -20; exit 1; }
timeout -k 10 200 python -u scripts/wgrad_probe.py 2>/dev/null | grep -v amdgpu || exit 1
DMC_WG_HALO3=0 timeout -k 10 200 python -u scripts/wgrad_probe.py 2>/dev/null | sed 's/^/  halo2 /' | grep -v amdgpu || exit 1
REPS=2 bash scripts/ab.sh $O "DMC_WG_HALO3=1" "DMC_WG_HALO3=0"
