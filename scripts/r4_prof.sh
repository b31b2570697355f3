#!/bin/bash
# round-4 per-kernel roofline of the train step (scripts/roofline_step.py under five rocprofv3 runs, joined by
# scripts/kernel_roofline.py). First: the fused one-pass GroupNorm backward tests and its same-box A/B.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4p}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "fused_one_pass or one_block_per_sample or stats_and_backward" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 180 python -u scripts/gemm_probe.py > $O/gemm_probe.txt 2>&1 || { tail -20 $O/gemm_probe.txt; exit 1; }
grep -v amdgpu.ids $O/gemm_probe.txt || true
REPS=2 bash scripts/ab.sh $O/ab "DMC_GN_BWD_FUSED=4" "DMC_GN_BWD_FUSED=0"
P="python3 scripts/roofline_step.py"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --kernel-rename -d $O/rA -o rA --output-format csv -- $P > $O/rA.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rB -o rB --output-format csv -- $P > $O/rB.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/rC -o rC --output-format csv -- $P > $O/rC.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/rD -o rD --output-format csv -- $P > $O/rD.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/rE -o rE --output-format csv -- $P > $O/rE.log 2>&1
python3 scripts/kernel_roofline.py $O/rA $O/rB $O/rC $O/rD $O/rE $O/train_kernel_roofline.csv
