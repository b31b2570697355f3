#!/bin/bash
# round-4 per-kernel roofline of the train step (scripts/roofline_step.py under five rocprofv3 runs, joined by
# scripts/kernel_roofline.py), then the graph-replay train / DDIM traces and the roofline conv stats + PMC
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4p}
mkdir -p $O
P="python3 scripts/roofline_step.py"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --kernel-rename -d $O/rA -o rA --output-format csv -- $P > $O/rA.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rB -o rB --output-format csv -- $P > $O/rB.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/rC -o rC --output-format csv -- $P > $O/rC.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/rD -o rD --output-format csv -- $P > $O/rD.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/rE -o rE --output-format csv -- $P > $O/rE.log 2>&1
python3 scripts/kernel_roofline.py $O/rA $O/rB $O/rC $O/rD $O/rE $O/train_kernel_roofline.csv
