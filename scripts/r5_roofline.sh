#!/bin/bash
# per-kernel roofline table of the eager B=128 bf16 train step (scripts/roofline_step.py under five rocprofv3 runs,
# joined by scripts/kernel_roofline.py) -> gpurun_out/<dir>/train_kernel_roofline.csv
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5rf}
mkdir -p $O
P=(python3 scripts/roofline_step.py)
timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --kernel-rename -d $O/A -o a --output-format csv -- "${P[@]}" > $O/A.log 2>&1 || { tail $O/A.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/B -o b --output-format csv -- "${P[@]}" > $O/B.log 2>&1 || { tail $O/B.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/C -o c --output-format csv -- "${P[@]}" > $O/C.log 2>&1 || { tail $O/C.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/D -o d --output-format csv -- "${P[@]}" > $O/D.log 2>&1 || { tail $O/D.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/E -o e --output-format csv -- "${P[@]}" > $O/E.log 2>&1 || { tail $O/E.log; exit 1; }
python3 scripts/kernel_roofline.py $O/A $O/B $O/C $O/D $O/E $O/train_kernel_roofline.csv --top 25 | tee $O/roofline.txt
