#!/bin/bash
# kernel trace + PMC passes of the weight gradient on one shape (default the 32x32 128->128 layer)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5wgpmc}
SHAPE=${2:-32 128-128}
ONLY=${3:-pipe}
mkdir -p $O
P=(python3 scripts/wgrad_probe2.py --iters 10 --shape "$SHAPE" --only "$ONLY")
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- "${P[@]}" > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq -o sq --output-format csv -- "${P[@]}" > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $O/sq2 -o sq2 --output-format csv -- "${P[@]}" > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- "${P[@]}" > $O/fetch.log 2>&1 || { tail $O/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- "${P[@]}" > $O/write.log 2>&1 || { tail $O/write.log; exit 1; }
find $O -name "*kernel_stats.csv" | head -3 | xargs cat
