#!/bin/bash
# kernel trace + PMC passes of one conv_probe shape (default the 8x8 256->256 conv on the small-map kernel)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5convpmc}
SHAPE=${2:-r256_8}
mkdir -p $O
P=(python3 scripts/conv_probe.py --shape $SHAPE --iters 10)
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- "${P[@]}" > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq -o sq --output-format csv -- "${P[@]}" > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $O/sq2 -o sq2 --output-format csv -- "${P[@]}" > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- "${P[@]}" > $O/fetch.log 2>&1 || { tail $O/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $O/tcp -o tcp --output-format csv -- "${P[@]}" > $O/tcp.log 2>&1 || { tail $O/tcp.log; exit 1; }
grep -h "small\|glds\|epilogue" $(find $O/kt -name "*kernel_stats.csv") | cut -d, -f1-4
