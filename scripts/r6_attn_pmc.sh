#!/bin/bash
# SQ counter passes over the L = 256 attention kernels (scripts/attn_probe.py --L 256), one rocprofv3 run per pass
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r6apmc}; mkdir -p $O
P=(python3 scripts/attn_probe.py --L 256)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq -o sq --output-format csv -- "${P[@]}" > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d $O/sq2 -o sq2 --output-format csv -- "${P[@]}" > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- "${P[@]}" > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
for k in attn_fwd_res attn_dq_res attn_dkdv_res; do echo "== $k"; python3 scripts/pmc_summary.py $O $k; done | tee $O/summary.txt
grep attn $(find $O/kt -name "*kernel_stats.csv") | cut -c1-160
