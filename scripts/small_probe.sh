#!/bin/bash
# small-level conv shapes: timing per option, then a kernel trace and SQ counters of the 8x8 split-K conv
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/small
mkdir -p $O
for cfg in "DMC_X=0" "DMC_NO_SPLITK=1" "DMC_GLDS_SKST=5"; do
  echo "== $cfg"
  env $cfg timeout -k 10 60 python3 scripts/conv_probe.py --shape all --iters 30 2>&1 | grep -v amdgpu.ids
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 scripts/conv_probe.py --shape r256_8 --iters 20 > /dev/null 2>&1
python3 scripts/prof_summary.py "$(find $O/kt -name '*kernel_stats.csv' | head -1)" 1 10
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq -o sq --output-format csv -- python3 scripts/conv_probe.py --shape r256_8 --iters 5 > /dev/null 2>&1
python3 scripts/pmc_summary.py $O/sq glds
