#!/bin/bash
# where the LDS-DMA GEMM kernel's waves spend their cycles on small-K / small-map shapes (SQ counters, one pass
# per shape) plus plain kernel-trace durations of the same probe commands
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4pmc}
mkdir -p $O
for sh in r256_4 qkv_8 p1_16 qkv_16 r128_32; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt_$sh -o kt --output-format csv -- python3 scripts/conv_probe.py --shape $sh --iters 20 > $O/kt_$sh.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT -d $O/pmc_$sh -o pmc --output-format csv -- python3 scripts/conv_probe.py --shape $sh --iters 20 > $O/pmc_$sh.log 2>&1 || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/gemm -o gemm --output-format csv -- python3 scripts/gemm_probe.py > $O/gemm.log 2>&1 || exit 1
echo done
