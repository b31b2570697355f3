#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3k}
mkdir -p $O
for rep in 1 2; do
for lib in default v 2; do
  for s in r128_32 r384_32 r128_64; do
    if [ $lib = default ]; then L=""; else L="DMC_LIB=abl_lib/libdmc_abl$lib.so"; fi
    env $L DMC_HALO_VER=4 timeout -k 10 120 python -u scripts/conv_probe.py --shape $s --iters 50 2>&1 | tail -1 | sed "s/^/abl$lib /" | tee -a $O/abl.txt
  done
done
done
P="python3 scripts/conv_probe.py --shape r128_32 --iters 5"
export DMC_HALO_VER=4
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$O/sq" -o sq --output-format csv -- $P > /dev/null 2>&1 || exit 1
python3 scripts/pmc_summary.py $O/sq hw_kernel | tee $O/pmc_hw.txt
