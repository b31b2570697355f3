#!/bin/bash
# PMC passes over one conv shape of scripts/conv_probe.py (default: the bench roofline conv r128_32);
# each pass is its own rocprofv3 run (counters only, no tracing domains).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
SHAPE=${2:-r128_32}
mkdir -p "$OUT"
P="python3 scripts/conv_probe.py --shape $SHAPE --iters 5"
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/sq" -o sq --output-format csv -- $P
timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d "$OUT/sq2" -o sq2 --output-format csv -- $P
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- $P
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- $P
