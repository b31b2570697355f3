#!/bin/bash
# PMC passes over the bench roofline conv (scripts/conv_probe.py r128_32); each pass its own rocprofv3 run.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/sq" -o sq --output-format csv -- python3 scripts/conv_probe.py --shape r128_32 --iters 5
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 scripts/conv_probe.py --shape r128_32 --iters 5
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 scripts/conv_probe.py --shape r128_32 --iters 5
