#!/bin/bash
# round-4 exploration: per-layer conv / wgrad table of the train step and of DDIM, the wgrad probe, PMC of the
# 32x32 128->128 wgrad (SQ occupancy / wait / MFMA counters; traffic)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4x}
mkdir -p $O
timeout -k 10 300 python -u scripts/layer_prof.py --steps 3 > $O/layers_train.txt 2>&1 || { tail -20 $O/layers_train.txt; exit 1; }
timeout -k 10 300 python -u scripts/layer_prof.py --steps 5 --sample > $O/layers_sample.txt 2>&1 || { tail -20 $O/layers_sample.txt; exit 1; }
timeout -k 10 200 python -u scripts/wgrad_probe.py > $O/wgrad_probe.txt 2>&1 || { tail -20 $O/wgrad_probe.txt; exit 1; }
cat $O/wgrad_probe.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/wgk -o wgk --output-format csv -- python3 scripts/wgrad_probe.py --iters 20 > /dev/null 2>&1 || exit 1
P="python3 scripts/wgrad_probe.py --shape w128_32 --iters 5"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/wsq -o wsq --output-format csv -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/wfetch -o wfetch --output-format csv -- $P > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/wwrite -o wwrite --output-format csv -- $P > /dev/null 2>&1 || exit 1
echo explore-done
