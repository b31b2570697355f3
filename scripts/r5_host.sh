#!/bin/bash
# DDIM-50 eager vs graphed step loop per batch, and the host enqueue time of one UNet forward
set -o pipefail
O=gpurun_out/${1:-r5host}
mkdir -p $O
timeout -k 10 400 python3 -u scripts/ddim_probe.py --batches 128,64,16 --host > $O/ddim.log 2>&1; r=$?
cat $O/ddim.log; exit $r
