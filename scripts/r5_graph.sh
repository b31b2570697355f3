#!/bin/bash
# sampling-loop graph tests, then DDIM-50 eager vs graphed per batch
set -o pipefail
O=gpurun_out/${1:-r5graph}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py \
  -k "graph or ddim or ddpm or sample or cfg" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python3 -u scripts/ddim_probe.py --batches 128,64,48,16 > $O/ddim.log 2>&1 || { tail -20 $O/ddim.log; exit 1; }
grep -v Sampling $O/ddim.log
