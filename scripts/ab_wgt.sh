#!/bin/bash
# tap-aware LDS-DMA weight-gradient kernel: tests, then UNet train DMC_WG_TAPS 1 vs 0 (same box)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wgt
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for cfg in "DMC_WG_TAPS=1" "DMC_WG_TAPS=0" "DMC_WG_TAPS=1" "DMC_WG_TAPS=0"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline --no-sample > $O/unet.json 2>/dev/null
  python3 -c "import json; u=json.load(open('$O/unet.json')); print('$cfg'.ljust(20), 'unet train', u['value'])"
done
