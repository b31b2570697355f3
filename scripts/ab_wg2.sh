#!/bin/bash
# 1x1 weight-gradient XCD mapping A/B: parity tests, then DiT + UNet train per setting (same box)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wg2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for cfg in "DMC_WG_1X1=1" "DMC_WG_1X1=4" "DMC_WG_1X1=1" "DMC_WG_1X1=4"; do
  env $cfg timeout -k 10 300 python -u bench.py --dit-only > $O/dit.json 2>/dev/null
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline --no-sample > $O/unet.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/dit.json')); u=json.load(open('$O/unet.json')); print('$cfg', 'dit train', d['train_img_s'], 'dit cfg', d['value'], 'unet train', u['value'])"
done
