#!/bin/bash
# 1x1 weight-gradient kernel: parity tests, then DiT train + UNet train per DMC_WG_1X1 setting (same box)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wg1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for v in ${VARIANTS:-0 1 2 3 0 1}; do
  DMC_WG_1X1=$v timeout -k 10 300 python -u bench.py --dit-only > $O/dit$v.json 2>/dev/null
  DMC_WG_1X1=$v timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline --no-sample > $O/unet$v.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/dit$v.json')); u=json.load(open('$O/unet$v.json')); print('WG_1X1=$v', 'dit train', d['train_img_s'], 'dit cfg', d['value'], 'unet train', u['value'])"
done
