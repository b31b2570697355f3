#!/bin/bash
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ge2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for cfg in "DMC_GELU_EPI=1" "DMC_GELU_EPI=0" "DMC_GELU_EPI=1" "DMC_GELU_EPI=0"; do
  env $cfg timeout -k 10 300 python -u bench.py --dit-only > $O/dit.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/dit.json')); print('$cfg'.ljust(24), 'dit train', d['train_img_s'], 'dit cfg', d['value'])"
done
