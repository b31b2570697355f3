#!/bin/bash
# same-box A/B of the DiT line: working tree vs the HEAD snapshot under _ab_head/
set -e -o pipefail
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_dit_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dh_t.log 2>&1 || { tail -30 gpurun_out/dh_t.log; exit 1; }
tail -1 gpurun_out/dh_t.log
for i in 1 2; do
  for v in new head; do
    if [ $v = head ]; then cd $R/_ab_head; else cd $R; fi
    timeout -k 10 300 python -u bench.py --dit-only > $R/gpurun_out/dh.json 2>/dev/null
    cd $R
    python3 -c "import json; d=json.load(open('gpurun_out/dh.json')); print('$v'.ljust(5), 'dit train', d['train_img_s'], 'dit cfg', d['value'])"
  done
done
