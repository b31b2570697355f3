#!/bin/bash
# same-box A/B: the working tree vs the HEAD snapshot built under _ab_head/ (train + sampling lines)
set -e -o pipefail
R=$(pwd)
for i in 1 2 3; do
  for v in new head; do
    if [ $v = head ]; then cd $R/_ab_head; else cd $R; fi
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline ${ABARGS} > $R/gpurun_out/ab.json 2>/dev/null
    cd $R
    python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v'.ljust(5), 'train', d['value'], 'ddim50', d.get('ddim50',{}).get('value'), 'cfg', d.get('ddim50_cfg',{}).get('value'))"
  done
done
