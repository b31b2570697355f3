#!/bin/bash
# one-rank RCCL step overhead (bench dp1_rccl line) at several GradSync bucket sizes
set -o pipefail
O=gpurun_out/${1:-r5dp}
mkdir -p $O
for b in 25 50 75 150; do
  DMC_DDP_BUCKET_MB=$b timeout -k 10 400 python3 bench.py --no-sample --no-cpu --no-cfg --no-dit --no-roofline > $O/b$b.json 2> $O/b$b.err || { tail -20 $O/b$b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$b.json').read().strip().splitlines()[-1]); r=d['dp1_rccl']; print('bucket $b', 'train', d['value'], 'dp1', r.get('train_img_s'), 'overhead', r.get('overhead_ms_per_step'), 'segs', r.get('graph_segments'), 'exposed', r.get('exposed_comm_ms_per_step'))"
done | tee $O/dp.txt
