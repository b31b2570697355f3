#!/bin/bash
# data-parallel segmentation overhead (bench.py's dp1_rccl line: one-rank RCCL, AVG forced) vs the bucket size
set -o pipefail
O=gpurun_out/${1:-r6bucket}; mkdir -p $O
for rep in 1 2; do
  for mb in 25 50 100; do
    DMC_DDP_BUCKET_MB=$mb timeout -k 10 600 python -u bench.py --no-sample --no-dit --no-cpu --no-roofline > $O/b${mb}_$rep.json 2> $O/b${mb}_$rep.err || { tail -20 $O/b${mb}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/b${mb}_$rep.json').read().splitlines() if l.startswith('{')][-1]); p=d.get('dp1_rccl', {}); print('bucket_mb $mb', 'train', d['value'], 'dp1', p.get('train_img_s'), 'overhead_ms', p.get('overhead_ms_per_step'), 'segments', p.get('graph_segments'), 'exposed', p.get('exposed_comm_ms_per_step'))"
  done
done
