#!/bin/bash
# one-rank RCCL step: host enqueue per step (segmented replay) vs the single-graph step, AVG and SUM
set -o pipefail
O=gpurun_out/${1:-r5dp4}
mkdir -p $O
A="--no-sample --no-extra --no-dit --no-cpu --no-roofline --steps 20 --warmup 5"
for v in "" "--dist-one-rank" "--dist-one-rank --dist-force-avg"; do
  timeout -k 10 300 python3 bench.py $v $A > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('graph_segments'), d.get('reduce_op'))"
done
