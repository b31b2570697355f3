#!/bin/bash
# one-rank RCCL step: SUM vs AVG, and the headline single-graph step, same box
set -o pipefail
O=gpurun_out/${1:-r5dp2}
mkdir -p $O
A="--no-sample --no-extra --no-dit --no-cpu --no-roofline"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $A > $O/base$i.json 2>$O/base$i.err || { tail $O/base$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --dist-one-rank $A > $O/sum$i.json 2>$O/sum$i.err || { tail $O/sum$i.err; exit 1; }
  timeout -k 10 300 python3 bench.py --dist-one-rank --dist-force-avg $A > $O/avg$i.json 2>$O/avg$i.err || { tail $O/avg$i.err; exit 1; }
  for k in base sum avg; do python3 -c "import json; d=json.loads(open('$O/$k$i.json').read().strip().splitlines()[-1]); print('$k', d['ms_per_step'], d.get('graph_segments'), d.get('reduce_op'), d.get('exposed_comm_ms_per_step'))"; done
done | tee $O/dp2.txt
