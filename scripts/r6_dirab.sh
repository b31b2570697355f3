#!/bin/bash
# model A/B of this tree against a copy of the previous commit's package and library in _ab_prev/ (for changes
# that touch the Python executor and the C ABI together, where DMC_LIB alone cannot select the old behaviour)
set -o pipefail
O=$PWD/gpurun_out/${1:-r6dirab}; mkdir -p $O
ARGS=${BENCH_ARGS:---no-extra --no-dit --no-cpu --no-roofline}
for rep in 1 2; do
  for arm in prev new; do
    d=.; [ $arm = prev ] && d=_ab_prev
    (cd $d && timeout -k 10 300 python -u bench.py $ARGS > $O/$arm$rep.json 2> $O/$arm$rep.err) || { tail -20 $O/$arm$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/$arm$rep.json').read().splitlines() if l.startswith('{')][-1]); print('$arm', 'train', d['value'], 'ddim50', d.get('ddim50', {}).get('value'))"
  done
done
