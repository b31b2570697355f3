#!/bin/bash
# quick GPU check: the given pytest selection, then N train-line benches
set -e -o pipefail
mkdir -p gpurun_out
SEL="$1"; NB="${2:-2}"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $SEL > gpurun_out/chk.log 2>&1 || { tail -40 gpurun_out/chk.log; exit 1; }
tail -2 gpurun_out/chk.log
for i in $(seq $NB); do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline > gpurun_out/b.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print('train', d['value'], 'ddim50', d.get('ddim50',{}).get('value'), 'cfg', d.get('ddim50_cfg',{}).get('value'))"
done
