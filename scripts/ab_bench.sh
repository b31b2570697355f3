#!/bin/bash
# A/B of launch options on the headline bench (train + DDIM-50 + CFG lines): one bench.py run per setting.
# usage: scripts/ab_bench.sh OUTDIR "ENV1=.. ENV2=.." "ENV3=.." ...
set -e -o pipefail
O=$1; shift
mkdir -p "$O"
i=0
for cfg in "$@"; do
  i=$((i + 1))
  env $cfg timeout -k 10 300 python -u bench.py --no-extra --no-dit --no-cpu --no-roofline > "$O/ab$i.json" 2> "$O/ab$i.err"
  python3 -c "import json,sys; d=json.load(open('$O/ab$i.json')); print('$cfg'.ljust(40), 'train', d['value'], 'ddim50', d['ddim50']['value'], 'cfg', d['ddim50_cfg']['value'])"
done
