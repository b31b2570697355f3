#!/bin/bash
# generic weight-gradient split sweep on the train line (same box): DMC_WG_BLOCKS / DMC_WG_MINPIX
set -e -o pipefail
for cfg in ${CFGS:-"DMC_WG_MINPIX=256" "DMC_WG_BLOCKS=512" "DMC_WG_BLOCKS=768" "DMC_WG_BLOCKS=1024" "DMC_WG_BLOCKS=1536" \
           "DMC_WG_MINPIX=256" "DMC_WG_BLOCKS=512" "DMC_WG_BLOCKS=768" "DMC_WG_BLOCKS=1024" "DMC_WG_BLOCKS=1536"}; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-sample --no-roofline > gpurun_out/wgb.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/wgb.json')); print('$cfg'.ljust(22), d['value'])"
done
