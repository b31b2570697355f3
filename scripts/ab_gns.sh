#!/bin/bash
# GroupNorm-backward statistics: channel slices per sample (DMC_GN_BWD_SLICES) and the one-block size limit
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gns
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
for cfg in "DMC_GN_BWD_SLICES=1" "DMC_GN_BWD_SLICES=2" "DMC_GN_BWD_SLICES=4" "DMC_GN_BWD_SLICES=4 DMC_GN_BWD_ONE_MAX=131072" "DMC_GN_BWD_SLICES=8 DMC_GN_BWD_ONE_MAX=131072"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline --no-sample > $O/unet.json 2>/dev/null
  python3 -c "import json; u=json.load(open('$O/unet.json')); print('$cfg'.ljust(48), 'unet train', u['value'])"
done
done
