#!/bin/bash
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wht
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "bench_size" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
for cfg in "DMC_WG_HALO_TARGET=256" "DMC_WG_HALO_TARGET=128" "DMC_WG_HALO_TARGET=192" "DMC_WG_HALO_TARGET=384"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline --no-sample > $O/unet.json 2>/dev/null
  python3 -c "import json; u=json.load(open('$O/unet.json')); print('$cfg'.ljust(28), 'unet train', u['value'])"
done
done
