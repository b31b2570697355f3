#!/bin/bash
# A/B of the GroupNorm-backward sums from the input-gradient convs (training line only) + kernel traces
set -e -o pipefail
O=gpurun_out/gnb
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "groupnorm_backward_partials" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
for cfg in "DMC_GNB_PARTIALS=1" "DMC_GNB_PARTIALS=0" "DMC_GNB_DROP=0" "DMC_GNB_PARTIALS=1" "DMC_GNB_PARTIALS=0" "DMC_GNB_DROP=0"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-sample --no-roofline > $O/tr.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/tr.json')); print('$cfg'.ljust(24), d['value'])"
done
for v in 1 0; do
  DMC_GNB_DROP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$v -o p$v --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline > /dev/null 2>&1
done
