#!/bin/bash
# roofline-conv A/B of the 3x3 kernels (halo2 vs register-weight hw kernel, tap rotation), + rocprof stats of both
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3i}
mkdir -p $O
for rep in 1 2; do
  for cfg in "DMC_HALO_VER=2" "DMC_HALO_VER=4" "DMC_HALO_VER=4 DMC_HALO_ROT=1" "DMC_HALO_VER=2 DMC_HALO_ROT=1"; do
    env $cfg timeout -k 10 120 python -u bench.py --roofline-only > $O/roof.json 2> $O/roof.err || { tail -20 $O/roof.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/roof.json')); print('$cfg'.ljust(34), d['avg_launch_ms'], d['frac'])" | tee -a $O/roof.txt
  done
done
for v in 2 4; do
  for s in r128_32 r384_32 r128_64; do
    DMC_HALO_VER=$v timeout -k 10 120 python -u scripts/conv_probe.py --shape $s --iters 50 2>&1 | tail -1 | sed "s/^/ver$v $s /" | tee -a $O/roof.txt
  done
done
