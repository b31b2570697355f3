#!/bin/bash
# round 3: register-weight 3x3 conv (conv3x3_hw_kernel, DMC_HALO_VER=4): parity tests, roofline A/B, step A/B,
# then the whole GPU suite, the smoke and the default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3f}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu \
  -k "halo_kernel or halo_gn_silu or groupnorm_partials or groupnorm_backward_partials" > $O/kern.log 2>&1 \
  || { tail -40 $O/kern.log; exit 1; }
tail -2 $O/kern.log
for rep in 1 2; do
  for cfg in "DMC_HALO_VER=2" "DMC_HALO_VER=4" "DMC_HALO_VER=4 DMC_HALO_ROT=1" "DMC_HALO_VER=2 DMC_HALO_ROT=1"; do
    env $cfg timeout -k 10 120 python -u bench.py --roofline-only > $O/roof.json 2> $O/roof.err || { tail -20 $O/roof.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/roof.json')); print('$cfg'.ljust(34), d['avg_launch_ms'], d['frac'])"
  done
done
REPS=2 bash scripts/ab.sh $O/ab "DMC_HALO_VER=2" "DMC_HALO_VER=4" || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -2 $O/gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
