#!/bin/bash
# halo conv with wave-private weight rows (DMC_HALO_LATE=1) vs the per-tap-barrier kernel: tests, probe, A/B
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/late
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo_kernel" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in 0 1 0 1; do
  echo "== DMC_HALO_LATE=$v"
  DMC_HALO_LATE=$v timeout -k 10 60 python3 scripts/conv_probe.py --shape all --iters 30 2>&1 | grep -E "r128_32|r384_32|r256_16"
done
bash scripts/ab_bench.sh $O "DMC_HALO_LATE=0" "DMC_HALO_LATE=1" "DMC_HALO_LATE=0" "DMC_HALO_LATE=1"
