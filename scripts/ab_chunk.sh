#!/bin/bash
# halo conv with a chunk's nine weight slices resident (DMC_HALO_CHUNK=1) vs the per-tap weight ring: tests, probe, A/B
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/chunk
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo_kernel" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in 0 1 0 1; do
  echo "== DMC_HALO_CHUNK=$v"
  DMC_HALO_CHUNK=$v timeout -k 10 60 python3 scripts/conv_probe.py --shape all --iters 30 2>&1 > $O/probe_$v.txt; grep -E "r128_32|r384_32|r256_16|r256_32" $O/probe_$v.txt || true
done
bash scripts/ab_bench.sh $O "DMC_HALO_CHUNK=0" "DMC_HALO_CHUNK=1" "DMC_HALO_CHUNK=0" "DMC_HALO_CHUNK=1"
