#!/bin/bash
# L2->LDS fill-rate check of the 3x3 conv kernels: the same layers on the 8-wave 256x128 kernel (DMC_HALO_VER=1),
# the two-blocks-per-CU 128x128 kernel (2) and the chunk-resident 256x64 kernel (DMC_HALO_CHUNK=1)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fill
mkdir -p $O
for cfg in "DMC_HALO_VER=2" "DMC_HALO_CHUNK=1" "DMC_HALO_CHUNK=2" "DMC_HALO_VER=2" "DMC_HALO_CHUNK=2"; do
  echo "== $cfg"
  env $cfg timeout -k 10 60 python3 scripts/conv_probe.py --shape all --iters 30 > $O/probe.txt 2>&1
  grep -E "r128_32|r384_32|r256_16|r256_32|r128_64" $O/probe.txt || true
done
