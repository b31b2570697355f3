#!/bin/bash
# reduce-batch timing (this build vs the coalesced-store timing variant) + 1x1 wgrad stage variants
set -o pipefail
O=gpurun_out/${1:-r5red2}
mkdir -p $O
for v in "" redcoal; do
  echo "== reduce ${v:-base}"
  DMC_LIB=diffusion_models_collection_amd/libdmc${v:+_$v}.so timeout -k 10 120 python3 scripts/wgrad_reduce_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done | tee $O/red.txt
for v in "" s64x3 s64x4 s32x4 s32x6; do
  echo "== 1x1 ${v:-base}"
  DMC_LIB=diffusion_models_collection_amd/libdmc${v:+_$v}.so timeout -k 10 120 python3 scripts/gemm_wgrad_probe.py --iters 20 2>&1 | grep -v amdgpu.ids | grep -E "x[0-9]:|per step" | sed 's/| mm.*//' || exit 1
done | tee $O/w1.txt
