#!/bin/bash
# timing of the wgrad ablation libraries (scripts/build_variant.sh) on two shapes
set -o pipefail
O=gpurun_out/${1:-r5abl}
mkdir -p $O
for v in "" abl1 abl2 abl4 abl7; do
  L=diffusion_models_collection_amd/libdmc${v:+_$v}.so
  for sh in "32 128-128" "16 256-256"; do
    echo "== ${v:-base} $sh"
    DMC_LIB=$L timeout -k 10 60 python3 scripts/wgrad_probe2.py --only pipe --shape "$sh" --iters 20 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee $O/abl.txt
