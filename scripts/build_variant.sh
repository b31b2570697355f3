#!/bin/bash
# build diffusion_models_collection_amd/libdmc_<name>.so with extra defines on dmc_conv.hip (timing ablations):
#   bash scripts/build_variant.sh <name> "-DWG_ABL=1"
set -e
N=$1; D=$2
R=$(cd "$(dirname "$0")/.." && pwd)
python -m diffusion_models_collection_amd.build > /dev/null
mkdir -p $R/build/var_$N
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-variable $D \
  -I $R/include -I $R/diffusion_models_collection_amd/csrc -c $R/diffusion_models_collection_amd/csrc/dmc_conv.hip \
  -o $R/build/var_$N/dmc_conv.o
O=""
for f in dmc_wgrad dmc_norm dmc_attn dmc_elem dmc_dit dmc_data; do O="$O $R/build/$f.o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/diffusion_models_collection_amd/libdmc_$N.so \
  $R/build/var_$N/dmc_conv.o $O
echo built libdmc_$N.so
