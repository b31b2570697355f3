#!/bin/bash
# Measurement build: libdmc_stamp.so = libdmc.so with -DDMC_STAMP (phase clocks in the halo conv). Never shipped:
# scripts/stamp_probe.py loads it through DMC_LIB.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/stamp_lib"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I $R/include -I $R/diffusion_models_collection_amd/csrc"
/opt/rocm/bin/hipcc $F -DDMC_STAMP -c "$R/diffusion_models_collection_amd/csrc/dmc_conv.hip" -o "$R/stamp_lib/dmc_conv.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/stamp_lib/libdmc_stamp.so" "$R/stamp_lib/dmc_conv.o" \
  "$R/build/dmc_norm.o" "$R/build/dmc_attn.o" "$R/build/dmc_elem.o" "$R/build/dmc_dit.o" "$R/build/dmc_data.o"
echo "$R/stamp_lib/libdmc_stamp.so"
