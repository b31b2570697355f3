#!/bin/bash
# Measurement builds of the register-weight 3x3 conv with parts removed (-DHW_ABL=N: 1 no MFMAs, 2 no epilogue,
# 3 no weight loads, v: accumulators in VGPRs); loaded through DMC_LIB by scripts/r3_abl.sh, never shipped.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/abl_lib"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I $R/include -I $R/diffusion_models_collection_amd/csrc"
for n in "$@"; do
  D="-DHW_ABL=$n"; [ "$n" = v ] && D="-DHW_ACC=\"v\""
  /opt/rocm/bin/hipcc $F $D -c "$R/diffusion_models_collection_amd/csrc/dmc_conv.hip" -o "$R/abl_lib/dmc_conv_$n.o" &
done
wait
for n in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/abl_lib/libdmc_abl$n.so" "$R/abl_lib/dmc_conv_$n.o" \
    "$R/build/dmc_norm.o" "$R/build/dmc_attn.o" "$R/build/dmc_elem.o" "$R/build/dmc_dit.o" "$R/build/dmc_data.o"
  rm "$R/abl_lib/dmc_conv_$n.o"
done
