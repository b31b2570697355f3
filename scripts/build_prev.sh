#!/bin/bash
# build diffusion_models_collection_amd/libdmc_prev.so from the committed sources of a git revision (default HEAD):
# a same-box A/B baseline for uncommitted kernel changes (DMC_LIB=.../libdmc_prev.so)
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/csrc $T/include
for f in $(git -C $R ls-tree --name-only $REV diffusion_models_collection_amd/csrc/); do git -C $R show $REV:$f > $T/csrc/$(basename $f); done
for f in $(git -C $R ls-tree --name-only $REV include/); do git -C $R show $REV:$f > $T/include/$(basename $f); done
O=""
for s in dmc_conv dmc_wgrad dmc_norm dmc_attn dmc_elem dmc_dit dmc_data; do
  X=""; [ $s = dmc_elem ] || [ $s = dmc_data ] && X="-ffp-contract=off"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-variable $X \
    -I $T/include -I $T/csrc -c $T/csrc/$s.hip -o $T/$s.o &
  O="$O $T/$s.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/diffusion_models_collection_amd/libdmc_prev.so $O
rm -rf $T
echo built libdmc_prev.so from $REV
