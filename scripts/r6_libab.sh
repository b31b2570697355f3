#!/bin/bash
# this build vs libdmc_prev.so (scripts/build_prev.sh): selected -m gpu tests, a probe script run under both builds,
# then the model A/B.   r6_libab.sh <outdir> "<pytest -k expr>" "<probe command>"
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
bash scripts/r6_sel.sh $1 -k "$2" || exit 1
if [ -n "$3" ]; then
  DMC_LIB=diffusion_models_collection_amd/libdmc_prev.so timeout -k 10 300 $3 > $O/probe_prev.txt 2>&1 || { tail -20 $O/probe_prev.txt; exit 1; }
  timeout -k 10 300 $3 > $O/probe_new.txt 2>&1 || { tail -20 $O/probe_new.txt; exit 1; }
  paste -d'|' $O/probe_prev.txt $O/probe_new.txt | grep -v amdgpu.ids
fi
REPS=2 BENCH_ARGS="${BENCH_ARGS:---no-extra --no-dit --no-cpu --no-roofline}" bash scripts/ab.sh $O "DMC_LIB=diffusion_models_collection_amd/libdmc_prev.so" "DMC_LIB=diffusion_models_collection_amd/libdmc.so"
