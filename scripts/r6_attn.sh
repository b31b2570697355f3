#!/bin/bash
# attention: parity tests, per-shape timing and bitwise comparison of this build against libdmc_prev.so, model A/B
set -o pipefail
O=gpurun_out/${1:-r6attn}; mkdir -p $O
bash scripts/r6_sel.sh ${1:-r6attn} -k "attention or attn or trainer_1k or graphed_train" || exit 1
DMC_LIB=diffusion_models_collection_amd/libdmc_prev.so timeout -k 10 300 python -u scripts/attn_probe.py --save $O/a.pt > $O/probe_prev.txt 2>&1 || { tail -20 $O/probe_prev.txt; exit 1; }
timeout -k 10 300 python -u scripts/attn_probe.py --save $O/b.pt > $O/probe_new.txt 2>&1 || { tail -20 $O/probe_new.txt; exit 1; }
paste -d'|' $O/probe_prev.txt $O/probe_new.txt
python scripts/attn_probe.py --compare $O/a.pt $O/b.pt > $O/compare.txt 2>&1; rc=$?
rm -f $O/a.pt $O/b.pt   # ~100 MB: gpurun copies back at most 64 MiB of gpurun_out/
cat $O/compare.txt; [ $rc = 0 ] || exit 1
REPS=2 BENCH_ARGS="--no-extra --no-dit --no-cpu --no-roofline" bash scripts/ab.sh $O "DMC_LIB=diffusion_models_collection_amd/libdmc_prev.so" "DMC_LIB=diffusion_models_collection_amd/libdmc.so"
