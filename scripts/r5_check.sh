#!/bin/bash
# round-5 GPU check: the whole -m gpu suite, then a same-box A/B of this tree's library against a reference build
# (DMC_LIB=$REF, default libdmc_base.so: the build this round started from, pruned) on the train + DDIM lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5chk}
REF=${REF:-$PWD/diffusion_models_collection_amd/libdmc_base.so}
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ ${TESTSEL} > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
BENCH_ARGS=${BENCH_ARGS:-"--no-extra --no-dit --no-cpu --no-roofline"} REPS=${REPS:-2} bash scripts/ab.sh $O \
  "DMC_LIB=$PWD/diffusion_models_collection_amd/libdmc.so" "DMC_LIB=$REF"
