#!/bin/bash
# default bench (as the driver runs it) + same-box A/B against a saved previous library (ab_lib/libdmc_prev.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3o}
mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
if [ -f ab_lib/libdmc_prev.so ]; then
  REPS=2 bash scripts/ab.sh $O/ab "DMC_LIB=ab_lib/libdmc_prev.so" "DMC_LIB=diffusion_models_collection_amd/libdmc.so" || exit 1
fi
