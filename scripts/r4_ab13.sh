#!/bin/bash
# GroupNorm prologue on the halo conv (1, default) vs the materialised apply (0) in the sampling loops; then the
# small-map conv latency probe (hot / one-at-a-time / cold caches)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab13}
mkdir -p $O
BENCH_ARGS="--no-extra --no-dit --no-cpu --no-roofline --no-train" REPS=2 bash scripts/ab.sh $O "DMC_HALO_PRO=1" "DMC_HALO_PRO=0" || exit 1
bash scripts/r4_probe_small.sh ${1:-r4ab13}
