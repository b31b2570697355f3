#!/bin/bash
# GroupNorm backward persistent form: parity, per-shape kernel time (both arms), model A/B
set -o pipefail
O=gpurun_out/${1:-r6gnpipe}; mkdir -p $O
bash scripts/r6_sel.sh ${1:-r6gnpipe} -k "gn_bwd or groupnorm or graphed_train" || exit 1
for p in 0 1; do
  DMC_GN_BWD_PIPE=$p timeout -k 10 300 python -u scripts/gn_probe.py --iters 50 > $O/probe_pipe$p.txt 2>&1 || { tail -20 $O/probe_pipe$p.txt; exit 1; }
done
paste -d'|' $O/probe_pipe0.txt $O/probe_pipe1.txt | grep bwd
REPS=2 BENCH_ARGS="--no-sample --no-extra --no-dit --no-cpu --no-roofline" bash scripts/ab.sh $O "DMC_GN_BWD_PIPE=0" "DMC_GN_BWD_PIPE=1"
