#!/bin/bash
# split-K ring depth: per-launch check + same-box A/B in the model
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab14}
mkdir -p $O
timeout -k 10 180 python3 -u scripts/sk_stages_check.py > $O/check.txt 2>&1 || { cat $O/check.txt; exit 1; }
grep -v amdgpu.ids $O/check.txt
REPS=2 bash scripts/ab.sh $O "DMC_SK_STAGES=0" "DMC_SK_STAGES=5" "DMC_SK_STAGES=4"
