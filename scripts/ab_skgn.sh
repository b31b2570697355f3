#!/bin/bash
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/skgn
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash scripts/ab_bench.sh $O "DMC_NO_SKGN=0" "DMC_NO_SKGN=1" "DMC_NO_SKGN=0" "DMC_NO_SKGN=1"
