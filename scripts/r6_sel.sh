#!/bin/bash
# run a selection of -m gpu tests: r6_sel.sh <outdir> <pytest -k expr or node ids...>
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu "$@" > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; exit $rc
