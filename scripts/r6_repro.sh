#!/bin/bash
set -o pipefail
O=gpurun_out/r6rep2; mkdir -p $O
for v in "on 0 0" "on 1 0" "on 1 1"; do
  timeout -k 10 120 python -u scripts/r6_drop_repro.py $v > $O/v_${v// /_}.log 2>&1; rc=$?
  echo "variant $v rc $rc"; tail -3 $O/v_${v// /_}.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
