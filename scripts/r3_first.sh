#!/bin/bash
# round 3, first GPU session: the new parity-protocol tests, the changed kernel / DDP tests, then the bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_protocol.py -q -s --timeout 300 --timeout-method thread -m gpu > $O/protocol.log 2>&1
rc=$?
tail -40 $O/protocol.log | grep -v "^$"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ddp.py tests/test_gpu_dit.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -2 $O/kern.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
