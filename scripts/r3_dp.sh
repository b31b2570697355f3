#!/bin/bash
# after the thread-local capture change: the DDP / RCCL GPU tests and the 2-rank gloo rehearsal of the bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3dp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_protocol.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "ddp or rccl" > $O/ddp.log 2>&1 || { tail -30 $O/ddp.log; exit 1; }
tail -1 $O/ddp.log
bash scripts/rehearse_dp.sh $O || exit 1
