#!/bin/bash
# round 3, first GPU session: the new parity-protocol tests, the changed kernel / DDP tests, the bench, then an
# A/B of the register-staged weight stream of the 3x3 halo conv (DMC_HALO_WREG)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_protocol.py -q -s --timeout 300 --timeout-method thread -m gpu > $O/protocol.log 2>&1
rc=$?
grep -E "passed|failed|PASS|FAIL|Error|error|1000 steps|teacher|bf16 vs|DDIM-50|RCCL" $O/protocol.log | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k "halo" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -1 $O/kern.log
for w in 0 1 0 1; do
  DMC_HALO_WREG=$w timeout -k 10 120 python -u bench.py --roofline-only > $O/roof_$w.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/roof_$w.json')); print('wreg $w', d['avg_launch_ms'], d['frac'])"
done
bash scripts/ab.sh $O/ab "DMC_HALO_WREG=0" "DMC_HALO_WREG=1" "DMC_HALO_WREG=0" "DMC_HALO_WREG=1" || exit 1
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_dit.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu > $O/rest.log 2>&1 || { tail -30 $O/rest.log; exit 1; }
tail -1 $O/rest.log
