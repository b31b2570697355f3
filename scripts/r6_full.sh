#!/bin/bash
# the whole -m gpu suite (no -x: every failure reported), smoke(), then the default bench line. Later GPU steps run
# only when pytest ended normally (rc 0 = green, 1 = assertion failures); a crash / abort / time limit ends the call.
set -o pipefail
O=gpurun_out/${1:-r6full}
SEL=${2:-tests/}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -rf --timeout 200 --timeout-method thread -m gpu $SEL > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
if [ $rc -gt 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
[ "${3:-bench}" = "nobench" ] && exit $rc
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('train', d['value'], 'ddim50', d['ddim50']['value'], 'cfg', d['ddim50_cfg']['value'], 'fp32', d['fp32'], 'c64', d['celeba64']['train_img_s'], d['celeba64']['ddim100_img_s'], 'dp1', d['dp1_rccl'].get('overhead_ms_per_step'))"
exit $rc
