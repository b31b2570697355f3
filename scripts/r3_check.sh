#!/bin/bash
# round 3: full GPU suite, smoke, default bench on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r3e}
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -3 $O/gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
