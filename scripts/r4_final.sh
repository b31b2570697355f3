#!/bin/bash
# round-4 final GPU evidence of the current tree: the whole -m gpu suite, the smoke, the default bench, then the
# profiles (roofline conv stats + PMC, DiT loop PMC, train / sample / 1-rank RCCL traces, per-kernel roofline CSV)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4z}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu.log 2>&1
tail -3 $O/gpu.log
grep -q " failed\| error" $O/gpu.log && { grep -E "^FAILED|^ERROR" $O/gpu.log | head; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
head -c 300 $O/bench.json; echo
