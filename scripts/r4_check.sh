#!/bin/bash
# round-4 quick GPU check: a pytest selection (parity first), then the default bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4c}
shift
mkdir -p $O
[ $# -eq 0 ] && set -- tests/test_gpu_protocol.py
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > $O/gpu.log 2>&1
rc=$?
tail -3 $O/gpu.log
[ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error" $O/gpu.log | head -20; exit 1; }
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("train", d["value"], "graphed", d.get("graphed"), "ddim50", d.get("ddim50", {}).get("value"),
      "cfg", d.get("ddim50_cfg", {}).get("value"), "roof", d.get("roofline", {}).get("avg_launch_ms"),
      "dp1", {k: d.get("dp1_rccl", {}).get(k) for k in ("ms_per_step", "overhead_ms_per_step", "reduce_op",
                                                          "exposed_comm_ms_per_step", "error")})
PY
