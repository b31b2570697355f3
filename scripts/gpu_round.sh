#!/bin/bash
# One GPU session: parity tests, the bench line, a kernel-trace profile of the bench, PMC traffic of the
# roofline conv. Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-round}
mkdir -p "$O"
STAGES=${STAGES:-tbpm}
if [[ $STAGES == *t* ]]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
    || { tail -30 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
fi
if [[ $STAGES == *b* ]]; then
  timeout -k 10 500 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
  cat "$O/bench.json"
fi
if [[ $STAGES == *p* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o prof --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit > "$O/prof_bench.json" 2> "$O/prof_bench.err" \
    || { tail -30 "$O/prof_bench.err"; exit 1; }
  f=$(find "$O/prof" -name '*kernel_stats.csv' | head -1); python3 scripts/prof_summary.py "$f" 10 20
fi
if [[ $STAGES == *s* ]]; then
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
fi
if [[ $STAGES == *T* ]]; then   # training-only kernel trace: 3 warm-up + 10 steps
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/proft" -o proft --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline > "$O/proft.json" 2> "$O/proft.err" \
    || { tail -30 "$O/proft.err"; exit 1; }
  python3 scripts/trace_summary.py "$(find "$O/proft" -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 45 > "$O/proft_summary.txt"
  head -30 "$O/proft_summary.txt"
fi
if [[ $STAGES == *S* ]]; then   # sampling-only kernel trace: 2 DDIM-50 runs
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/profs" -o profs --output-format csv -- \
    python3 bench.py --no-train --no-cpu --no-extra --no-dit --no-roofline > "$O/profs.json" 2> "$O/profs.err" \
    || { tail -30 "$O/profs.err"; exit 1; }
  python3 scripts/trace_summary.py "$(find "$O/profs" -name '*kernel_trace.csv' | head -1)" --steps 100 --top 40 > "$O/profs_summary.txt"
  head -25 "$O/profs_summary.txt"
fi
if [[ $STAGES == *D* ]]; then   # DiT-S/2 kernel trace: 2 DDIM-50 CFG loops + 13 train steps
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/profd" -o profd --output-format csv -- \
    python3 bench.py --dit-only > "$O/profd.json" 2> "$O/profd.err" || { tail -30 "$O/profd.err"; exit 1; }
  python3 scripts/trace_summary.py "$(find "$O/profd" -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 30 > "$O/profd_train.txt"
  python3 scripts/prof_summary.py "$(find "$O/profd" -name '*kernel_stats.csv' | head -1)" 1 30 > "$O/profd_stats.txt"
  head -20 "$O/profd_train.txt"
fi
if [[ $STAGES == *r* ]]; then   # kernel stats of the roofline conv alone (bench.py --roofline-only), for profiles/
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/profr" -o profr --output-format csv -- \
    python3 bench.py --roofline-only > "$O/profr.json" 2> "$O/profr.err" || { tail -30 "$O/profr.err"; exit 1; }
  cat "$O/profr.json"; cat "$(find "$O/profr" -name '*kernel_stats.csv' | head -1)"
fi
if [[ $STAGES == *m* ]]; then
  P="python3 bench.py --roofline-only"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$O/fetch" -o fetch --output-format csv -- $P > /dev/null
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$O/write" -o write --output-format csv -- $P > /dev/null
  python3 scripts/pmc_to_json.py "$O/fetch" "$O/write" conv3x3_halo2_kernel "$O/pmc_roofline_conv.json"
fi
