#!/bin/bash
# round 3 session b: GroupNorm statistics folded into the consumers (DMC_GN_LAZY), parity + A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k "halo or gn_ or groupnorm" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -1 $O/kern.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_protocol.py -q -s --timeout 300 --timeout-method thread -m gpu > $O/model.log 2>&1 || { grep -E "passed|failed|Error" $O/model.log | tail -5; tail -40 $O/model.log; exit 1; }
grep -E "passed|failed|DDIM-50|1000 steps" $O/model.log | tail -6
for d in 0 1 2 0 1 2; do
  DMC_HALO_DPOS=$d timeout -k 10 120 python -u bench.py --roofline-only > $O/roof_$d.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/roof_$d.json')); print('dpos $d', d['avg_launch_ms'], d['frac'])"
done
bash scripts/ab.sh $O/ab "DMC_GN_LAZY=0" "DMC_GN_LAZY=1" "DMC_HALO_DPOS=1" "DMC_HALO_DPOS=2" "DMC_SIDE_STREAM=1" "DMC_GN_LAZY=0" "DMC_GN_LAZY=1" "DMC_HALO_DPOS=1" "DMC_HALO_DPOS=2" "DMC_SIDE_STREAM=1" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_dit.py tests/test_gpu_dit_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/rest.log 2>&1 || { tail -30 $O/rest.log; exit 1; }
tail -1 $O/rest.log
for mode in plain dist; do
  F=""; [ $mode = dist ] && F="--dist-one-rank"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$mode -o tr --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline $F > $O/tr_$mode.json 2> $O/tr_$mode.err || { tail -20 $O/tr_$mode.err; exit 1; }
  python3 scripts/trace_summary.py "$(find $O/tr_$mode -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 60 > $O/tr_${mode}_summary.txt
  head -1 $O/tr_${mode}_summary.txt
done
