#!/bin/bash
# round 3 session c: same-box regression vs the round-2 tree (_ab_prev, built from f3862a0), the DDP tests, and the
# kernel traces of the single-graph step vs the 1-rank RCCL segmented step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k "gn_ or halo_gn" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -1 $O/kern.log
for i in 1 2; do
  for v in prev cur lazy; do
    if [ $v = prev ]; then D=_ab_prev; else D=.; fi
    L=0; [ $v = lazy ] && L=1
    (cd $D && DMC_GN_LAZY=$L timeout -k 10 300 python -u bench.py --no-extra --no-dit --no-cpu --no-roofline) > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { tail -20 $O/ab_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_${v}_$i.json')); print('$v', d['value'], d['ddim50']['value'], d['ddim50_cfg']['value'])"
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_dit.py tests/test_gpu_dit_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/rest.log 2>&1 || { tail -30 $O/rest.log; exit 1; }
tail -1 $O/rest.log
for mode in plain dist; do
  F=""; [ $mode = dist ] && F="--dist-one-rank"
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$mode -o tr --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline $F > $O/tr_$mode.json 2> $O/tr_$mode.err || { tail -20 $O/tr_$mode.err; exit 1; }
  python3 scripts/trace_summary.py "$(find $O/tr_$mode -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 60 > $O/tr_${mode}_summary.txt
  head -1 $O/tr_${mode}_summary.txt
done
