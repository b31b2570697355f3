#!/bin/bash
# round 3 session d: after dropping the lazy-GN / DMA-position code -- halo + GN kernel tests, the dropout and
# 1-rank RCCL protocol tests, then a same-box A/B against the round-2 tree (_ab_prev) and the 1-rank RCCL step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -m gpu -k "halo or gn_" > $O/kern.log 2>&1 || { tail -30 $O/kern.log; exit 1; }
tail -1 $O/kern.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_protocol.py -x -q --timeout 300 --timeout-method thread -m gpu -k "dropout or rccl" > $O/proto.log 2>&1 || { tail -30 $O/proto.log; exit 1; }
tail -1 $O/proto.log
for i in 1 2 3; do
  for v in prev cur; do
    if [ $v = prev ]; then D=_ab_prev; else D=.; fi
    (cd $D && timeout -k 10 300 python -u bench.py --no-extra --no-dit --no-cpu --no-roofline) > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { tail -20 $O/ab_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_${v}_$i.json')); print('$v', d['value'], d['ddim50']['value'], d['ddim50_cfg']['value'])"
  done
done
timeout -k 10 300 python -u bench.py --no-extra --no-dit --no-cpu --no-roofline --no-sample --dist-one-rank > $O/dist1.json 2> $O/dist1.err || { tail -20 $O/dist1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dist1.json')); print('dist1', d['value'], d.get('ms_per_step'))"
