#!/bin/bash
set -e -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cd_t.log 2>&1 || { tail -30 gpurun_out/cd_t.log; exit 1; }
tail -1 gpurun_out/cd_t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cd -o cd --output-format csv -- python3 bench.py --no-train --no-cpu --no-extra --no-dit --no-roofline --no-cfg > gpurun_out/cd.json 2>/dev/null
grep -h "ddim_step" $(find gpurun_out/cd -name '*kernel_stats.csv') | cut -d, -f1-4
python3 -c "import json; d=json.load(open('gpurun_out/cd.json')); print('ddim50', d['ddim50']['value'])"
