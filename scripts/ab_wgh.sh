#!/bin/bash
# halo weight-gradient kernel A/B (DMC_WG_HALO_VER 1: 8-wave one block per CU, 2: 4-wave two blocks per CU)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wgh
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
DMC_WG_HALO_VER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -k "wgrad or halo or bench_size" > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
for cfg in "DMC_WG_HALO_VER=2" "DMC_WG_HALO_VER=1" "DMC_WG_HALO_VER=2" "DMC_WG_HALO_VER=1"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-roofline --no-sample > $O/unet.json 2>/dev/null
  python3 -c "import json; u=json.load(open('$O/unet.json')); print('$cfg', 'unet train', u['value'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/proft -o proft --output-format csv -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline > /dev/null 2>&1
python3 scripts/trace_summary.py "$(find $O/proft -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 60 > $O/proft_summary.txt
grep -E "window|wgrad" $O/proft_summary.txt
