#!/bin/bash
# dmc_gn_stats_apply: its tests, then a same-box A/B of the module switch (train + DDIM-50 bench lines)
set -o pipefail
O=gpurun_out/${1:-r5gsa}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_model.py -k "gn_stats_apply or stats_one_block or small_map_gn or halo_prologue_bitwise" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
A="--no-cpu --no-extra --no-dit --no-roofline --no-cfg"
for r in 1 2; do
  for on in 8192 0; do
    timeout -k 10 300 python3 -c "
import sys, runpy
import diffusion_models_collection_amd.models._unet_exec as E
E._GN_SMALL_FUSE = int(sys.argv[1])
sys.argv = ['bench.py'] + sys.argv[2:]
runpy.run_path('bench.py', run_name='__main__')" $on $A > $O/b$on.json 2> $O/b$on.err || { tail $O/b$on.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/b$on.json').read().strip().splitlines()[-1]); print('fuse=$on', d['value'], d['ddim50']['value'])"
  done
done
