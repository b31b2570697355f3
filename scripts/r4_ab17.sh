#!/bin/bash
# GroupNorm statistics combined once per block in the prologue conv (DMC_PRO_PART) vs the finalize launch; parity first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ab17}
mkdir -p $O
timeout -k 10 300 python -u scripts/dbg_propart.py 2>&1 | grep "kernel N" | grep -v "equal=True" && { echo "kernel mismatch"; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_model.py \
  tests/test_gpu_kernels.py -k "halo_gn_silu_prologue or unet" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
BENCH_ARGS="--no-extra --no-dit --no-cpu --no-roofline --no-train" REPS=2 bash scripts/ab.sh $O "DMC_PRO_PART=1" "DMC_PRO_PART=0"
