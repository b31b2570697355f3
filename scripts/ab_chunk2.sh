#!/bin/bash
# chunk-resident 3x3 conv with per-tap progressive waits (DMC_HALO_CHUNK=2): parity tests, then the fill probe
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/chunk2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "halo_kernel" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
bash scripts/fill_probe.sh
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_all.log 2>&1 || { tail -30 $O/gpu_all.log; exit 1; }
tail -1 $O/gpu_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
