set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2e
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_model.py -x -v -s --timeout 300 --timeout-method thread -k "ddp or graph or trajectory or flat_adamw" > gpurun_out/r2e/pytest.log 2>&1 || { tail -80 gpurun_out/r2e/pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r2e/pytest.log | tail -20
