set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
timeout -k 10 300 python -u scripts/dbg/nan_b128.py bf16 > gpurun_out/r2b/nan.log 2>&1 || { tail -20 gpurun_out/r2b/nan.log; exit 1; }
cat gpurun_out/r2b/nan.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -v -s --timeout 300 --timeout-method thread -k "halo_kernel or bench_size or resume_from or plain_torch or unfused_ema" > gpurun_out/r2b/pytest.log 2>&1 || { tail -60 gpurun_out/r2b/pytest.log; exit 1; }
grep -E "rel|PASS|FAIL|passed|failed|bf16 vs" gpurun_out/r2b/pytest.log | tail -40
