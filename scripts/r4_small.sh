#!/bin/bash
# small-map conv: parity, then the conv probe on the 8x8 / 4x4 shapes with and without it, then the bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4s}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "small_kernel or narrow_halo or halo_kernel or conv_forward or dgrad_wgrad" > $O/gpu.log 2>&1
rc=$?; tail -3 $O/gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error|assert" $O/gpu.log | head -20; exit 1; }
for sh in r512_8 r256_8 r512_4 r256_4 nin_32 nout_32; do
  timeout -k 10 120 python -u scripts/conv_probe.py --shape $sh --epi full >> $O/probe.txt 2>&1 || exit 1
  DMC_NO_SMALL=1 DMC_NO_NHALO=1 timeout -k 10 120 python -u scripts/conv_probe.py --shape $sh --epi full >> $O/probe_nosmall.txt 2>&1 || exit 1
done
echo "small:"; grep -v amdgpu.ids $O/probe.txt; echo "split-K:"; grep -v amdgpu.ids $O/probe_nosmall.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py -k "cifar or bf16 or graphed or finalize_in_producing" > $O/gpu2.log 2>&1
rc=$?; tail -3 $O/gpu2.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR|Error|assert" $O/gpu2.log | head -20; exit 1; }
timeout -k 10 600 python -u bench.py --no-extra --no-dit --no-cpu > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('train', d['value'], 'ddim50', d['ddim50']['value'], 'cfg', d['ddim50_cfg']['value'], 'roof_us', d['roofline']['avg_launch_ms'])"
