#!/bin/bash
set -e -o pipefail
for w in ${PROBES:-none chsum gnfin none chsum gnfin}; do
  timeout -k 10 200 python -u scripts/probe_skip.py $w --steps 30 --warmup 5 --no-cpu --no-extra --no-dit --no-sample --no-roofline > gpurun_out/probe.json 2>gpurun_out/probe.err || { tail -20 gpurun_out/probe.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/probe.json')); print('$w'.ljust(8), d['value'], d['ms_per_step'])"
done
