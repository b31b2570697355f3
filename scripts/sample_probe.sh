#!/bin/bash
# DDIM-50 at B=128: graph replay on/off, and a sampling-only kernel trace (2 DDIM-50 runs, no CFG)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/samp
mkdir -p $O
for g in 0 1 0 1; do
  DMC_GRAPH=$g timeout -k 10 200 python -u bench.py --no-train --no-cpu --no-extra --no-dit --no-roofline --no-cfg > $O/g$g.json 2>/dev/null
  python3 -c "import json; d=json.load(open('$O/g$g.json')); print('DMC_GRAPH=$g ddim50', d['ddim50'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profs -o profs --output-format csv -- \
    python3 bench.py --no-train --no-cpu --no-extra --no-dit --no-roofline --no-cfg > $O/profs.json 2> $O/profs.err
python3 scripts/trace_summary.py "$(find $O/profs -name '*kernel_trace.csv' | head -1)" --steps 100 --top 40 > $O/profs_summary.txt
head -45 $O/profs_summary.txt
