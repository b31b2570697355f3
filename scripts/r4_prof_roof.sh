#!/bin/bash
# the headline roofline conv only: kernel-trace stats + FETCH / WRITE passes (first part of r4_prof_final.sh)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4pr}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/profr -o profr --output-format csv -- \
  python3 bench.py --roofline-only > $O/profr.json 2> $O/profr.err || { tail -30 $O/profr.err; exit 1; }
cat $O/profr.json; cp "$(find $O/profr -name '*kernel_stats.csv' | head -1)" $O/roofline_kernel_stats.csv
P="python3 bench.py --roofline-only"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- $P > /dev/null
python3 scripts/pmc_to_json.py $O/fetch $O/write conv3x3_halo2_kernel $O/pmc_roofline_conv.json
head -3 $O/roofline_kernel_stats.csv
