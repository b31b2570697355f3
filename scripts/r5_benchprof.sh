#!/bin/bash
# round-5 profiles the bench line reads: the roofline conv's kernel-trace stats and its FETCH/WRITE passes, the
# DiT loop's PMC traffic, and kernel-trace summaries of the graphed train step and the DDIM-50 loop
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5bp}
mkdir -p $O
R=(python3 bench.py --roofline-only)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rf -o rf --output-format csv -- "${R[@]}" > $O/rf.log 2>&1 || { tail $O/rf.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/rff -o f --output-format csv -- "${R[@]}" > $O/rff.log 2>&1 || { tail $O/rff.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/rfw -o w --output-format csv -- "${R[@]}" > $O/rfw.log 2>&1 || { tail $O/rfw.log; exit 1; }
python3 scripts/pmc_to_json.py $O/rff $O/rfw conv3x3_halo2_kernel $O/pmc_roofline_conv.json
D=(python3 bench.py --dit-only --no-train)
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $O/dtf -o f --output-format csv -- "${D[@]}" > $O/dtf.log 2>&1 || { tail $O/dtf.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $O/dtw -o w --output-format csv -- "${D[@]}" > $O/dtw.log 2>&1 || { tail $O/dtw.log; exit 1; }
python3 scripts/pmc_loop.py $O/dtf $O/dtw 2 $O/pmc_dit_loop.json
S=(python3 bench.py --no-train --no-cpu --no-cfg --no-extra --no-dit --no-roofline)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/smp -o smp --output-format csv -- "${S[@]}" > $O/smp.log 2>&1 || { tail $O/smp.log; exit 1; }
T=(python3 bench.py --no-sample --no-cpu --no-cfg --no-extra --no-dit --no-roofline)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trn -o trn --output-format csv -- "${T[@]}" > $O/trn.log 2>&1 || { tail $O/trn.log; exit 1; }
find $O -name "*kernel_stats.csv" | sort
