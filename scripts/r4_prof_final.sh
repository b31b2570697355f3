#!/bin/bash
# round 4 profiles for profiles/: roofline conv kernel stats + PMC traffic, DiT loop traffic, train / sample /
# 1-rank RCCL traces, and the per-kernel roofline CSV of the train step (scripts/roofline_step.py, 5 passes)
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4pf}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/profr -o profr --output-format csv -- \
  python3 bench.py --roofline-only > $O/profr.json 2> $O/profr.err || { tail -30 $O/profr.err; exit 1; }
cat $O/profr.json; cp "$(find $O/profr -name '*kernel_stats.csv' | head -1)" $O/roofline_kernel_stats.csv
P="python3 bench.py --roofline-only"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- $P > /dev/null
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- $P > /dev/null
python3 scripts/pmc_to_json.py $O/fetch $O/write conv3x3_halo2_kernel $O/pmc_roofline_conv.json
P="python3 bench.py --dit-only --no-train"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/dfetch -o dfetch --output-format csv -- $P > /dev/null
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/dwrite -o dwrite --output-format csv -- $P > /dev/null
python3 scripts/pmc_loop.py $O/dfetch $O/dwrite 2 $O/pmc_dit_loop.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/proft -o proft --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline > $O/proft.json 2> $O/proft.err \
  || { tail -30 $O/proft.err; exit 1; }
python3 scripts/trace_summary.py "$(find $O/proft -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 60 > $O/train_summary.txt
head -3 $O/train_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profs -o profs --output-format csv -- \
  python3 bench.py --no-train --no-cpu --no-extra --no-dit --no-roofline --no-cfg > $O/profs.json 2> $O/profs.err \
  || { tail -30 $O/profs.err; exit 1; }
python3 scripts/trace_summary.py "$(find $O/profs -name '*kernel_trace.csv' | head -1)" --steps 100 --top 50 > $O/sample_summary.txt
head -3 $O/sample_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/profd -o profd --output-format csv -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu --no-extra --no-dit --no-sample --no-roofline --dist-one-rank > $O/profd.json 2> $O/profd.err \
  || { tail -30 $O/profd.err; exit 1; }
python3 scripts/trace_summary.py "$(find $O/profd -name '*kernel_trace.csv' | head -1)" --steps 9 --marker adamw_flat --top 60 > $O/train_dist1_summary.txt
head -3 $O/train_dist1_summary.txt
P="python3 scripts/roofline_step.py"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --kernel-rename -d $O/rA -o rA --output-format csv -- $P > $O/rA.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/rB -o rB --output-format csv -- $P > $O/rB.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/rC -o rC --output-format csv -- $P > $O/rC.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/rD -o rD --output-format csv -- $P > $O/rD.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/rE -o rE --output-format csv -- $P > $O/rE.log 2>&1
python3 scripts/kernel_roofline.py $O/rA $O/rB $O/rC $O/rD $O/rE $O/train_kernel_roofline.csv
