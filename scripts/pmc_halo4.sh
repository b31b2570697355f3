set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc/a -o a --output-format csv -- python3 scripts/halo_probe.py 0 > gpurun_out/pmc/a.log 2>&1
f=$(find gpurun_out/pmc/a -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r['Kernel_Name'][:60]
    agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    if 'halo4' not in k: continue
    print(k)
    for c, v in d.items():
        print(f"  {c:28s} {sum(v)/len(v):14.0f}  (n={len(v)})")
PY
