"""Average the PMC counters of the kernels whose name contains a pattern (rocprofv3 counter_collection CSVs)."""
import collections
import csv
import glob
import sys

root, pat = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "conv"
agg = collections.defaultdict(list)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    print(f"{k:28s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
