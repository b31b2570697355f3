"""Per-launch-shape timing of kernels matching a pattern in a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2])
rows = list(csv.DictReader(open(path)))
for pat in sys.argv[3:]:
    d = collections.defaultdict(list)
    for r in rows:
        if pat in r["Kernel_Name"]:
            d[(r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])].append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(pat)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"   grid {k} n/step {len(v) / steps:5.1f} avg {sum(v) / len(v) / 1e3:8.1f} us  tot {sum(v) / steps / 1e6:.3f} ms/step")
