"""Per-kernel-family time of the graphed train steps in a rocprofv3 kernel trace (steps between the last
N+1 adamw_flat_kernel markers). usage: step_families.py kernel_trace.csv [N]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]][-(nsteps + 1):]
fam = collections.defaultdict(lambda: [0.0, 0])
for r in rows[idx[0] + 1: idx[-1] + 1]:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    m = re.match(r"[\w:]+(<[^()]*>)?", n)
    key = m.group(0) if m else n[:40]
    fam[key][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / nsteps
    fam[key][1] += 1 / nsteps
wall = (int(rows[idx[-1]]["End_Timestamp"]) - int(rows[idx[0]]["End_Timestamp"])) / 1e3 / nsteps
tot = sum(v[0] for v in fam.values())
print(f"steps {nsteps}: kernel sum {tot:.0f} us/step, wall {wall:.0f} us/step")
for k, v in sorted(fam.items(), key=lambda x: -x[1][0]):
    print(f"{v[0]:8.1f} us {v[1]:6.1f}/step {100 * v[0] / tot:5.1f}%  {k}")
