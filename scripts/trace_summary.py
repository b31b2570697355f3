"""Group a rocprofv3 kernel_trace.csv by (kernel, grid, block) over the last `--last` fraction of dispatches:
time per step per group, plus busy vs. wall time of that window (launch gaps).

    python scripts/trace_summary.py <kernel_trace.csv> --steps N [--skip-frac F] [--top K]
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=float, required=True, help="steps inside the window")
ap.add_argument("--skip", type=int, default=0, help="dispatches to skip at the start (warm-up)")
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--by-name", action="store_true")
ap.add_argument("--marker", default=None, help="kernel-name substring that ends every step (e.g. adamw_flat)")
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))[a.skip:]
if a.marker:
    # window = the last `steps` steps: after the (steps+1)-th last marker up to the last marker
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    n = int(a.steps)
    if len(idx) < n + 1:
        raise SystemExit(f"only {len(idx)} markers for {n} steps")
    rows = rows[idx[-n - 1] + 1: idx[-1] + 1]
g = collections.defaultdict(lambda: [0, 0.0])
busy = 0.0
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\((?!\)).*$", "", name)[:60]
    key = name if a.by_name else (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
    g[key][0] += 1
    g[key][1] += d
    busy += d
wall = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
print(f"window: {len(rows)} dispatches, busy {busy / a.steps / 1e3:.3f} ms/step, wall {wall / a.steps / 1e3:.3f} ms/step")
for k, (n, t) in sorted(g.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print(f"{t / a.steps:9.1f} us/step  n/step {n / a.steps:6.1f}  avg {t / n:8.1f} us  {k}")
