"""Per-kernel roofline table of the B=128 bf16 train step from five rocprofv3 runs of scripts/roofline_step.py (the
eager step; the last of its steps is used, delimited by the AdamW launch):
  A: --kernel-trace --marker-trace --kernel-rename   (each dispatch tagged with the op + algorithmic work that launched it)
  B: --kernel-trace                                   (kernel names, grids, durations)
  C: --pmc FETCH_SIZE     D: --pmc WRITE_SIZE     E: --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
aligned by dispatch index. HBM bytes = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half the bytes of a wide streaming
read, MI355X_MICROARCH.md) + WRITE_SIZE, both reported in KiB. MFMA busy = MFMA busy cycles summed over the 1024 SIMDs
/ (1024 x GRBM_GUI_ACTIVE / 8). Algorithmic work is attributed to the longest kernel of each op (the others are
marked aux); bound = mfma for ops with FLOPs (peak 2.5 PFLOP/s dense bf16), else hbm (8 TB/s).

    python scripts/kernel_roofline.py A B C D E OUT.csv [--top 20]
"""
import argparse
import collections
import csv
import glob
import re

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs=5)
ap.add_argument("out")
ap.add_argument("--top", type=int, default=20)
a = ap.parse_args()


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return re.sub(r"\((?!\)).*$", "", n)[:70]


def trace(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]


def pmc(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    by = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(f)):
        i = int(r["Dispatch_Id"])
        by[i][r["Counter_Name"]] = by[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[i] = r["Kernel_Name"]
    return [(names[i], by[i]) for i in sorted(by)]


def last_step(seq, key):
    idx = [i for i, x in enumerate(seq) if "adamw_flat" in key(x)]
    return seq[idx[-2] + 1: idx[-1] + 1]


A = last_step(trace(a.dirs[0]), lambda x: x[0])
B = last_step(trace(a.dirs[1]), lambda x: x[0])
C = last_step(pmc(a.dirs[2]), lambda x: x[0])
D = last_step(pmc(a.dirs[3]), lambda x: x[0])
E = last_step(pmc(a.dirs[4]), lambda x: x[0])
n = min(len(A), len(B), len(C), len(D), len(E))
if len({len(A), len(B), len(C), len(D), len(E)}) != 1:
    print("warning: dispatch counts differ", len(A), len(B), len(C), len(D), len(E), "- aligned from the end")
A, B, C, D, E = A[-n:], B[-n:], C[-n:], D[-n:], E[-n:]
for i in range(n):
    if B[i][1] != A[i][1]:
        raise SystemExit(f"dispatch {i}: grids differ between the runs ({A[i]} vs {B[i]})")
# ops: consecutive dispatches with the same range tag; algorithmic work to the longest kernel of the op
alg = [None] * n
i = 0
while i < n:
    tag = A[i][0]
    j = i
    while j + 1 < n and A[j + 1][0] == tag and tag.startswith("dmc:"):
        j += 1
    if tag.startswith("dmc:"):
        _, op, fl, by, shp = tag.split(":", 4)
        main = max(range(i, j + 1), key=lambda k: B[k][2])
        for k in range(i, j + 1):
            alg[k] = (op, float(fl), float(by), shp) if k == main else (op + " (aux)", 0.0, 0.0, shp)
    i = j + 1
agg = collections.OrderedDict()
for k in range(n):
    name, grid, us = B[k]
    key = (short(name), grid)
    g = agg.setdefault(key, dict(calls=0, us=0.0, fl=0.0, by=0.0, hbm=0.0, mf=0.0, gr=0.0, ops=collections.Counter()))
    g["calls"] += 1
    g["us"] += us
    if alg[k]:
        g["fl"] += alg[k][1]
        g["by"] += alg[k][2]
        g["ops"][f"{alg[k][0]} {alg[k][3]}".strip()] += 1
    c, d, e = C[k][1], D[k][1], E[k][1]
    g["hbm"] += (2 * c.get("FETCH_SIZE", 0.0) + d.get("WRITE_SIZE", 0.0)) * 1024
    g["mf"] += e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    g["gr"] += e.get("GRBM_GUI_ACTIVE", 0.0)
tot = sum(g["us"] for g in agg.values())
rows = sorted(agg.items(), key=lambda kv: -kv[1]["us"])
cols = ["rank", "kernel", "grid_threads", "calls_per_step", "avg_us", "us_per_step", "share_of_step", "ops",
        "alg_gflop_per_launch", "alg_mb_per_launch", "bound", "achieved", "unit", "peak", "frac",
        "pmc_hbm_mb_per_launch", "pmc_over_alg", "pmc_hbm_tbps", "pmc_hbm_frac_of_8tbps", "mfma_busy_frac"]
with open(a.out, "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(cols)
    for r, ((name, grid), g) in enumerate(rows, 1):
        c = g["calls"]
        avg = g["us"] / c
        fl, by, hbm = g["fl"] / c, g["by"] / c, g["hbm"] / c
        if fl > 0:
            bound, ach, unit, peak = "mfma", fl / (avg * 1e-6) / 1e12, "TFLOP/s", 2500.0
        elif by > 0:
            bound, ach, unit, peak = "hbm", by / (avg * 1e-6) / 1e12, "TB/s", 8.0
        else:
            bound, ach, unit, peak = "hbm (aux: PMC bytes)", hbm / (avg * 1e-6) / 1e12, "TB/s", 8.0
        mfb = g["mf"] / (1024 * g["gr"] / 8) if g["gr"] > 0 else 0.0
        w.writerow([r, name, grid, c, round(avg, 2), round(g["us"], 1), round(g["us"] / tot, 4),
                    "; ".join(f"{k} x{v}" for k, v in g["ops"].most_common(3)), round(fl / 1e9, 3),
                    round(by / 1e6, 2), bound, round(ach, 2), unit, peak, round(ach / peak, 4), round(hbm / 1e6, 2),
                    round(hbm / by, 3) if by else "", round(hbm / (avg * 1e-6) / 1e12, 2),
                    round(hbm / (avg * 1e-6) / 8e12, 4), round(mfb, 4)])
print(f"{len(rows)} kernels, {n} dispatches, {tot / 1e3:.3f} ms of kernel time in the step -> {a.out}")
for r, ((name, grid), g) in enumerate(rows[:a.top], 1):
    print(f"{r:3d} {g['us']:8.1f} us {g['calls']:3d}x {name[:48]:48s} {grid}")
