"""HBM traffic of a whole sampling loop from rocprofv3 --pmc passes over `bench.py --dit-only --no-train` (two
50-step CFG loops: the warm-up call and the timed call): FETCH_SIZE (KB, doubled: gfx950 tallies 128-B requests at
64 B, MI355X_MICROARCH.md 'HBM') + WRITE_SIZE (KB), summed over every dispatch, divided by the loop count.

    python scripts/pmc_loop.py <fetch_dir> <write_dir> <loops> <out.json>
"""
import csv
import glob
import json
import sys


def total(root, counter):
    v, n = 0.0, 0
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                v += float(r["Counter_Value"])
                n += 1
    return v, n


fetch_dir, write_dir, loops, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
fk, nf = total(fetch_dir, "FETCH_SIZE")
wk, nw = total(write_dir, "WRITE_SIZE")
res = {"scope": f"all dispatches of {loops} DiT-S/2 DDIM-50 CFG loops (B=128, 256-row forwards)",
       "dispatches": [nf, nw], "FETCH_SIZE_KB_total": fk, "WRITE_SIZE_KB_total": wk,
       "hbm_bytes_per_loop": int((2 * fk * 1024 + wk * 1024) / loops)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
