"""HBM traffic per kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over bench.py.

Usage: traffic_summary.py DIR CONFIG N_IMG K LAUNCHES_PER_STEP STEPS
Units and corrections follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE under-counts wide (16 B/lane) coalesced reads by exactly 2x, so it is doubled;
WRITE_SIZE is exact for 16 B/lane stores.  Only the last STEPS x LAUNCHES_PER_STEP dispatches of
each kernel (the timed steps) are used: `hbm_bytes_per_step` is their sum / STEPS (bench.py's
roofline `traffic` is per step, like its `achieved`), `hbm_bytes` the mean per launch.
"""
import collections
import csv
import glob
import json
import re
import sys

root, cfg = sys.argv[1], sys.argv[2]
n_img, k, per_step, steps = (int(x) for x in sys.argv[3:7])
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(root + "/**/*counter_collection.csv", recursive=True)):
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id", 0)))
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        kn = re.sub(r"[<(].*", "", name)
        if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"config": cfg, "n_img": n_img, "k": k, "launches_per_step": per_step, "steps": steps,
       "units": "bytes", "fetch_correction": 2.0,
       "note": "FETCH_SIZE (KB) x 2 (gfx950 wide-read under-count) + WRITE_SIZE (KB); last "
               "steps x launches_per_step dispatches of each kernel",
       "kernels": {}}
n = per_step * steps
for kn, d in sorted(vals.items()):
    f = d.get("FETCH_SIZE", [])[-n:]
    w = d.get("WRITE_SIZE", [])[-n:]
    if not f or not w:
        continue
    fb, wb = 2.0 * 1024.0 * sum(f), 1024.0 * sum(w)
    out["kernels"][kn] = {"fetch_bytes_per_step": fb / steps, "write_bytes_per_step": wb / steps,
                          "hbm_bytes_per_step": (fb + wb) / steps,
                          "hbm_bytes": (fb + wb) / len(f), "launches_used": len(f)}
print(json.dumps(out, indent=1))
