#!/usr/bin/env python3
"""Per-launch PMC of the largest launches of one kernel (a pmc_passes.sh
output directory) → an entry of profiles/pmc_gram_latest.json, which
bench.py reads for its roofline "traffic" field.

    python scripts/pmc_latest.py <pmc dir> <kernel key> <source tag>

Only the launches with the largest grid are averaged (a bench script also
runs small sample launches).  FETCH_SIZE is doubled: on gfx950 it reports
half the bytes of wide streaming reads (MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import glob
import json
import os
import sys

src, key, tag = sys.argv[1], sys.argv[2], sys.argv[3]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rows = []
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if key + "(" in r["Kernel_Name"] or key + "<" in r["Kernel_Name"]]
if not rows:
    sys.exit(f"no {key} launches under {src}")
gmax = max(int(r["Grid_Size"]) for r in rows)
per = collections.defaultdict(list)
for r in rows:
    if int(r["Grid_Size"]) == gmax:
        per[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {n: sum(v) / len(v) for n, v in per.items()}
ent = {"source": tag, "grid_size": gmax, "launches_averaged": max(len(v) for v in per.values()),
       "counters_mean_per_launch": m}
if "FETCH_SIZE" in m:
    ent["fetch_bytes_x2"] = m["FETCH_SIZE"] * 1024 * 2
    ent["hbm_bytes_per_launch"] = ent["fetch_bytes_x2"] + m.get("WRITE_SIZE", 0.0) * 1024
if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
    ent["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
    ent["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
out = os.path.join(REPO, "profiles", "pmc_gram_latest.json")
lat = json.load(open(out)) if os.path.exists(out) else {}
lat[key] = ent
json.dump(lat, open(out, "w"), indent=1)
print(json.dumps({key: {k: v for k, v in ent.items() if k != "counters_mean_per_launch"}}))
