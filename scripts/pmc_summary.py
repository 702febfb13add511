#!/usr/bin/env python3
"""Summarise a gpurun_out/prof run into profiles/: kernel stats (top kernels)
and per-launch PMC for k_gram / k_score (FETCH_SIZE doubled: on gfx950 it
reports half the bytes of wide streaming reads, MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "prof")
tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
prof = os.path.join(REPO, "profiles")
os.makedirs(prof, exist_ok=True)


def short(name):
    for key in ("k_gram_reduce", "k_gram8d", "k_gram8", "k_gram3", "k_gram", "k_q8_quant", "k_score_direct", "k_score"):
        if key + "<" in name or key + "(" in name:
            return key
    return name[:60]


# kernel stats
if not os.path.exists(os.path.join(src, "trace", "run_kernel_stats.csv")):
    raise SystemExit("no trace stats under " + src)
stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
lines = ["| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
for r in stats[:25]:
    lines.append(f"| `{r['Name'][:80]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.4f} | "
                 f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |")
open(os.path.join(prof, f"{tag}_kernel_stats.md"), "w").write(
    "# rocprofv3 --kernel-trace --stats: `python3 bench.py --steps 5 --warmup 2 --no-cpu`\n\n" + "\n".join(lines) + "\n")

# PMC
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in ("pmc1", "pmc2", "pmc3"):
    path = os.path.join(src, d, "p_counter_collection.csv")
    if not os.path.exists(path):
        continue
    for r in csv.DictReader(open(path)):
        agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for kname, cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    rec = {"counters_mean_per_launch": m}
    if "FETCH_SIZE" in m:
        rec["hbm_read_bytes_per_launch"] = 2 * m["FETCH_SIZE"] * 1024  # gfx950: FETCH_SIZE = ½ bytes
    if "WRITE_SIZE" in m:
        rec["hbm_write_bytes_per_launch"] = m["WRITE_SIZE"] * 1024
    if "hbm_read_bytes_per_launch" in rec and "hbm_write_bytes_per_launch" in rec:
        rec["hbm_bytes_per_launch"] = rec["hbm_read_bytes_per_launch"] + rec["hbm_write_bytes_per_launch"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
        # GRBM_GUI_ACTIVE is summed over 8 XCDs; 1024 SIMDs
        rec["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
    if "TCC_HIT_sum" in m:
        rec["l2_hit_rate"] = m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        rec["wave_cycle_split"] = {k: m[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in m}
    out[kname] = rec
json.dump(out, open(os.path.join(prof, f"{tag}_pmc.json"), "w"), indent=1)
latest_path = os.path.join(prof, "pmc_gram_latest.json")
latest = json.load(open(latest_path)) if os.path.exists(latest_path) else {}
if "kernel" in latest:  # older single-kernel format
    latest = {latest["kernel"]: {"hbm_bytes_per_launch": latest["hbm_bytes_per_launch"], "source": latest["source"]}}
for kname in ("k_gram", "k_gram3", "k_gram8", "k_gram8d", "k_q8_quant", "k_score_direct"):
    if kname in out and "hbm_bytes_per_launch" in out[kname]:
        latest[kname] = {"hbm_bytes_per_launch": out[kname]["hbm_bytes_per_launch"], "source": f"{tag}_pmc.json"}
json.dump(latest, open(latest_path, "w"), indent=1)
print(json.dumps(out, indent=1)[:3000])
