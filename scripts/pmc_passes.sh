#!/bin/bash
# PMC of one kernel, one counter group per rocprofv3 pass (gfx950 slot limits:
# ≤ 8 SQ, ≤ 4 TCC per pass), then a per-launch mean summary (JSON) on stdout.
#   bash scripts/pmc_passes.sh <kernel-regex> <outdir> <python script + args...>
set -u
RX=$1; OUT=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$OUT"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
P3="FETCH_SIZE TCC_HIT_sum"
P4="WRITE_SIZE TCC_MISS_sum"
i=0
for G in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i + 1))
  # shellcheck disable=SC2086
  timeout -s KILL 180 rocprofv3 --kernel-include-regex "$RX" --pmc $G -d "$OUT/p$i" -o p --output-format csv \
    -- python3 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$OUT" "$RX" <<'PY'
import csv, collections, glob, json, re, sys
out, rx = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if re.search(rx, r["Kernel_Name"]):
            agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    d = {"counters_mean_per_launch": m}
    if "FETCH_SIZE" in m:  # KiB; ×2 on gfx950 for wide streaming reads (MI355X_MICROARCH.md)
        d["fetch_bytes_x2"] = m["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in m:
        d["write_bytes"] = m["WRITE_SIZE"] * 1024
    if "SQ_WAVE_CYCLES" in m:
        d["wave_cycle_split"] = {n: m.get(n, 0) / m["SQ_WAVE_CYCLES"] for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        d["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
    res[k] = d
print(json.dumps(res, indent=1))
PY
