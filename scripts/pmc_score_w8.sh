#!/bin/bash
# PMC of k_score_1p, four waves (product) vs eight waves per workgroup (exp
# build with -DOCM_S1P_W8), one process and one counter pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05f}; mkdir -p "$O"
E=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_w8.so
for on in 0 1; do
  OCM_S1P_W8_ON=$on OCM_ALLOW_EXP_LIB=1 OCM_LIB=$E timeout -s KILL 120 rocprofv3 --kernel-include-regex k_score_1p \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    -d "$O/pmc_w$on" -o p --output-format csv -- python3 scripts/bench_score.py --k 20 --reps 3 --kernels diag > "$O/pmc_w$on.log" 2>&1 || exit 4
done
python3 - "$O" <<'PY'
import csv, collections, glob, json, sys
out = {}
for on in (0, 1):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/pmc_w{on}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    m["wait_inst_frac"] = m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]
    m["wait_any_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
    m["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 256 * 4 / 8) if m.get("GRBM_GUI_ACTIVE") else None
    out["waves_per_wg_" + ("8" if on else "4")] = m
print(json.dumps(out, indent=1))
json.dump(out, open(f"{sys.argv[1]}/pmc_score_w4_w8.json", "w"), indent=1)
PY
