#!/bin/bash
# k_score_1p A/B: the product libocm.so against an experiment build
# (EXP=build/exp/libocm_<name>.so), alternating in separate processes, then
# the LDS counter pass of the product kernel.
#   TAG=r03d EXP=libocm_r02score.so bash scripts/score_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-score_ab}; mkdir -p "$O"
E=$PWD/ocm-vae-simca_amd/csrc/build/exp/${EXP:-libocm_r02score.so}
for i in 1 2 3; do
  timeout -k 10 120 python3 -u scripts/bench_score.py --k 20 --reps 20 --kernels diag --tag product >> "$O/ab.log" 2>&1 || exit 2
  OCM_ALLOW_EXP_LIB=1 OCM_LIB=$E timeout -k 10 120 python3 -u scripts/bench_score.py --k 20 --reps 20 --kernels diag --tag "$(basename "$E")" >> "$O/ab.log" 2>&1 || exit 3
done
grep '^{' "$O/ab.log"
if [ "${PMC:-1}" = 1 ]; then
  timeout -s KILL 120 rocprofv3 --kernel-include-regex k_score_1p \
    --pmc SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d "$O/pmc" -o p --output-format csv -- python3 scripts/bench_score.py --k 20 --reps 3 --kernels diag > "$O/pmc.log" 2>&1 || exit 4
  python3 - "$O" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, sum(v) / len(v))
PY
fi
