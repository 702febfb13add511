# PMC of the i8x3 Gram variants (k_gram8d direct vs k_gram8s shared): one counter group per pass.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmcg8
mkdir -p $OUT
K="--kernel-include-regex k_gram8"
A="scripts/gram_once.py --reps 2"
for V in direct shared; do
  OCM_GRAM8_VARIANT=$V timeout -s KILL 120 rocprofv3 $K --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA -d $OUT/$V.1 -o p --output-format csv -- python3 $A > $OUT/$V.1.log 2>&1 || exit 1
  OCM_GRAM8_VARIANT=$V timeout -s KILL 120 rocprofv3 $K --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/$V.2 -o p --output-format csv -- python3 $A > $OUT/$V.2.log 2>&1 || exit 2
  OCM_GRAM8_VARIANT=$V timeout -s KILL 120 rocprofv3 $K --pmc FETCH_SIZE TA_BUSY_avr -d $OUT/$V.3 -o p --output-format csv -- python3 $A > $OUT/$V.3.log 2>&1 || exit 3
done
python3 - <<'PY'
import csv, collections, glob, os
out = "gpurun_out/pmcg8"
for v in ("direct", "shared"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for d in glob.glob(f"{out}/{v}.*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(d)):
            if "k_gram8" not in r["Kernel_Name"]: continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(v, {k: f"{agg[k]/max(1,n[k]):.4g}" for k in sorted(agg)})
PY
