set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r02_bandpmc; mkdir -p $O
for L in product band; do
  if [ "$L" = product ]; then unset OCM_LIB; else export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_$L.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-include-regex gram8d --pmc FETCH_SIZE TCC_HIT_sum -d $O/$L -o p --output-format csv -- python3 scripts/bench_gram.py --variants i8x3:0 --rounds 1 > $O/$L.log 2>&1 || { echo "$L failed"; exit 1; }
  python3 - $O/$L <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        print(sys.argv[1].split("/")[-1], r["Dispatch_Id"], r["Counter_Name"], r["Counter_Value"])
PY
done
