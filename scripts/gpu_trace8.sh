cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc8
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc8/trace -o run --output-format csv -- python3 scripts/gram_once.py --reps 2 > gpurun_out/pmc8/trace.log 2>&1 || exit 7
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/pmc8/trace/run_kernel_stats.csv')))[:4]:
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6, 3), 'ms')
PY
