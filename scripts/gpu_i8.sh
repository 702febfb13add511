cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc8
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "gram" > gpurun_out/pytest_i8.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_i8.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_gram.py --rounds 2 > gpurun_out/bench_gram.log 2>&1 || { echo bench_gram failed; tail -20 gpurun_out/bench_gram.log; exit 6; }
grep -v amdgpu.ids gpurun_out/bench_gram.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc8/trace -o run --output-format csv -- python3 scripts/gram_once.py --reps 2 > gpurun_out/pmc8/trace.log 2>&1 || exit 7
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/pmc8/trace/run_kernel_stats.csv')))[:4]:
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6, 3), 'ms')
PY
