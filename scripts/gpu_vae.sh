cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/vae
timeout -k 10 300 python -u -m pytest tests/test_vae_train.py tests/test_gpu_vae.py tests/test_vae_model.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/vae/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/vae/pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/vae_only.py 300 2>&1 | grep -v amdgpu.ids | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/vae/trace -o run --output-format csv -- python3 scripts/vae_only.py 100 > gpurun_out/vae/trace.log 2>&1 || exit 7
python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/vae/trace/run_kernel_stats.csv')))[:12]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us', r['Percentage'][:5])"
