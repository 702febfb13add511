# GPU check: parity tests, score A/B, bench, kernel-trace of the bench.
# Any failing GPU step ends the script (no further GPU work after a fault).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_simca.py -q -p no:cacheprovider > gpurun_out/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_kernels.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench.log; exit 2; }
grep "^{" gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'], d['score_kernel']['achieved_GBs'], d['score_kernel']['avg_launch_ms'])"
if [ "${TRACE:-1}" = 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_trace.log 2>&1 || { echo "trace failed"; exit 3; }
fi
echo done
