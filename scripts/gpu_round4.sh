# GPU tests + bench line + kernel trace (current defaults).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail gpurun_out/bench.log; exit 6; }
tail -1 gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-vae > gpurun_out/prof/bench_trace.log 2>&1 || { echo "prof failed"; exit 7; }
echo done
