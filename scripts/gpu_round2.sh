# Bench line + kernel trace of the bench (current defaults).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo bench failed; tail gpurun_out/bench.log; exit 6; }
tail -1 gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-vae > gpurun_out/prof/bench_trace.log 2>&1 || { echo "prof failed"; exit 7; }
echo done
