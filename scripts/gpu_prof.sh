cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"
tail -2 gpurun_out/prof_bench.log
find gpurun_out/prof_bench -name "*stats*" | head
