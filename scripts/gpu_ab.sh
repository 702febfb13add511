cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_simca.py -q -p no:cacheprovider > gpurun_out/pytest_kernels.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest_kernels.log
timeout -k 10 300 python scripts/bench_score.py > gpurun_out/bench_score.log 2>&1
echo "bench_score rc=$?"; cat gpurun_out/bench_score.log | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1
echo "bench rc=$?"; grep "^{" gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'], d['score_kernel']['achieved_GBs'], d['score_kernel']['avg_launch_ms'])"
