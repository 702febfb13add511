cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider > gpurun_out/pytest_kernels.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest_kernels.log
timeout -k 10 300 python scripts/bench_gram.py > gpurun_out/bench_gram.log 2>&1
echo "bench_gram rc=$?"; cat gpurun_out/bench_gram.log | grep -v amdgpu.ids
