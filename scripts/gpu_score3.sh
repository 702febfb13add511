# score kernel A/B: current build vs the variants (parity first)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_simca.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "score or simca or predict or transform" > gpurun_out/score3_tests.log 2>&1
rc=$?; tail -2 gpurun_out/score3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_score.py --rounds 5 --variants direct,lds > gpurun_out/score3_bench.log 2>&1 || { tail -5 gpurun_out/score3_bench.log; exit 3; }
grep -v amdgpu.ids gpurun_out/score3_bench.log
