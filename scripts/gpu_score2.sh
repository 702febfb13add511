# k_score_coop: parity (kernel + SIMCA tests under the variant), then A/B vs direct.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
OCM_SCORE_VARIANT=${SV:-coop} timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_simca.py tests/test_gpu_cv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/score2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/score2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_score.py --rounds 3 --variants direct,${SV:-coop} > gpurun_out/score2_bench.log 2>&1 || { echo "bench_score failed"; tail -20 gpurun_out/score2_bench.log; exit 3; }
grep -v amdgpu.ids gpurun_out/score2_bench.log
echo done
