cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/score
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_simca.py tests/test_gpu_cv.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/score/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/score/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_score.py --variants direct,cs --rounds 3 2>&1 | grep -v amdgpu.ids | tail -6
