# Gram bf16x3 A/B (speed + accuracy) and the GPU test suite.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_gram.py --rounds 3 --variants f32:256x32:2048,bf16x3:256x32:2048 > gpurun_out/bench_gram.log 2>&1 || { echo "bench_gram failed"; tail -20 gpurun_out/bench_gram.log; exit 3; }
grep -v amdgpu.ids gpurun_out/bench_gram.log
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_gpu.log | tail -15
[ $rc -le 1 ] || exit 1
echo done
