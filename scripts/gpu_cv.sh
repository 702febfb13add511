# GPU: full -m gpu suite, then the C3 CV benchmark (1M x 2048, 10 folds).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/diag_gemm.py > gpurun_out/diag_gemm.log 2>&1 || { echo "diag gemm failed"; tail gpurun_out/diag_gemm.log; exit 8; }
grep -v amdgpu.ids gpurun_out/diag_gemm.log
timeout -k 10 120 python scripts/diag_vae_conv.py > gpurun_out/diag_vae.log 2>&1 || { echo "diag failed"; tail -20 gpurun_out/diag_vae.log; exit 9; }
grep "rel err" gpurun_out/diag_vae.log
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/pytest_gpu.log | tail -15
# rc 1 = assertion failures (keep measuring); anything else (crash, timeout) ends the call
[ $rc -le 1 ] || exit 1
timeout -k 10 600 python scripts/bench_cv.py > gpurun_out/bench_cv.log 2>&1 || { echo "bench_cv failed"; tail -20 gpurun_out/bench_cv.log; exit 2; }
grep "^{" gpurun_out/bench_cv.log
timeout -k 10 600 python scripts/bench_cv.py --lv-min 2 --lv-max 20 --reps 2 > gpurun_out/bench_cv_sweep.log 2>&1 || { echo "bench_cv sweep failed"; tail -20 gpurun_out/bench_cv_sweep.log; exit 3; }
grep "^{" gpurun_out/bench_cv_sweep.log

timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
grep "^{" gpurun_out/bench.log
timeout -k 10 600 python scripts/bench_e2e.py > gpurun_out/bench_e2e.log 2>&1 || { echo "bench_e2e failed"; tail -20 gpurun_out/bench_e2e.log; exit 5; }
grep "^{" gpurun_out/bench_e2e.log
echo done
