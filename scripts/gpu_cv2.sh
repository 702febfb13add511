# C3 CV benchmark (1M x 2048, 10 folds) and the PCIe-inclusive drop-in rate.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_cv.py > gpurun_out/bench_cv.log 2>&1 || { echo "bench_cv failed"; tail -20 gpurun_out/bench_cv.log; exit 2; }
grep "^{" gpurun_out/bench_cv.log
timeout -k 10 600 python scripts/bench_cv.py --lv-min 2 --lv-max 20 --reps 2 > gpurun_out/bench_cv_sweep.log 2>&1 || { echo "bench_cv sweep failed"; tail -20 gpurun_out/bench_cv_sweep.log; exit 3; }
grep "^{" gpurun_out/bench_cv_sweep.log
timeout -k 10 600 python scripts/bench_e2e.py > gpurun_out/bench_e2e.log 2>&1 || { echo "bench_e2e failed"; tail -20 gpurun_out/bench_e2e.log; exit 5; }
grep "^{" gpurun_out/bench_e2e.log
