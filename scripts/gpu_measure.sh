# Round measurements: full bench line (SIMCA + VAE + CPU baseline), C3 CV, PCIe-inclusive drop-in.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { echo bench failed; tail gpurun_out/bench_full.log; exit 6; }
tail -1 gpurun_out/bench_full.log
bash scripts/gpu_cv2.sh
