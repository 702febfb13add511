# MFMA accumulation-rounding microtest + Gram mode A/B (speed and accuracy).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O2 scripts/mfma_rounding.hip -o /tmp/mfma_rounding > /dev/null 2>&1 || { echo "compile failed"; exit 1; }
timeout -k 10 60 /tmp/mfma_rounding || { echo "microtest failed"; exit 2; }
timeout -k 10 600 python scripts/bench_gram.py --rounds 3 > gpurun_out/bench_gram.log 2>&1 || { echo "bench_gram failed"; tail -20 gpurun_out/bench_gram.log; exit 3; }
grep -v amdgpu.ids gpurun_out/bench_gram.log
echo done
