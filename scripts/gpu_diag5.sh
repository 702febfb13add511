cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/diag_vae_bench.py > gpurun_out/diag_vae_bench.log 2>&1 || { echo "diag failed"; tail -20 gpurun_out/diag_vae_bench.log; exit 3; }
grep -v amdgpu.ids gpurun_out/diag_vae_bench.log
echo done
