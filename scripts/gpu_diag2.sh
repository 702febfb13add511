# MFMA internal-precision microtest + VAE training-mode diagnostic.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O2 scripts/mfma_rounding2.hip -o /tmp/mfma_rounding2 > /dev/null 2>&1 || { echo "compile failed"; exit 1; }
timeout -k 10 60 /tmp/mfma_rounding2 || { echo "microtest failed"; exit 2; }
timeout -k 10 600 python scripts/diag_vae_train.py > gpurun_out/diag_vae_train.log 2>&1 || { echo "vae diag failed"; tail -20 gpurun_out/diag_vae_train.log; exit 3; }
grep -v amdgpu.ids gpurun_out/diag_vae_train.log
echo done
