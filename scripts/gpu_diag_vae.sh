cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in vae simca+vae canary; do
  timeout -k 10 300 python scripts/diag_vae_after_simca.py $m > gpurun_out/diag_after_$m.log 2>&1 || { echo "diag $m failed"; tail -20 gpurun_out/diag_after_$m.log; exit 3; }
  grep -v amdgpu.ids gpurun_out/diag_after_$m.log
done
timeout -k 10 400 python scripts/diag_vae_train.py > gpurun_out/diag_vae_train.log 2>&1 || { echo "diag train failed"; tail -20 gpurun_out/diag_vae_train.log; exit 4; }
grep -v amdgpu.ids gpurun_out/diag_vae_train.log
echo done
