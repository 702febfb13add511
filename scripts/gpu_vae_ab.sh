cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in foreach fused foreach fused; do
  OCM_VAE_ADAM=$v timeout -k 10 200 python scripts/vae_only.py 300 > gpurun_out/vae_$v.log 2>&1 || { echo "vae $v failed"; tail -5 gpurun_out/vae_$v.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/vae_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['final_loss'], d['params_finite'])"
done
