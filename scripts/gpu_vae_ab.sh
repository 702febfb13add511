# VAE: GPU tests (model parity, trainer, conv kernels) then the train-steps/s line (twice).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_vae.py tests/test_vae_train.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/vae_tests.log 2>&1
rc=$?; tail -3 gpurun_out/vae_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 2; do
  timeout -k 10 300 python scripts/vae_only.py 300 > gpurun_out/vae_$v.log 2>&1 || { echo "vae failed"; tail -5 gpurun_out/vae_$v.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/vae_$v.log').read().strip().splitlines()[-1]); print(d['value'], d['loss_after_warmup'], d['final_loss'], d['params_finite'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vae -o run --output-format csv -- python3 scripts/vae_only.py 100 > gpurun_out/vae_prof.log 2>&1 || echo "prof failed"
