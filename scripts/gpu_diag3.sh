cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in vae simca+vae canary; do
  timeout -k 10 300 python scripts/diag_vae_after_simca.py $mode > gpurun_out/diag_$mode.log 2>&1 || { echo "diag $mode failed"; tail -20 gpurun_out/diag_$mode.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/diag_$mode.log
done
timeout -k 10 600 python scripts/bench_gram.py --rounds 2 --variants f32:256x32:2048,bf16x3:256x32:2048 > gpurun_out/bench_gram.log 2>&1 || { echo "bench_gram failed"; exit 3; }
grep -v amdgpu.ids gpurun_out/bench_gram.log
echo done
