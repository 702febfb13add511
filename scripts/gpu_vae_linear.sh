set -u
# Round 6: the bf16 VAE step's bottleneck Linear layers through
# vae_fused.linear_act — VAE tests, steps/s A/B, kernel trace of the step.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06zj}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_vae_train.py tests/test_gpu_vae.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
grep "rel err" $OUT/tests.log | head -12
timeout -k 10 400 python -u scripts/vae_linear_ab.py --steps 300 --rounds 2 > $OUT/ab.jsonl 2>&1 || { tail -20 $OUT/ab.jsonl; exit 1; }
cat $OUT/ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 scripts/vae_step_trace.py 50 > $OUT/trace.log 2>&1 || exit 1
python3 scripts/vae_step_trace.py --summarize $OUT/prof/run_kernel_trace.csv 50 > $OUT/vae_step_trace.md && head -12 $OUT/vae_step_trace.md
rm -f $OUT/prof/*_kernel_trace.csv
