# Gram add-form A/B, then the default bench (bf16x3) and its kernel trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_gram.py --rounds 3 --variants f32:256x32:2048,bf16x3:256x32:2048,bf16x3pk:256x32:2048 > gpurun_out/bench_gram.log 2>&1 || { echo "bench_gram failed"; tail -20 gpurun_out/bench_gram.log; exit 3; }
grep -v amdgpu.ids gpurun_out/bench_gram.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 4; }
grep "^{" gpurun_out/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-vae > gpurun_out/bench_trace.log 2>&1 || { echo "trace failed"; exit 5; }
echo done
