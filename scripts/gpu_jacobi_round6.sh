set -u
# Round 6: the Jacobi round with its LDS reads batched and branch-free
# rotations — eigensolver tests, isolated eigensolve, share timeline and line.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06r}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_eig_wait.py tests/test_gpu_northstar.py tests/test_gpu_f64.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for S in bench geom nuts; do
  timeout -k 10 120 python scripts/bench_eig.py --reps 20 --spectrum $S > $OUT/eig_$S.log 2>&1 || exit 1
  tail -1 $OUT/eig_$S.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --rows 125000 --steps 3 --warmup 1 --no-cpu --no-vae --no-cv --no-prep --phase-steps 0 > $OUT/trace_bench.log 2>&1 || exit 1
python scripts/trace_timeline.py $OUT/prof/run_kernel_trace.csv k_randn > $OUT/timeline.txt 2>&1; tail -60 $OUT/timeline.txt
grep -i jacobi $OUT/prof/run_kernel_stats.csv | cut -c1-220
rm -f $OUT/prof/*_kernel_trace.csv
timeout -k 10 200 python bench.py --rows 125000 --steps 20 --no-cpu --no-vae --no-cv --no-prep > $OUT/share.log 2>&1 && tail -1 $OUT/share.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])"
