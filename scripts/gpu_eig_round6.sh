set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06e}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_northstar.py tests/test_gpu_simca.py tests/test_gpu_cv.py tests/test_gpu_dist.py tests/test_gpu_vae.py tests/test_gpu_prep.py tests/test_gpu_f64.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python scripts/bench_eig.py --reps 20 > $OUT/eig.log 2>&1 && cat $OUT/eig.log | tail -1
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --rows 125000 --steps 3 --warmup 1 --no-cpu --no-vae --no-cv --no-prep --phase-steps 0 > $OUT/trace_bench.log 2>&1 && tail -1 $OUT/trace_bench.log | cut -c1-300
python scripts/trace_timeline.py $OUT/prof/run_kernel_trace.csv k_randn > $OUT/timeline.txt 2>&1; tail -60 $OUT/timeline.txt
rm -f $OUT/prof/*_kernel_trace.csv
timeout -k 10 200 python bench.py --rows 125000 --steps 20 --no-cpu --no-vae --no-cv --no-prep > $OUT/share.log 2>&1 && tail -1 $OUT/share.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])"
# quantiser: the product kernel against the copy-only timing build, alternating
for L in product qcopy product qcopy; do
  if [ "$L" = product ]; then unset OCM_LIB OCM_ALLOW_EXP_LIB; else export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_$L.so; fi
  timeout -k 10 120 python scripts/quant_ab.py --reps 10 >> $OUT/quant_ab.jsonl 2>> $OUT/quant_ab.err || exit 1
done
unset OCM_LIB OCM_ALLOW_EXP_LIB
cat $OUT/quant_ab.jsonl
