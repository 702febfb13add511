# Chebyshev-filtered eigensolver: tests, then product vs the plain-iteration
# exp build on three spectra, the share line and the preprocessing bench line
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06g}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_northstar.py tests/test_gpu_simca.py tests/test_gpu_cv.py tests/test_gpu_prep.py tests/test_gpu_f64.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for S in bench nuts geom; do
  for L in product nocheb; do
    if [ "$L" = product ]; then unset OCM_LIB OCM_ALLOW_EXP_LIB; else export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_$L.so; fi
    timeout -k 10 120 python scripts/bench_eig.py --reps 10 --spectrum $S >> $OUT/eig_ab.jsonl 2>> $OUT/eig_ab.err || exit 1
  done
done
unset OCM_LIB OCM_ALLOW_EXP_LIB
cat $OUT/eig_ab.jsonl
timeout -k 10 300 python -u bench.py --rows 125000 --steps 20 --warmup 3 --no-cpu --no-vae --no-cv --no-prep > $OUT/share.log 2>&1 && tail -1 $OUT/share.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-vae --no-cv > $OUT/bench_prep.log 2>&1 && tail -1 $OUT/bench_prep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], json.dumps(d.get('prep_fit_score')))"
