# fused-quantiser neighbour exchange: the product (LDS row image) against the
# DPP-shift exp build — prep tests on the exp build, then alternating bench lines
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06k}
mkdir -p $OUT
EXP=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_${EXPN:-qpdpp}.so
OCM_ALLOW_EXP_LIB=1 OCM_LIB=$EXP timeout -k 10 400 python -u -m pytest tests/test_gpu_prep.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests_exp.log 2>&1 || { tail -30 $OUT/tests_exp.log; exit 1; }
tail -1 $OUT/tests_exp.log
for L in product exp product exp; do
  if [ $L = product ]; then unset OCM_LIB OCM_ALLOW_EXP_LIB; else export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$EXP; fi
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-vae --no-cv > $OUT/bench_$L.log 2>&1 || exit 1
  tail -1 $OUT/bench_$L.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); p=d['prep_fit_score']
print('$L', d['ms_per_step'], *[(s, m, p[s][m]['ms_per_step'], p[s][m]['quantise_ms']) for s in ('nuts_snv_sg5_d1','cheese_sg15_d1') for m in ('materialised','fused','fused_write')])" | tee -a $OUT/ab.txt
done
