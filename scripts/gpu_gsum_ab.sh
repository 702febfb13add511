# Gram group sums: tests, then the headline bench alternating with the exp
# build that reduces every chunk partial (OCM_GRAM_NO_GSUM)
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06l}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_simca.py tests/test_gpu_northstar.py tests/test_gpu_cv.py tests/test_gpu_prep.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
EXP=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_nogsum.so
for L in product nogsum product nogsum; do
  if [ $L = product ]; then unset OCM_LIB OCM_ALLOW_EXP_LIB; else export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$EXP; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-vae --no-cv --no-prep > $OUT/bench_$L.log 2>&1 || exit 1
  tail -1 $OUT/bench_$L.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases_ms']['rank0']
print('$L', d['ms_per_step'], d['roofline']['avg_launch_ms'], 'gram phase', ph['gram'])" | tee -a $OUT/ab.txt
done
