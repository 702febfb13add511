set -u
# Round 6: wall-clock phase stamps of k_jacobi_1b (`make exp EXP_NAME=jstamp
# EXP_FLAGS=-DOCM_JACOBI_STAMPS`): a 32×32 problem alone (scripts/jacobi_micro.py)
# and the Rayleigh–Ritz Jacobi + fused test of isolated eigensolves.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06x}
mkdir -p $OUT
export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_jstamp.so
timeout -k 10 120 python scripts/jacobi_micro.py --reps 4 > $OUT/micro.log 2>&1 || { tail -5 $OUT/micro.log; exit 1; }
grep jacobi32 $OUT/micro.log | tail -2
for S in bench geom; do
  timeout -k 10 120 python scripts/bench_eig.py --reps 3 --spectrum $S > $OUT/stamps_$S.log 2>&1 || exit 1
  echo "== $S"; grep jacobi32 $OUT/stamps_$S.log | tail -4
done
