#!/bin/bash
# score-kernel iteration: parity tests, timing, phase stamps (diagnostic build)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-score}; mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -k "${TESTK:-score}" -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$O/test.log" 2>&1; rc=$?
tail -3 "$O/test.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u scripts/bench_score.py --k ${KS:-16,20} --reps 10 --kernels diag > "$O/score.log" 2>&1 || exit 2
grep '^{' "$O/score.log"
if [ -f ocm-vae-simca_amd/csrc/build/exp/libocm_stamps.so ]; then
  OCM_STAMPS=1 OCM_ALLOW_EXP_LIB=1 OCM_LIB=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_stamps.so timeout -k 10 200 python3 scripts/bench_score.py \
    --k ${KS:-16,20} --kernels diag --reps 3 --tag stamps > "$O/stamps.log" 2>&1 || exit 3
  grep '^{' "$O/stamps.log"
fi
