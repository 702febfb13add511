#!/bin/bash
# Short GPU iteration (through gpurun): selected tests, then optional extra
# commands, each under its own time limit; stops at the first failure.
#   TAG=r03c TESTS="tests/test_gpu_kernels.py -k eig" EXTRA1="python scripts/bench_eig.py" bash scripts/gpu_quick.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="gpurun_out/${TAG:-quick}"
mkdir -p "$OUT"
step() {  # name seconds command...
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  if [ "$rc" != 0 ]; then echo "stopping"; exit "$rc"; fi
}
if [ -n "${TESTS:-}" ]; then
  # shellcheck disable=SC2086
  step tests "${TEST_SECS:-400}" python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
fi
for i in 1 2 3 4; do
  v="EXTRA$i"
  if [ -n "${!v:-}" ]; then
    # shellcheck disable=SC2086
    step "extra$i" "${EXTRA_SECS:-300}" ${!v}
  fi
done
rm -f "$OUT"/*/*_kernel_trace.csv
echo "done"
