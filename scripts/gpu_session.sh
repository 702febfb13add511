#!/bin/bash
# One GPU session on the box (run through gpurun): GPU tests, smoke, bench
# line, kernel trace.  Every GPU step runs under its own time limit; the
# session stops at the first step that crashes, aborts or times out (pytest's
# exit status 1 = failed assertions still lets the later steps run).
#   TAG=r02a TESTS="tests -m gpu" BENCH=1 PROF=1 bash scripts/gpu_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="gpurun_out/${TAG:-run}"
mkdir -p "$OUT"

run() {  # name seconds ok_codes command...
  local name=$1 secs=$2 ok=$3
  shift 3
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(date +%T))"
  tail -n 3 "$OUT/$name.log"
  case " $ok " in *" $rc "*) return 0 ;; esac
  echo "stopping: $name exited $rc"
  exit "$rc"
}

if [ -n "${TESTS:-}" ]; then
  # shellcheck disable=SC2086
  run gputest "${TEST_SECS:-900}" "0 1" python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread -p no:cacheprovider
fi
if [ "${SMOKE:-0}" = 1 ]; then
  run smoke 300 "0" python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BENCH:-0}" = 1 ]; then
  run bench 600 "0" python -u bench.py ${BENCH_ARGS:-}
fi
if [ "${PROF:-0}" = 1 ]; then
  run prof 600 "0" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-vae
  rm -f "$OUT"/prof/*_kernel_trace.csv  # large; the stats file is the record
fi
if [ -n "${EXTRA:-}" ]; then
  # shellcheck disable=SC2086
  run extra "${EXTRA_SECS:-600}" "0" $EXTRA
fi
echo "session done"
