#!/bin/bash
# Eigensolver iteration (through gpurun): the eigensolver / SIMCA tests, the
# bench_eig timing and its kernel trace.  TAG names the output directory.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="gpurun_out/${TAG:-eig}"
mkdir -p "$OUT"
echo "== tests ($(date +%T))"
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_northstar.py} -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests.log" 2>&1
tail -n 2 "$OUT/tests.log"
echo "== eig trace ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 scripts/bench_eig.py --reps 10 > "$OUT/eig.log" 2>&1
tail -n 2 "$OUT/eig.log"
rm -f "$OUT"/prof/*_kernel_trace.csv
echo "done"
