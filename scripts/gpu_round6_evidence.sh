#!/bin/bash
# Round-6 closing evidence (through gpurun): GPU tests, smoke, the default
# bench line, the 125k-row share line, the headline kernel trace by launch
# shape, and the PMC passes of the bench kernels (k_gram8e, k_q8_quant,
# k_score_1p) on this tree.  Stops at the first failing step.
#   TAG=r06m bash scripts/gpu_round5_evidence.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06m}
mkdir -p "$O"
step() {  # name seconds command...
  local name=$1 secs=$2
  shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(date +%T))"
  tail -n 2 "$O/$name.log"
  if [ "$rc" != 0 ]; then exit "$rc"; fi
}
if [ "${TESTS:-1}" = 1 ]; then
  step tests 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench 500 python3 -u bench.py
  step share125k 300 python3 -u bench.py --rows 125000 --no-cpu --no-vae --no-cv --no-prep --steps 20
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 -u bench.py --no-cpu --no-vae --no-cv --no-prep --steps 5
  python3 scripts/trace_by_grid.py "$O/prof/run_kernel_trace.csv" "$O/headline_by_grid.md" "headline workload (bench.py --no-cpu --no-vae --no-cv --no-prep --steps 5): kernel trace by launch shape" || exit 6
  rm -f "$O/prof/run_kernel_trace.csv"
fi
if [ "${PMC:-1}" = 1 ]; then
  step pmc_gram 600 bash scripts/pmc_passes.sh "k_gram8e|k_q8_quant" "$O/pmc_gram" scripts/bench_gram.py --rounds 1 --variants i8x3:0
  step pmc_score 400 bash scripts/pmc_passes.sh "k_score_1p" "$O/pmc_score" scripts/bench_score.py --k 20 --reps 3 --kernels diag
fi
echo done
