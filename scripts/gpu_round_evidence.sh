#!/bin/bash
# A round's closing evidence on one MI355X (run through gpurun):
#   GPU tests, the default bench line, the 125k-row share line, a rocprofv3
#   kernel trace of the headline workload alone (stats + per-grid summary: the
#   1M-row launches' averages are what the bench line's hipEvent timing is
#   compared against) and the VAE step trace.
#     bash scripts/gpu_round_evidence.sh gpurun_out/<tag>
set -o pipefail
O=${1:-gpurun_out/evidence}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1 || exit 1
tail -2 "$O/tests.log"
timeout -k 10 400 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 2
timeout -k 10 300 python3 -u bench.py --rows 125000 --no-cpu --no-vae --no-cv --no-prep --steps 20 > "$O/share125k.json" 2>> "$O/bench.err" || exit 3
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R" || exit 4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 -u bench.py --no-cpu --no-vae --no-cv --no-prep --steps 5 > "$O/bench_prof.json" 2> "$O/bench_prof.err" || exit 5
python3 scripts/trace_by_grid.py "$O/prof/run_kernel_trace.csv" "$O/headline_by_grid.md" "headline workload (bench.py --no-cpu --no-vae --no-cv --no-prep --steps 5): kernel trace by launch shape" || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/vprof" -o run --output-format csv -- python3 scripts/vae_step_trace.py 50 > "$O/vrun.log" 2>&1 || exit 7
python3 scripts/vae_step_trace.py --summarize "$O/vprof/run_kernel_trace.csv" 50 > "$O/vae_trace.md" || exit 8
rm -f "$O/prof/run_kernel_trace.csv" "$O/vprof/run_kernel_trace.csv"
echo done
