#!/bin/bash
# Evidence runs (through gpurun): the strong-scaling one-rank share (bench at
# 125k rows with the per-phase split) and the kernel trace of the graphed VAE
# step.  Each GPU step has its own time limit; the script stops at the first
# failure.   TAG=r03b bash scripts/gpu_evidence.sh
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="gpurun_out/${TAG:-evidence}"
mkdir -p "$OUT"
echo "== share125k ($(date +%T))"
timeout -k 10 300 python -u bench.py --rows 125000 --steps 20 --warmup 3 --phase-steps 5 --no-cpu --no-vae --no-cv \
  > "$OUT/share125k.log" 2>&1
tail -n 1 "$OUT/share125k.log"
echo "== vae trace ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/vaeprof" -o run --output-format csv -- \
  python3 scripts/vae_only.py 100 > "$OUT/vaeprof.log" 2>&1
tail -n 2 "$OUT/vaeprof.log"
rm -f "$OUT"/vaeprof/*_kernel_trace.csv  # the per-dispatch trace is large; the stats file is the record
echo "done"
