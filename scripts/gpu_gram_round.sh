#!/bin/bash
# Gram evidence for one library build (through gpurun): chunk A/B of the
# default kernel against the 32x32x32 one in one process, the PMC passes of
# the default kernel, the bench line and its kernel trace.  Each GPU step
# has its own time limit; the script stops at the first failure.
#   TAG=r03q bash scripts/gpu_gram_round.sh
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="gpurun_out/${TAG:-gramround}"
mkdir -p "$OUT"
echo "== gram A/B ($(date +%T))"
timeout -k 10 300 python -u scripts/bench_gram.py --rounds 3 \
  --variants "${VARIANTS:-i8x3:0,i8x3k32:0,i8x3:3072,i8x3:6144}" > "$OUT/gram_ab.log" 2>&1
grep -E "TFLOP|err" "$OUT/gram_ab.log"
if [ "${PMC:-1}" = 1 ]; then
  echo "== pmc ($(date +%T))"
  timeout -k 10 600 bash scripts/pmc_passes.sh "k_gram8e|k_q8_quant" "$OUT/pmc" scripts/bench_gram.py \
    --variants i8x3:0 --rounds 1 > "$OUT/pmc.json" 2> "$OUT/pmc.err"
  head -c 600 "$OUT/pmc.json"; echo
fi
if [ "${BENCH:-1}" = 1 ]; then
  echo "== bench ($(date +%T))"
  timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1
  tail -n 1 "$OUT/bench.log" | head -c 1500; echo
  echo "== prof ($(date +%T))"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-vae > "$OUT/prof.log" 2>&1
  rm -f "$OUT"/prof/*/*_kernel_trace.csv "$OUT"/prof/*_kernel_trace.csv
fi
echo "done"
