#!/bin/bash
# Gram chunking / variant A/B: per-kernel times (rocprofv3 kernel trace) for
# each VARIANTS entry (× LIBS: "product" or build/exp/libocm_<name>.so) in its
# own process.  TAG names the output directory.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-gram}; mkdir -p "$O"
for L in ${LIBS:-product}; do
for V in ${VARIANTS:-i8x3:0}; do
  N=${L}_$(echo "$V" | tr ':' '_')
  if [ "$L" = product ]; then unset OCM_LIB; else export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_$L.so; fi
  echo "== $N"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/$N" -o p --output-format csv \
    -- python3 scripts/bench_gram.py --variants "$V" --rounds 2 > "$O/$N.log" 2>&1 || { echo "variant $V failed"; exit 1; }
  grep -E "TFLOP|err" "$O/$N.log"
  python3 - "$O/$N" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("gram", "q8", "colblk", "fixup", "colexp")):
            print(f'  {r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg_ms {float(r["AverageNs"]) / 1e6:8.3f}')
PY
done
done
