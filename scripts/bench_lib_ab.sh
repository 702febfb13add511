#!/bin/bash
# bench.py (no CPU leg, no VAE) alternating between the product libocm and
# exp builds (LIBS: "product" or build/exp/libocm_<name>.so), one process each.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-benchab}; mkdir -p "$O"
for L in ${LIBS:-product}; do
  if [ "$L" = product ]; then unset OCM_LIB; else export OCM_ALLOW_EXP_LIB=1 OCM_LIB=$PWD/ocm-vae-simca_amd/csrc/build/exp/libocm_$L.so; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-vae > "$O/$L.json" 2> "$O/$L.err" || { echo "$L failed"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])" "$O/$L.json" "$L"
done
