#!/bin/bash
# Kernel trace of the graphed C4 VAE step alone (scripts/vae_step_trace.py) → gpurun_out/$TAG/vae_step_trace.md
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-vae_trace}
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/prof" -o run --output-format csv -- python3 scripts/vae_step_trace.py 50 > "$O/trace.log" 2>&1 || { tail -20 "$O/trace.log"; exit 1; }
python3 scripts/vae_step_trace.py --summarize "$O/prof/run_kernel_trace.csv" 50 > "$O/vae_step_trace.md" && head -60 "$O/vae_step_trace.md"
rm -f "$O"/prof/*_kernel_trace.csv
