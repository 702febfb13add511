#!/usr/bin/env python3
"""Per-call durations and grids of the hipBLASLt GEMMs (Cijk_*) in one replay
of the graphed VAE step, from a rocprofv3 kernel trace of
scripts/vae_step_trace.py (between its sentinel launches).

    python scripts/vae_gemm_calls.py OUT/run_kernel_trace.csv
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sent = [i for i, r in enumerate(rows) if "k_cast_f64_f32" in r["Kernel_Name"]]
lo, hi = sent[-2], sent[-1]
win = rows[lo + 1:hi]
# one replay: the last 1/50 of the window
step = win[-(len(win) // 50):]
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"]
    if "Cijk" in name or "act_bias" in name or "elu" in name:
        print(f"{d:7.2f} us  grid {r.get('Grid_Size', '?'):>8}  wg {r.get('Workgroup_Size', '?'):>5}  {name[:90]}")
