#!/usr/bin/env python3
"""rocprofv3 kernel trace (CSV) → markdown table grouped by (kernel, grid
size), so a kernel launched at several sizes (the Gram at 1M rows and on the
θ3 rows, for example) shows each launch shape's own average — the figure the
bench line's hipEvent timing of the 1M-row launches is compared against.

    python scripts/trace_by_grid.py <run_kernel_trace.csv> <out.md> "<title>"
"""
import collections
import csv
import sys

src, dst, title = sys.argv[1], sys.argv[2], sys.argv[3]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(src)):
    name = r["Kernel_Name"]
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    acc[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
total = sum(sum(v) for v in acc.values())
rows = sorted(acc.items(), key=lambda kv: -sum(kv[1]))
lines = [f"# {title}", "", "| kernel | grid (work-items) | calls | avg ms | total ms | % |", "|---|---|---|---|---|---|"]
for (name, grid), v in rows[:40]:
    lines.append(f"| `{name[:90]}` | {grid} | {len(v)} | {sum(v) / len(v):.4f} | {sum(v):.3f} | "
                 f"{100 * sum(v) / total:.2f} |")
open(dst, "w").write("\n".join(lines) + "\n")
