#!/usr/bin/env python3
"""rocprofv3 --kernel-trace --stats output → markdown table (profiles/).

    python scripts/trace_summary.py <kernel_stats.csv | results.db> <out.md> "<title>"

Reads the CSV stats file, or the rocpd SQLite database rocprofv3 writes when
no --output-format is given (its top_kernels view)."""
import csv
import sqlite3
import sys

src, dst, title = sys.argv[1], sys.argv[2], sys.argv[3]
if src.endswith(".db"):
    con = sqlite3.connect(src)
    rows = [{"Name": n, "Calls": c, "TotalDurationNs": t * 1e3, "AverageNs": a * 1e3, "Percentage": p}
            for n, c, t, a, p in con.execute("select name, total_calls, total_duration, average, percentage "
                                             "from top_kernels order by total_duration desc")]
else:
    rows = list(csv.DictReader(open(src)))
lines = [f"# {title}", "", "| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
for r in rows[:30]:
    lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.4f} | "
                 f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |")
open(dst, "w").write("\n".join(lines) + "\n")
