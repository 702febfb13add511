#!/usr/bin/env python3
"""rocprofv3 --kernel-trace --stats CSV → markdown table (profiles/)."""
import csv
import sys

src, dst, title = sys.argv[1], sys.argv[2], sys.argv[3]
rows = list(csv.DictReader(open(src)))
lines = [f"# {title}", "", "| kernel | calls | avg ms | total ms | % |", "|---|---|---|---|---|"]
for r in rows[:30]:
    lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.4f} | "
                 f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |")
open(dst, "w").write("\n".join(lines) + "\n")
