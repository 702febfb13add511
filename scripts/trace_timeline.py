#!/usr/bin/env python3
"""Print a kernel timeline (start offset, duration, gap before) for the
launches between the last two occurrences of a marker kernel in a rocprofv3
kernel_trace.csv — e.g. one eigensolve of scripts/bench_eig.py:

    python scripts/trace_timeline.py gpurun_out/x/prof/run_kernel_trace.csv k_randn
"""
import csv
import sys


def main():
    path, marker = sys.argv[1], sys.argv[2]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(idx) < 2:
        sys.exit(f"fewer than two '{marker}' launches")
    a, b = idx[-2], idx[-1]
    t0 = int(rows[a]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        busy += e - s
        q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        print(f"{(s - t0) / 1e3:9.1f} us  +{(e - s) / 1e3:7.1f}  gap {(s - prev_end) / 1e3:6.1f}  q{q:>3}  {r['Kernel_Name'][:80]}")
        prev_end = e
    span = int(rows[b]["Start_Timestamp"]) - t0
    print(f"span {span / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
