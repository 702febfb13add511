#!/usr/bin/env python3
"""GPU idle gaps inside the timed steps of a rocprofv3 kernel_trace.csv:
every interval of at least --min-us during which no kernel runs, with the
kernels on either side, for the last --steps steps (a step starts at each
launch whose name contains --marker, e.g. the headline's k_colsum_part).

    python scripts/step_gaps.py run_kernel_trace.csv --marker k_colsum_part --steps 2
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="k_colsum_part")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--min-us", type=float, default=3.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    for si in range(max(0, len(marks) - a.steps - 1), len(marks) - 1):
        lo, hi = marks[si], marks[si + 1]
        t0 = int(rows[lo]["Start_Timestamp"])
        busy_end = t0
        prev = None
        tot = 0.0
        print(f"--- step from {rows[lo]['Kernel_Name'][:40]}: span {(int(rows[hi]['Start_Timestamp']) - t0) / 1e3:.1f} us")
        for r in rows[lo:hi + 1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - busy_end) / 1e3
            if gap >= a.min_us and prev is not None:
                tot += gap
                print(f"  {(busy_end - t0) / 1e3:9.1f} us  idle {gap:7.1f}  after {prev[:45]:45s} before {r['Kernel_Name'][:45]}")
            if e > busy_end:
                busy_end = e
                prev = r["Kernel_Name"]
        print(f"  idle total {tot:.1f} us")


if __name__ == "__main__":
    main()
