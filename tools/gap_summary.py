#!/usr/bin/env python3
"""Per-kernel durations and the gaps between consecutive dispatches (the command processor's view) from a
rocprofv3 --kernel-trace CSV: for every kernel name, the median duration and the median gap from the previous
dispatch's end to its start, over the last N dispatches of the timed GN loop.
usage: gap_summary.py DIR [N]   (DIR holds **/*kernel_trace.csv)"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    rows = rows[-n:]
    dur, gap = defaultdict(list), defaultdict(list)
    for i, (s, e, k) in enumerate(rows):
        dur[k].append((e - s) / 1e3)
        if i > 0:
            gap[k].append((s - rows[i - 1][1]) / 1e3)
    for k in sorted(dur, key=lambda k: -statistics.median(dur[k])):
        print(f"{k:24s} n {len(dur[k]):4d}  dur med {statistics.median(dur[k]):7.2f} us  "
              f"gap before med {statistics.median(gap[k]) if gap[k] else 0:6.2f} us")


if __name__ == "__main__":
    main()
