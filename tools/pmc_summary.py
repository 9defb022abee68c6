#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel (bytes per launch).

FETCH_SIZE / WRITE_SIZE are reported by rocprofv3 in KB.  Per MI355X_MICROARCH.md, on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads (TCC_EA0_RDREQ x 64 B for 128-B
requests): the corrected read bytes are 2 x FETCH_SIZE.  WRITE_SIZE is taken as reported.
usage: pmc_summary.py DIR  (DIR/FETCH_SIZE/**/*counter_collection.csv, DIR/WRITE_SIZE/...)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return acc


def summarise(d):
    fetch = per_kernel(d, "FETCH_SIZE")
    write = per_kernel(d, "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        out[k.split("(")[0]] = {
            "launches": max(len(f), len(w)),
            "fetch_size_kb_raw": fk,
            "write_size_kb": wk,
            "hbm_bytes_per_launch": 2.0 * fk * 1024.0 + wk * 1024.0,
        }
    return out


def main():
    if sys.argv[1] == "--sizes":  # DIR/p<N>/{FETCH_SIZE,WRITE_SIZE} for each size N -> bench.py's committed format
        d, sizes = sys.argv[2], sys.argv[3:]
        print(json.dumps({
            "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes over `python3 bench.py --no-cpu "
                      "--points N` (tools/archive/r03_pmc.sh; keys: C4 point counts, kitti<N>, trace, track); hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE (gfx950 "
                      "FETCH_SIZE half-count correction, MI355X_MICROARCH.md); FETCH_SIZE counts memory-side requests "
                      "incl. Infinity-Cache hits",
            "points_per_gpu": {n: summarise(os.path.join(d, "p" + n)) for n in sizes}}, indent=1))
    else:
        print(json.dumps(summarise(sys.argv[1]), indent=1))


if __name__ == "__main__":
    main()
