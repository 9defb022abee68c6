#!/usr/bin/env python3
"""Roof evidence per kernel from tools/archive/r04_pmc.sh's passes (DIR/p<KEY>/{FETCH_SIZE,WRITE_SIZE,SQ}).

Per kernel and key:
* hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (FETCH_SIZE in KB, half-counted on gfx950 per
  MI355X_MICROARCH.md; memory-side requests, Infinity-Cache hits included);
* avg_launch_us from the same passes' kernel trace, dram_gbs = bytes / that duration, dram_frac of the 8 TB/s spec;
* SQ split (quad-cycle counters summed over the device): valu_issue_frac = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  (share of resident-wave time issuing VALU), wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt /
  barrier), issue_stall_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES; valu_busy_per_simd = 4 * SQ_ACTIVE_INST_VALU /
  (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs) (GRBM_GUI_ACTIVE is summed over the 8 XCDs) and the effective clock
  GRBM_GUI_ACTIVE / 8 / duration.
usage: pmc_roof.py DIR KEY..."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PEAK_GBS = 8000.0
SIMDS = 256 * 4


def counters(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[row["Kernel_Name"].split("(")[0]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return acc


def durations(d):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[row["Kernel_Name"].split("(")[0]].append(
                    (float(row["End_Timestamp"]) - float(row["Start_Timestamp"])) * 1e-3)
    return acc


def mean(v):
    return sum(v) / len(v) if v else None


def summarise(d):
    out = {}
    pas = {p: counters(os.path.join(d, p)) for p in ("FETCH_SIZE", "WRITE_SIZE", "SQ")}
    dur = durations(d)
    for k in sorted(set(pas["FETCH_SIZE"]) | set(pas["SQ"])):
        f = mean(pas["FETCH_SIZE"].get(k, {}).get("FETCH_SIZE", []))
        w = mean(pas["WRITE_SIZE"].get(k, {}).get("WRITE_SIZE", []))
        sq = {c: mean(v) for c, v in pas["SQ"].get(k, {}).items()}
        us = mean(dur.get(k, []))
        r = {"launches": len(dur.get(k, [])), "avg_launch_us": us}
        if f is not None and w is not None:
            b = 2.0 * f * 1024.0 + w * 1024.0
            r["hbm_bytes_per_launch"] = b
            if us:
                r["dram_gbs"] = b / (us * 1e-6) / 1e9
                r["dram_frac"] = r["dram_gbs"] / PEAK_GBS
        wc = sq.get("SQ_WAVE_CYCLES")
        if wc:
            for name, c in (("valu_issue_frac", "SQ_ACTIVE_INST_VALU"), ("any_issue_frac", "SQ_ACTIVE_INST_ANY"),
                            ("wait_frac", "SQ_WAIT_ANY"), ("issue_stall_frac", "SQ_WAIT_INST_ANY")):
                if sq.get(c) is not None:
                    r[name] = sq[c] / wc
        g = sq.get("GRBM_GUI_ACTIVE")
        if g and sq.get("SQ_ACTIVE_INST_VALU") is not None:
            r["valu_busy_per_simd"] = 4.0 * sq["SQ_ACTIVE_INST_VALU"] / (g / 8.0 * SIMDS)
            if us:
                r["effective_clock_mhz"] = g / 8.0 / us
        r["sq_raw"] = sq
        out[k] = r
    return out


def main():
    d, keys = sys.argv[1], sys.argv[2:]
    print(json.dumps({"source": "tools/archive/r04_pmc.sh: rocprofv3 --kernel-trace --stats --pmc, separate FETCH_SIZE / "
                                "WRITE_SIZE / SQ+GRBM passes over `python3 bench.py --no-cpu` (see pmc_roof.py)",
                      "keys": {k: summarise(os.path.join(d, "p" + k)) for k in keys}}, indent=1))


if __name__ == "__main__":
    main()
