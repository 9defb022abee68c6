#!/usr/bin/env python3
"""Per-kernel mean of every SQ counter collected by tools/sq_pass.sh (DIR/pass*/**/*counter_collection.csv)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "pass*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            acc[row["Kernel_Name"].split("(")[0]][row["Counter_Name"]].append(float(row["Counter_Value"]))
print(json.dumps({k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}, indent=1))
