#!/usr/bin/env python3
"""Per-kernel averages of the PMC passes (rocprofv3 --pmc ... -o run --output-format csv)
under an output dir, e.g. tools/r05_walk_pmc.sh's."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "?")
            acc[name][row["Counter_Name"]].append((row.get("Dispatch_Id"), float(row["Counter_Value"])))
res = {}
for k, ctrs in acc.items():
    res[k] = {}
    for c, vals in ctrs.items():
        per = defaultdict(float)
        for d, v in vals:
            per[d] += v  # sum over XCD/SE instances of one dispatch
        res[k][c] = sum(per.values()) / len(per)
        # per dispatch in launch order: a kernel launched on different inputs in
        # one run (bench.py's C4 steps, then its random-source A/B) has one
        # value per input, which the mean above mixes
        res[k][c + "_by_dispatch"] = [per[d] for d in sorted(per, key=lambda x: int(x or 0))]
print(json.dumps(res, indent=1))
