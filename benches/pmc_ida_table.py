#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/ida_pmc.sh output): per kernel, the
mean of each counter over its dispatches (counters summed over dimensions)."""
import collections
import csv
import json
import sys


def load(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"].split("(")[0].replace("void ", ""), r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


out = collections.defaultdict(dict)
for p in sys.argv[1:]:
    for k, cs in load(p).items():
        out[k].update(cs)
print(json.dumps(out, indent=1))
