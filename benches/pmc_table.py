#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, the mean per
dispatch of every counter (summed over the per-XCD/SE instances)."""
import collections
import csv
import json
import sys


def summarise(paths):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            per[(k, r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
            seen[k].add(r["Dispatch_Id"])
    out = collections.defaultdict(dict)
    for (k, c), d in per.items():
        out[k][c] = sum(d.values()) / len(d)
        out[k]["dispatches"] = len(seen[k])
    return out


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1:]), indent=1))
