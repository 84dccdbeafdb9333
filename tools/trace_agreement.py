#!/usr/bin/env python3
"""Agreement of bench.py's HIP-event kernel time with the rocprofv3 kernel
trace of the same run: the timed route kernel's launches W+1 .. W+K (after W
warm-up launches) from <trace dir>/*kernel_trace.csv vs the bench line's
roofline.kernel_ms.
    python tools/trace_agreement.py <trace dir> <bench json line file> [W K]
"""
import csv
import glob
import json
import os
import sys

KERNEL = "k_walk<false, false, false>"


def main():
    tdir, bfile = sys.argv[1], sys.argv[2]
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    rows = []
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if KERNEL in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    ms = [(e - s) / 1e6 for s, e in rows]
    timed = ms[W:W + K]
    with open(bfile) as fh:
        line = json.loads([ln for ln in fh if ln.startswith("{")][-1])
    kms = line["roofline"]["per_gpu"]["kernel_ms"] if "per_gpu" in line["roofline"] \
        else line["roofline"]["kernel_ms"]
    mean = sum(timed) / len(timed)
    print(f"{KERNEL} launches under rocprofv3 (ms): {[round(x, 3) for x in ms]}")
    print(f"launches {W + 1}..{W + K} = the bench's {K} timed steps (after {W} warm-up): "
          f"mean {mean:.4f} ms")
    print(f"bench.py kernel_ms (HIP events, same run): {kms:.4f} ms")
    print(f"ratio {mean / kms:.4f}")


if __name__ == "__main__":
    main()
