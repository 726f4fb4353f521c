#!/usr/bin/env python3
"""Summarise a tools/profile.sh directory: per kernel, average duration from
the kernel trace and the average of every PMC counter per dispatch.  FETCH_SIZE
and WRITE_SIZE are reported in bytes (rocprofv3 reports KiB); HBM_READ_B is
FETCH_SIZE * 2 (gfx950 reports half of a wide coalesced read stream,
MI355X_MICROARCH.md §HBM)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("smj::", "")


def main(d):
    res = defaultdict(dict)
    st = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        for r in csv.DictReader(open(st)):
            k = short(r["Name"])
            res[k]["calls"] = int(r["Calls"])
            res[k]["avg_us"] = round(float(r["AverageNs"]) / 1e3, 2)
            res[k]["total_ms"] = round(float(r["TotalDurationNs"]) / 1e6, 3)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        acc = defaultdict(list)
        for r in csv.DictReader(open(f)):
            acc[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in acc.items():
            val = sum(v) / len(v)
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                val *= 1024
            res[k][c] = val
            if c == "FETCH_SIZE":
                res[k]["HBM_READ_B"] = 2 * val
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
