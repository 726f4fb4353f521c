#!/usr/bin/env python3
"""Average PMC counters per kernel over tools/lab_run.sh pmc* dirs (FETCH/WRITE in bytes)."""
import csv, collections, glob, sys
d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(d + "/pmc*/run_counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-48:]
        acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        if flt in k:
            val = sum(v) / len(v)
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                val *= 1024
            print(f"{k:50s} {c:24s} {val:.4g}")
