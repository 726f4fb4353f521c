#!/usr/bin/env python3
"""Per-launch HBM traffic of every kernel from separate rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE each in its own pass, as MI355X_MICROARCH.md §HBM
prescribes).  rocprofv3 reports both in KiB; gfx950 counts half of a wide
coalesced read stream in FETCH_SIZE, so read bytes = 2 * FETCH_SIZE * 1024.

    python tools/make_traffic.py CFG_KEY FETCH_DIR WRITE_DIR [OUT_JSON]

merges {CFG_KEY: {kernel: {"read_B", "write_B", "bytes", "launches"}}} into
OUT_JSON (default profiles/pmc_traffic.json), the file bench.py reads."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


ALIAS = {"k_scatter_res": "k_scatter", "k_scatter_wc": "k_scatter",
         "k_scatter_u": "k_scatter", "k_sample_hist": "k_sample",
         "k_scatter_swa": "k_scatter", "k_hist_c": "k_hist",
         "k_scatter_swp": "k_scatter", "k_hist_p": "k_hist", "k_hist_v": "k_hist"}


def short(name):
    """Kernel symbol -> the name the library's HIP-event trace uses."""
    n = name.split("(")[0].replace("void ", "").replace("smj::", "")
    n = n.split("<")[0]
    return ALIAS.get(n, n)


def per_launch(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                acc[(short(r["Kernel_Name"]), r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
    out = defaultdict(list)
    for (k, _), v in acc.items():
        out[k].append(sum(v))  # summed over XCD/agent instances of one dispatch
    return {k: (sum(v) / len(v), len(v)) for k, v in out.items()}


def main():
    key, fdir, wdir = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    fetch, write = per_launch(fdir, "FETCH_SIZE"), per_launch(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        rb = 2 * fetch.get(k, (0, 0))[0] * 1024
        wb = write.get(k, (0, 0))[0] * 1024
        res[k] = {"read_B": round(rb), "write_B": round(wb), "bytes": round(rb + wb),
                  "launches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    d = {}
    if os.path.exists(out):
        d = json.load(open(out))
    d[key] = res
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: res}, indent=1))


if __name__ == "__main__":
    main()
