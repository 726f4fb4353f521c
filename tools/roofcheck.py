#!/usr/bin/env python3
"""Check every bench line's roofline against the rocprofv3 kernel stats of the
SAME command (VERDICT r02 "Next round" #1).

    python tools/roofcheck.py DIR NAME [NAME ...] > DIR/roofcheck.json

DIR holds, per NAME, `NAME.json` (the line printed by `rocprofv3 --kernel-trace
--stats -- python3 bench.py ...`), `trace_NAME/**/run_kernel_stats.csv` (that
run's stats) and optionally `NAME_noprof.json` (the same bench command without
the profiler, same box).  For the line's dominant kernel it recomputes
    frac_rocprof = alg_bytes_per_launch / rocprof AverageNs / 8000 GB/s
and reports the relative gap to the line's own `roofline.frac` (HIP events),
plus the gap between the profiled and the unprofiled line."""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_traffic import short  # noqa: E402

PEAK = 8000.0


def stats(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        return {}
    out, main = {}, {}
    for r in csv.DictReader(open(files[0])):
        k = short(r["Name"])
        calls, tot = int(r["Calls"]), float(r["TotalDurationNs"])
        c0, t0 = out.get(k, (0, 0.0))
        out[k] = (c0 + calls, t0 + tot)
        # the instantiation with the most time (a layout probe that stops at
        # its first check, e.g. a 32-bit-word try whose payloads do not fit,
        # is another instantiation of a few microseconds)
        if tot > main.get(k, ("", 0, 0.0))[2]:
            main[k] = (r["Name"], calls, tot)
    return {k: (c, t / c, main[k]) for k, (c, t) in out.items()}


def load(p):
    try:
        with open(p) as f:
            return json.loads(f.read().strip().splitlines()[-1])
    except Exception:
        return None


def main():
    d, names = sys.argv[1], sys.argv[2:]
    res = {}
    for nm in names:
        line = load(os.path.join(d, nm + ".json"))
        st = stats(os.path.join(d, "trace_" + nm))
        e = {"line": nm + ".json"}
        if line and line.get("roofline"):
            rf = line["roofline"]
            k = rf["kernel"]
            e.update(kernel=k, line_frac=rf["frac"], line_avg_ms=rf["avg_launch_ms"],
                     alg_bytes_per_launch=rf["alg_bytes_per_launch"])
            if k in st:
                calls, avg_ns, (mname, mcalls, mtot) = st[k]
                fr = rf["alg_bytes_per_launch"] / avg_ns / PEAK
                e.update(rocprof_calls=calls, rocprof_avg_ms=round(avg_ns / 1e6, 4),
                         rocprof_frac=round(fr, 4))
                # the gap is taken on the main instantiation when others ran
                if mcalls != calls:
                    avg_ns = mtot / mcalls
                    fr = rf["alg_bytes_per_launch"] / avg_ns / PEAK
                    e.update(rocprof_main=mname, rocprof_main_calls=mcalls,
                             rocprof_main_avg_ms=round(avg_ns / 1e6, 4),
                             rocprof_main_frac=round(fr, 4))
                e.update(rel_gap=round(abs(fr - rf["frac"]) / rf["frac"], 4),
                         within_5pct=abs(fr - rf["frac"]) <= 0.05 * rf["frac"])
            e["ms_per_step"] = line.get("ms_per_step")
        nop = load(os.path.join(d, nm + "_noprof.json"))
        if nop and nop.get("roofline"):
            e.update(noprof_ms_per_step=nop["ms_per_step"], noprof_frac=nop["roofline"]["frac"],
                     noprof_avg_ms=nop["roofline"]["avg_launch_ms"])
        res[nm] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
