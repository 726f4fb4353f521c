#!/usr/bin/env python3
"""Tail of a rocprofv3 kernel trace as a timeline: every dispatch of the last
`ms` milliseconds with the idle gap before it, and the totals.

    python tools/timeline.py TRACE_CSV [ms] [OUT_CSV] [STEP_START]

With STEP_START (a kernel-name substring, e.g. k_join_begin) the window is the
last step instead: from that kernel's last dispatch up to the first idle gap
above 100 us (the host work after the timed loop).
"""
import csv
import sys


def main(src, ms=10.0, dst=None, start=None):
    rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
    if start:
        i = max(k for k, r in enumerate(rows) if start in r["Kernel_Name"])
        step = [rows[i]]
        for r in rows[i + 1:]:
            if int(r["Start_Timestamp"]) - int(step[-1]["End_Timestamp"]) > 100_000:
                break
            step.append(r)
        rows = step
    else:
        end = max(int(r["End_Timestamp"]) for r in rows)
        rows = [r for r in rows if int(r["Start_Timestamp"]) >= end - ms * 1e6]
    out = ["gap_before_us,duration_us,kernel"]
    prev = None
    gaps = busy = 0.0
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        gaps += max(gap, 0.0)
        busy += (e - s) / 1e3
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:90]
        out.append(f"{gap:.1f},{(e - s) / 1e3:.1f},{name}")
        prev = e if prev is None else max(prev, e)
    out.append(f"# {len(rows)} dispatches, busy {busy:.1f} us, gaps {gaps:.1f} us")
    text = "\n".join(out)
    if dst:
        open(dst, "w").write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 10.0,
         sys.argv[3] if len(sys.argv) > 3 else None,
         sys.argv[4] if len(sys.argv) > 4 else None)
