#!/usr/bin/env python3
"""One join step's timeline from a rocprofv3 kernel trace: the launches from
the last `k_join_begin` to the status readback after the group pass, each
with the idle gap before it.

    python tools/step_timeline.py TRACE_CSV [OUT_CSV]
"""
import csv
import sys


def main(src, dst=None):
    rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_join_begin" in r["Kernel_Name"]]
    if not starts:
        print("no k_join_begin in the trace", file=sys.stderr)
        return 1
    step = rows[starts[-1]:]
    # the step ends with its status readback (the first copy after the group
    # pass); what follows belongs to the bench's epilogue
    gs = [i for i, r in enumerate(step) if "k_groupsort" in r["Kernel_Name"]]
    if gs:
        for i in range(gs[-1] + 1, len(step)):
            if "copyBuffer" in step[i]["Kernel_Name"]:
                step = step[:i + 1]
                break
    out = ["gap_before_us,duration_us,kernel"]
    prev_end = None
    gaps = busy = 0.0
    for r in step:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = 0.0 if prev_end is None else max(s - prev_end, 0) / 1e3
        dur = (e - s) / 1e3
        gaps += gap
        busy += dur
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        out.append(f'{gap:.1f},{dur:.1f},"{name}"')
        prev_end = e if prev_end is None else max(prev_end, e)
    text = "\n".join(out) + "\n"
    if dst:
        open(dst, "w").write(text)
    else:
        sys.stdout.write(text)
    print(f"{len(step)} launches, {busy:.1f} us busy, {gaps:.1f} us of gaps", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
