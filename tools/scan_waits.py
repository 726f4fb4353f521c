#!/usr/bin/env python3
"""Scan the device assembly of the library for loads that wait alone.

For every kernel, count the global/buffer loads followed directly (before any
other load) by an `s_waitcnt vmcnt(0)`, and the flat / scratch memory
instructions.  A gather whose loads each wait alone, or that goes through
flat loads (they count against lgkmcnt too, so every LDS wait drains them),
shows up here.

    python tools/scan_waits.py [--min 6]

Compiles csrc/*.hip for gfx950 with --cuda-device-only -S into /tmp.
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "avx-sort-merge-joins_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def scan(path):
    fn, prev = None, None
    waits, flat = {}, {}
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*;\s*@", line)
        if m:
            fn, prev = m.group(1), None
            continue
        if fn is None:
            continue
        t = line.strip()
        if t.startswith(("flat_", "scratch_")):
            flat[fn] = flat.get(fn, 0) + 1
        if t.startswith(("global_load", "buffer_load")):
            prev = "L"
        elif t.startswith("s_waitcnt") and "vmcnt(0)" in t:
            if prev == "L":
                waits[fn] = waits.get(fn, 0) + 1
            prev = "W"
    return waits, flat


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min", type=int, default=6, help="report kernels with at least this many")
    a = ap.parse_args()
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(".hip"):
            continue
        for d in ("", "-DKEY_8B"):
            out = f"/tmp/scan_{f}{d}.s"
            subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950",
                            "--cuda-device-only", "-S", *([d] if d else []),
                            os.path.join(CSRC, f), "-o", out],
                           check=True, stderr=subprocess.DEVNULL)
            waits, flat = scan(out)
            tag = f + (" (16 B)" if d else " (8 B)")
            for k, v in sorted(waits.items(), key=lambda x: -x[1]):
                if v >= a.min:
                    print(f"{tag:28s} lone waits {v:4d}  {k[:100]}")
            for k, v in sorted(flat.items(), key=lambda x: -x[1]):
                print(f"{tag:28s} flat/scratch {v:3d}  {k[:100]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
