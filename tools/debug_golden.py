"""Run the golden sort/join cases one by one outside pytest (no output capture),
printing progress, to locate an abort."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import torch  # noqa: F401,E402
import smj  # noqa: E402

for w in (8, 16):
    lib = smj.Library(w)
    g = np.load(os.path.join(ROOT, "tests", "golden", f"golden_w{w}.npz"))
    for n in (16, 255, 16384, 2 * 16384 + 77):
        print(f"w{w} sort n={n}", flush=True)
        got = lib.avxsort_tuples(g[f"sort_in_{n}"])
        want = g[f"sort_out_{n}"]
        print("  keys equal:", np.array_equal(got["key"], want["key"]), flush=True)
