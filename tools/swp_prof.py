"""Per-phase cycle counts of the stable scatter k_scatter_swp (lab build with
-DSMJ_SWP_PROF):

    make -C avx-sort-merge-joins_amd BUILD=build_prof LIBOUT=build_prof/lib EXTRA=-DSMJ_SWP_PROF
    SMJ_LIB_DIR=$PWD/avx-sort-merge-joins_amd/build_prof/lib python tools/swp_prof.py --width 8

Prints thread 0's average cycles per tile in each phase (barrier waits
included), over bench_partitioning's workload (2^27 tuples, 10 bits)."""
import argparse
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import smj  # noqa: E402

PHASES = ["rank", "barrier1", "owner scan + info", "prefetch + barrier2", "stage + barrier3",
          "wait loads", "segment stores", "barrier4", "carry"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--width", type=int, default=8)
    p.add_argument("--n", type=int, default=1 << 27)
    p.add_argument("--bits", type=int, default=10)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    lib = smj.Library(a.width)
    R = lib.empty(a.n)
    lib.dev_gen_pk(R, 0, a.n, 12345, with_payload=False)
    fan = 1 << a.bits
    out = lib.empty(a.n + fan * 64 // a.width)
    hist = torch.zeros(fan, dtype=torch.int64, device="cuda")
    off = torch.zeros_like(hist)
    f = lib.lib.smj_swp_prof
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 16)()
    lib.dev_partition(R, out, a.bits, 0, True, hist, off)  # warm-up
    torch.cuda.synchronize()
    f(buf)
    for _ in range(a.reps):
        lib.dev_partition(R, out, a.bits, 0, True, hist, off)
    torch.cuda.synchronize()
    f(buf)
    tile = 512 * (16 if a.width == 8 else 8)
    ntiles = (a.n + tile - 1) // tile * a.reps
    tot = sum(buf[k] for k in range(9))
    print(f"width {a.width}: {ntiles} tiles, {tot / ntiles:.0f} cycles per tile (thread 0)")
    for k, name in enumerate(PHASES):
        print(f"  {name:22s} {buf[k] / ntiles:8.0f}  {100.0 * buf[k] / tot:5.1f} %")


if __name__ == "__main__":
    main()
