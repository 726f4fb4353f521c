#!/usr/bin/env python3
"""Kernel micro-benchmarks on device-resident synthetic data (one process per
configuration; per-kernel times from the library's HIP-event trace).

  python tools/microbench.py partition --n 134217728 --bits 10
  python tools/microbench.py sort --n 134217728 --width 8
  python tools/microbench.py join --n 128000000
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import torch  # noqa: E402
import smj  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("what", choices=["partition", "sort", "join", "merge", "copy"])
    p.add_argument("--n", type=int, default=1 << 27)
    p.add_argument("--width", type=int, default=16)
    p.add_argument("--bits", type=int, default=9)
    p.add_argument("--shift", type=int, default=0)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--dist", default="uniform")
    p.add_argument("--nohint", action="store_true",
                   help="join without the key-range hint (the reference API path)")
    a = p.parse_args()
    lib = smj.load(a.width)
    n = a.n
    R = lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345, with_payload=a.what != "sort")
    res = {"what": a.what, "n": n, "width": a.width,
           "variant": os.environ.get("SMJ_PT_VARIANT", "default")}
    if a.what == "copy":
        # achievable-bandwidth reference: device-to-device copy of one relation
        out = lib.empty(n)
        f = lambda: out.copy_(R)
        alg = 2 * n * a.width
    elif a.what == "partition":
        out = lib.empty(n + (1 << a.bits) * 64 // a.width)
        h = torch.zeros(1 << a.bits, dtype=torch.int64, device="cuda")
        o = torch.zeros_like(h)
        f = lambda: lib.dev_partition(R, out, a.bits, a.shift, True, h, o)
        alg = 2 * n * a.width
    elif a.what == "sort":
        out = lib.empty(n)
        f = lambda: lib.dev_sort(R, out)
        alg = 2 * n * a.width
    elif a.what == "merge":
        A = lib.empty(n // 2)
        B = lib.empty(n - n // 2)
        lib.dev_sort(R[: n // 2], A)
        lib.dev_sort(R[n // 2:], B)
        out = lib.empty(n)
        f = lambda: lib.dev_merge2(A, B, out)
        alg = 2 * n * a.width
    else:
        S = lib.empty(n)
        if a.dist == "uniform":
            lib.dev_gen_fk(S, 0, n, n, 54321)
        else:
            lib.dev_gen_zipf(S, 0, n, 0.75, 54321)
        sR, sS = lib.empty(n), lib.empty(n)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        kmax = 0 if a.nohint else n
        f = lambda: lib.dev_join(R, S, sR, sS, cnt, a.bits, 1, kmax)
        alg = 5 * 2 * n * a.width
    f()
    torch.cuda.synchronize()
    lib.trace(True)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        f()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    k = lib.trace_read()
    lib.trace(False)
    res["ms"] = round(dt * 1e3, 4)
    res["alg_GBps"] = round(alg / dt / 1e9, 1)
    res["kernels_ms"] = {name: round(v[0] / a.reps, 4) for name, v in k.items()}
    if a.what == "join":
        res["count"] = int(cnt.item())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
