#!/usr/bin/env python3
"""Time smj_dev_materialize over the device join's sorted outputs at
128M x 128M (PK/FK uniform and Zipf 0.75 S), 16- and 8-byte tuples.

Algorithmic bytes per call: read sorted R and S once and write every output
tuple once, (|R| + |S| + out) * w."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import torch  # noqa: E402
import smj  # noqa: E402


def run(w, dist, n=128_000_000, reps=5):
    lib = smj.load(w)
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    if dist == "uniform":
        lib.dev_gen_fk(S, 0, n, n, 54321)
    else:
        lib.dev_gen_zipf(S, 0, n, 0.75, 54321)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.dev_join(R, S, sR, sS, cnt, 9, 1, n)
    del R, S
    out = lib.empty(n)
    total = lib.dev_materialize(sR, sS, out)
    torch.cuda.synchronize()
    ok = total == n and torch.equal(out, sS)  # PK/FK: the sorted S, once
    lib.trace(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lib.dev_materialize(sR, sS, out)
    e1.record()
    torch.cuda.synchronize()
    k = lib.trace_read()
    lib.trace(False)
    ms = e0.elapsed_time(e1) / reps
    alg = (2 * n + total) * w
    return {"width": w, "dist": dist, "n": n, "outputs": total, "ok": bool(ok),
            "ms": round(ms, 3), "alg_GBps": round(alg / ms / 1e6, 1),
            "frac_of_8TBps": round(alg / ms / 1e6 / 8000, 3),
            "kernels_ms": {a: round(b[0] / reps, 3) for a, b in k.items()}}


def main():
    for w in (16, 8):
        for dist in ("uniform", "zipf"):
            print(json.dumps(run(w, dist)), flush=True)
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
