#!/usr/bin/env python3
"""Time the multi-GPU exchange partition (smj_dev_partition_range[_packed])
at the partition widths of 1..8 GPUs (2^9..2^12 partitions), 128M tuples."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import torch  # noqa: E402
import smj  # noqa: E402


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    n = 128_000_000
    lib = smj.load(w)
    R = lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    out = lib.empty(n)
    words = torch.empty(n, dtype=torch.int64, device="cuda")
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    for bits in (9, 10, 11, 12):
        hist = torch.zeros(1 << bits, dtype=torch.int64, device="cuda")
        for packed in ((False, True) if w == 16 else (False,)):
            def f():
                if packed:
                    lib.dev_partition_range_packed(R, words, bits, 1, n, hist, bad)
                else:
                    lib.dev_partition_range(R, out, bits, 1, n, hist)
            f()
            torch.cuda.synchronize()
            lib.trace(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            torch.cuda.synchronize()
            k = lib.trace_read()
            lib.trace(False)
            print(f"bits {bits} packed {packed}: {e0.elapsed_time(e1) / 5:.3f} ms",
                  {a: round(b[0] / 5, 3) for a, b in k.items()}, flush=True)


if __name__ == "__main__":
    main()
