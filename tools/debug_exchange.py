#!/usr/bin/env python3
"""Isolate the exchange path at full size on one GPU: range partition of R
and S, then the segmented local join straight on the partition buffers (no
collective), checked for digit order, row checksums and the join count."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "avx-sort-merge-joins_amd"))
import torch  # noqa: E402
import smj  # noqa: E402
from smj.dist import plan_shift  # noqa: E402


def checksum(t):
    k = t[:, 1].to(torch.int64)
    p = t[:, 0].to(torch.int64)
    return int(k.sum()), int(p.sum()), int(((k * 0x9E3779B1) ^ p).sum())


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 128_000_000
    bits = 9
    lib = smj.load(w)
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    lib.dev_gen_fk(S, 0, n, n, 54321)
    parts, segs = [], []
    s1 = plan_shift(1, n, bits)
    for rel in (R, S):
        out = lib.empty(n)
        hist = torch.zeros(1 << bits, dtype=torch.int64, device="cuda")
        lib.dev_partition_range(rel, out, bits, 1, n, hist)
        torch.cuda.synchronize()
        d = (out[:, 1].to(torch.int64) - 1) >> s1
        print("partition: digits sorted", bool((d[1:] >= d[:-1]).all()),
              "hist ok", torch.equal(torch.bincount(d, minlength=1 << bits), hist),
              "checksum ok", checksum(out) == checksum(rel), flush=True)
        parts.append(out)
        segs.append(hist.view(1, -1).contiguous())
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    key_hi = 1 + (1 << (s1 + bits)) - 1
    lib.dev_join_segmented(parts[0], segs[0], parts[1], segs[1], bits, 1, key_hi, sR, sS, cnt)
    torch.cuda.synchronize()
    print("segmented join count", int(cnt.item()), "expect", n, flush=True)
    for src, o in ((R, sR), (S, sS)):
        k = o[:, 1].to(torch.int64)
        print("sorted", bool((k[1:] >= k[:-1]).all()), "checksum ok",
              checksum(o) == checksum(src), flush=True)


if __name__ == "__main__" and not os.environ.get("DIST"):
    main()


def dist_main(w, n):
    """The same through DistributedJoin on a one-rank RCCL group."""
    import torch.distributed as dist
    from smj.dist import DeviceOps, DistributedJoin
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    lib = smj.load(w)
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    lib.dev_gen_fk(S, 0, n, n, 54321)
    dj = DistributedJoin(DeviceOps(lib), 9, 1, n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for it in range(3):
        rR, segR, wR = dj._exchange(R, "R")
        rS, segS, wS = dj._exchange(S, "S")
        wR.wait()
        wS.wait()
        torch.cuda.synchronize()
        print(it, "recv == part:", torch.equal(rR, dj.buf["partR"][:n]),
              torch.equal(rS, dj.buf["partS"][:n]), "checksums",
              checksum(rR) == checksum(R), checksum(rS) == checksum(S), flush=True)
        sR = dj._grow("sortR", rR.shape[0])
        sS = dj._grow("sortS", rS.shape[0])
        dj.ops.join_segmented(rR, segR, rS, segS, dj.lbits, dj.key_lo, dj.key_hi, sR, sS, cnt)
        torch.cuda.synchronize()
        print(it, "count", int(cnt.item()), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__" and os.environ.get("DIST"):
    dist_main(int(sys.argv[1]), int(sys.argv[2]))
