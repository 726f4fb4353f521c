"""Multi-process test of the multi-GPU join orchestration (smj/dist.py) on CPU.

world_size 2 and 3 over gloo (127.0.0.1).  The device ops are replaced by host
stand-ins (a monotone range partition in torch, the oracle's join count), so
this checks the part that is host logic: partition ownership, the count and
row all-to-alls, buffer reuse across steps and the count all-reduce.  The GPU
run of the same class is bench.py --gpus N.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


class HostOps:
    """Host stand-ins for DeviceOps (16-byte tuples as (n, 2) int64 rows)."""

    def __init__(self, orc):
        self.orc = orc

    def empty(self, n):
        return torch.empty((n, 2), dtype=torch.int64)

    def partition_range(self, inp, out, nbits, key_min, key_max, hist):
        F = 1 << nbits
        span = key_max - key_min + 1
        d = ((inp[:, 1] - key_min).clamp(0, span - 1) * F) // span
        order = torch.argsort(d, stable=True)
        out[: inp.shape[0]] = inp[order]
        hist.copy_(torch.bincount(d, minlength=F))

    def join(self, R, S, sR, sS, count):
        r = R.numpy().reshape(-1).view(self.orc.dtype)
        s = S.numpy().reshape(-1).view(self.orc.dtype)
        c, a, b = self.orc.sortmergejoin(r, s)
        sR.copy_(torch.from_numpy(a.view(np.int64).reshape(-1, 2)))
        sS.copy_(torch.from_numpy(b.view(np.int64).reshape(-1, 2)))
        count.fill_(c)


def _worker(rank, world, port, n, q):
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import oracle
    from smj.dist import DistributedJoin, owners

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world)
    try:
        orc = oracle.Oracle(16)
        total = n * world
        # global relations, identical on every rank; each rank keeps its slice
        orc.seed(12345)
        R = orc.create_relation_pk(total)
        R["payload"] = np.arange(total)
        orc.seed(54321)
        S = orc.create_relation_zipf(total, total, 0.5)
        S["payload"] = -np.arange(total)
        expect = orc.merge_join(np.sort(R, order="key"), np.sort(S, order="key"))

        def rows(t):
            return torch.from_numpy(t[rank * n:(rank + 1) * n].view(np.int64).reshape(-1, 2).copy())

        dj = DistributedJoin(HostOps(orc), 6, 1, total)
        count = torch.zeros(1, dtype=torch.int64)
        for _ in range(2):  # second step reuses the grown buffers
            rR, rS = dj.step(rows(R), rows(S), count)
            assert int(count.item()) == expect
        # every received key is in this rank's contiguous share of the range
        F, span = 64, total
        own = owners(F, world)
        for got in (rR, rS):
            d = ((got[:, 1] - 1).clamp(0, span - 1) * F) // span
            assert bool((own[d] == rank).all())
        # no row lost or duplicated
        sizes = torch.tensor([rR.shape[0], rS.shape[0]])
        dist.all_reduce(sizes)
        assert sizes.tolist() == [total, total]
        q.put((rank, "ok"))
    except BaseException as e:  # report to the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_join_gloo(world, oracles):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 5000, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    res = dict(q.get(timeout=5) for _ in range(world))
    for p in procs:
        if p.is_alive():
            p.kill()
    assert res == {r: "ok" for r in range(world)}, res


def test_owners_and_send_counts():
    import sys
    sys.path.insert(0, PKG)
    from smj.dist import owners, send_counts
    assert owners(8, 2).tolist() == [0, 0, 0, 0, 1, 1, 1, 1]
    assert owners(8, 3).tolist() == [0, 0, 0, 1, 1, 1, 2, 2]
    h = torch.arange(8)
    assert send_counts(h, 2).tolist() == [6, 22]
    assert send_counts(h, 3).tolist() == [3, 12, 13]
