"""Multi-GPU m-way sort-merge join: one process per GPU over torch.distributed.

SURVEY.md §8(e).  The reference scales over the threads of one host: thread i
range-partitions its chunk of R and S, the co-partitions are redistributed so
that every thread owns whole key ranges, each thread sorts, merges and joins
its own ranges, and the per-thread counts are summed
(src/joins/sortmergejoin_multiway.c:195-330, threads joined in
src/joins/joincommon.c:140-260).  Here a rank plays the part of a thread:

1. range-partition the local slices of R and S on the device
   (``smj_dev_partition_range``: monotone digit of the key over the global key
   range, so partition p holds a contiguous key interval);
2. partition p is owned by rank ``p * world // F`` -- contiguous, balanced
   ownership, so every key lands on exactly one rank;
3. one ``all_to_all_single`` of the per-owner counts, then one of the rows
   (RCCL over xGMI on the GPU, gloo in the CPU tests): each rank receives its
   whole key ranges of R and S;
4. the local join (``smj_dev_join``), then an ``all_reduce`` of the count.

The class is written against a small ``ops`` interface (``empty``,
``partition_range``, ``join``) so that the orchestration the GPU bench runs is
the same code the CPU multi-process tests run (with host stand-ins for the
device ops that live in tests/).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def owners(fanout: int, world: int) -> torch.Tensor:
    """Owner rank of each of the `fanout` range partitions (contiguous)."""
    return torch.arange(fanout, dtype=torch.int64) * world // fanout


def send_counts(hist: torch.Tensor, world: int) -> torch.Tensor:
    """Rows this rank sends to every rank: per-partition counts summed by owner."""
    own = owners(hist.numel(), world).to(hist.device)
    out = torch.zeros(world, dtype=torch.int64, device=hist.device)
    return out.index_add_(0, own, hist.to(torch.int64))


class DeviceOps:
    """The device implementation of the ops interface (libsmj_hip*.so)."""

    def __init__(self, lib):
        self.lib = lib

    def empty(self, n):
        return self.lib.empty(n)

    def partition_range(self, inp, out, nbits, key_min, key_max, hist):
        self.lib.dev_partition_range(inp, out, nbits, key_min, key_max, hist)

    def join(self, R, S, sR, sS, count):
        # the local key range is a 1/world slice of the global one: let the
        # library sample it (key_max = 0) rather than plan for the global span
        self.lib.dev_join(R, S, sR, sS, count, 9, 1, 0)


class DistributedJoin:
    """One process per device; `step` joins the local slices of R and S
    against the slices on all other ranks and leaves the GLOBAL match count in
    `count` on every rank."""

    def __init__(self, ops, fanout_bits: int, key_min: int, key_max: int,
                 group=None):
        self.ops = ops
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.bits = fanout_bits
        self.fanout = 1 << fanout_bits
        if self.fanout < self.world:
            raise ValueError(f"fanout 2^{fanout_bits} < world size {self.world}")
        self.key_min = key_min
        self.key_max = key_max
        self.buf = {}
        self.last_recv = {}

    def _grow(self, key, n):
        b = self.buf.get(key)
        if b is None or b.shape[0] < n:
            b = self.ops.empty(max(n, 1))
            self.buf[key] = b
        return b[:n]

    def exchange(self, part, hist, key):
        """All-to-all of the range partitions; returns this rank's rows."""
        send = send_counts(hist, self.world)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        sl, rl = send.tolist(), recv.tolist()
        out = self._grow("recv" + key, sum(rl))
        dist.all_to_all_single(out, part, rl, sl, group=self.group)
        self.last_recv[key] = (sl, rl)
        return out

    def step(self, R, S, count):
        dev = count.device
        parts = []
        for key, rel in (("R", R), ("S", S)):
            part = self._grow("part" + key, rel.shape[0])
            hist = torch.zeros(self.fanout, dtype=torch.int64, device=dev)
            self.ops.partition_range(rel, part, self.bits, self.key_min,
                                     self.key_max, hist)
            parts.append(self.exchange(part, hist, key))
        rR, rS = parts
        sR = self._grow("sortR", rR.shape[0])
        sS = self._grow("sortS", rS.shape[0])
        self.ops.join(rR, rS, sR, sS, count)
        dist.all_reduce(count, group=self.group)
        return rR, rS
