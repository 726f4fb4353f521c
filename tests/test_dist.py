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
    """Host stand-ins for DeviceOps (16-byte tuples as (n, 2) int64 rows; the
    packed exchange as int64 words, like smj_dev_partition_range_packed; 48-bit
    words in two planes, like smj_dev_partition_range_planes)."""

    can_pack = True
    K = 3  # shards of the sampled layout (the device uses smj_sampled_shards())

    def __init__(self, orc, sampled=True, overflow=False, not_applicable=False, planes=True,
                 shards=True):
        self.orc = orc
        self.shards_ok = shards  # the exact form by exact shard regions (else histogram)
        self.can_sample = sampled
        self.can_planes = planes and sampled
        self.overflow = overflow  # report a region overflow from the sampled form
        self.not_applicable = not_applicable  # the sampled form returns False

    def shards(self):
        return self.K

    def sampled_capacity(self, n, nbits):
        return n + n // 8 + (1 << nbits) * self.K * 5 + 16

    def partition_range_sampled(self, inp, out, nbits, key_min, key_max, packed, seg_start,
                                seg_cnt, flags):
        """The device's sampled layout: partition p is K consecutive shard
        regions (shard = position / n * K), each followed by slack that holds
        garbage; partitions in order."""
        from smj.dist import range_digit
        F, K, n = 1 << nbits, self.K, inp.shape[0]
        if self.not_applicable:
            return False
        flags.zero_()
        if packed:
            words = torch.empty(n, dtype=torch.int64)
            hist = torch.zeros(F, dtype=torch.int64)
            bad = torch.zeros(1, dtype=torch.int32)
            if not self.partition_range_packed(inp, words, nbits, key_min, key_max, hist, bad):
                return False
            flags[1] = int(bad[0])
            # back in input order: the packed partition above sorted by digit
            d = range_digit(inp[:, 1], key_min, key_max, nbits)
            vals = torch.empty_like(words)
            vals[torch.argsort(d, stable=True)] = words
        else:
            vals = inp
        pos, order = self._place(inp, nbits, key_min, key_max, seg_start, seg_cnt, flags)
        out.fill_(-7)  # the slack must never be read
        out[pos] = vals[order]
        return True

    def partition_range_shards(self, inp, out, nbits, key_min, key_max, packed, seg_start,
                               seg_cnt, flags):
        """smj_dev_partition_range_shards: the sampled layout with exactly
        sized regions back to back (no slack, no overflow); `out` holds n."""
        from smj.dist import range_digit
        F, n = 1 << nbits, inp.shape[0]
        if not self.shards_ok or self.not_applicable:
            return False
        flags.zero_()
        if packed:
            words = torch.empty(n, dtype=torch.int64)
            hist = torch.zeros(F, dtype=torch.int64)
            bad = torch.zeros(1, dtype=torch.int32)
            if not self.partition_range_packed(inp, words, nbits, key_min, key_max, hist, bad):
                return False
            flags[1] = int(bad[0])
            d = range_digit(inp[:, 1], key_min, key_max, nbits)
            vals = torch.empty_like(words)
            vals[torch.argsort(d, stable=True)] = words
        else:
            vals = inp
        pos, order = self._place(inp, nbits, key_min, key_max, seg_start, seg_cnt, flags,
                                 slack=False)
        assert out.shape[0] >= n and (n == 0 or int(pos.max()) < n)
        out[pos] = vals[order]
        return True

    def _place(self, inp, nbits, key_min, key_max, seg_start, seg_cnt, flags, slack=True):
        """The sampled layout's element positions: partition p is K
        consecutive shard regions (shard = position / n * K), each followed by
        slack; returns (positions, input order) and fills the tables."""
        from smj.dist import range_digit
        F, K, n = 1 << nbits, self.K, inp.shape[0]
        d = range_digit(inp[:, 1], key_min, key_max, nbits)
        q = torch.arange(n) * K // max(n, 1)
        idx = d * K + q
        cnt = torch.bincount(idx, minlength=F * K)
        cap = cnt + (cnt // 8 + torch.arange(F * K) % 5 if slack else 0)
        start = torch.cumsum(cap, 0) - cap
        order = torch.argsort(idx, stable=True)
        first = torch.cumsum(cnt, 0) - cnt
        si = idx[order]
        pos = start[si] + torch.arange(n) - first[si]
        seg_start.copy_(start)
        seg_cnt.copy_(cnt)
        if self.overflow and slack:
            flags[0] = 1
        return pos, order

    def partition_range_planes(self, inp, out, nbits, key_min, key_max, seg_start, seg_cnt,
                               flags):
        """smj_dev_partition_range_planes: the sampled layout of 48-bit words
        w = (key - base) mod 2^s1 << (48 - s1) | payload, lo 32 bits in
        out.lo, hi 16 in out.hi; flags[1] or-s 1 / 2 / 4 (payload over 64 -
        s1 bits / key outside the range / payload over 48 - s1 bits)."""
        if self.not_applicable or nbits > 10:
            return False
        s1 = self._s1(key_min, key_max, nbits)
        if not 1 <= s1 <= 32:
            return False
        n = inp.shape[0]
        assert out.stride >= self.sampled_capacity(n, nbits) and out.stride % 32 == 0
        flags.zero_()
        L = max(key_max - key_min, 0).bit_length()
        k = inp[:, 1].numpy().astype(np.int64)
        pu = inp[:, 0].numpy().astype(np.int64).view(np.uint64)
        rel = (k - key_min).astype(np.uint64)
        bad = 0
        if ((k < key_min) | (rel > np.uint64((1 << L) - 1))).any():
            bad |= 2
        if (pu >> np.uint64(64 - s1)).any():
            bad |= 1
        if (pu >> np.uint64(48 - s1)).any():
            bad |= 4
        w = ((rel & np.uint64((1 << s1) - 1)) << np.uint64(48 - s1)) | \
            (pu & np.uint64((1 << (48 - s1)) - 1))
        pos, order = self._place(inp, nbits, key_min, key_max, seg_start, seg_cnt, flags)
        flags[1] = bad
        lo = torch.from_numpy((w & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32))
        hi = torch.from_numpy((w >> np.uint64(32)).astype(np.uint16).view(np.int16))
        out.lo.fill_(-7)  # the slack must never be read
        out.hi.fill_(-7)
        out.lo[pos] = lo[order]
        out.hi[pos] = hi[order]
        return True

    @staticmethod
    def _take(X, a, c):
        """Elements [a, a + c) of an exchange buffer (planes: as int64 words)."""
        from smj.dist import Planes
        if isinstance(X, Planes):
            lo = X.lo[a:a + c].numpy().view(np.uint32).astype(np.uint64)
            hi = X.hi[a:a + c].numpy().view(np.uint16).astype(np.uint64)
            return torch.from_numpy((lo | (hi << np.uint64(32))).view(np.int64))
        return X[a:a + c]

    def join_segmented_tables(self, R, nR, startR, cntR, S, nS, startS, cntS, bucket_bits,
                              key_lo, key_hi, sR, sS, count, packed=False, stage=None):
        """Gather every bucket's segments (bucket-major) and join the dense
        relations with the checks of join_segmented.  The staged form (the
        device sorts R's tiles first): a "R" call must precede the "REST" call
        of the same step, with the same tables; the join happens at "REST"."""
        if stage == "R":
            self.staged_r = (R.data_ptr(), startR.data_ptr(), nR)
            self.stage_calls = getattr(self, "stage_calls", 0) + 1
            return
        if stage == "REST":
            assert getattr(self, "staged_r", None) == (R.data_ptr(), startR.data_ptr(), nR)
            self.staged_r = None
        else:
            self.whole_calls = getattr(self, "whole_calls", 0) + 1
        from smj.dist import Planes
        planes = isinstance(R, Planes)
        assert planes == isinstance(S, Planes) and not (planes and packed)
        dense = []
        for X, n, st, ct in ((R, nR, startR, cntR), (S, nS, startS, cntS)):
            assert st.shape == ct.shape and st.shape[0] == 1 << bucket_bits
            rows, seg = [], torch.zeros(1, st.shape[0], dtype=torch.int64)
            for b in range(st.shape[0]):
                for j in range(st.shape[1]):
                    a, c = int(st[b, j]), int(ct[b, j])
                    if c:
                        rows.append(self._take(X, a, c))
                        seg[0, b] += c
            Xd = torch.cat(rows) if rows else self._take(X, 0, 0)
            assert Xd.shape[0] == n
            if not packed and not planes:
                assert bool((Xd[:, 1] != -7).all()), "a gap was read"  # keys are >= 1
            dense.append((Xd, seg))
        (Rd, segR), (Sd, segS) = dense
        self.join_segmented(Rd, segR, Sd, segS, bucket_bits, key_lo, key_hi, sR, sS, count,
                            packed=packed, bits=48 if planes else 64)

    def empty(self, n):
        return torch.empty((n, 2), dtype=torch.int64)

    def empty_words(self, n):
        return torch.empty(n, dtype=torch.int64)

    @staticmethod
    def _s1(key_min, key_max, bits):
        from smj.dist import plan_shift
        return plan_shift(key_min, key_max, bits)

    def partition_range_packed(self, inp, out, nbits, key_min, key_max, hist, bad):
        from smj.dist import range_digit
        s1 = self._s1(key_min, key_max, nbits)
        if not 1 <= s1 <= 32:
            return False
        L = max(key_max - key_min, 0).bit_length()
        k = inp[:, 1].numpy().astype(np.int64)
        p = inp[:, 0].numpy().astype(np.int64)
        rel = k - key_min
        if ((k < key_min) | (rel > (1 << L) - 1) | (p < 0) | (p >= (1 << (64 - s1)))).any():
            bad.fill_(1)
        d = range_digit(inp[:, 1], key_min, key_max, nbits)
        w = ((rel.astype(np.uint64) & np.uint64((1 << s1) - 1)) << np.uint64(64 - s1)) | \
            p.astype(np.uint64)
        order = torch.argsort(d, stable=True)
        out[: inp.shape[0]] = torch.from_numpy(w.view(np.int64))[order]
        hist.copy_(torch.bincount(d, minlength=1 << nbits))
        return True

    def _unpack(self, words, seg, key_lo, key_hi, bucket_bits, bits=64):
        s1 = self._s1(key_lo, key_hi, bucket_bits)
        b = torch.repeat_interleave(torch.arange(seg.shape[1]).repeat(seg.shape[0]),
                                    seg.reshape(-1)).numpy().astype(np.uint64)
        w = words.numpy().view(np.uint64)
        rel = (b << np.uint64(s1)) | (w >> np.uint64(bits - s1))
        rows = np.empty((len(w), 2), np.int64)
        rows[:, 1] = key_lo + rel.astype(np.int64)
        rows[:, 0] = (w & np.uint64((1 << (bits - s1)) - 1)).astype(np.int64)
        return torch.from_numpy(rows)

    def partition_range(self, inp, out, nbits, key_min, key_max, hist):
        from smj.dist import range_digit
        d = range_digit(inp[:, 1], key_min, key_max, nbits)
        order = torch.argsort(d, stable=True)
        out[: inp.shape[0]] = inp[order]
        hist.copy_(torch.bincount(d, minlength=1 << nbits))

    def join_segmented(self, R, segR, S, segS, bucket_bits, key_lo, key_hi, sR, sS, count,
                       packed=False, bits=64):
        from smj.dist import range_digit
        if packed or bits == 48:
            R = self._unpack(R, segR, key_lo, key_hi, bucket_bits, bits)
            S = self._unpack(S, segS, key_lo, key_hi, bucket_bits, bits)
        # the receive layout the device join relies on: source by source,
        # local bucket b holds exactly the keys of local digit b
        for rows, seg in ((R, segR), (S, segS)):
            assert seg.shape[1] == 1 << bucket_bits
            assert int(seg.sum()) == rows.shape[0]
            d = range_digit(rows[:, 1], key_lo, key_hi, bucket_bits)
            expect = torch.repeat_interleave(
                torch.arange(seg.shape[1]).repeat(seg.shape[0]), seg.reshape(-1))
            assert torch.equal(d, expect)
        r = R.numpy().reshape(-1).view(self.orc.dtype)
        s = S.numpy().reshape(-1).view(self.orc.dtype)
        c, a, b = self.orc.sortmergejoin(r, s)
        sR.copy_(torch.from_numpy(a.view(np.int64).reshape(-1, 2)))
        sS.copy_(torch.from_numpy(b.view(np.int64).reshape(-1, 2)))
        count.fill_(c)


def _worker(rank, world, port, n, q, s_payload="negative", mode="sampled", planes=True,
            wide=False, chunk_mb=None, staged=True, shards=True):
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import oracle
    import smj.dist as sd
    from smj.dist import DistributedJoin, Planes, owners, range_digit
    if chunk_mb is not None:  # every row message over the limit: chunked
        sd.CHUNK_BYTES = chunk_mb << 20

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
        # negative S payloads cannot be packed: R goes packed first, then both
        # as tuples; non-negative ones: both relations travel as packed words
        S["payload"] = -np.arange(total) if s_payload == "negative" else np.arange(total)
        if s_payload == "r_negative":  # R cannot be packed, S can
            R["payload"] = -np.arange(total)
        if s_payload == "wide48":  # 64-bit words hold S's payloads, 48-bit ones do not
            S["payload"] = (1 << 45) + np.arange(total)
        expect = orc.merge_join(np.sort(R, order="key"), np.sort(S, order="key"))

        def rows(t):
            return torch.from_numpy(t[rank * n:(rank + 1) * n].view(np.int64).reshape(-1, 2).copy())

        # mode: "sampled" (every rank), "exact", "mixed" (rank 0 exact, the
        # others sampled: receivers read either form), "overflow" (rank 1's
        # sampled regions overflow: every rank repeats exactly)
        ops = HostOps(orc, sampled=mode != "exact", overflow=mode == "overflow" and rank == 1,
                      not_applicable=mode == "mixed" and rank == 0, planes=planes,
                      shards=shards)
        if wide:  # 2^9 buckets per rank: 2^10 partitions across ranks, planes too
            dj = DistributedJoin(ops, 9, 1, total, n_hint=n, staged=staged)
            assert dj.pbits == 9 + (world > 1)
        else:
            dj = DistributedJoin(ops, 6, 1, total, staged=staged)
        # the layout both relations reach the local join in: planes when the
        # payloads fit 48-bit words on every rank (a rank where the planes do
        # not apply, or a sampled overflow, sends every rank to words)
        if s_payload in ("negative", "r_negative"):
            want = "tuples"
        elif s_payload == "wide48" or not ops.can_planes or mode in ("mixed", "overflow"):
            want = "words"
        else:
            want = "planes"
        assert dj.layout == ("planes" if ops.can_planes else "words")
        count = torch.zeros(1, dtype=torch.int64)
        for _ in range(2):  # second step reuses the grown buffers
            sR, sS = dj.step(rows(R), rows(S), count)
            assert int(count.item()) == expect
            assert dj.last_layout == want, (dj.last_layout, want)
            assert dj.last_packed == (want != "tuples")
        # the local join: two calls per step (R's tile stage while S's rows
        # fly, then the rest) across ranks unless staged=False, one call on
        # one rank
        if world > 1 and staged:
            assert getattr(ops, "stage_calls", 0) == 2 and getattr(ops, "whole_calls", 0) == 0
        else:
            assert getattr(ops, "whole_calls", 0) == 2 and getattr(ops, "stage_calls", 0) == 0
        # every key this rank sorted is in its contiguous share of the range
        own = owners(dj.fanout, world, dj.used)
        for got in (sR, sS):
            d = range_digit(got[:, 1], 1, total, dj.pbits)
            assert bool((own[d] == rank).all())
            k = got[:, 1]
            assert bool((k[1:] >= k[:-1]).all())
        # the row exchange alone (bench.py --op exchange repeats it): the last
        # step's transfer again lands the same rows in the same places, and the
        # own chunk is never copied
        xb, cap, cs, sl, rl, gmax = dj.last_rows["S"]
        assert isinstance(xb, Planes) == (want == "planes")
        remote = sum(rl) - rl[rank]
        planes_ = xb.planes if isinstance(xb, Planes) else (xb,)
        before = [p[:cap + remote].clone() for p in planes_]
        for p in planes_:
            p[cap:cap + remote] = -9
        dj._rows(xb, cap, cs, sl, rl, gmax).wait()
        # every rank agrees on the largest message (the RCCL rounds)
        t = torch.tensor([gmax])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        assert int(t) == gmax >= max(sl + rl)
        assert all(torch.equal(p[:cap + remote], b) for p, b in zip(planes_, before))
        # no row lost or duplicated
        sizes = torch.tensor([sR.shape[0], sS.shape[0]])
        dist.all_reduce(sizes)
        assert sizes.tolist() == [total, total]
        q.put((rank, "ok"))
    except BaseException as e:  # report to the parent
        q.put((rank, repr(e)))
        raise
    finally:
        from smj.dist import release_row_groups
        release_row_groups()
        dist.destroy_process_group()


def _sub_worker(rank, world, port, n, q):
    """A DistributedJoin on the sub-group {0, 1} of a world of 3: rank 2
    takes no part in it (the row communicator is created with
    use_local_synchronization, only by the members), and two joins on the
    same group share one cached row communicator."""
    import sys
    for p in (ROOT, PKG):
        sys.path.insert(0, p)
    import oracle
    from smj import dist as sd
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world)
    try:
        if rank < 2:
            sub = dist.new_group(ranks=[0, 1], use_local_synchronization=True)
            orc = oracle.Oracle(16)
            total = 2 * n
            orc.seed(12345)
            R = orc.create_relation_pk(total)
            R["payload"] = np.arange(total)
            orc.seed(54321)
            S = orc.create_relation_fk(total, total)
            S["payload"] = np.arange(total)
            expect = orc.merge_join(np.sort(R, order="key"), np.sort(S, order="key"))

            def rows(t):
                return torch.from_numpy(
                    t[rank * n:(rank + 1) * n].view(np.int64).reshape(-1, 2).copy())
            joins = [sd.DistributedJoin(HostOps(orc), 6, 1, total, group=sub) for _ in range(2)]
            assert joins[0].row_group is joins[1].row_group and len(sd._ROW_GROUPS) == 1
            count = torch.zeros(1, dtype=torch.int64)
            for dj in joins:
                dj.step(rows(R), rows(S), count)
                assert int(count.item()) == expect
            sd.release_row_groups()
            assert not sd._ROW_GROUPS
        q.put((rank, "ok"))
    except BaseException as e:
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_distributed_join_subgroup():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sub_worker, args=(r, 3, port, 4000, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    res = dict(q.get(timeout=5) for _ in range(3))
    for p in procs:
        if p.is_alive():
            p.kill()
    assert res == {r: "ok" for r in range(3)}, res


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,chunk_mb,s_payload,mode", [
    (1, None, "negative", "sampled"), (1, None, "rowid", "exact"),
    (1, None, "r_negative", "sampled"),
    (2, None, "negative", "sampled"), (3, None, "negative", "sampled"),
    (2, 0, "negative", "sampled"), (3, 0, "rowid", "sampled"),
    (2, None, "rowid", "sampled"), (3, None, "rowid", "sampled"),
    (2, None, "r_negative", "sampled"), (3, None, "r_negative", "sampled"),
    (2, None, "rowid", "exact"), (3, None, "negative", "exact"),
    (3, None, "rowid", "mixed"), (2, None, "negative", "mixed"),
    (3, None, "rowid", "overflow"), (2, None, "rowid", "sampled-onecall"),
    (3, None, "negative", "exact-onecall"), (2, None, "rowid", "exact-hist"),
    (3, None, "negative", "exact-hist"),
    (1, None, "wide48", "sampled"), (2, None, "wide48", "sampled"),
    (2, 0, "rowid", "sampled-noplanes"), (3, None, "rowid", "sampled-noplanes"),
    (1, None, "rowid", "sampled-noplanes"), (2, None, "rowid", "sampled-wide"),
    (2, None, "rowid", "sampled-noplanes-wide")])
def test_distributed_join_gloo(world, chunk_mb, s_payload, mode, oracles, monkeypatch):
    """chunk_mb 0: every row message over the chunk limit, so the exchange
    takes the chunked isend/irecv path (the one RCCL needs for >1 GiB).
    mode: the exchange partition's form (sampled with gaps, exact, a mix of
    the two, or a sampled overflow that sends every rank back to exact).
    s_payload "rowid": both relations exchanged as 48-bit planes (packed
    words with "-noplanes" ops, a rank where the planes do not apply, or an
    overflow); "negative": S cannot be packed, every rank falls back to tuples
    for both; "r_negative": R cannot be packed but S can (S goes again, as
    tuples); "wide48": S's payloads need 64-bit words (both go as words)."""
    staged = True
    shards = not mode.endswith("-hist")  # the exact form by histogram + scatter
    mode = mode.replace("-hist", "")
    if mode.endswith("-onecall"):  # the local join in one call (no staging)
        staged = False
        mode = mode[:-len("-onecall")]
    planes = not mode.endswith("-noplanes")  # ops without the 48-bit planes
    mode = mode.replace("-noplanes", "")
    wide = mode.endswith("-wide")  # 2^9 buckets per rank and an n hint
    mode = mode.replace("-wide", "")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 5000, q, s_payload, mode,
                                               planes, wide, chunk_mb, staged, shards))
             for r in range(world)]
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
    from smj.dist import owned, owners, plan_shift, send_counts
    assert owners(8, 2).tolist() == [0, 0, 0, 0, 1, 1, 1, 1]
    assert owners(8, 3).tolist() == [0, 0, 0, 1, 1, 1, 2, 2]
    # 5 of 8 partitions hold keys: those split, the empty top to the last rank
    assert owners(8, 2, 5).tolist() == [0, 0, 0, 1, 1, 1, 1, 1]
    assert owners(8, 3, 5).tolist() == [0, 0, 1, 1, 2, 2, 2, 2]
    for F, G, U in ((8, 3, 8), (4096, 8, 4096), (2048, 3, 2048), (64, 5, 64), (1024, 8, 977),
                    (1024, 3, 977), (16, 8, 3), (8, 8, 1)):
        own = owners(F, G, U)
        for g in range(G):
            lo, hi = owned(F, G, g, U)
            assert own[lo:hi].eq(g).all() and int(own.eq(g).sum()) == hi - lo
    # 1..2^30 in 4096 partitions of 2^18 keys (make_plan's s1)
    assert plan_shift(1, 1 << 30, 12) == 18
    h = torch.arange(8)
    assert send_counts(h, 2).tolist() == [6, 22]
    assert send_counts(h, 3).tolist() == [3, 12, 13]


def test_local_range_int64_edges():
    """Every rank's local plan has the global partition width (its buckets
    ARE the exchanged partitions) and stays inside int64, also for key
    ranges that reach INT64_MIN / INT64_MAX."""
    import sys
    sys.path.insert(0, PKG)
    from smj.dist import INT64_MAX, local_range, owned, plan_shift, used_parts
    lo64 = -(1 << 63)
    cases = [(1, 128_000_000), (lo64, INT64_MAX), (1, (1 << 62) + 1), (lo64, 5),
             (INT64_MAX - 1000, INT64_MAX), (7, 7)]
    for kmin, kmax in cases:
        for pbits, world in ((9, 1), (10, 2), (11, 3), (11, 8), (4, 5)):
            base, s1 = None, None
            for rank in range(world):
                b, klo, khi, lbits = local_range(kmin, kmax, pbits, world, rank)
                assert base is None or b == base  # one base on every rank
                base = b
                assert b <= kmin and lo64 <= klo <= khi <= INT64_MAX
                gs1 = plan_shift(b, kmax, pbits)
                assert plan_shift(klo, khi, lbits) == gs1  # same partition width
                p_lo, p_hi = owned(1 << pbits, world, rank, used_parts(kmin, kmax, pbits))
                if (p_lo << gs1) < (1 << max(kmax - kmin, 0).bit_length()):
                    assert klo == b + (p_lo << gs1)
                assert (1 << lbits) >= p_hi - p_lo
            assert kmax - base < (1 << max(kmax - kmin, 0).bit_length())


def test_partition_bits():
    """The exchange's partition width: bucket_bits + log2 G up to 2^10.  Since
    round 6 the 48-bit planes' scatter takes 2^10 partitions (16-byte
    segments), so no bit is given up for them; whether the planes are tried
    is planes_hold's: 48-bit words hold payloads as wide as the key span."""
    import sys
    sys.path.insert(0, PKG)
    from smj.dist import partition_bits, planes_hold
    n = 128_000_000
    assert partition_bits(9, 1, True, n) == 9
    assert partition_bits(9, 2, False, n) == 10
    assert partition_bits(9, 2, True, None) == 10
    assert partition_bits(9, 2, True, n) == 10
    assert partition_bits(9, 8, True, n) == 10
    assert partition_bits(6, 3, True, n) == 8
    assert partition_bits(9, 16, True, 1000) == 10
    assert partition_bits(8, 2, True, n, (1, 2 * n)) == 9
    assert partition_bits(8, 4, True, n, (1, 4 * n)) == 10
    assert partition_bits(8, 8, True, n, (1, 8 * n)) == 10
    # the benchmark's row ids (payloads within the key span): planes hold at
    # G = 1, 2, 4 (keys 1..512M at 2^10: s1 = 19, 29 payload bits), not at
    # G = 8 (keys 1..1024M: s1 = 20, 28 payload bits)
    assert planes_hold(1, n, 8) and planes_hold(1, 2 * n, 9) and planes_hold(1, 4 * n, 10)
    assert not planes_hold(1, 8 * n, 10)
    assert not planes_hold(1, 4 * n, 9) and not planes_hold(1, 8 * n, 9)


def test_next_layout_ladder():
    """DistributedJoin._next_layout: the layout and form an invalid attempt
    repeats with (bad / ovf are maxima over the ranks): planes -> words when
    only the 48-bit payload limit failed or a region overflowed (exact form),
    -> tuples when a payload needs more than 64 - s1 bits or a key lies
    outside the plan; words -> tuples on any bad bit; tuples stay."""
    import sys
    sys.path.insert(0, PKG)
    from smj.dist import (BAD_PAYLOAD, BAD_PAYLOAD48, BAD_RANGE, DistributedJoin)

    class J:
        _next_layout = DistributedJoin._next_layout

        def __init__(self, can_pack, sampled):
            self.can_pack, self.sampled = can_pack, sampled
    j = J(True, True)
    assert j._next_layout("planes", True, BAD_PAYLOAD48, 0) == ("words", True)
    assert j._next_layout("planes", True, BAD_PAYLOAD | BAD_PAYLOAD48, 0) == ("tuples", True)
    assert j._next_layout("planes", True, BAD_RANGE, 0) == ("tuples", True)
    assert j._next_layout("planes", True, 0, 1) == ("words", False)  # overflow: exact words
    assert j._next_layout("words", True, BAD_PAYLOAD, 0) == ("tuples", True)
    assert j._next_layout("words", True, 0, 1) == ("words", False)
    assert j._next_layout("tuples", True, 0, 1) == ("tuples", False)
    # 8-byte tuples (no 64-bit words) and an exact default form
    k = J(False, False)
    assert k._next_layout("planes", True, BAD_PAYLOAD48, 0) == ("tuples", False)
    assert k._next_layout("planes", True, 0, 1) == ("tuples", False)


@pytest.mark.parametrize("G", [2, 3, 4, 8])
@pytest.mark.parametrize("total", [None, 1_024_000_000, 128_000_000, 3_000_000])
def test_rank_key_balance(G, total):
    """Keys 1..total over G ranks (None: the weak-scaled benchmark, 128M per
    rank): every rank owns one contiguous key range of whole partitions, at
    most one partition more than its share of the partitions the keys reach,
    and on the benchmark's shapes the largest holds at most 1 % more keys
    than the mean (uniform keys: the rank loads).  The power-of-two partition
    space split evenly would give ranks 0-6 134M keys each and rank 7 85M at
    keys 1..1024M (1.048x the mean)."""
    bench_shape = total is None
    total = total or 128_000_000 * G
    import sys
    sys.path.insert(0, PKG)
    from smj.dist import local_range, owned, partition_bits, used_parts
    kmin, kmax = 1, total
    pbits = partition_bits(8, G, True, total // G, (kmin, kmax))
    F, U = 1 << pbits, used_parts(kmin, kmax, pbits)
    base = local_range(kmin, kmax, pbits, G, 0)[0]
    s1 = max((kmax - base).bit_length() - pbits, 0)
    keys = []
    for g in range(G):
        lo, hi = owned(F, G, g, U)
        a, b = max(base + (lo << s1), kmin), min(base + (hi << s1) - 1, kmax)
        keys.append(max(b - a + 1, 0))
    assert sum(keys) == total
    assert max(keys) <= -(-U // G) << s1, keys
    if bench_shape:
        assert max(keys) / (total / G) <= 1.01, keys
