"""GPU side of the multi-GPU join (smj/dist.py) on one device.

* The exchange is simulated on one GPU: every "source rank" range-partitions
  its slice with smj_dev_partition_range, the receive buffer of a rank is the
  concatenation of the sources' owned partitions, and smj_dev_join_segmented
  joins it; per-rank counts and sorted outputs are checked against the oracle.
* The same for the sampled exchange partition (regions with slack, gaps on
  the wire) and the table-driven local join.
* DistributedJoin itself runs over a one-rank NCCL (RCCL) group: the same
  code path bench.py --gpus N runs, with the collectives degenerate.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _inputs(orc, kind, n):
    orc.seed(12345)
    R = orc.create_relation_mway(n, n)
    orc.seed(54321)
    if kind == "zipf":
        S = orc.create_relation_zipf(n, n, 0.75)
    else:
        S = orc.create_relation_mway(n, n)
    return R, S


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kind", ["pk_fk", "zipf"])
@pytest.mark.parametrize("packed", [False, True])
def test_segmented_join_simulated_exchange(libs, oracles, width, world, kind, packed):
    import torch
    from smj.dist import DistributedJoin, ceil_log2, owned, plan_shift, used_parts
    orc, lib = oracles[width], libs[width]
    if packed and width != 16:
        pytest.skip("packed words are the 16-byte layout")
    n = 600_000
    R, S = _inputs(orc, kind, n)
    total, _, _ = orc.sortmergejoin(R, S)
    bucket_bits = 6
    pbits = min(bucket_bits + ceil_log2(world), 12)
    F = 1 << pbits
    s1 = plan_shift(1, n, pbits)
    # every source partitions its slice of R and S
    parts = {}
    for key, rel in (("R", R), ("S", S)):
        for s in range(world):
            sl = rel[s * n // world:(s + 1) * n // world]
            d_in = lib.to_device(sl)
            hist = torch.zeros(F, dtype=torch.int64, device="cuda")
            if packed:
                out = torch.empty(len(sl), dtype=torch.int64, device="cuda")
                bad = torch.zeros(1, dtype=torch.int32, device="cuda")
                assert lib.dev_partition_range_packed(d_in, out, pbits, 1, n, hist, bad)
                torch.cuda.synchronize()
                assert int(bad.item()) == 0
            else:
                out = lib.empty(len(sl))
                lib.dev_partition_range(d_in, out, pbits, 1, n, hist)
                torch.cuda.synchronize()
            parts[key, s] = (out, hist)
    got_total = 0
    for g in range(world):
        p_lo, p_hi = owned(F, world, g, used_parts(1, n, pbits))
        lbits = ceil_log2(max(p_hi - p_lo, 1))
        key_lo = 1 + (p_lo << s1)
        key_hi = key_lo + (1 << (s1 + lbits)) - 1
        recv, segs = {}, {}
        for key in ("R", "S"):
            rows, seg = [], torch.zeros(world, 1 << lbits, dtype=torch.int64, device="cuda")
            for s in range(world):
                out, hist = parts[key, s]
                start = int(hist[:p_lo].sum())
                cnt = int(hist[p_lo:p_hi].sum())
                rows.append(out[start:start + cnt])
                seg[s, :p_hi - p_lo] = hist[p_lo:p_hi]
            recv[key] = torch.cat(rows).contiguous()
            segs[key] = seg
        nR, nS = recv["R"].shape[0], recv["S"].shape[0]
        sR, sS = lib.empty(nR), lib.empty(nS)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        lib.dev_join_segmented(recv["R"], segs["R"], recv["S"], segs["S"], lbits,
                               key_lo, key_hi, sR, sS, cnt, packed=packed)
        torch.cuda.synchronize()
        # the oracle on this rank's share of the key range
        lo_k, hi_k = 1 + (p_lo << s1), 1 + (p_hi << s1)
        mR = R[(R["key"] >= lo_k) & (R["key"] < hi_k)] if g < world - 1 else R[R["key"] >= lo_k]
        mS = S[(S["key"] >= lo_k) & (S["key"] < hi_k)] if g < world - 1 else S[S["key"] >= lo_k]
        exp, eR, eS = orc.sortmergejoin(mR, mS)
        assert int(cnt.item()) == exp, (g, int(cnt.item()), exp)
        assert np.array_equal(lib.to_host(sR), eR)
        assert np.array_equal(lib.to_host(sS), eS)
        got_total += exp
    assert got_total == total


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("kind", ["pk_fk", "zipf"])
@pytest.mark.parametrize("layout", ["tuples", "words", "planes"])
@pytest.mark.parametrize("staged", [False, True], ids=["onecall", "staged"])
def test_sampled_exchange_simulated(libs, oracles, width, world, kind, layout, staged):
    """The sampled exchange partition (smj_dev_partition_range_sampled: K shard
    regions per partition, slack between them) simulated on one GPU: rank g
    receives from every source the chunk [start of its first owned region,
    start of the next rank's first region) -- gaps included -- and joins it
    through smj_dev_join_segmented_tables with the sources' region tables.
    staged: the join in two calls (SMJ_SEG_STAGE_R, then _REST), S's receive
    buffer holding garbage during the first (the multi-GPU join runs R's tile
    stage while S's rows are still in flight).  layout "planes": 48-bit words
    in two planes (smj_dev_partition_range_planes and
    smj_dev_join_segmented_planes), both widths."""
    import torch
    from smj.dist import Planes, ceil_log2, owned, plan_shift, used_parts
    orc, lib = oracles[width], libs[width]
    packed = layout == "words"
    if packed and width != 16:
        pytest.skip("packed words are the 16-byte layout")
    if staged and world == 1:
        pytest.skip("one rank: nothing in flight, the join is one call")
    n = 600_000
    R, S = _inputs(orc, kind, n)
    total, _, _ = orc.sortmergejoin(R, S)
    bucket_bits = 6
    pbits = min(bucket_bits + ceil_log2(world), 10)
    F, K = 1 << pbits, lib.sampled_shards()
    s1 = plan_shift(1, n, pbits)
    parts = {}
    for key, rel in (("R", R), ("S", S)):
        for s in range(world):
            sl = rel[s * n // world:(s + 1) * n // world]
            d_in = lib.to_device(sl)
            cap = lib.sampled_capacity(len(sl), pbits)
            ss = torch.empty(F * K, dtype=torch.int64, device="cuda")
            sc = torch.empty(F * K, dtype=torch.int64, device="cuda")
            fl = torch.ones(2, dtype=torch.int32, device="cuda")
            if layout == "planes":
                out = Planes(-(-cap // 32) * 32, device="cuda")
                out.buf.fill_(-7)
                assert lib.dev_partition_range_planes(d_in, out.buf, out.stride, pbits, 1, n,
                                                      ss, sc, fl)
            else:
                out = (torch.full((cap,), -7, dtype=torch.int64, device="cuda") if packed
                       else lib.empty(cap))
                assert lib.dev_partition_range_sampled(d_in, out, pbits, 1, n, packed, ss, sc,
                                                       fl)
            torch.cuda.synchronize()
            assert fl.tolist() == [0, 0]
            assert int(sc.sum()) == len(sl)
            ss, sc = ss.view(F, K), sc.view(F, K)
            # regions in (partition, shard) order, no overlap
            ends = (ss + sc).reshape(-1)
            assert bool((ends[:-1] <= ss.reshape(-1)[1:]).all())
            parts[key, s] = (out, ss, sc)
    got_total = 0
    for g in range(world):
        p_lo, p_hi = owned(F, world, g, used_parts(1, n, pbits))
        mine = p_hi - p_lo
        lbits = ceil_log2(max(mine, 1))
        key_lo = 1 + (p_lo << s1)
        key_hi = key_lo + (1 << (s1 + lbits)) - 1
        recv, tabs, used = {}, {}, {}
        for key in ("R", "S"):
            rows, tst, tct, base, nused = [], [], [], 0, 0
            for s in range(world):
                out, ss, sc = parts[key, s]
                c0 = int(ss[p_lo, 0])
                c1 = int(ss[p_hi, 0]) if p_hi < F else int((ss + sc).max())
                rows.append([p[c0:c1] for p in out.planes] if layout == "planes"
                            else out[c0:c1])
                tst.append(ss[p_lo:p_hi] - c0 + base)
                tct.append(sc[p_lo:p_hi])
                base += c1 - c0
                nused += int(sc[p_lo:p_hi].sum())
            if layout == "planes":  # the chunks back to back in both planes
                rb = Planes(-(-max(base, 1) // 32) * 32, device="cuda")
                for i in range(2):
                    rb.planes[i][:base].copy_(torch.cat([r[i] for r in rows]))
                recv[key] = rb
            else:
                recv[key] = torch.cat(rows).contiguous()
            st_ = torch.zeros(1 << lbits, world * K, dtype=torch.int64, device="cuda")
            ct_ = torch.zeros_like(st_)
            st_[:mine] = torch.stack(tst, 1).reshape(mine, world * K)
            ct_[:mine] = torch.stack(tct, 1).reshape(mine, world * K)
            tabs[key] = (st_.contiguous(), ct_.contiguous())
            used[key] = nused
        sR, sS = lib.empty(used["R"]), lib.empty(used["S"])
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        if layout == "planes":
            rR, rS = recv["R"], recv["S"]
            args = (rR.buf, rR.stride, used["R"], *tabs["R"], rS.buf, rS.stride, used["S"],
                    *tabs["S"], lbits, key_lo, key_hi, sR, sS, cnt)
            join = lib.dev_join_segmented_planes
            s_buf = rS.buf
        else:
            args = (recv["R"], used["R"], *tabs["R"], recv["S"], used["S"], *tabs["S"],
                    lbits, key_lo, key_hi, sR, sS, cnt)

            def join(*a, stage=None):
                lib.dev_join_segmented_tables(*a, packed=packed, stage=stage)
            s_buf = recv["S"]
        if staged:
            s_rows = s_buf.clone()
            s_buf.fill_(-3)  # S has not arrived yet
            join(*args, stage="R")
            torch.cuda.synchronize()
            s_buf.copy_(s_rows)
            join(*args, stage="REST")
        else:
            join(*args)
        torch.cuda.synchronize()
        lo_k, hi_k = 1 + (p_lo << s1), 1 + (p_hi << s1)
        mR = R[(R["key"] >= lo_k) & (R["key"] < hi_k)] if g < world - 1 else R[R["key"] >= lo_k]
        mS = S[(S["key"] >= lo_k) & (S["key"] < hi_k)] if g < world - 1 else S[S["key"] >= lo_k]
        exp, eR, eS = orc.sortmergejoin(mR, mS)
        assert int(cnt.item()) == exp, (g, int(cnt.item()), exp)
        assert np.array_equal(lib.to_host(sR), eR)
        assert np.array_equal(lib.to_host(sS), eS)
        got_total += exp
    assert got_total == total


def _init_one_rank(dist, torch):
    """A one-rank RCCL group over an in-process store: no TCP port (a port
    probed free can be taken by another process before the store binds it)."""
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(),
                            device_id=torch.device("cuda", 0))


@pytest.mark.parametrize("xsampled", ["1", "0"])
def test_distributed_join_one_rank_rccl(libs, width, xsampled, monkeypatch):
    """DistributedJoin over a one-rank RCCL group, device ops, 4M x 4M, with
    the sampled (1) and the exact (0) exchange partition."""
    import torch
    import torch.distributed as dist
    from smj.dist import DeviceOps, DistributedJoin
    lib = libs[width]
    _init_one_rank(dist, torch)
    try:
        n = 4_000_000
        R, S = lib.empty(n), lib.empty(n)
        lib.dev_gen_pk(R, 0, n, 12345)
        lib.dev_gen_fk(S, 0, n, n, 54321)
        dj = DistributedJoin(DeviceOps(lib, sampled=xsampled == "1"), 9, 1, n)
        count = torch.zeros(1, dtype=torch.int64, device="cuda")
        for _ in range(2):
            sR, sS = dj.step(R, S, count)
            torch.cuda.synchronize()
            assert int(count.item()) == n
            # one rank: 48-bit planes unless the exact partition is forced
            # (planes are a sampled form); else packed words at 16 bytes
            want = "planes" if xsampled == "1" else "words" if width == 16 else "tuples"
            assert dj.last_layout == want
        ref = torch.sort(S[:, 1].to(torch.int64)).values
        assert torch.equal(sS[:, 1].to(torch.int64), ref)
        assert torch.equal(sR[:, 1].to(torch.int64), torch.arange(1, n + 1, device="cuda"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("F,G,U", [(256, 1, 256), (512, 2, 512), (1024, 3, 1024), (1024, 8, 1024),
                                   (16, 16, 16), (1024, 8, 977), (1024, 3, 977), (512, 2, 489),
                                   (16, 4, 3)])
def test_exchange_table_kernels(libs, F, G, U):
    """smj_dev_xsend / smj_dev_xrecv (exchange.hip) against their framework-op
    statement in smj/dist.py (xsend_torch / xrecv_torch, which the gloo tests
    run): random region tables with empty regions, every rank's view; U of
    the F partitions reach the key range (the ranks split those)."""
    import torch
    from smj.dist import HEAD, owned, xrecv_torch, xsend_torch
    lib = libs[16]
    K = 8
    g = torch.Generator().manual_seed(F * 31 + G)
    cnt = torch.randint(0, 50, (F, K), generator=g, dtype=torch.int64)
    cnt[torch.rand(F, K, generator=g) < 0.2] = 0
    slack = torch.randint(0, 9, (F, K), generator=g, dtype=torch.int64)
    size = cnt + slack
    start = (torch.cumsum(size.reshape(-1), 0) - size.reshape(-1)).view(F, K)
    flags = torch.tensor([0, 1], dtype=torch.int32)  # [overflow, not packable]
    per = [owned(F, G, r, U)[1] - owned(F, G, r, U)[0] for r in range(G)]
    mlen = sum(HEAD + 2 * K * m for m in per)
    want_msg, want_chunk = torch.empty(mlen, dtype=torch.int64), torch.empty(2 * G, dtype=torch.int64)
    xsend_torch(start, cnt, flags, G, want_msg, want_chunk, U)
    d = {k: v.cuda() for k, v in dict(start=start, cnt=cnt, flags=flags).items()}
    msg = torch.full((mlen,), -5, dtype=torch.int64, device="cuda")
    chunk = torch.empty(2 * G, dtype=torch.int64, device="cuda")
    lib.dev_xsend(d["start"], d["cnt"], d["flags"], G, msg, chunk, U)
    torch.cuda.synchronize()
    assert torch.equal(msg.cpu(), want_msg) and torch.equal(chunk.cpu(), want_chunk)
    # rank r receives, from every source, that source's message to r (here:
    # the same sender's tables stand in for every source)
    offs = [sum(HEAD + 2 * K * m for m in per[:r]) for r in range(G)]
    for r in range(G):
        mine = per[r]
        one = want_msg[offs[r]:offs[r] + HEAD + 2 * K * mine]
        rmsg = one.repeat(G)
        nb = 1 << max(mine - 1, 0).bit_length()
        cap = int((start + size).max()) + 3
        wt, wc = torch.empty(nb, G * K, dtype=torch.int64), torch.empty(nb, G * K, dtype=torch.int64)
        ws = torch.empty(4 * G + 2, dtype=torch.int64)
        xrecv_torch(rmsg, want_chunk, G, r, mine, K, wt, wc, cap, ws)
        t = torch.full((nb, G * K), -1, dtype=torch.int64, device="cuda")
        c = torch.full((nb, G * K), -1, dtype=torch.int64, device="cuda")
        sm = torch.empty(4 * G + 2, dtype=torch.int64, device="cuda")
        lib.dev_xrecv(rmsg.cuda(), chunk, G, r, mine, K, t, c, cap, sm)
        torch.cuda.synchronize()
        assert torch.equal(t.cpu(), wt) and torch.equal(c.cpu(), wc) and torch.equal(sm.cpu(), ws)


def test_rccl_list_all_to_all_views(libs, monkeypatch):
    """The row exchange's RCCL form (smj/dist.py _rows: list all_to_all of
    views into one buffer, empty views for ranks with nothing to send, several
    rounds): on a one-rank group the call shape and the view semantics."""
    import torch
    import torch.distributed as dist
    _init_one_rank(dist, torch)
    try:
        buf = torch.arange(1000, dtype=torch.int64, device="cuda")
        out = torch.full((1000,), -1, dtype=torch.int64, device="cuda")
        for lo, hi in ((0, 300), (300, 300), (300, 1000)):  # a piece, an empty one, the rest
            dist.all_to_all([out[lo:hi]], [buf[lo:hi]], async_op=True).wait()
        torch.cuda.synchronize()
        assert torch.equal(out, buf)
        e = buf[:0]
        dist.all_to_all([e], [e], async_op=True).wait()
        torch.cuda.synchronize()
        # the 48-bit planes' pieces as _rows sends them: the lo plane as
        # int32, the hi plane's int16 as bytes (RCCL has no 16-bit integer)
        from smj.dist import Planes, _wire
        a, b = Planes(1024, device="cuda"), Planes(1024, device="cuda")
        a.buf.copy_(torch.arange(a.buf.numel(), dtype=torch.int32, device="cuda") * 7919)
        b.buf.fill_(-1)
        for lo, hi in ((0, 300), (300, 300), (300, 1000)):
            for pa, pb in zip(a.planes, b.planes):
                dist.all_to_all([_wire(pb[lo:hi])], [_wire(pa[lo:hi])], async_op=True).wait()
        torch.cuda.synchronize()
        for pa, pb in zip(a.planes, b.planes):
            assert torch.equal(pa[:1000], pb[:1000])
    finally:
        dist.destroy_process_group()


def test_partition_range_planes_flags(libs, width):
    """smj_dev_partition_range_planes' not-packable flags and its limits: a
    payload wider than 48 - s1 bits sets 4 (and 1 past 64 - s1 bits), a key
    outside the range 2; more than 2^10 partitions: not applicable (False,
    nothing launched).  Clean input: every element comes back unpacked from
    its region (the words restated here)."""
    import torch
    from smj.dist import Planes, plan_shift
    lib = libs[width]
    n, nbits, kmax = 100_000, 8, 1 << 30  # s1 = 22: payloads up to 2^26
    K = lib.sampled_shards()
    F = 1 << nbits
    s1 = plan_shift(1, kmax, nbits)
    g = torch.Generator().manual_seed(7)
    keys = torch.randint(1, kmax + 1, (n,), generator=g)
    pays = torch.randint(0, 1 << 20, (n,), generator=g)

    def run(k, p, bits=nbits):
        h = np.zeros(n, dtype=lib.dtype)
        h["key"], h["payload"] = k.numpy(), p.numpy()
        d = lib.to_device(h)
        cap = lib.sampled_capacity(n, bits)
        out = Planes(-(-cap // 32) * 32, device="cuda")
        ss = torch.empty((1 << bits) * K, dtype=torch.int64, device="cuda")
        sc = torch.empty_like(ss)
        fl = torch.full((2,), 9, dtype=torch.int32, device="cuda")
        ok = lib.dev_partition_range_planes(d, out.buf, out.stride, bits, 1, kmax, ss, sc, fl)
        torch.cuda.synchronize()
        return ok, out, ss, sc, fl.tolist()

    ok, out, ss, sc, fl = run(keys, pays)
    assert ok and fl == [0, 0] and int(sc.sum()) == n
    lo = out.lo.cpu().numpy().view(np.uint32).astype(np.uint64)
    hi = out.hi.cpu().numpy().view(np.uint16).astype(np.uint64)
    w = lo | (hi << np.uint64(32))
    got = []
    for i, (a, c) in enumerate(zip(ss.cpu().tolist(), sc.cpu().tolist())):
        x = w[a:a + c]
        rel = (np.uint64(i // K) << np.uint64(s1)) | (x >> np.uint64(48 - s1))
        got.append(np.stack([(rel + np.uint64(1)).astype(np.int64),
                             (x & np.uint64((1 << (48 - s1)) - 1)).astype(np.int64)], 1))
    got = np.concatenate(got)
    want = np.stack([keys.numpy(), pays.numpy()], 1)
    assert np.array_equal(got[np.lexsort((got[:, 1], got[:, 0]))],
                          want[np.lexsort((want[:, 1], want[:, 0]))])
    wide = pays.clone()
    wide[5] = 1 << (48 - s1)  # fits 64 - s1 bits, not 48 - s1
    assert run(keys, wide)[4][1] == 4
    if width == 16:  # 8-byte tuples carry 32-bit payloads: never past 64 - s1
        wider = pays.clone()
        wider[9] = 1 << (64 - s1)
        assert run(keys, wider)[4][1] == 5
    out_of_range = keys.clone()
    out_of_range[3] = kmax + 5
    assert run(out_of_range, pays)[4][1] & 2
    # 2^10 partitions apply since round 6 (16-byte segments), 2^11 do not
    ok10, _, _, sc10, fl10 = run(keys, pays, bits=10)
    assert ok10 and fl10 == [0, 0] and int(sc10.sum()) == n
    assert not run(keys, pays, bits=11)[0]
