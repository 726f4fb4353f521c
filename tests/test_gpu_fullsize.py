"""BASELINE configs at their full sizes, bit-compared with the oracle
restatement (oracle/smj_oracle.c, pinned to the reference by tests/golden/):

* bench_sort on 1 MI355X: 2^27 tuples through smj_dev_sort (the device form of
  avxsort_tuples, src/bench/sortbench.c:85-202);
* bench_partitioning on 1 MI355X: 2^27 tuples, 10 radix bits, shift 0,
  through smj_dev_partition (partition_relation_optimized: stable, 64-byte
  padded, src/bench/partitioningbench.c:128-196);
* sortmergejoin_multiway 128M x 128M: sorted R, sorted S and the count.

Inputs come from the device generators (keys 1..N permuted, the shape of
create_relation_pk) and are copied to the host for the oracle.  The oracle's
sorts are its stable LSD radix sort (orc_sort_tuples_radix, checked against
the qsort restatement in tests/test_oracle.py); the join's two run on two host
threads (ctypes drops the GIL).
"""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N27 = 1 << 27


def _free(torch):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("payload", [False, True], ids=["payload0", "payload"])
def test_bench_sort_full(libs, oracles, width, payload):
    import torch
    lib, orc = libs[width], oracles[width]
    R = lib.empty(N27)
    # bench_sort leaves the payload 0 (create_relation_pk); the second case
    # carries payloads 5+i so that the (key, payload) order is exercised too
    lib.dev_gen_pk(R, 0, N27, 12345, with_payload=payload)
    out = lib.empty(N27)
    lib.dev_sort(R, out)
    torch.cuda.synchronize()
    host_in = lib.to_host(R)
    got = lib.to_host(out)
    del R, out
    _free(torch)
    want = orc.sort_radix(host_in)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("payload", ["fits48", "wide48"])
def test_sort_p48_fallback(libs, oracles, width, payload):
    """The 48-bit layout (LayP48) and its fallbacks at a size where the plan's
    s1 is 17 (2^25 keys over 256 partitions): payloads below 2^(48 - 17) go as
    48-bit words; a payload of 2^31 and above (8-byte tuples: any negative
    int32, as the unsigned value their order uses; 16-byte: 2^40) sends the
    sort to tuples (8 B) or 64-bit words (16 B).  Bit-exact against the
    oracle either way."""
    import torch
    lib, orc = libs[width], oracles[width]
    n = 1 << 25
    R = lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 777, with_payload=True)
    if payload == "wide48":
        big = -(1 << 30) if width == 8 else (1 << 40)
        R[::4096, 0] = big
    out = lib.empty(n)
    lib.dev_sort(R, out)
    torch.cuda.synchronize()
    host_in = lib.to_host(R)
    got = lib.to_host(out)
    del R, out
    _free(torch)
    np.testing.assert_array_equal(got, orc.sort_radix(host_in))


@pytest.mark.parametrize("bits,shift", [(10, 0), (10, 7)])
def test_bench_partition_full(libs, oracles, width, bits, shift):
    import torch
    lib, orc = libs[width], oracles[width]
    fan = 1 << bits
    R = lib.empty(N27)
    lib.dev_gen_pk(R, 0, N27, 12345, with_payload=True)
    out = lib.empty(N27 + fan * 64 // width)
    hist = torch.zeros(fan, dtype=torch.int64, device="cuda")
    off = torch.zeros_like(hist)
    lib.dev_partition(R, out, bits, shift, True, hist, off)
    torch.cuda.synchronize()
    host_in = lib.to_host(R)
    got = lib.to_host(out)
    cnt, offs = hist.cpu().numpy(), off.cpu().numpy()
    del R, out
    _free(torch)
    want, wcnt, woff = orc.partition(host_in, bits, shift, True)
    np.testing.assert_array_equal(cnt, wcnt)
    np.testing.assert_array_equal(offs, woff)
    # every partition's tuples, in order (the padding between them is unset)
    mask = np.zeros(len(want), bool)
    for o, c in zip(woff.tolist(), wcnt.tolist()):
        mask[o:o + c] = True
    np.testing.assert_array_equal(got[:len(want)][mask], want[mask])


@pytest.mark.parametrize("dist_,fanout_bits", [
    ("uniform", 8),     # bench.py's plan: D1 = 8, D2 = 8, packed words at s1 = 19
    ("zipf_ref", 8),    # the Zipf line's S: create_relation_zipf after srand(54321)
    ("uniform", 9),
    ("zipf", 9),        # the fast rejection-inversion sampler (N1024 tests' S)
])
def test_headline_join_full_bitexact(libs, oracles, width, dist_, fanout_bits):
    """BASELINE configs[3] (R = S = 128M): the device join's sorted R, sorted S
    and count against the oracle's sortmergejoin on the same inputs, at the
    exact plan bench.py times (fanout_bits 8) and at 9."""
    import torch
    lib, orc = libs[width], oracles[width]
    n = 128_000_000
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    if dist_ == "uniform":
        lib.dev_gen_fk(S, 0, n, n, 54321)
    elif dist_ == "zipf_ref":
        lib.dev_gen_zipf_ref(S, 0, n, 0.75, 54321)
    else:
        lib.dev_gen_zipf(S, 0, n, 0.75, 54321)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.dev_join(R, S, sR, sS, cnt, fanout_bits, 1, n)
    torch.cuda.synchronize()
    count = int(cnt.item())
    hR, hS = lib.to_host(R), lib.to_host(S)
    gR, gS = lib.to_host(sR), lib.to_host(sS)
    del R, S, sR, sS
    _free(torch)
    with ThreadPoolExecutor(2) as ex:
        fR = ex.submit(orc.sort_radix, hR)
        fS = ex.submit(orc.sort_radix, hS)
        wR, wS = fR.result(), fS.result()
    assert count == orc.merge_join(wR, wS) == n
    np.testing.assert_array_equal(gR, wR)
    np.testing.assert_array_equal(gS, wS)


@pytest.mark.parametrize("payload,layout", [("wide48", "words"), ("full64", "p96")])
def test_headline_join_full_payload_layouts(libs, oracles, payload, layout):
    """The headline join (128M x 128M, 16-byte tuples, bench.py's plan) with
    payloads the 48-bit words cannot hold: 2^40 + row id (64-bit packed
    words) and random 64-bit values, negative ones included (12-byte
    elements, LayP96, through the persistent tile pass k_tilepass_p).  bench.py
    --payload sets the same payloads; sorted R, sorted S and the count
    against the oracle's full (key, payload) radix sort."""
    import torch
    import bench
    lib, orc = libs[16], oracles[16]
    n = 128_000_000
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    lib.dev_gen_fk(S, 0, n, n, 54321)
    bench.set_payloads(R, S, payload, 0)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.dev_join(R, S, sR, sS, cnt, 8, 1, n)
    torch.cuda.synchronize()
    assert lib.last_layout() == layout
    count = int(cnt.item())
    hR, hS = lib.to_host(R), lib.to_host(S)
    gR, gS = lib.to_host(sR), lib.to_host(sS)
    del R, S, sR, sS
    _free(torch)
    with ThreadPoolExecutor(2) as ex:
        fR = ex.submit(orc.sort_radix, hR)
        fS = ex.submit(orc.sort_radix, hS)
        wR, wS = fR.result(), fS.result()
    assert count == orc.merge_join(wR, wS) == n
    np.testing.assert_array_equal(gR, wR)
    np.testing.assert_array_equal(gS, wS)


def _checksum(torch, t):
    """Order-independent checksum of (n, 2) rows: wrapping int64 sums of the
    keys, the payloads and of two 64-bit avalanche hashes of each row (a row
    lost and another duplicated changes the hash sums unless the two rows'
    hashes collide: ~2^-64 per such pair)."""
    k = t[:, 1].to(torch.int64)
    p = t[:, 0].to(torch.int64)
    z = (k * 0x2545F4914F6CDD1D) ^ (p + 0x632BE59BD9B4E019)
    z = (z ^ (z >> 31)) * 0x1B873593CA5A7E35
    z = (z ^ (z >> 29)) * 0x3C79AC492BA7B653
    z = z ^ (z >> 32)
    h1 = int(z.sum())
    h2 = int((z * (z | 1)).sum())
    return (int(k.sum()), int(p.sum()), h1, h2)


@pytest.mark.parametrize("dist_", ["uniform", "zipf"])
def test_n1024_join_properties(libs, dist_):
    """BASELINE configs[4] on one GPU (its 1-GPU point): R = S = 1024M
    16-byte tuples, S uniform or Zipf 0.75.  The plan keeps 2^10 level-1
    partitions (the sampled, packed path) with up to 256 tiles per bucket.
    Count = |S|, outputs sorted by (key, payload), each a permutation of its
    input (checksums); the oracle would need minutes on the host at this size."""
    import torch
    lib = libs[16]
    n = 1_024_000_000
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    if dist_ == "uniform":
        lib.dev_gen_fk(S, 0, n, n, 54321)
    else:
        # the reference's own create_relation_zipf stream (genzipf.c:97-159,
        # bit-exact, refgen.hip), the relation configs[4] names
        t0 = time.time()
        lib.dev_gen_zipf_ref(S, 0, n, 0.75, 54321)
        torch.cuda.synchronize()
        print(f"[n1024] create_relation_zipf stream generated in {time.time() - t0:.1f} s")
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.dev_join(R, S, sR, sS, cnt, 9, 1, n)
    torch.cuda.synchronize()
    assert int(cnt.item()) == n
    for src, out in ((R, sR), (S, sS)):
        k = out[:, 1]
        dk = k[1:] - k[:-1]
        assert bool((dk >= 0).all())
        tie = dk == 0
        p = out[:, 0]
        assert bool((p[1:][tie] >= p[:-1][tie]).all())
        del dk, tie
        assert _checksum(torch, src) == _checksum(torch, out)
    del R, S, sR, sS
    _free(torch)


def test_distributed_join_n1024_one_rank():
    """The multi-GPU code path (smj/dist.py DistributedJoin: range partition,
    table exchange, the rank's own rows read in place, the segmented local
    join) on BASELINE configs[4]'s size, R = S = 1024M 16-byte tuples, S
    Zipf 0.75, over a one-rank RCCL group: count = |S|, both outputs sorted
    and permutations of their inputs (checksums), two steps (buffer reuse)."""
    import torch
    import torch.distributed as dist
    import smj
    from smj.dist import DeviceOps, DistributedJoin
    lib = smj.load(16)
    # one rank: an in-process store (no TCP port to collide with)
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(),
                            device_id=torch.device("cuda", 0))
    try:
        n = 1_024_000_000
        R, S = lib.empty(n), lib.empty(n)
        lib.dev_gen_pk(R, 0, n, 12345)
        lib.dev_gen_zipf_ref(S, 0, n, 0.75, 54321)  # create_relation_zipf's stream
        dj = DistributedJoin(DeviceOps(lib), 9, 1, n)
        count = torch.zeros(1, dtype=torch.int64, device="cuda")
        for _ in range(2):
            sR, sS = dj.step(R, S, count)
            torch.cuda.synchronize()
            assert int(count.item()) == n
        for src, out in ((R, sR), (S, sS)):
            assert out.shape[0] == n
            k = out[:, 1]
            assert bool((k[1:] >= k[:-1]).all())
            assert _checksum(torch, src) == _checksum(torch, out)
        del R, S, sR, sS, dj
    finally:
        dist.destroy_process_group()
    _free(torch)


def test_mpsm_n1024_zipf_ref(libs):
    """BASELINE configs[4] through the C API's multi-GPU join
    (smj_mgpu_join, the sortmergejoin_mpsm path: one RCCL rank per visible
    GPU): R = S = 1024M 16-byte tuples, S the reference's create_relation_zipf
    stream (theta 0.75, seed 54321).  Count = |S|, both outputs sorted and
    permutations of their inputs (checksums)."""
    import torch
    lib = libs[16]
    n = 1_024_000_000
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    lib.dev_gen_zipf_ref(S, 0, n, 0.75, 54321)
    torch.cuda.synchronize()
    try:
        c, sR, sS, counts, st = lib.mgpu_join(R, S, 0)
        assert c == n and st["replans"] == 0
        for src, out in ((R, sR), (S, sS)):
            k = out[:, 1]
            assert bool((k[1:] >= k[:-1]).all())
            assert _checksum(torch, src) == _checksum(torch, out)
        del sR, sS
    finally:
        lib.lib.smj_mgpu_release()
        del R, S
        _free(torch)


@pytest.mark.parametrize("width", [16, 8])
def test_mgpu_copy8_zipf_32m(libs, oracles, width):
    """The G = 8 rank protocol (smj_mgpu_join, ranks sharing the one GPU with
    device-copy collectives, SMJ_MG_COPY) at 32M x 32M with the reference's
    create_relation_zipf S (theta 0.75, seed 54321): count, and the ranks'
    sorted shares in rank order, bit-exact against the oracle."""
    import torch
    from smj import MG_COPY
    lib, orc = libs[width], oracles[width]
    n = 32 << 20
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    lib.dev_gen_zipf_ref(S, 0, n, 0.75, 54321)
    torch.cuda.synchronize()
    try:
        c, sR, sS, counts, st = lib.mgpu_join(R, S, 8, MG_COPY)
        assert counts[:, 0].sum() == n and counts[:, 1].sum() == n
        assert (counts > 0).all()  # every rank owns a share of both
        hR, hS = lib.to_host(R), lib.to_host(S)
        gR, gS = lib.to_host(sR), lib.to_host(sS)
    finally:
        lib.lib.smj_mgpu_release()
        del R, S
        _free(torch)
    with ThreadPoolExecutor(2) as ex:
        fR = ex.submit(orc.sort_radix, hR)
        fS = ex.submit(orc.sort_radix, hS)
        wR, wS = fR.result(), fS.result()
    assert c == orc.merge_join(wR, wS) == n
    np.testing.assert_array_equal(gR, wR)
    np.testing.assert_array_equal(gS, wS)
