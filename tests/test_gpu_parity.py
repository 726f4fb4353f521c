"""GPU parity of the HIP path against the CPU oracle (bit-exact).

Mirrors the reference's own Check suites (tests/check_partitioning.c,
check_avxsort.c, check_merge.c, check_scalarsort.c) but with exact
comparisons instead of sortedness-only asserts, on seeded inputs from the
reference generators (restated in oracle/smj_oracle.c and pinned by
tests/golden/), plus the edge cases those suites never hit: empty and tiny
inputs, ragged sizes, negative/full-range keys, heavy duplicates (Zipf), wide
digits.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def rand_tuples(width, n, seed, lo=None, hi=None):
    rng = np.random.default_rng(seed)
    dt = np.dtype([("payload", "<i4"), ("key", "<i4")]) if width == 8 else \
        np.dtype([("payload", "<i8"), ("key", "<i8")])
    t = np.zeros(n, dt)
    if width == 8:
        lo = -(1 << 31) if lo is None else lo
        hi = (1 << 31) - 1 if hi is None else hi
        t["key"] = rng.integers(lo, hi, n, dtype=np.int64)
        t["payload"] = rng.integers(-(1 << 31), (1 << 31) - 1, n, dtype=np.int64)
    else:
        lo = -(1 << 62) if lo is None else lo
        hi = (1 << 62) if hi is None else hi
        t["key"] = rng.integers(lo, hi, n, dtype=np.int64)
        t["payload"] = rng.integers(-(1 << 62), 1 << 62, n, dtype=np.int64)
    return t


# ------------------------------------------------------------- partitioning
PART_CASES = [(0, 4, 0), (1, 4, 0), (7, 2, 0), (1000, 4, 0), (20000, 10, 0),
              (100003, 7, 3), (300001, 10, 17), (65536, 12, 0),
              (200000, 13, 0), (70000, 16, 0)]


@pytest.mark.parametrize("n,nbits,shift", PART_CASES)
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_partition_matches_oracle(libs, oracles, width, n, nbits, shift, variant):
    orc, lib = oracles[width], libs[width]
    orc.seed(12345 + n)
    t = orc.create_relation_pk(n)
    t["payload"] = np.arange(n) + 5
    out, cnt, off = lib.partition(t, nbits, shift, variant)
    eout, ecnt, eoff = orc.partition(t, nbits, shift, padded=variant != 0)
    np.testing.assert_array_equal(cnt, ecnt)
    np.testing.assert_array_equal(off, eoff)
    if variant:
        assert np.all((off * width) % 64 == 0)  # check_partitioning.c:72-76
    for i in range(1 << nbits):
        a = out[off[i]:off[i] + cnt[i]]
        b = eout[eoff[i]:eoff[i] + ecnt[i]]
        assert np.array_equal(a, b), f"partition {i} differs"


def test_lds_order_selfcheck(libs, width):
    """The hardware property the stable partition's ranks rely on
    (k_scatter_swa): lane-ordered returns of colliding LDS atomic adds."""
    assert libs[width].selfcheck_lds_order() == 0


@pytest.mark.parametrize("n,nbits,shift,kind", [
    (5_000_003, 10, 0, "pk"),         # several tiles per workgroup chunk
    (3_000_017, 1, 0, "pk"),          # two partitions, long runs
    (2_500_000, 10, 0, "hot"),        # 90 % of the tuples in one partition
    (2_000_001, 9, 4, "dups"),        # few distinct keys: equal digits everywhere
    (777_777, 10, 22, "pk"),          # digit above every key: one partition
])
def test_partition_stable_large(libs, oracles, width, n, nbits, shift, kind):
    """Multi-tile chunks, carries that live over many tiles, skew: the stable
    write-combining scatter against the oracle, every partition in order."""
    orc, lib = oracles[width], libs[width]
    orc.seed(4242 + n)
    t = orc.create_relation_pk(n)
    rng = np.random.default_rng(n)
    if kind == "hot":
        hot = rng.random(n) < 0.9
        t["key"][hot] = 1 + (t["key"][hot] << nbits)  # digit 0 (key - 1 = k << nbits)
    elif kind == "dups":
        t["key"] = rng.integers(1, 40, n)
    t["payload"] = np.arange(n) - n // 2
    out, cnt, off = lib.partition(t, nbits, shift, 1)
    eout, ecnt, eoff = orc.partition(t, nbits, shift, padded=True)
    np.testing.assert_array_equal(cnt, ecnt)
    np.testing.assert_array_equal(off, eoff)
    mask = np.zeros(len(eout), bool)
    for o, c in zip(eoff.tolist(), ecnt.tolist()):
        mask[o:o + c] = True
    np.testing.assert_array_equal(out[:len(eout)][mask], eout[mask])


def test_partition_random_keys(libs, oracles, width):
    orc, lib = oracles[width], libs[width]
    t = rand_tuples(width, 123457, 7)
    out, cnt, off = lib.partition(t, 10, 5, 1)
    eout, ecnt, eoff = orc.partition(t, 10, 5, padded=True)
    np.testing.assert_array_equal(cnt, ecnt)
    for i in range(1024):
        assert np.array_equal(out[off[i]:off[i] + cnt[i]], eout[eoff[i]:eoff[i] + ecnt[i]])


# ------------------------------------------------------------------ sorting
SORT_SIZES = [0, 1, 2, 15, 16, 255, 4096, 16384, 49229, 3 * 16384 + 77, 1 << 20,
              1000003]


@pytest.mark.parametrize("n", SORT_SIZES)
def test_sort_pk(libs, oracles, width, n):
    orc, lib = oracles[width], libs[width]
    orc.seed(12345)
    t = orc.create_relation_pk(n)  # payload left 0 like bench_sort
    got = lib.avxsort_tuples(t)
    assert np.array_equal(got, orc.sort(t))


@pytest.mark.parametrize("n", [100, 5000, 262145, 1 << 21])
@pytest.mark.parametrize("kind", ["nonunique", "random", "narrow"])
def test_sort_other_inputs(libs, oracles, width, n, kind):
    orc, lib = oracles[width], libs[width]
    if kind == "nonunique":
        orc.seed(54321)
        t = orc.create_relation_nonunique(n, max(1, n // 3))
    elif kind == "random":
        t = rand_tuples(width, n, n)
    else:  # tiny key range, many payload ties to break
        t = rand_tuples(width, n, n + 1, 0, 40)
    for fn in ("avxsort_tuples", "avxsortmultiway_tuples", "scalarsort_tuples"):
        got = lib.avxsort_tuples(t, fn)
        assert np.array_equal(got, orc.sort(t)), fn


def test_sort_zipf_skew(libs, oracles, width):
    orc, lib = oracles[width], libs[width]
    orc.seed(54321)
    t = orc.create_relation_zipf(400000, 5000, 0.75)
    t["payload"] = np.random.default_rng(3).integers(0, 1000, len(t))
    got = lib.avxsort_tuples(t)
    assert np.array_equal(got, orc.sort(t))


@pytest.mark.parametrize("copies", [40, 100, 700])
def test_sort_long_equal_key_runs(libs, oracles, width, copies):
    """One relation, groups that fit in LDS but hold equal-key runs longer than
    the group pass fixes in place, payloads shuffled: the slot of the pair
    mode (two groups per iteration) that fails is queued for the skew path on
    its own while the other slot's group is written."""
    orc, lib = oracles[width], libs[width]
    rng = np.random.default_rng(copies)
    n = (1 << 20) + 37
    t = rand_tuples(width, n, 2)
    t["key"] = 1 + (rng.permutation(n) // copies)
    t["payload"] = rng.integers(0, 1 << 30, n)
    got = lib.avxsort_tuples(t)
    assert np.array_equal(got, orc.sort(t))


def non_nan_words(rng, n):
    """int64 patterns that are neither NaN nor -0 as IEEE doubles."""
    v = rng.integers(-(1 << 63), (1 << 63) - 1, 2 * n, dtype=np.int64)
    v = v[(((v >> 52) & 0x7FF) != 0x7FF) & (v != np.int64(-2 ** 63))]
    return v[:n]


def test_sort_int64_int32(libs, oracles, width):
    """avx* int64 entry points: IEEE-double order, like the reference's AVX
    networks (oracle pinned in test_oracle.py); scalar ones: integer order."""
    orc, lib = oracles[width], libs[width]
    rng = np.random.default_rng(11)
    v = non_nan_words(rng, 300001)
    for fn in ("avxsort_int64", "avxsortmultiway_int64"):
        assert np.array_equal(lib.sort_int(v, fn), orc.sort_int64_fp64(v)), fn
    assert np.array_equal(lib.sort_int(v, "scalarsort_int64"), np.sort(v))
    w = rng.integers(-(1 << 31), (1 << 31) - 1, 100003, dtype=np.int64).astype(np.int32)
    for fn in ("avxsort_int32", "scalarsort_int32"):
        assert np.array_equal(lib.sort_int(w, fn), np.sort(w)), fn


def test_int64_fp64_golden(libs, width):
    """This fork's signed (key, ptr) carriers (src/bench/sortbench.c:267-298)
    through avxsort_int64 / avx_merge_int64: the reference's own outputs."""
    import os
    from conftest import ROOT
    lib = libs[width]
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_int64.npz"),
                 allow_pickle=False) as d:
        g = {k: d[k] for k in d.files}
    for k in g:
        if k.startswith("carrier_in_"):
            n = k.rsplit("_", 1)[1]
            v = g[k]
            want = v[g[f"carrier_perm_{n}"]]
            for fn in ("avxsort_int64", "avxsortmultiway_int64"):
                assert np.array_equal(lib.sort_int(v, fn), want), (fn, n)
    v = g["words_in"]
    assert np.array_equal(lib.sort_int(v), v[g["words_perm"]])
    a, b = g["merge_a"], g["merge_b"]
    assert np.array_equal(lib.merge_int64(a, b),
                          np.concatenate([a, b])[g["merge_perm"]])


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 9), (5, 0), (70000, 33333)])
def test_merge_int64(libs, oracles, width, la, lb):
    orc, lib = oracles[width], libs[width]
    rng = np.random.default_rng(la + 7 * lb)
    a = orc.sort_int64_fp64(non_nan_words(rng, la))
    b = orc.sort_int64_fp64(non_nan_words(rng, lb))
    assert np.array_equal(lib.merge_int64(a, b), orc.merge_int64_fp64(a, b))
    a, b = np.sort(a), np.sort(b)
    assert np.array_equal(lib.merge_int64(a, b, "scalar_merge_int64"),
                          np.sort(np.concatenate([a, b])))


# ------------------------------------------------------------------ merging
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 5), (7, 0), (1, 1), (1000, 1),
                                   (4096, 4096), (100000, 3333), (77777, 200001)])
def test_merge2(libs, oracles, width, la, lb):
    orc, lib = oracles[width], libs[width]
    a = orc.sort(rand_tuples(width, la, la, 0, 5000))
    b = orc.sort(rand_tuples(width, lb, lb + 1, 0, 5000))
    exp = orc.merge(a, b)
    for fn in ("avx_merge_tuples", "scalar_merge_tuples"):
        assert np.array_equal(lib.avx_merge_tuples(a, b, fn), exp)


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 64, 128, 255, 256, 257, 1024, 2048])
def test_multiway_merge(libs, oracles, width, k):
    orc, lib = oracles[width], libs[width]
    rng = np.random.default_rng(k)
    maxlen = 3000 if k <= 256 else 300
    runs = [orc.sort(rand_tuples(width, int(rng.integers(0, maxlen)), 100 * k + i, 0, 10000))
            for i in range(k)]
    exp = orc.multiway_merge(runs)
    for fn in ("avx_multiway_merge", "scalar_multiway_merge"):
        out, n, consumed = lib.avx_multiway_merge(runs, fn)
        assert n == len(exp)
        assert consumed  # parts[] advanced like avx_multiwaymerge.c:268-272
        assert np.array_equal(out, exp)


def test_multiway_merge_skew_and_large(libs, oracles, width):
    """One hot key over every run (a value bucket larger than LDS: k_km_over
    ranks its elements by binary searches), keys spanning the whole signed range, empty
    runs between full ones, and the bench_multiwaymerge shape 64 x 65536."""
    orc, lib = oracles[width], libs[width]
    rng = np.random.default_rng(77)
    hot = []
    for i in range(8):
        t = rand_tuples(width, 5000, 300 + i, 7, 8)
        hot.append(orc.sort(t))
    lo, hi = (-2 ** 31, 2 ** 31 - 1) if width == 8 else (-2 ** 62, 2 ** 62)
    wide = [orc.sort(rand_tuples(width, int(rng.integers(0, 4000)), 400 + i, lo, hi))
            if i % 3 else np.zeros(0, lib.dtype) for i in range(40)]
    big = [orc.sort(rand_tuples(width, 65536, 500 + i, 1, 1 << 30)) for i in range(64)]
    for runs in (hot, wide, big):
        exp = orc.multiway_merge(runs)
        out, n, consumed = lib.avx_multiway_merge(runs)
        assert n == len(exp) and consumed
        assert np.array_equal(out, exp)


def test_multiway_merge_long_equal_runs(libs, oracles, width):
    """A value bucket within LDS whose equal-key run (480 copies of one key
    across 4 runs, payloads interleaved) is longer than the serial fix
    handles: the one-pass merge sorts that bucket in LDS (bitonic)."""
    orc, lib = oracles[width], libs[width]
    runs = []
    for i in range(4):
        t = rand_tuples(width, 3000, 900 + i, 0, 100000)
        t["key"][:120] = 50000
        runs.append(orc.sort(t))
    exp = orc.multiway_merge(runs)
    out, n, consumed = lib.avx_multiway_merge(runs)
    assert n == len(exp) and consumed
    assert np.array_equal(out, exp)


def test_dev_multiway_merge_back_to_back(libs, oracles, width):
    """The device k-way merge does not wait for the stream: merges of
    different run tables issued back to back (a hot-key bucket past LDS in
    every other one) all land, each in its own output."""
    import torch
    orc, lib = oracles[width], libs[width]
    cases = []
    for c in range(6):
        rng = np.random.default_rng(1000 + c)
        k = int(rng.integers(3, 80))
        runs = []
        for i in range(k):
            hi = 9 if c % 2 else 1 << 20
            runs.append(orc.sort(rand_tuples(width, int(rng.integers(0, 2000)), 50 * c + i, 7, hi)))
        exp = orc.multiway_merge(runs)
        druns = [lib.to_device(r) for r in runs]
        out = lib.empty(max(len(exp), 1))
        cases.append((druns, out, exp))
    for druns, out, _ in cases:
        lib.dev_multiway_merge(druns, out)
    torch.cuda.synchronize()
    for druns, out, exp in cases:
        assert np.array_equal(lib.to_host(out)[:len(exp)], exp)


# -------------------------------------------------------------------- joins
def test_merge_join_dups(libs, oracles, width):
    orc, lib = oracles[width], libs[width]
    for seed, n in [(1, 0), (2, 1), (3, 1000), (4, 200000)]:
        r = orc.sort(rand_tuples(width, n, seed, 0, max(1, n // 4)))
        s = orc.sort(rand_tuples(width, n + 3, seed + 9, 0, max(1, n // 4)))
        assert lib.merge_join(r, s) == orc.merge_join(r, s)


JOIN_CASES = [("pk_fk", 0, 0), ("pk_fk", 1, 1), ("pk_fk", 1000, 1000),
              ("pk_fk", 1 << 20, 1 << 20), ("pk_fk", 300000, 1200000),
              ("nonunique", 250000, 250000), ("zipf", 200000, 400000),
              ("random", 100000, 100000)]


def make_join_inputs(orc, width, kind, nr, ns):
    if kind == "pk_fk":
        orc.seed(12345)
        R = orc.create_relation_mway(nr, max(nr, 1))
        orc.seed(54321)
        S = orc.create_relation_mway(ns, max(nr, 1))
    elif kind == "nonunique":
        orc.seed(12345)
        R = orc.create_relation_nonunique(nr, nr)
        orc.seed(54321)
        S = orc.create_relation_nonunique(ns, nr)
    elif kind == "zipf":
        orc.seed(12345)
        R = orc.create_relation_mway(nr, nr)
        orc.seed(54321)
        S = orc.create_relation_zipf(ns, nr, 0.75)
    else:
        R = rand_tuples(width, nr, 5, -50000, 50000)
        S = rand_tuples(width, ns, 6, -50000, 50000)
    return R, S


@pytest.mark.parametrize("kind,nr,ns", JOIN_CASES)
def test_sortmergejoin_count(libs, oracles, width, kind, nr, ns):
    orc, lib = oracles[width], libs[width]
    R, S = make_join_inputs(orc, width, kind, nr, ns)
    exp, _, _ = orc.sortmergejoin(R, S)
    for nthr in (1, 8):
        assert lib.sortmergejoin_multiway(R, S, nthreads=nthr) == exp
    assert lib.sortmergejoin_multiway(R, S, nthreads=3) is None  # pow-2 check
    assert lib.sortmergejoin_multiway(R, S, nthreads=2, mpsm=True) == exp
    # m-pass (src/joins/sortmergejoin_multipass.c): sort both, then one scan
    assert lib.sortmergejoin_multiway(R, S, nthreads=4, algo="m-pass") == exp
    assert lib.sortmergejoin_multiway(R, S, nthreads=3, algo="m-pass") is None


@pytest.mark.parametrize("kind,nr,ns", JOIN_CASES[2:])
def test_device_join_sorted_outputs(libs, oracles, width, kind, nr, ns):
    import torch
    orc, lib = oracles[width], libs[width]
    R, S = make_join_inputs(orc, width, kind, nr, ns)
    exp, eR, eS = orc.sortmergejoin(R, S)
    dR, dS = lib.to_device(R), lib.to_device(S)
    sR, sS = lib.empty(nr), lib.empty(ns)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.dev_join(dR, dS, sR, sS, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == exp
    assert np.array_equal(lib.to_host(sR), eR)
    assert np.array_equal(lib.to_host(sS), eS)
    # inputs untouched
    assert np.array_equal(lib.to_host(dR), R)


# --------------------------------------------------------------- generators
def test_device_generators(libs, width):
    import torch
    lib = libs[width]
    n = 1 << 20
    t = lib.empty(n)
    lib.dev_gen_pk(t, 0, n, 12345)
    h = lib.to_host(t)
    assert np.array_equal(np.sort(h["key"]), np.arange(1, n + 1))
    assert np.array_equal(h["payload"], np.arange(n) + 5)
    # shards of one relation compose to the same relation
    a, b = lib.empty(n // 2), lib.empty(n - n // 2)
    lib.dev_gen_pk(a, 0, n, 12345)
    lib.dev_gen_pk(b, n // 2, n, 12345)
    assert np.array_equal(np.concatenate([lib.to_host(a), lib.to_host(b)]), h)
    z = lib.empty(n)
    lib.dev_gen_zipf(z, 0, 100000, 0.75, 54321)
    torch.cuda.synchronize()
    zk = lib.to_host(z)["key"]
    assert zk.min() >= 1 and zk.max() <= 100000
    counts = np.bincount(zk)
    top = np.sort(counts)[::-1]
    # Zipf(0.75): rank-1 share = 1/H(100000, 0.75)
    H = np.sum(1.0 / np.arange(1, 100001) ** 0.75)
    assert abs(top[0] / n - 1 / H) < 0.15 / H


@pytest.mark.parametrize("first,n,total,maxid,seed", [
    (0, 1 << 20, 1 << 20, 1 << 20, 12345),          # PK
    (777777, 300001, 128000000, 128000000, 12345),  # a shard of the 128M bench R
    (5, 200000, 1000000, 333333, 54321)])           # FK over a smaller domain
def test_device_generators_vs_restatement(libs, oracles, width, first, n, total, maxid, seed):
    """datagen.hip against its C restatement (oracle orc_dev_gen_*): the
    integer generators are bit-exact for every shard."""
    import torch
    lib, orc = libs[width], oracles[width]
    t = lib.empty(n)
    if maxid == total:
        lib.dev_gen_pk(t, first, total, seed)
    else:
        lib.dev_gen_fk(t, first, total, maxid, seed)
    torch.cuda.synchronize()
    assert np.array_equal(lib.to_host(t), orc.dev_gen_perm(n, first, total, maxid, seed))
    lib.dev_gen_pk(t, first, total, seed, with_payload=False)
    torch.cuda.synchronize()
    assert np.array_equal(lib.to_host(t), orc.dev_gen_perm(n, first, total, total, seed, False))


@pytest.mark.parametrize("theta,maxid", [(0.75, 100000), (0.75, 128000000), (0.25, 5000),
                                         (1.0, 1 << 20)])
def test_device_zipf_vs_restatement(libs, oracles, width, theta, maxid):
    """Zipf by rejection-inversion against the restatement: the sample
    decisions rest on libm log/exp/log1p/expm1, which the device library may
    round differently from glibc by an ulp, so an accept/reject near a
    boundary can flip; the draws must agree except for such rare flips
    (tolerance: 1 in 10^5 of the draws)."""
    import torch
    lib, orc = libs[width], oracles[width]
    n, first = 1 << 20, 4242
    z = lib.empty(n)
    lib.dev_gen_zipf(z, first, maxid, theta, 54321)
    torch.cuda.synchronize()
    got = lib.to_host(z)
    exp = orc.dev_gen_zipf(n, first, maxid, theta, 54321)
    assert np.array_equal(got["payload"], exp["payload"])
    bad = int(np.count_nonzero(got["key"] != exp["key"]))
    assert bad <= n // 100000, bad


# ------------------------------------------------------------ skew path
def _hot_inputs(orc, width, n, payload):
    """R = PK 1..n; half of S is key 7 (one group far beyond LDS: the split
    skew kernels), a tenth is key 1000 (a small skew group), the rest FK."""
    orc.seed(12345)
    R = orc.create_relation_mway(n, n)
    orc.seed(54321)
    S = orc.create_relation_mway(n, n)
    S["key"][: n // 2] = 7
    S["key"][n // 2: n // 2 + n // 10] = 1000
    if payload == "equal":
        S["payload"] = 0
    elif payload == "random64":  # no packed word holds them (16 B: LayP96)
        info = np.iinfo(S["payload"].dtype)
        rng = np.random.default_rng(64)
        R["payload"] = rng.integers(info.min, info.max, n, dtype=S["payload"].dtype)
        S["payload"] = rng.integers(info.min, info.max, n, dtype=S["payload"].dtype)
    else:  # descending payloads: equal-key runs come out of order
        S["payload"] = np.arange(n, 0, -1)
    return R, S


@pytest.mark.parametrize("payload", ["equal", "descending", "random64"])
@pytest.mark.parametrize("hint", [True, False])
def test_device_join_hot_keys(libs, oracles, width, payload, hint):
    """Groups too large for LDS: counting-sorted on the device (exact last
    digit); equal-key runs out of payload order fall back to the segmented
    merge sort.  With the key-range hint the host-planned path runs, without
    it the sampled plan.  Random full-width payloads take the skew kernels in
    the 12-byte elements at 16 bytes (LayP96)."""
    import torch
    orc, lib = oracles[width], libs[width]
    n = 1 << 20
    R, S = _hot_inputs(orc, width, n, payload)
    exp, eR, eS = orc.sortmergejoin(R, S)
    dR, dS = lib.to_device(R), lib.to_device(S)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    if hint:
        lib.dev_join(dR, dS, sR, sS, cnt, 9, 1, n)
    else:
        lib.dev_join(dR, dS, sR, sS, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == exp
    assert np.array_equal(lib.to_host(sR), eR)
    assert np.array_equal(lib.to_host(sS), eS)
    if payload == "random64" and width == 16:
        assert lib.last_layout() == "p96"


def test_device_join_keys_outside_hint(libs, oracles, width):
    """A key-range hint narrower than the data: keys outside clamp to the end
    digits (order kept), the last digit is then not exact and the clamped
    groups take the merge-sort and merge-join fallback."""
    import torch
    orc, lib = oracles[width], libs[width]
    n = 300000
    R, S = make_join_inputs(orc, width, "pk_fk", n, n)
    exp, eR, eS = orc.sortmergejoin(R, S)
    dR, dS = lib.to_device(R), lib.to_device(S)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.dev_join(dR, dS, sR, sS, cnt, 9, n // 4, n // 2)
    torch.cuda.synchronize()
    assert int(cnt.item()) == exp
    assert np.array_equal(lib.to_host(sR), eR)
    assert np.array_equal(lib.to_host(sS), eS)


@pytest.mark.parametrize("payload", ["rowid", "negative", "wide", "wide48", "p48off"])
def test_device_join_packed_words(libs, oracles, width, payload):
    """With a key-range hint the 16-byte join carries packed words (key offset
    in the bucket + payload) through the intermediate passes: 48-bit words in
    two planes first (LayP48), 64-bit words when a payload needs more than
    48 - s1 bits ("wide48": 2^44 here, s1 = 11), tuples when it needs more
    than 64 - s1 or is negative.  "p48off": the workspace's layouts without
    the 48-bit planes (smj_workspace_set_layouts: 64-bit words from the
    start).  The result is the same on every path."""
    if payload == "p48off":
        if width != 16:
            pytest.skip("packed words are the 16-byte layout")
        import smj
        libs[16].set_layouts(smj.LAYOUT_NO_P48)
        try:
            _packed_join_case(libs, oracles, width, "rowid")
        finally:
            libs[16].set_layouts(0)
        return
    _packed_join_case(libs, oracles, width, payload)


def _packed_join_case(libs, oracles, width, payload):
    import torch
    orc, lib = oracles[width], libs[width]
    n = 500_000
    R, S = make_join_inputs(orc, width, "pk_fk", n, n)
    if payload == "negative":
        S["payload"][n // 3] = -5
    elif payload == "wide" and width == 16:
        R["payload"][7] = np.int64(1) << 60
    elif payload == "wide48" and width == 16:
        R["payload"][7] = np.int64(1) << 44
    exp, eR, eS = orc.sortmergejoin(R, S)
    dR, dS = lib.to_device(R), lib.to_device(S)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for _ in range(2):
        lib.dev_join(dR, dS, sR, sS, cnt, 9, 1, n)
        torch.cuda.synchronize()
        assert int(cnt.item()) == exp
        assert np.array_equal(lib.to_host(sR), eR)
        assert np.array_equal(lib.to_host(sS), eS)


# ------------------------------------------- reference entry points, no hint
def _api_join_device(lib, dR, dS, nthreads=1):
    """sortmergejoin_multiway on relation_t over device-resident tuples (the
    library uses them in place, bench.py --api)."""
    import ctypes
    import smj
    os.environ["SMJ_QUIET"] = "1"
    rR = smj.Relation(dR.data_ptr(), dR.shape[0])
    rS = smj.Relation(dS.data_ptr(), dS.shape[0])
    cfg = smj.JoinConfig(nthreads, 128, int(lib.width == 16), int(lib.width == 16), 20 << 20, 2)
    res = lib.lib.sortmergejoin_multiway(ctypes.byref(rR), ctypes.byref(rS), ctypes.byref(cfg))
    total = int(res.contents.totalresults)
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    libc.free(res.contents.resultlist)
    libc.free(ctypes.cast(res, ctypes.c_void_p))
    return total


@pytest.mark.parametrize("case", ["pk_fk", "s_above", "r_negative", "wide_payload", "zipf"])
def test_api_join_size_guess(libs, oracles, width, case):
    """sortmergejoin_multiway takes no key-range hint: its plan is guessed from
    |R| (keys 1..|R|, the reference's own assumption,
    src/joins/sortmergejoin_multiway.c:372-376) and verified by the level-1
    scatter.  Keys outside the guess (above |R|, negative) send the join back
    to the exact key range; an unpackable payload (16 B) to tuples.  The count
    and the device-resident form must match the oracle either way."""
    import torch
    orc, lib = oracles[width], libs[width]
    n = 400_000
    R, S = make_join_inputs(orc, width, "zipf" if case == "zipf" else "pk_fk", n, n)
    if case == "s_above":
        S["key"][::1000] = n + 17
    elif case == "r_negative":
        R["key"][5] = -3
    elif case == "wide_payload" and width == 16:
        R["payload"][9] = np.int64(1) << 61
    exp, _, _ = orc.sortmergejoin(R, S)
    assert lib.sortmergejoin_multiway(R, S) == exp  # host buffers (staged)
    dR, dS = lib.to_device(R), lib.to_device(S)
    for _ in range(2):  # the second call reuses the context's workspace
        assert _api_join_device(lib, dR, dS) == exp
    torch.cuda.synchronize()
    assert np.array_equal(lib.to_host(dR), R)  # inputs untouched


@pytest.mark.parametrize("case", ["pk", "one_above", "negative", "wide_payload"])
def test_sort_size_guess(libs, oracles, width, case):
    """avxsort_tuples guesses keys 1..n (create_relation_pk's shape) and falls
    back to the exact key range when a key lies outside."""
    orc, lib = oracles[width], libs[width]
    n = 300_001
    orc.seed(777)
    t = orc.create_relation_pk(n)
    t["payload"] = np.arange(n) + 5
    if case == "one_above":
        t["key"][n // 2] = 3 * n
    elif case == "negative":
        t["key"][:10] = -np.arange(10)
    elif case == "wide_payload" and width == 16:
        t["payload"][3] = np.int64(1) << 62
    assert np.array_equal(lib.avxsort_tuples(t), orc.sort(t))


@pytest.mark.parametrize("nbits", [0, 1, 2, 3])
@pytest.mark.parametrize("n", [1, 513, 4097, 65536 + 511, 1 << 20])
@pytest.mark.parametrize("packed", [False, True])
def test_partition_range_sampled_small_bits(libs, oracles, width, nbits, n, packed):
    """smj_dev_partition_range_sampled at few partitions, where the sample's
    overestimate is largest against the per-region slack: every region must
    stay inside smj_sampled_capacity() (a canary after it stays intact) and
    the partitions must hold exactly the input, each key in its range."""
    import torch
    orc, lib = oracles[width], libs[width]
    if packed and width != 16:
        pytest.skip("packed words are the 16-byte layout")
    orc.seed(99 + n)
    t = orc.create_relation_pk(n)
    d_in = lib.to_device(t)
    F, K = 1 << nbits, lib.sampled_shards()
    cap = lib.sampled_capacity(n, nbits)
    canary = 4096
    if packed:
        buf = torch.full((cap + canary,), -7, dtype=torch.int64, device="cuda")
    else:
        buf = lib.empty(cap + canary)
        buf.fill_(-7)
    ss = torch.empty(F * K, dtype=torch.int64, device="cuda")
    sc = torch.empty(F * K, dtype=torch.int64, device="cuda")
    fl = torch.ones(2, dtype=torch.int32, device="cuda")
    if not lib.dev_partition_range_sampled(d_in, buf, nbits, 1, n, packed, ss, sc, fl):
        # packed words need 1 <= s1 <= 32: a one-key range has s1 = 0
        assert packed and int(n - 1).bit_length() - nbits < 1
        return
    torch.cuda.synchronize()
    assert bool((buf[cap:] == -7).all())
    if fl[0]:
        # a region overflowed (few workgroups fill few of a partition's shards:
        # the join then repeats the exact partition); nothing passed the buffer
        assert n < 1 << 20
        return
    assert fl.tolist() == [0, 0]
    assert int(sc.sum()) == n
    ssh, sch = ss.cpu().numpy(), sc.cpu().numpy()
    assert int((ssh + sch).max()) <= cap
    if packed:
        return  # the word layout is covered by the exchange tests
    h = lib.to_host(buf[:cap])
    keys = []
    s1 = max(int(n - 1).bit_length() - nbits, 0)  # make_plan over [1, n]
    for i in range(F * K):
        seg = h[ssh[i]:ssh[i] + sch[i]]
        p = i // K
        rel = seg["key"].astype(np.int64) - 1
        assert np.all(np.minimum(rel >> s1, F - 1) == p)
        keys.append(seg["key"])
    assert np.array_equal(np.sort(np.concatenate(keys)), np.arange(1, n + 1))


@pytest.mark.parametrize("nbits", [0, 3, 8, 10])
@pytest.mark.parametrize("n", [1, 4097, 1 << 20, 3_000_017])
@pytest.mark.parametrize("packed", [False, True])
def test_partition_range_shards(libs, oracles, width, nbits, n, packed):
    """smj_dev_partition_range_shards (the exchange's exact form across ranks,
    round 6): regions exactly sized and back to back, covering [0, n) with no
    gap, partition-major; every element in its partition's key range; the
    partitions together are exactly the input (16-byte tuples: the (key,
    payload) multiset; packed words: per partition the same sorted words as
    smj_dev_partition_range_packed writes)."""
    import torch
    orc, lib = oracles[width], libs[width]
    if packed and width != 16:
        pytest.skip("packed words are the 16-byte layout")
    orc.seed(7 + n + nbits)
    t = orc.create_relation_fk(n, 5 * n)
    t["payload"] = np.arange(n)
    d_in = lib.to_device(t)
    F, K = 1 << nbits, lib.sampled_shards()
    canary = 4096
    if packed:
        buf = torch.full((n + canary,), -7, dtype=torch.int64, device="cuda")
    else:
        buf = lib.empty(n + canary)
        buf.fill_(-7)
    ss = torch.empty(F * K, dtype=torch.int64, device="cuda")
    sc = torch.empty(F * K, dtype=torch.int64, device="cuda")
    fl = torch.ones(2, dtype=torch.int32, device="cuda")
    kmax = 5 * n
    if not lib.dev_partition_range_shards(d_in, buf, nbits, 1, kmax, packed, ss, sc, fl):
        assert packed and int(kmax - 1).bit_length() - nbits < 1
        return
    torch.cuda.synchronize()
    assert fl.tolist() == [0, 0]
    assert bool((buf[n:] == -7).all())  # nothing past n
    ssh, sch = ss.cpu().numpy(), sc.cpu().numpy()
    assert int(sch.sum()) == n
    # back to back: region i starts where region i - 1 ends
    assert ssh[0] == 0 and np.array_equal(ssh[1:], (ssh + sch)[:-1])
    s1 = max(int(kmax - 1).bit_length() - nbits, 0)
    if packed:
        words = torch.empty(n, dtype=torch.int64, device="cuda")
        hist = torch.zeros(F, dtype=torch.int64, device="cuda")
        bad = torch.zeros(1, dtype=torch.int32, device="cuda")
        assert lib.dev_partition_range_packed(d_in, words, nbits, 1, kmax, hist, bad)
        torch.cuda.synchronize()
        hs = hist.cpu().numpy()
        got, want = buf[:n].cpu().numpy(), words.cpu().numpy()
        pc = sch.reshape(F, K).sum(1)
        assert np.array_equal(pc, hs)
        o = 0
        for p in range(F):
            assert np.array_equal(np.sort(got[o:o + hs[p]]), np.sort(want[o:o + hs[p]])), p
            o += hs[p]
        return
    h = lib.to_host(buf[:n])
    for i in range(F * K):
        seg = h[ssh[i]:ssh[i] + sch[i]]
        rel = seg["key"].astype(np.int64) - 1
        assert np.all(np.minimum(rel >> s1, F - 1) == i // K)
    o = np.argsort(h["payload"], kind="stable")
    assert np.array_equal(h["payload"][o], np.arange(n))
    assert np.array_equal(h["key"][o], t["key"])


@pytest.mark.parametrize("kind,n,maxid,skip,first", [
    ("nonunique", 1 << 20, 1 << 20, 0, 0), ("nonunique", 1 << 20, 1000, 17, 0),
    ("nonunique", 300001, 1 << 20, 0, 700000), ("zipf", 1 << 20, 1 << 20, 0, 0),
    ("zipf", 250000, 100000, 5, 123457)])
def test_reference_generators_vs_oracle(libs, oracles, width, kind, n, maxid, skip, first):
    """refgen.hip against the oracle's glibc-driven restatement of the
    reference generators (pinned to the compiled reference by the golden
    vectors): a 1M-tuple relation, an inner shard [first, first + n) of a
    larger one, and `skip` rand() calls consumed before the relation."""
    import ctypes
    import torch
    lib, orc = libs[width], oracles[width]
    total = first + n + 1000
    libc = ctypes.CDLL(None)
    orc.seed(4242)
    for _ in range(skip):
        libc.rand()
    if kind == "nonunique":
        exp = orc.create_relation_nonunique(total, maxid)
    else:
        exp = orc.create_relation_zipf(total, maxid, 0.75)
    t = lib.empty(n)
    if kind == "nonunique":
        lib.dev_gen_nonunique(t, first, total, maxid, 4242, skip)
    else:
        lib.dev_gen_zipf_ref(t, first, maxid, 0.75, 4242, skip)
    torch.cuda.synchronize()
    assert np.array_equal(lib.to_host(t), exp[first:first + n])


def test_layout_hint_alternating_payloads(libs, oracles):
    """The workspace's layout hint (capi.hip device_bucket): joins of one
    shape whose payloads alternate between 48-bit, 64-bit-word and unpackable
    values.  A call after a payload fallback starts at the layout the last one
    reached (every 16th re-probes from the top); every call must still give
    the oracle's count and sorted relations, whichever layout it runs in."""
    import torch
    orc, lib = oracles[16], libs[16]
    n = 300_000
    R, S = make_join_inputs(orc, 16, "pk_fk", n, n)
    cases = {}
    for kind in ("rowid", "wide48", "negative"):
        r, s = R.copy(), S.copy()
        if kind == "wide48":
            r["payload"] += np.int64(1) << 44
        elif kind == "negative":
            s["payload"] = -1 - s["payload"]
        exp, eR, eS = orc.sortmergejoin(r, s)
        cases[kind] = (lib.to_device(r), lib.to_device(s), exp, eR, eS)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    seq = ["wide48", "wide48", "rowid", "negative", "negative", "rowid", "wide48"] * 3
    for kind in seq:
        dR, dS, exp, eR, eS = cases[kind]
        lib.dev_join(dR, dS, sR, sS, cnt, 9, 1, n)
        torch.cuda.synchronize()
        assert int(cnt.item()) == exp, kind
        assert np.array_equal(lib.to_host(sR), eR), kind
        assert np.array_equal(lib.to_host(sS), eS), kind


# ------------------------------------------------- 32-bit words (LayP32)
@pytest.mark.parametrize("case", ["pk", "tiny", "wide", "negative"])
def test_sort_p32_words(libs, oracles, width, case):
    """Sorts whose payloads fit 32 - s1 bits (the sort benchmark's payload 0)
    carry 32-bit words through the intermediate passes (LayP32); a wider
    payload sends the call to the next layout that holds it (48-bit words,
    or 12-byte elements for a negative 16-byte payload), and later calls of that shape
    start there.  The result is the oracle's on every path."""
    import torch
    orc, lib = oracles[width], libs[width]
    n = (1 << 20) + 77
    orc.seed(4242)
    t = orc.create_relation_pk(n)  # payload 0
    rng = np.random.default_rng(7)
    if case == "tiny":
        t["payload"] = rng.integers(0, 16, n)
    elif case == "wide":
        t["payload"][n // 3] = 1 << 28
    elif case == "negative":
        t["payload"][5] = -1
    want = {"pk": "p32", "tiny": "p32", "wide": "p48",
            "negative": "p48" if width == 8 else "p96"}[case]
    exp = orc.sort(t)
    lib.reset_workspace()  # no layout remembered
    d = lib.to_device(t)
    out = lib.empty(n)
    for call in range(2):
        lib.dev_sort(d, out)
        torch.cuda.synchronize()
        assert np.array_equal(lib.to_host(out), exp), (case, call)
        assert lib.last_layout() == want, (case, call, lib.last_layout())
    if case != "pk":
        # the shape that failed 32-bit words does not try them again, a new
        # shape does
        t2 = t[:n - 1].copy()
        t2["payload"] = 0
        d2, o2 = lib.to_device(t2), lib.empty(n - 1)
        lib.dev_sort(d2, o2)
        torch.cuda.synchronize()
        assert np.array_equal(lib.to_host(o2), orc.sort(t2))
        assert lib.last_layout() == "p32"
    import smj
    lib.set_layouts(smj.LAYOUT_NO_P32)
    lib.dev_sort(d, out)
    torch.cuda.synchronize()
    assert np.array_equal(lib.to_host(out), exp)
    assert lib.last_layout() != "p32"
    lib.set_layouts(0)


@pytest.mark.parametrize("n", [300_000, 4_000_000])
def test_join_p32_words(libs, oracles, width, n):
    """A join whose row-id payloads fit 32 - s1 bits (300K tuples: s1 = 11
    at 2^8 buckets) runs on 32-bit words; at 4M they do not and the join
    takes the 48-bit words.  Count and sorted relations as the oracle's."""
    import torch
    orc, lib = oracles[width], libs[width]
    R, S = make_join_inputs(orc, width, "pk_fk", n, n)
    exp, eR, eS = orc.sortmergejoin(R, S)
    lib.reset_workspace()
    dR, dS = lib.to_device(R), lib.to_device(S)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for call in range(2):
        lib.dev_join(dR, dS, sR, sS, cnt, 8, 1, n)
        torch.cuda.synchronize()
        assert int(cnt.item()) == exp
        assert np.array_equal(lib.to_host(sR), eR)
        assert np.array_equal(lib.to_host(sS), eS)
        assert lib.last_layout() == ("p32" if n < 1_000_000 else "p48"), (call, lib.last_layout())


@pytest.mark.parametrize("case", ["equal", "ragged", "wide_span", "no_p96"])
def test_join_p96(libs, oracles, case):
    """16-byte joins whose payloads no packed word holds (random 64-bit
    values, negative ones included) carry 12-byte elements through the
    intermediate passes (LayP96: the payload plane and a 32-bit key-offset
    plane) where the plan spans < 2^32 keys; relations of different sizes
    partition one at a time (one plane stride a launch).  A plan spanning
    2^32 keys or more, or SMJ_LAYOUT_NO_P96, takes the 16-byte tuples.
    Count and sorted relations as the oracle's on every path."""
    import torch
    import smj
    orc, lib = oracles[16], libs[16]
    nR, nS = {"ragged": (700_001, 1_300_003)}.get(case, (1_000_003, 1_000_003))
    R, S = make_join_inputs(orc, 16, "pk_fk", nR, nS)
    rng = np.random.default_rng(96)
    R["payload"] = rng.integers(-(1 << 63), (1 << 63) - 1, nR, dtype=np.int64)
    S["payload"] = rng.integers(-(1 << 63), (1 << 63) - 1, nS, dtype=np.int64)
    if case == "wide_span":
        R["key"][nR // 2] += np.int64(1) << 33  # one unmatched key far away
    exp, eR, eS = orc.sortmergejoin(R, S)
    lib.reset_workspace()
    lib.set_layouts(smj.LAYOUT_NO_P96 if case == "no_p96" else 0)
    try:
        dR, dS = lib.to_device(R), lib.to_device(S)
        sR, sS = lib.empty(nR), lib.empty(nS)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        for call in range(2):
            lib.dev_join(dR, dS, sR, sS, cnt, 8, 1, max(nR, nS))
            torch.cuda.synchronize()
            assert int(cnt.item()) == exp, call
            assert np.array_equal(lib.to_host(sR), eR), call
            assert np.array_equal(lib.to_host(sS), eS), call
            want = "tuples" if case in ("wide_span", "no_p96") else "p96"
            assert lib.last_layout() == want, (call, lib.last_layout())
    finally:
        lib.set_layouts(0)


def test_layout_hints_per_shape(libs, oracles):
    """A workspace alternating two join shapes whose payloads do not fit
    32-bit words (row ids + 2^30) tries the 32-bit words once per shape, not
    on every call: the workspace keeps each shape's hint (capi.hip
    device_bucket, Workspace::ShapeHint).  A call that skips them partitions
    each relation once (two k_scatter launches); every call gives the
    oracle's count and sorted relations in the 48-bit words."""
    import torch
    orc, lib = oracles[16], libs[16]
    cases = []
    for nR, nS in ((300_007, 300_007), (200_003, 500_009)):
        R, S = make_join_inputs(orc, 16, "pk_fk", nR, nS)
        R["payload"] += np.int64(1) << 30
        S["payload"] += np.int64(1) << 30
        exp, eR, eS = orc.sortmergejoin(R, S)
        cases.append((lib.to_device(R), lib.to_device(S), lib.empty(nR), lib.empty(nS),
                      nR, exp, eR, eS))
    lib.reset_workspace()
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    for call in range(6):
        dR, dS, sR, sS, nR, exp, eR, eS = cases[call % 2]
        lib.trace(True)
        lib.dev_join(dR, dS, sR, sS, cnt, 8, 1, nR)
        torch.cuda.synchronize()
        launches = lib.trace_read().get("k_scatter", (0, 0))[1]
        lib.trace(False)
        assert int(cnt.item()) == exp, call
        assert np.array_equal(lib.to_host(sR), eR), call
        assert np.array_equal(lib.to_host(sS), eS), call
        assert lib.last_layout() == "p48", (call, lib.last_layout())
        if call >= 2:
            assert launches == 2, (call, launches)
