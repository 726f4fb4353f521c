"""Pin the CPU oracle (oracle/smj_oracle.c) to the reference's golden vectors.

tests/golden/golden_w{8,16}.npz were produced by tests/golden/make_golden.py
from the reference itself (compiled from /root/reference by
oracle/build_ref.sh).  These tests run on CPU only; the GPU parity tests then
compare the HIP library with the oracle pinned here (and with the fixtures
directly, tests/test_gpu_parity.py::test_golden_*).

Ordering contract: 8-byte tuples sort as the packed 64-bit word
(key, payload), a total order, so outputs compare exactly.  The reference's
16-byte path sorts by key only and leaves equal keys in an implementation
order; those outputs compare keys exactly and the (key, payload) multiset.
"""
import os

import numpy as np
import pytest

from conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden")
PART_CASES = [(4, 0), (10, 0), (7, 3), (4, 20)]
SORT_NS = [16, 255, 16384, 2 * 16384 + 77]
KINDS = ["pk", "nonunique", "zipf"]


@pytest.fixture(scope="module", params=[8, 16], ids=["w8", "w16"])
def case(request, oracles):
    w = request.param
    with np.load(os.path.join(GOLD, f"golden_w{w}.npz"), allow_pickle=False) as d:
        gold = {k: d[k] for k in d.files}
    return w, oracles[w], gold


def canon(t):
    return np.sort(t, order=["key", "payload"])


def same_order(w, got, want):
    """Exact for 8-byte tuples; keys exact + canonical multiset for 16-byte."""
    assert len(got) == len(want)
    if w == 8:
        np.testing.assert_array_equal(got, want)
    else:
        np.testing.assert_array_equal(got["key"], want["key"])
        np.testing.assert_array_equal(canon(got), canon(want))


def test_generators(case):
    w, orc, g = case
    orc.seed(12345)
    np.testing.assert_array_equal(orc.create_relation_pk(1000), g["gen_pk"])
    orc.seed(54321)
    np.testing.assert_array_equal(orc.create_relation_nonunique(1000, 300), g["gen_nonunique"])
    orc.seed(777)
    np.testing.assert_array_equal(orc.create_relation_zipf(2000, 500, 0.75), g["gen_zipf"])
    orc.seed(99)
    np.testing.assert_array_equal(orc.create_relation_fk(1500, 400), g["gen_fk"])


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("nbits,shift", PART_CASES)
def test_partition(case, nbits, shift, variant):
    w, orc, g = case
    tag = f"part_b{nbits}_s{shift}_v{variant}"
    out, cnt, off = orc.partition(g["part_in"], nbits, shift, padded=variant > 0)
    np.testing.assert_array_equal(cnt, g[tag + "_cnt"])
    np.testing.assert_array_equal(off, g[tag + "_off"])
    dense = np.concatenate([out[off[i]:off[i] + cnt[i]] for i in range(1 << nbits)])
    # every variant of the reference partitioner is stable: exact order
    np.testing.assert_array_equal(dense, g[tag + "_dense"])


@pytest.mark.parametrize("n", SORT_NS)
def test_sort(case, n):
    w, orc, g = case
    same_order(w, orc.sort(g[f"sort_in_{n}"]), g[f"sort_out_{n}"])


@pytest.mark.parametrize("n", SORT_NS)
def test_sort_radix_golden(case, n):
    """The full-size checker (LSD radix) on the reference's sort vectors."""
    w, orc, g = case
    same_order(w, orc.sort_radix(g[f"sort_in_{n}"]), g[f"sort_out_{n}"])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sort_radix_matches_sort(case, seed):
    """sort_radix == sort (qsort on tup_cmp) bit for bit: signed keys and
    payloads, heavy duplicates, both halves of the words varying."""
    w, orc, _ = case
    rng = np.random.default_rng(seed)
    n = 200_003
    t = np.zeros(n, orc.dtype)
    info = np.iinfo(t["key"].dtype)
    t["key"] = rng.integers(info.min, info.max, n, endpoint=True)
    t["key"][: n // 2] = rng.integers(-50, 50, n // 2)
    t["payload"] = rng.integers(info.min, info.max, n, endpoint=True)
    t["payload"][n // 3:] = rng.integers(-3, 3, n - n // 3)
    np.testing.assert_array_equal(orc.sort_radix(t), orc.sort(t))


def test_merge(case):
    w, orc, g = case
    same_order(w, orc.merge(g["merge_a"], g["merge_b"]), g["merge_out"])


@pytest.mark.parametrize("k", [4, 64])
def test_multiway_merge(case, k):
    w, orc, g = case
    runs = np.split(g[f"mw{k}_runs"], np.cumsum(g[f"mw{k}_lens"])[:-1])
    assert len(runs) == k
    out = orc.multiway_merge(runs)
    assert int(g[f"mw{k}_n"][0]) == len(out)
    same_order(w, out, g[f"mw{k}_out"])


def test_merge_join(case):
    w, orc, g = case
    got = [orc.merge_join(g[f"mj{s}_R"], g[f"mj{s}_S"]) for s in (1, 2, 3)]
    np.testing.assert_array_equal(got, g["mj_counts"])


def test_merge_join_materialize(case):
    """The materialising restatement (joincommon.c:256-289) on the golden
    merge-join inputs: as many tuples as the reference counted, equal to an
    independent numpy construction (per key, the S run repeated |R_k| times)."""
    from test_gpu_materialize import numpy_materialize
    w, orc, g = case
    for s, count in zip((1, 2, 3), g["mj_counts"].tolist()):
        R, S = g[f"mj{s}_R"], g[f"mj{s}_S"]
        out = orc.merge_join_materialize(R, S)
        assert len(out) == count
        assert np.array_equal(out, numpy_materialize(R, S))


def join_inputs(gen, kind, nr, ns):
    """Same inputs as tests/golden/make_golden.py:join_inputs."""
    gen.seed(12345)
    R = gen.create_relation_nonunique(nr, nr) if kind == "nonunique" else gen.create_relation_pk(nr)
    gen.seed(54321)
    if kind == "pk":
        S = gen.create_relation_pk(ns)
    elif kind == "nonunique":
        S = gen.create_relation_nonunique(ns, nr)
    else:
        S = gen.create_relation_zipf(ns, nr, 0.75)
    return R, S


def test_sortmergejoin_counts(case):
    w, orc, g = case
    rows = g["join_cases"]
    seen = set()
    for kind_i, nr, ns, T, count in rows.tolist():
        if count < 0:  # the reference crashed on this case (make_golden.py)
            continue
        key = (kind_i, nr, ns)
        R, S = join_inputs(orc, KINDS[kind_i], nr, ns)
        c, sR, sS = orc.sortmergejoin(R, S)
        assert c == count, (KINDS[kind_i], nr, ns, T)
        if key not in seen:
            seen.add(key)
            assert np.all(np.diff(sR["key"]) >= 0) and np.all(np.diff(sS["key"]) >= 0)
            np.testing.assert_array_equal(canon(sR), canon(R))
    assert len(seen) == 4


# -- live cross-check against the compiled reference (this container only) ----
def _reference(w):
    import oracle
    if not oracle.reference_available(w):
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    return oracle.Reference(w)


@pytest.mark.parametrize("w", [8, 16])
def test_live_reference_partition_sort(w, oracles):
    ref, orc = _reference(w), oracles[w]
    rng = np.random.default_rng(7 + w)
    t = np.zeros(20000, orc.dtype)
    # the reference's AVX sort compares tuples as doubles
    # (src/avxsort/avxsort_core.h:2259-2266), so its domain is non-negative
    # keys below the NaN range; the device library sorts all signed keys
    t["key"] = rng.integers(0, 1 << 20, len(t))
    t["payload"] = np.arange(len(t))
    for nbits, shift in [(6, 0), (5, 9)]:
        o1, c1, f1 = ref.partition(t, nbits, shift, 1)
        o2, c2, f2 = orc.partition(t, nbits, shift, padded=True)
        np.testing.assert_array_equal(c1, c2)
        np.testing.assert_array_equal(f1, f2)
        np.testing.assert_array_equal(o1[: f1[-1] + c1[-1]], o2[: f2[-1] + c2[-1]])
    fn = "avxsort_tuples" if w == 8 else "scalarsort_tuples"
    same_order(w, orc.sort(t), ref.sort(t, fn))


# ------------------------------------------- int64 items in the AVX (FP64) order
def int64_gold():
    with np.load(os.path.join(GOLD, "golden_int64.npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def test_int64_fp64_order_golden(oracles):
    """avxsort_int64 / avx_merge_int64 order items as IEEE doubles
    (src/avxsort/avxcommon.h:79-190): this fork's signed (key, ptr) carriers
    (src/bench/sortbench.c:267-298) come out key-ascending, negative keys
    included.  Pins orc_sort_int64_fp64 / orc_merge_int64_fp64."""
    g = int64_gold()
    orc = oracles[8]
    ns = [int(k.rsplit("_", 1)[1]) for k in g if k.startswith("carrier_in_")]
    assert ns
    for n in ns:
        v = g[f"carrier_in_{n}"]
        want = v[g[f"carrier_perm_{n}"]]
        np.testing.assert_array_equal(orc.sort_int64_fp64(v), want)
        assert not np.array_equal(np.sort(v), want)  # not the integer order
    v = g["words_in"]
    np.testing.assert_array_equal(orc.sort_int64_fp64(v), v[g["words_perm"]])
    a, b = g["merge_a"], g["merge_b"]
    np.testing.assert_array_equal(orc.merge_int64_fp64(a, b),
                                  np.concatenate([a, b])[g["merge_perm"]])


def test_int64_fp64_order_live_reference(oracles):
    ref = _reference(8)
    rng = np.random.default_rng(77)
    key = rng.integers(-(2 ** 31 - 1), 2 ** 31 - 1, 40000)
    w = (np.abs(key).astype(np.int64) << 20) | (np.arange(40000) & 0xFFFFF)
    v = np.where(key < 0, w | np.int64(-2 ** 63), w).astype(np.int64)
    np.testing.assert_array_equal(oracles[8].sort_int64_fp64(v), ref.sort_int64(v))


# ---- large cases pinned by digests (tests/golden/golden_big.npz): the sort of
# 2^20 tuples and multiway merges of fan-in 128..2048
def _big():
    with np.load(os.path.join(GOLD, "golden_big.npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


def _mg():
    import importlib
    import sys
    sys.path.insert(0, GOLD)
    return importlib.import_module("make_golden")


def check_big(w, got, g, tag):
    mg = _mg()
    if w == 8:
        assert bytes(mg.digest(got)) == bytes(g[f"{tag}_out_digest"])
    assert bytes(mg.digest(got["key"])) == bytes(g[f"{tag}_out_key_digest"])
    assert bytes(mg.digest(canon(got))) == bytes(g[f"{tag}_out_canon_digest"])


@pytest.mark.parametrize("w", [8, 16])
def test_big_sort(w, oracles):
    g, mg, orc = _big(), _mg(), oracles[w]
    t = mg.big_sort_input(orc)
    assert bytes(mg.digest(t)) == bytes(g[f"w{w}_sort_in_digest"])
    check_big(w, orc.sort(t), g, f"w{w}_sort")


@pytest.mark.parametrize("w", [8, 16])
@pytest.mark.parametrize("k,maxlen", [(128, 900), (1024, 200), (2048, 100)])
def test_big_multiway(w, k, maxlen, oracles):
    g, mg, orc = _big(), _mg(), oracles[w]
    runs = mg.sorted_runs(np.random.default_rng(k), k, maxlen, orc.dtype)
    assert bytes(mg.digest(np.concatenate(runs))) == bytes(g[f"w{w}_mw{k}_in_digest"])
    out = orc.multiway_merge(runs)
    assert len(out) == int(g[f"w{w}_mw{k}_n"][0])
    check_big(w, out, g, f"w{w}_mw{k}")


def test_inregister_network_restatement_vs_golden():
    """orc_inregister_sort_keyval32 against the reference's AVX kernel
    (avxsort_core.h:1213-1274, tests/golden/golden_avxcore.npz): NaNs, signed
    zeros, infinities, denormals and duplicates included."""
    import oracle
    g = np.load(os.path.join(ROOT, "tests", "golden", "golden_avxcore.npz"))
    got = oracle.Oracle(8).inregister_sort_keyval32(g["inreg_in"])
    assert np.array_equal(got, g["inreg_out"])
