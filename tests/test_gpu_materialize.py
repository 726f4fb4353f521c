"""Materialised merge join (smj_dev_materialize).

The oracle is orc_merge_join_materialize, the C restatement of merge_join
built with JOIN_MATERIALIZE (src/joins/joincommon.c:256-289: one
<S.key, S.payload> per match, R-major).  The reference's chained result
buffer (tuple_buffer.h) is not in its tree, so the reference cannot be built
with materialisation: the restatement is cross-checked here against an
independent numpy construction (per key, the S run repeated |R_k| times)
instead of reference output -- the output ORDER is parity-unpinned, the
count is pinned through merge_join.  Comparisons are bit-exact.
"""
import numpy as np
import pytest

from test_gpu_parity import JOIN_CASES, make_join_inputs, rand_tuples

pytestmark = pytest.mark.gpu


def numpy_materialize(R, S):
    """Independent construction over sorted R, S."""
    if len(R) == 0 or len(S) == 0:
        return S[:0].copy()
    keys, s0, sc = np.unique(S["key"], return_index=True, return_counts=True)
    rc = np.searchsorted(R["key"], keys, "right") - np.searchsorted(R["key"], keys, "left")
    per = rc * sc
    total = int(per.sum())
    run = np.repeat(np.arange(len(keys)), per)
    start = np.concatenate([[0], np.cumsum(per)[:-1]])
    pos = np.arange(total) - start[run]
    return S[s0[run] + pos % sc[run]]


def check(lib, orc, R, S):
    import torch
    R, S = orc.sort(R), orc.sort(S)
    exp = orc.merge_join_materialize(R, S)
    assert len(exp) == orc.merge_join(R, S)
    assert np.array_equal(exp, numpy_materialize(R, S))
    dR, dS = lib.to_device(R), lib.to_device(S)
    assert lib.dev_materialize(dR, dS) == len(exp)  # count only
    out = lib.empty(len(exp) + 5)
    got = lib.dev_materialize(dR, dS, out)
    torch.cuda.synchronize()
    assert got == len(exp)
    assert np.array_equal(lib.to_host(out)[:got], exp)
    return exp, dR, dS


@pytest.mark.parametrize("kind,nr,ns", JOIN_CASES)
def test_materialize_join_cases(libs, oracles, width, kind, nr, ns):
    orc, lib = oracles[width], libs[width]
    R, S = make_join_inputs(orc, width, kind, nr, ns)
    check(lib, orc, R, S)


def test_materialize_hot_keys(libs, oracles, width):
    """A hot key on both sides: one run's output spans many tiles and work
    items; an S run crossing tile boundaries; keys present on one side only."""
    orc, lib = oracles[width], libs[width]
    rng = np.random.default_rng(7)
    R = rand_tuples(width, 30000, 1, 0, 2000)
    S = rand_tuples(width, 50000, 2, 0, 2000)
    R["key"][:5000] = 777          # |R_777| >= 5000
    S["key"][:9000] = 777          # S run of 9000 crosses several tiles
    S["payload"][:9000] = rng.integers(0, 1 << 20, 9000)
    S["key"][9000:9100] = 5000     # no partner in R
    check(lib, orc, R, S)


def test_materialize_single_key_and_capacity(libs, oracles, width):
    import torch
    orc, lib = oracles[width], libs[width]
    R = rand_tuples(width, 3000, 3, 42, 43)   # every key 42
    S = rand_tuples(width, 2500, 4, 42, 43)
    exp, dR, dS = check(lib, orc, R, S)
    assert len(exp) == 3000 * 2500
    # a short output buffer receives the prefix, the total is still returned
    cap = len(exp) // 3 + 17
    out = lib.empty(cap)
    assert lib.dev_materialize(dR, dS, out) == len(exp)
    torch.cuda.synchronize()
    assert np.array_equal(lib.to_host(out), exp[:cap])


def test_materialize_after_device_join(libs, oracles, width):
    """The device join's sorted outputs feed the materialisation directly."""
    import torch
    orc, lib = oracles[width], libs[width]
    n = 1 << 20
    R, S = lib.empty(n), lib.empty(n)
    lib.dev_gen_pk(R, 0, n, 12345)
    lib.dev_gen_fk(S, 0, n, n, 54321)
    sR, sS = lib.empty(n), lib.empty(n)
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lib.dev_join(R, S, sR, sS, cnt, 10, 1, n)
    out = lib.empty(n)
    assert lib.dev_materialize(sR, sS, out) == n
    torch.cuda.synchronize()
    # PK/FK: every S tuple matches exactly once, in sorted order
    assert np.array_equal(lib.to_host(out), lib.to_host(sS))


# ---- the reference-named materialisation path: merge_join(..., output),
# the join entry points with materialisation on, write_result_relation
MAT_CASES = [("nonunique", 50000, 60000), ("zipf", 20000, 40000),
             ("random", 30000, 30000), ("pk_fk", 0, 0)]


@pytest.mark.parametrize("kind,nr,ns", MAT_CASES)
def test_merge_join_output_buffer(libs, oracles, width, kind, nr, ns):
    """merge_join with a chainedtuplebuffer_t appends one <S.key, S.payload>
    per match (joincommon.c:273-279) after what the buffer already holds."""
    orc, lib = oracles[width], libs[width]
    R, S = make_join_inputs(orc, width, kind, nr, ns)
    R, S = orc.sort(R), orc.sort(S)
    exp = orc.merge_join_materialize(R, S)
    prefix = rand_tuples(width, 3, 9)
    n, buf = lib.merge_join_materialize(R, S, prefix=prefix)
    assert n == len(exp) == orc.merge_join(R, S)
    assert np.array_equal(buf[:3], prefix)
    assert np.array_equal(buf[3:], exp)


def persisted(path):
    """Out.tbl as write_relation's text format: '#KEY, VAL', then 'key payload'."""
    lines = open(path).read().splitlines()
    assert lines[0] == "#KEY, VAL"
    if len(lines) == 1:
        return np.zeros((0, 2), np.int64)
    return np.array([ln.split() for ln in lines[1:]], dtype=np.int64)


def low32(a):
    """what %d prints for an int64 argument on x86-64: the low 32 bits"""
    return np.asarray(a, dtype=np.int64).astype(np.int32).astype(np.int64)


def mpass_expected(orc, R, S, T, F):
    """m-pass output order (src/joins/sortmergejoin_multipass.c): thread t owns
    partitions [t F / T, (t + 1) F / T) of the digit ((key - 1) & mask) >>
    shift, shift = ceil(log2(chunk * T)) - log2(F) - 1 (:323-328), and writes
    the R-major matches of its own sorted relations; the threads' lists
    follow one another."""
    import math
    bits = int(math.log2(F))

    # the shift comes from each thread's chunk of R, for R and S alike
    chunk = len(R) // T
    sh = [max(math.ceil(math.log2(c * T)) - bits - 1, 0) if c else 0
          for c in [chunk] * (T - 1) + [len(R) - chunk * (T - 1)]]
    assert len(set(sh)) == 1 or len(R) < T

    def owner(rel):
        d = ((rel["key"].astype(np.int64) - 1) & (((1 << bits) - 1) << sh[0])) >> sh[0]
        return d // (F // T)

    oR, oS = owner(R), owner(S)
    parts = [orc.merge_join_materialize(orc.sort(R[oR == t]), orc.sort(S[oS == t]))
             for t in range(T)]
    return np.concatenate(parts)


@pytest.mark.parametrize("algo", ["m-way", "m-pass", "mpsm"])
@pytest.mark.parametrize("kind,nr,ns", MAT_CASES)
def test_join_materialize_and_persist(libs, oracles, width, algo, kind, nr, ns, tmp_path):
    """sortmergejoin_* with materialisation on hand the output in
    resultlist[0].results; write_result_relation appends it to Out.tbl
    (main.c:609-614) in write_relation's format (generator.c:200-213)."""
    orc, lib = oracles[width], libs[width]
    R, S = make_join_inputs(orc, width, kind, nr, ns)
    if algo == "m-pass":
        exp = mpass_expected(orc, R, S, 4, 128)
    else:
        exp = orc.merge_join_materialize(orc.sort(R), orc.sort(S))
    out = tmp_path / "Out.tbl"
    n, got = lib.sortmergejoin_multiway(R, S, nthreads=4, algo=algo, materialize=True,
                                        persist=str(out))
    assert n == len(exp)
    assert np.array_equal(got, exp)
    rows = persisted(out)
    assert len(rows) == len(exp)
    assert np.array_equal(rows[:, 0], low32(exp["key"]))
    assert np.array_equal(rows[:, 1], low32(exp["payload"]))
    # materialisation is off again: a plain join returns the count only
    assert lib.sortmergejoin_multiway(R, S, nthreads=4, algo=algo) == len(exp)
