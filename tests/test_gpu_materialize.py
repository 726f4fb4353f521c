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
