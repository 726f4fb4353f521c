"""CPU tests of the multi-GPU join's C++ orchestration (csrc/mgpu_orch.hpp).

sortmergejoin_mpsm runs mg::Rank on G GPUs with the library's kernels and
RCCL.  Here the SAME template runs on G host threads with host stand-ins for
the device contracts (tests/orch_host/host_orch.cpp: range partitions in the
three exchange layouts, the exchange table kernels, the segmented local join)
and memcpy collectives (mg::CopyColl), at G = 1, 2, 3 and 8.  The globally
sorted relations (the ranks' shares concatenated) and the count are compared
with the oracle's sort-merge join.  What this covers is the host logic: plan
and ownership arithmetic, the table messages and their exchange, agreement on
the exchange layout across ranks (planes -> words -> tuples, sampled ->
exact), the guessed key range and its replacement, buffer growth across calls
and the placement of the received rows.  The GPU run of the same template is
tests/test_gpu_mgpu.py.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "orch_host", "host_orch.cpp")
HDR = os.path.join(ROOT, "avx-sort-merge-joins_amd", "csrc", "mgpu_orch.hpp")
LAYOUT = {0: "tuples", 1: "words", 2: "planes"}
NOPLANES, ONECALL, SAMPLED, EXACT = 1, 2, 4, 8


@pytest.fixture(scope="session")
def host_libs(tmp_path_factory):
    d = tmp_path_factory.mktemp("orch_host")
    libs = {}
    for w in (8, 16):
        out = str(d / f"libhost_orch{w}.so")
        cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-pthread", "-shared", "-fPIC",
               SRC, "-o", out] + (["-DKEY_8B"] if w == 16 else [])
        subprocess.check_call(cmd)
        lib = C.CDLL(out)
        f = lib.host_mpsm_join
        f.restype = C.c_int64
        f.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int, C.c_uint32,
                      C.c_uint32, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_void_p,
                      C.c_void_p, C.c_void_p, C.c_char_p, C.c_int]
        libs[w] = f
    return libs


def run(f, R, S, G, flags=0, bucket_bits=4, key_range=None, ovf=-1, na=-1, calls=1):
    dt = R.dtype
    sR = np.zeros(len(R), dt)
    sS = np.zeros(len(S), dt)
    info = np.zeros(8 + 2 * G + 7, np.int64)
    err = C.create_string_buffer(512)
    kmin, kmax = key_range if key_range else (1, 0)
    c = f(R.ctypes.data, len(R), S.ctypes.data, len(S), G, flags, bucket_bits, kmin, kmax,
          ovf, na, calls, sR.ctypes.data, sS.ctypes.data, info.ctypes.data, err, 512)
    assert info[6] == 0, err.value.decode()
    return int(c), sR, sS, info


def relations(orc, w, n, kind, seed=12345):
    orc.seed(seed)
    R = orc.create_relation_pk(n)
    R["payload"] = np.arange(n)
    orc.seed(seed + 1)
    if kind == "zipf":
        S = orc.create_relation_zipf(n, n, 0.75)
        S["payload"] = np.arange(n)[::-1]
    else:
        S = orc.create_relation_fk(n, n)
        S["payload"] = np.arange(n) * 3
    if kind == "negative":  # no packing: 16-byte tuples travel as tuples
        S["payload"] = -1 - np.arange(n)
    if kind == "wide48" and w == 16:  # 64-bit words hold these, 48-bit ones do not
        S["payload"] = (1 << 45) + np.arange(n)
    if kind == "dupdup":  # duplicates on both sides
        R["key"] = R["key"] % (n // 7) + 1
        S["key"] = S["key"] % (n // 5) + 1
    if kind == "outside":  # keys beyond the guessed 1..|R|: the measured range
        S["key"] = S["key"] + 3 * n
    if kind == "negkeys":
        R["key"] = R["key"] - n // 2
        S["key"] = S["key"] - n // 2
    return R, S


def check(orc, R, S, got):
    c, sR, sS, info = got
    want, eR, eS = orc.sortmergejoin(R, S)
    assert c == want
    assert np.array_equal(sR, eR)
    assert np.array_equal(sS, eS)


@pytest.mark.parametrize("G", [1, 2, 3, 8])
@pytest.mark.parametrize("kind", ["uniform", "zipf", "negative", "wide48", "dupdup"])
def test_orchestration_vs_oracle(host_libs, oracles, width, G, kind):
    orc = oracles[width]
    R, S = relations(orc, width, 20000 + 13 * G, kind)
    got = run(host_libs[width], R, S, G, calls=2)
    check(orc, R, S, got)
    info = got[3]
    # the exchange layout every rank agreed on: 48-bit planes unless a payload
    # needs more bits (64-bit words), or cannot be packed (tuples)
    if width == 16 and kind == "negative":
        assert LAYOUT[info[0]] == "tuples"
    elif width == 16 and kind == "wide48":
        assert LAYOUT[info[0]] == "words"
    else:
        assert LAYOUT[info[0]] == "planes"
    # the local join: R's tile stage, then the rest, on every rank that holds
    # rows (G > 1; with keys 1..|R| planned as 2^L keys the top ranks of an
    # uneven share may own none)
    busy = int(((info[8::2][:G] + info[9::2][:G]) > 0).sum())
    assert (info[4], info[5]) == ((2 * busy, 0) if G > 1 else (0, 2))
    # one contiguous share per rank, every tuple once
    assert info[8::2][:G].sum() == len(R) and info[9::2][:G].sum() == len(S)
    # rank 0's phases (mg::Stats; a logical clock here, one unit per mark):
    # consecutive on the main stream, so they add up to its busy span; the
    # rows are timed on their own stream, only when something travels
    part, tables, wait, join, reduce_, busy, rows = info[8 + 2 * G:]
    assert part + tables + wait + join + reduce_ == busy
    assert min(part, tables, join, reduce_) > 0 and wait >= 0
    assert (rows > 0) == (G > 1)


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("flags,name", [(NOPLANES, "noplanes"), (ONECALL, "onecall"),
                                        (SAMPLED, "sampled"), (EXACT | NOPLANES, "exact")])
def test_orchestration_forms(host_libs, oracles, width, G, flags, name):
    orc = oracles[width]
    R, S = relations(orc, width, 30000, "uniform", seed=777)
    got = run(host_libs[width], R, S, G, flags=flags)
    check(orc, R, S, got)
    info = got[3]
    if flags & NOPLANES:
        assert LAYOUT[info[0]] == ("words" if width == 16 else "tuples")
    busy = int(((info[8::2][:G] + info[9::2][:G]) > 0).sum())
    if flags & ONECALL:
        assert (info[4], info[5]) == (0, busy)
    else:
        assert (info[4], info[5]) == (busy, 0)


@pytest.mark.parametrize("G", [2, 3, 8])
def test_orchestration_overflow_and_not_applicable(host_libs, oracles, width, G):
    """A sampled region overflow on one rank sends every rank to the exact
    partition (64-bit words, or tuples at 8 B); a rank where the sampled and
    planes forms do not apply makes every rank drop the planes."""
    orc = oracles[width]
    R, S = relations(orc, width, 25000, "uniform", seed=99)
    want = "words" if width == 16 else "tuples"
    got = run(host_libs[width], R, S, G, ovf=G - 1)
    check(orc, R, S, got)
    assert LAYOUT[got[3][0]] == want and got[3][2] == 4  # both relations once more
    got = run(host_libs[width], R, S, G, na=0)
    check(orc, R, S, got)
    assert LAYOUT[got[3][0]] == want


@pytest.mark.parametrize("G", [1, 3, 8])
@pytest.mark.parametrize("kind", ["outside", "negkeys"])
def test_orchestration_guessed_range_replan(host_libs, oracles, width, G, kind):
    """Keys outside the guessed 1..|R| (the reference's assumption): the
    48-bit partition flags them and every rank restarts with the measured
    range; a given range is used as is."""
    orc = oracles[width]
    R, S = relations(orc, width, 24000, kind, seed=4242)
    got = run(host_libs[width], R, S, G)
    check(orc, R, S, got)
    assert got[3][3] == 1  # one replan
    lo = int(min(R["key"].min(), S["key"].min()))
    hi = int(max(R["key"].max(), S["key"].max()))
    got = run(host_libs[width], R, S, G, key_range=(lo, hi))
    check(orc, R, S, got)
    assert got[3][3] == 0


@pytest.mark.parametrize("G", [2, 3, 8])
@pytest.mark.parametrize("nR,nS", [(7, 5), (0, 100), (100, 0), (0, 0), (1, 1), (9, 1000)])
def test_orchestration_ragged_and_empty(host_libs, oracles, width, G, nR, nS):
    """Chunks of n / G tuples (the last rank the rest): ranks with nothing to
    send, ranks that receive nothing, empty relations."""
    orc = oracles[width]
    orc.seed(5)
    R = orc.create_relation_pk(max(nR, 1))[:nR].copy()
    orc.seed(6)
    S = orc.create_relation_fk(max(nS, 1), max(nR, 1))[:nS].copy()
    got = run(host_libs[width], R, S, G)
    check(orc, R, S, got)


def test_orchestration_wide_keys(host_libs, oracles):
    """16-byte keys spanning most of int64 with the range given: partitions
    wider than 2^32 keys (no packed words: tuples), the plan base moved below
    INT64_MAX's edge (mg::local_range)."""
    orc = oracles[16]
    rng = np.random.default_rng(3)
    n = 20000
    R = np.zeros(n, orc.dtype)
    S = np.zeros(n, orc.dtype)
    R["key"] = rng.integers(-(1 << 62), (1 << 62), n)
    S["key"] = np.concatenate([R["key"][: n // 2], rng.integers(-(1 << 62), 1 << 62, n // 2)])
    R["payload"] = np.arange(n)
    S["payload"] = np.arange(n)
    lo = int(min(R["key"].min(), S["key"].min()))
    hi = int(max(R["key"].max(), S["key"].max()))
    for G in (2, 3, 8):
        got = run(host_libs[16], R, S, G, key_range=(lo, hi))
        check(orc, R, S, got)
        assert LAYOUT[got[3][0]] == "tuples"


def test_plan_arithmetic_matches_dist_py():
    """mgpu_orch.hpp restates smj/dist.py's plan functions; both must agree
    (checked here through a tiny g++ probe of the header)."""
    import sys
    import tempfile
    from conftest import PKG
    sys.path.insert(0, PKG)
    from smj.dist import local_range, partition_bits, used_parts
    probe = r'''
#include "%s"
#include <stdio.h>
int main() {
    long long cases[][2] = {{1, 128000000}, {-9223372036854775807LL - 1, 9223372036854775807LL},
                            {1, (1LL << 62) + 1}, {9223372036854775807LL - 1000, 9223372036854775807LL},
                            {7, 7}, {1, 1024000000}};
    unsigned pb[][2] = {{9, 1}, {10, 2}, {11, 3}, {11, 8}, {4, 5}, {9, 8}};
    for (auto& c : cases) for (auto& p : pb) for (unsigned r = 0; r < p[1]; r++) {
        auto l = smj::mg::local_range(c[0], c[1], p[0], p[1], r);
        printf("%%lld %%lld %%lld %%u %%u\n", (long long)l.base, (long long)l.key_lo, (long long)l.key_hi, l.lbits,
               smj::mg::used_parts(c[0], c[1], p[0]));
    }
    unsigned long long ns[] = {0, 1000, 128000000, 256000000};
    for (unsigned bb = 6; bb <= 9; bb++) for (unsigned G = 1; G <= 16; G *= 2)
        for (auto n : ns) for (int pl = 0; pl < 2; pl++)
            printf("%%u\n", smj::mg::partition_bits(bb, G, pl, n, true, 1, (long long)(G * 128000000ull)));
}
''' % HDR
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "p.cpp"), os.path.join(d, "p")
        open(src, "w").write(probe)
        subprocess.check_call(["g++", "-std=c++17", "-O1", src, "-o", exe])
        out = subprocess.check_output([exe], text=True).split("\n")
    want = []
    cases = [(1, 128000000), (-(1 << 63), (1 << 63) - 1), (1, (1 << 62) + 1),
             ((1 << 63) - 1001, (1 << 63) - 1), (7, 7), (1, 1024000000)]
    for kmin, kmax in cases:
        for pbits, world in ((9, 1), (10, 2), (11, 3), (11, 8), (4, 5), (9, 8)):
            for rank in range(world):
                b, klo, khi, lb = local_range(kmin, kmax, pbits, world, rank)
                want.append(f"{b} {klo} {khi} {lb} {used_parts(kmin, kmax, pbits)}")
    for bb in range(6, 10):
        G = 1
        while G <= 16:
            for n in (0, 1000, 128000000, 256000000):
                for pl in (0, 1):
                    want.append(str(partition_bits(bb, G, bool(pl), n or None,
                                                   (1, G * 128000000))))
            G *= 2
    assert out[:len(want)] == want
