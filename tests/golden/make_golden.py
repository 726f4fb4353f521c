#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE implementation.

Runs in the container that has /root/reference: oracle/build_ref.sh compiles
the reference sources into oracle/_ref/libref{8,16}.so, and this script calls
them through oracle.Reference (ctypes).  The fixtures are plain arrays (inputs
and the reference's outputs), loaded with numpy.load(allow_pickle=False) by
tests/test_oracle.py, which pins oracle/smj_oracle.c (the CPU restatement) to
them.  Nothing here runs on the GPU box.

    python tests/golden/make_golden.py           # golden_w8/w16.npz
    python tests/golden/make_golden.py --int64   # golden_int64.npz
    python tests/golden/make_golden.py --avxcore # golden_avxcore.npz
    python tests/golden/make_golden.py --big     # golden_big.npz (digests)
"""
import hashlib
import os
import re
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

PART_N = 5000
PART_CASES = [(4, 0), (10, 0), (7, 3), (4, 20)]
SORT_NS = [16, 255, 16384, 2 * 16384 + 77]
MW_FANIN = [4, 64]
JOIN_CASES = [("pk", 200000, 200000), ("pk", 300000, 100000),
              ("nonunique", 100000, 150000), ("zipf", 100000, 200000)]


def join_inputs(gen, kind, nr, ns):
    """R and S of a join case; gen is oracle.Reference or oracle.Oracle."""
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


def join_case(w, ki, T):
    ref = oracle.Reference(w)
    kind, nr, ns = JOIN_CASES[ki]
    R, S = join_inputs(ref, kind, nr, ns)
    print("\nCOUNT", ref.sortmergejoin_multiway(R, S, nthreads=T, fanout=128), flush=True)


def sorted_runs(rng, k, maxlen, dtype, keymax=100000):
    runs = []
    for _ in range(k):
        n = int(rng.integers(1, maxlen))
        t = np.zeros(n, dtype)
        t["key"] = np.sort(rng.integers(1, keymax, n))
        t["payload"] = rng.integers(0, 1 << 20, n)
        # canonical order (key, payload) so 8- and 16-byte semantics agree
        t = np.sort(t, order=["key", "payload"])
        runs.append(t)
    return runs


def main():
    for w in (8, 16):
        ref = oracle.Reference(w)
        out = {}
        # ---- generators (src/datagen/generator.c, genzipf.c)
        ref.seed(12345)
        out["gen_pk"] = ref.create_relation_pk(1000)
        ref.seed(54321)
        out["gen_nonunique"] = ref.create_relation_nonunique(1000, 300)
        ref.seed(777)
        out["gen_zipf"] = ref.create_relation_zipf(2000, 500, 0.75)
        ref.seed(99)
        out["gen_fk"] = ref.create_relation_fk(1500, 400)

        # ---- partitioning (src/partition/partition.c)
        ref.seed(12345)
        pin = ref.create_relation_pk(PART_N)
        pin["payload"] = np.arange(PART_N) + 5
        out["part_in"] = pin
        for nbits, shift in PART_CASES:
            for variant in (0, 1, 2):
                o, cnt, off = ref.partition(pin, nbits, shift, variant)
                dense = np.concatenate([o[off[i]:off[i] + cnt[i]] for i in range(1 << nbits)])
                tag = f"part_b{nbits}_s{shift}_v{variant}"
                out[tag + "_cnt"] = cnt
                out[tag + "_off"] = off
                out[tag + "_dense"] = dense

        # ---- sorting: AVX path for 8-byte tuples, scalar for 16-byte
        for n in SORT_NS:
            ref.seed(1000 + n)
            t = ref.create_relation_nonunique(n, max(2, n // 2))
            out[f"sort_in_{n}"] = t
            if w == 8:
                out[f"sort_out_{n}"] = ref.sort(t, "avxsort_tuples")
            else:
                out[f"sort_out_{n}"] = ref.sort(t, "scalarsort_tuples")

        # ---- 2-way merge (src/merge/merge.c)
        rng = np.random.default_rng(5)
        a, b = sorted_runs(rng, 2, 1200, ref.dtype)
        out["merge_a"], out["merge_b"] = a, b
        out["merge_out"] = ref.merge(a, b, "avx_merge_tuples" if w == 8 else "scalar_merge_tuples")

        # ---- multiway merge (src/merge/avx_multiwaymerge.c, scalar_multiwaymerge.c)
        for k in MW_FANIN:
            runs = sorted_runs(np.random.default_rng(k), k, 900, ref.dtype)
            mo, mn = ref.multiway_merge(runs, 4 << 20, scalar=(w == 16))
            out[f"mw{k}_runs"] = np.concatenate(runs)
            out[f"mw{k}_lens"] = np.array([len(r) for r in runs], np.int64)
            out[f"mw{k}_out"] = mo
            out[f"mw{k}_n"] = np.array([mn], np.int64)

        # ---- merge_join on dup x dup sorted runs (src/joins/joincommon.c)
        mj = []
        for seed, n in [(1, 10), (2, 1000), (3, 20000)]:
            r = np.random.default_rng(seed)
            R = np.zeros(n, ref.dtype)
            S = np.zeros(n + 7, ref.dtype)
            R["key"] = np.sort(r.integers(0, max(2, n // 4), n))
            S["key"] = np.sort(r.integers(0, max(2, n // 4), n + 7))
            out[f"mj{seed}_R"], out[f"mj{seed}_S"] = R, S
            mj.append(ref.merge_join(R, S))
        out["mj_counts"] = np.array(mj, np.int64)

        # ---- sortmergejoin_multiway counts (src/joins/sortmergejoin_multiway.c)
        # inputs are regenerated by the oracle from the seeds (pinned above).
        # Each case runs in a child process: the reference's 8-byte AVX path
        # segfaults deterministically on (nonunique, NTHREADS=8) here; such a
        # case is recorded with count -1 and skipped by the tests.
        cases = []
        for ki, (kind, nr, ns) in enumerate(JOIN_CASES):
            for T in (1, 2, 4, 8):
                r = subprocess.run([sys.executable, __file__, "--join-case",
                                    str(w), str(ki), str(T)],
                                   capture_output=True, text=True, timeout=600)
                c = -1
                m = re.search(r"COUNT (-?\d+)", r.stdout)
                if r.returncode == 0 and m:
                    c = int(m.group(1))
                cases.append((["pk", "nonunique", "zipf"].index(kind), nr, ns, T, c))
        out["join_cases"] = np.array(cases, np.int64)

        path = os.path.join(HERE, f"golden_w{w}.npz")
        np.savez_compressed(path, **out)
        print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(out)} arrays)")


BIG_SORT_N = 1 << 20            # sorts up to 2^20
BIG_MW = [(128, 900), (1024, 200), (2048, 100)]  # fan-in, max run length


def digest(a) -> np.ndarray:
    """SHA-256 of an array's bytes, as 32 uint8 (fixtures stay small)."""
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def big_sort_input(gen, n=BIG_SORT_N):
    """the 2^20 sort case: create_relation_nonunique(n, n/2), seed 4242"""
    gen.seed(4242)
    return gen.create_relation_nonunique(n, n // 2)


def big_fixtures():
    """Reference outputs too big to commit, kept as digests: the inputs are
    regenerated by the tests (the seeded generator restatement, pinned by
    golden_w*.npz, and sorted_runs over numpy's seeded generator); the
    fixture holds the reference's output digest, length and head/tail."""
    out = {}
    for w in (8, 16):
        ref = oracle.Reference(w)
        t = big_sort_input(ref)
        o = ref.sort(t, "avxsort_tuples" if w == 8 else "scalarsort_tuples")
        out[f"w{w}_sort_in_digest"] = digest(t)
        # exact order (8-byte tuples: the packed word is a total order), and
        # for both widths the key column and the (key, payload) multiset (the
        # 16-byte path leaves equal keys in an implementation order)
        out[f"w{w}_sort_out_digest"] = digest(o)
        out[f"w{w}_sort_out_key_digest"] = digest(o["key"])
        out[f"w{w}_sort_out_canon_digest"] = digest(np.sort(o, order=["key", "payload"]))
        out[f"w{w}_sort_out_head"] = o[:64]
        out[f"w{w}_sort_out_tail"] = o[-64:]
        for k, maxlen in BIG_MW:
            runs = sorted_runs(np.random.default_rng(k), k, maxlen, ref.dtype)
            mo, mn = ref.multiway_merge(runs, 4 << 20, scalar=(w == 16))
            out[f"w{w}_mw{k}_in_digest"] = digest(np.concatenate(runs))
            out[f"w{w}_mw{k}_out_digest"] = digest(mo)
            out[f"w{w}_mw{k}_out_key_digest"] = digest(mo["key"])
            out[f"w{w}_mw{k}_out_canon_digest"] = digest(np.sort(mo, order=["key", "payload"]))
            out[f"w{w}_mw{k}_n"] = np.array([mn, len(mo)], np.int64)
    path = os.path.join(HERE, "golden_big.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(out)} arrays)")


def carriers(rng, n):
    """This fork's (key, ptr) int64 carriers with signed keys, built as
    src/bench/sortbench.c:267-298 does (gen_random_int, SetPtr, SetKeyInt):
    sign bit | |key| << 20 | (i & 0xFFFFF)."""
    key = rng.integers(-(2 ** 31 - 1), 2 ** 31 - 1, n)
    w = (np.abs(key).astype(np.int64) << 20) | (np.arange(n, dtype=np.int64) & 0xFFFFF)
    return np.where(key < 0, w | np.int64(-2 ** 63), w).astype(np.int64)


def non_nan_words(rng, n):
    """Random int64 patterns that are no NaN and not -0 as doubles."""
    v = rng.integers(-(1 << 63), (1 << 63) - 1, 2 * n, dtype=np.int64)
    v = v[(((v >> 52) & 0x7FF) != 0x7FF) & (v != np.int64(-2 ** 63))]
    return v[:n]


def int64_fixtures():
    """avxsort_int64 / avx_merge_int64 on signed items: the AVX networks order
    int64 items as IEEE doubles (sign-magnitude), not as integers."""
    ref = oracle.Reference(8)
    rng = np.random.default_rng(2012)
    out = {}

    def perm(inp, res):
        # the reference's output as indices into the input (distinct items)
        order = {int(x): i for i, x in enumerate(inp)}
        assert len(order) == len(inp)
        return np.array([order[int(x)] for x in res], np.uint32)

    for n in (100, 16384 + 255, 2 * 16384 + 77):
        v = carriers(rng, n)
        out[f"carrier_in_{n}"] = v
        out[f"carrier_perm_{n}"] = perm(v, ref.sort_int64(v))
    v = non_nan_words(rng, 5000)
    out["words_in"] = v
    out["words_perm"] = perm(v, ref.sort_int64(v))
    a = ref.sort_int64(carriers(rng, 1500))
    b = ref.sort_int64(carriers(rng, 2001))
    b = b[~np.isin(b, a)]
    out["merge_a"], out["merge_b"] = a, b
    ab = np.concatenate([a, b])
    out["merge_perm"] = perm(ab, ref.merge_int64(a, b))
    path = os.path.join(HERE, "golden_int64.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(out)} arrays)")


def special_words():
    """Bit patterns the FP64 networks treat specially: NaNs (quiet, signalling,
    negative), +-0, +-inf, denormals, the extremes of the int64 range."""
    v = [0, -2 ** 63, 0x7FF0000000000000, -0x0010000000000000, 0x7FF8000000000000,
         0x7FF0000000000001, -0x0008000000000000, 0x7FFFFFFFFFFFFFFF, 1, -2 ** 63 + 1,
         0x000FFFFFFFFFFFFF, 0x0010000000000000, 2 ** 62, -(2 ** 62), 42, -42]
    return np.array(v, dtype=np.int64)


def avxcore_fixtures():
    """The reference's AVX register kernels the compat header
    include/compat/avxsort_core.h maps (check_merge.c calls them):
    inregister_sort_keyval32 (avxsort_core.h:1213-1274) on 16-item blocks of
    random, special and duplicate patterns, and merge16_varlen
    (:388-500) with the inputs as it leaves them (its register flush into
    consumed input slots, :461-475)."""
    ref = oracle.Reference(8)
    rng = np.random.default_rng(1213)
    sp = special_words()
    blocks = [carriers(rng, 16 * 200), non_nan_words(rng, 16 * 200),
              rng.integers(-(1 << 63), (1 << 63) - 1, 16 * 300, dtype=np.int64),
              rng.choice(sp, 16 * 300), rng.integers(-3, 4, 16 * 100).astype(np.int64),
              np.tile(np.arange(16, dtype=np.int64), 10), np.tile(np.arange(16, 0, -1), 10)]
    inp = np.concatenate(blocks).astype(np.int64)
    out = {"inreg_in": inp, "inreg_out": ref.inregister_sort_keyval32(inp)}
    for i, (la, lb) in enumerate(((100, 77), (1000, 1003), (16 * 40 + 3, 16 * 17 + 15),
                                  (4096, 33), (33, 4096))):
        a = ref.sort_int64(carriers(rng, la))
        b = ref.sort_int64(carriers(rng, lb))
        o, a2, b2 = ref.merge16_varlen(a, b)
        out[f"varlen{i}_a"], out[f"varlen{i}_b"] = a, b
        out[f"varlen{i}_out"], out[f"varlen{i}_a_after"], out[f"varlen{i}_b_after"] = o, a2, b2
    path = os.path.join(HERE, "golden_avxcore.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB, {len(out)} arrays)")


if __name__ == "__main__":
    if len(sys.argv) == 5 and sys.argv[1] == "--join-case":
        join_case(*map(int, sys.argv[2:]))
    elif len(sys.argv) == 2 and sys.argv[1] == "--int64":
        int64_fixtures()
    elif len(sys.argv) == 2 and sys.argv[1] == "--avxcore":
        avxcore_fixtures()
    elif len(sys.argv) == 2 and sys.argv[1] == "--big":
        big_fixtures()
    else:
        main()
