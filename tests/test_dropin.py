"""Drop-in check on the GPU: the reference's own drivers and check_* tests,
compiled unchanged from their sources against include/compat/ and linked with
libsmj_hip[_k8].so (oracle/build_dropin.sh, run by __graft_entry__.build()
where /root/reference exists; the binaries travel with the tree).

check_merge.c unit-tests the reference's AVX merge kernels through
avxsort_core.h, internal to the AVX implementation; include/compat/
avxsort_core.h maps those kernel names onto the device merges, so it is built
and run too (check_merge8)."""
import os
import re
import subprocess

import numpy as np

import pytest

from conftest import ROOT

DROPIN = os.path.join(ROOT, "oracle", "_ref", "dropin")


def binary(name):
    p = os.path.join(DROPIN, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (oracle/build_dropin.sh needs /root/reference)")
    return p


def run(args, timeout=300):
    env = dict(os.environ, SMJ_QUIET="1")
    return subprocess.run(args, capture_output=True, text=True, timeout=timeout,
                          cwd="/tmp", env=env)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["check_partitioning8", "check_partitioning16",
                                  "check_scalarsort8", "check_scalarsort16",
                                  "check_avxsort8", "check_merge8"])
def test_reference_check_suite(name):
    r = run([binary(name)])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert re.search(r"Failures: 0", r.stdout), r.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("w", [8, 16])
@pytest.mark.parametrize("algo", ["m-way", "m-pass", "mpsm"])
def test_reference_sortmergejoins_driver(w, algo):
    """src/main.c unchanged, PK/FK 1M x 1M: Results = |S|."""
    exe = binary(f"sortmergejoins{w}")
    r = run([exe, "-a", algo, "-n", "8", "-r", "1000000", "-s", "1000000"]
            + SCALAR[w])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Results = 1000000." in r.stdout, r.stdout[-2000:]


def results(r):
    m = re.search(r"Results = (\d+)\. DONE", r.stdout)
    assert r.returncode == 0 and m, r.stdout[-2000:] + r.stderr[-2000:]
    return int(m.group(1))


# KEY_8B builds of main.c refuse to run without these (src/main.c:871-877)
SCALAR = {8: [], 16: ["--scalarsort", "--scalarmerge"]}
AB_CASES = {
    "non-unique": ["-r", "2000000", "-s", "3000000", "--non-unique"],
    "full-range": ["-r", "1500000", "-s", "2500000", "--full-range"],
    "seeds": ["-r", "1000000", "-s", "4000000", "--non-unique",
              "-x", "777", "-y", "999"],
    "fanout": ["-r", "1000000", "-s", "1000000", "--non-unique", "-f", "64"],
}


@pytest.mark.gpu
@pytest.mark.parametrize("w", [8, 16])
@pytest.mark.parametrize("case", sorted(AB_CASES))
def test_driver_ab_against_reference(w, case):
    """A/B: the same src/main.c, once on the reference's own AVX/scalar
    objects (oracle/_ref/sortmergejoins_ref*, CPU) and once on the MI355X
    library; seeded generators, so both must print the same Results."""
    ref = os.path.join(ROOT, "oracle", "_ref", f"sortmergejoins_ref{w}")
    if not os.path.exists(ref):
        pytest.skip("reference driver not built")
    exe = binary(f"sortmergejoins{w}")
    args = ["-n", "8"] + AB_CASES[case] + SCALAR[w]
    want = results(run([ref, "-a", "m-way"] + args))
    for algo in ("m-way", "m-pass", "mpsm"):
        assert results(run([exe, "-a", algo] + args)) == want, algo


@pytest.mark.gpu
@pytest.mark.parametrize("w", [8, 16])
def test_reference_partitioning_bench(w):
    exe = binary(f"bench_partitioning{w}")
    for what in (0, 1, 2):
        r = run([exe, "4194304", str(what), "10"])
        assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("w", [8, 16])
def test_reference_multiwaymerge_bench(w):
    exe = binary(f"bench_multiwaymerge{w}")
    r = run([exe, "65536", "16", str(1 << 20)])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Output relation is now sorted" in r.stderr, r.stderr[-2000:]
    assert "not sorted" not in r.stderr


@pytest.mark.gpu
def test_reference_sortbench_posneg():
    """src/bench/sortbench.c unchanged: this fork's signed (key, ptr)
    carriers through avxsort_int64, checked by the bench itself."""
    r = run([binary("bench_sort8"), "1", "0", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "[dbg] PASS" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
@pytest.mark.parametrize("w", [8, 16])
@pytest.mark.parametrize("nthreads", [2, 4, 8])
def test_tputbench_ab_against_reference(w, nthreads):
    """src/bench/tputbench.c unchanged: its own join thread (partition, sort,
    multiway merge, merge_join per thread) on sortmergejoin_initrun.  A/B
    against the same driver on the reference's objects; T threads call the
    library concurrently.

    T = 1 is not compared: that path joins R with itself
    (tputbench.c:485, ``partsS[i]->tuples = rels->R.tuples``) and reads |S_i|
    tuples from R_i's place, past its end into padding and the next
    partition, so merge_join gets unsorted input and the count depends on
    the scan's behaviour outside its contract (the reference itself prints
    1993423 there for 999597 true matches)."""
    ref = os.path.join(ROOT, "oracle", "_ref", f"tputbench_ref{w}")
    if not os.path.exists(ref):
        pytest.skip("reference tputbench not built")
    exe = binary(f"tputbench{w}")
    args = ["-a", "tputbench", "-n", str(nthreads), "-r", "1000000", "-s", "1000000",
            "--non-unique"] + SCALAR[w]
    assert results(run([exe] + args)) == results(run([ref] + args))


def _table(path):
    """a write_relation file (generator.c:200-213): '#KEY, VAL' + 'key payload'"""
    lines = open(path).read().splitlines()
    assert lines[0] == "#KEY, VAL"
    a = np.array([ln.split() for ln in lines[1:]], dtype=np.int64).reshape(-1, 2)
    t = np.zeros(len(a), [("payload", "<i8"), ("key", "<i8")])
    t["key"], t["payload"] = a[:, 0], a[:, 1]
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("w", [8, 16])
def test_reference_driver_materialize_persist(w, tmp_path):
    """src/main.c built with JOIN_MATERIALIZE + PERSIST_RELATIONS (the
    reference's --enable-materialize --enable-persist) on the MI355X library:
    it writes its generated R.tbl and S.tbl, joins, and persists the matches
    with write_result_relation to Out.tbl.  Out.tbl must hold, per key in
    ascending order, the S run (in (key, payload) order) |R_k| times --
    merge_join's R-major output (joincommon.c:267-287) over the sorted
    relations the driver itself wrote."""
    from test_gpu_materialize import numpy_materialize
    exe = binary(f"sortmergejoins_mat{w}")
    env = dict(os.environ, SMJ_QUIET="1")
    r = subprocess.run([exe, "-a", "m-way", "-n", "4", "-r", "200000", "-s", "300000"]
                       + SCALAR[w], capture_output=True, text=True, timeout=300,
                       cwd=str(tmp_path), env=env)
    total = results(r)
    R, S = _table(tmp_path / "R.tbl"), _table(tmp_path / "S.tbl")
    assert len(R) == 200000 and len(S) == 300000
    out = _table(tmp_path / "Out.tbl")
    exp = numpy_materialize(np.sort(R, order=["key", "payload"]),
                            np.sort(S, order=["key", "payload"]))
    assert total == len(exp) == len(out)
    assert np.array_equal(out["key"], exp["key"])
    assert np.array_equal(out["payload"], exp["payload"])
