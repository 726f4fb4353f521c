"""The three reference-header exports added in round 4 (missing
#3), on the GPU:

* radix_cluster (/root/reference/src/partition/partition.h:38-43, defined
  partition.c:93-149): the naive stable radix cluster, against the oracle's
  unpadded partition (oracle/smj_oracle.c, pinned by tests/golden/) and with a
  caller hist that is not zero (the reference adds to it and shifts every
  partition's start by it);
* is_sorted_helper / check_sorted (joincommon.h:99-103, joincommon.c:397-515).

Plus a plain C caller linked against the libraries through the compat headers
(tests/compat_check/abi_extras.c, built by the Makefile), run as the
reference's drivers would call these functions.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,shift,bits", [(0, 0, 4), (1, 0, 3), (100_003, 0, 7),
                                          (1_000_003, 5, 10), (300_001, 20, 6),
                                          (65_536, 0, 12)])
def test_radix_cluster_vs_oracle(libs, oracles, width, n, shift, bits):
    lib, orc = libs[width], oracles[width]
    orc.seed(777 + n)
    t = orc.create_relation_pk(n)
    t["payload"] = np.arange(n) + 5
    out, hist = lib.radix_cluster(t, shift, bits)
    want, cnt, off = orc.partition(t, bits, shift, False)
    np.testing.assert_array_equal(hist, cnt.astype(np.int32))
    np.testing.assert_array_equal(out[:n], want[:n])


def test_radix_cluster_nonzero_hist(libs, oracles, width):
    """partition.c:111-122: counts are added to the caller's hist and the
    starts are the prefix sums of the updated hist."""
    lib, orc = libs[width], oracles[width]
    n, bits, shift = 50_000, 5, 2
    orc.seed(99)
    t = orc.create_relation_pk(n)
    t["payload"] = np.arange(n)
    h0 = (np.arange(1 << bits, dtype=np.int32) * 7) % 11
    out, hist = lib.radix_cluster(t, shift, bits, hist=h0)
    want, cnt, _ = orc.partition(t, bits, shift, False)
    np.testing.assert_array_equal(hist, h0 + cnt.astype(np.int32))
    start = np.concatenate([[0], np.cumsum(hist)[:-1]])
    pos = 0
    for i in range(1 << bits):
        c = int(cnt[i])
        np.testing.assert_array_equal(out[start[i]:start[i] + c], want[pos:pos + c])
        pos += c


def test_is_sorted_helper(libs, width):
    lib = libs[width]
    dt = lib.dtype
    n = 300_001
    t = np.zeros(n, dt)
    t["key"] = np.arange(n) // 4 + 1
    t["payload"] = -np.arange(n)  # payload order plays no part
    assert lib.is_sorted_helper(t) == 1
    assert lib.is_sorted_helper(t[:0]) == 1
    u = t.copy()
    u["key"][n - 1] = 0
    assert lib.is_sorted_helper(u) == 0
    u = t.copy()
    u["key"][0] = -1  # below the reference's start key 0
    assert lib.is_sorted_helper(u) == 0


def test_is_sorted_helper_messages(libs, capfd):
    """The 8-byte build prints the reference's lines (joincommon.c:456-476)."""
    lib = libs[8]
    t = np.zeros(10, lib.dtype)
    t["key"] = [1, 2, 2, 3, 4, 3, 5, 6, 7, 8]
    assert lib.is_sorted_helper(t) == 0
    out = capfd.readouterr().out
    assert "[WARN ] Equal items, still ok... item[2].key=2 is equal to item[1].key=2" in out
    assert "[ERROR] item[5].key=3 is less than item[4].key=4" in out


@pytest.mark.parametrize("w", [8, 16])
def test_c_caller(w):
    exe = os.path.join(PKG, "lib", f"abi_extras{w}")
    if not os.path.exists(exe):
        pytest.fail(f"{exe} missing: make -C {PKG}")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "ABI-EXTRAS OK" in r.stdout
    assert "3-thread -> R is sorted, size = 100003" in r.stdout
    assert "3-thread -> S is NOT sorted, size = 100003" in r.stdout
