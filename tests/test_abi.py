"""The C ABI (include/smj.h) on CPU: both libraries load, report their tuple
width, and export every function the header declares.  No compute call is made
here -- the library aborts without a HIP device (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "smj.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"#[^\n]*", "", src)
    # a declaration: <type> name(args);  -- skip typedef'd function pointers
    names = set(re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{}()]*(?:\([^()]*\)[^;{}()]*)*\)\s*;", src))
    return {n for n in names if n not in ("sizeof",)}


@pytest.fixture(scope="module")
def smj_mod():
    import smj
    for w in (8, 16):
        if not os.path.exists(smj.lib_path(w)):
            smj.build()
            break
    return smj


def test_header_lists_match_binding(smj_mod):
    decl = declared_functions()
    listed = set(smj_mod.REFERENCE_SYMBOLS) | set(smj_mod.DEVICE_SYMBOLS)
    assert decl == listed, (sorted(decl - listed), sorted(listed - decl))


@pytest.mark.parametrize("width", [8, 16])
def test_library_exports(smj_mod, width):
    path = smj_mod.lib_path(width)
    lib = ctypes.CDLL(path)
    missing = [s for s in declared_functions() if not hasattr(lib, s)]
    assert not missing, missing
    lib.smj_tuple_bytes.restype = ctypes.c_int
    assert lib.smj_tuple_bytes() == width


@pytest.mark.parametrize("width", [8, 16])
def test_binding_loads(smj_mod, width):
    L = smj_mod.Library(width)  # binds every signature; no device call
    assert L.dtype.itemsize == width


def test_binding_fails_loudly_without_library(smj_mod, tmp_path):
    with pytest.raises(FileNotFoundError):
        smj_mod.Library(16, path=str(tmp_path / "nope.so"))


def test_product_does_not_reference_oracle():
    """The shipped path never imports or links the oracle."""
    for root, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".h", ".cpp")) or f == "Makefile":
                text = open(os.path.join(root, f), errors="ignore").read()
                assert "oracle" not in text.replace("no oracle", ""), os.path.join(root, f)


@pytest.mark.parametrize("width", [8, 16])
def test_glibc_rand_jump_ahead(smj_mod, width):
    """smj_glibc_rand (the jump-ahead behind the reference-exact device
    generators, refgen.hip) against glibc's own srand/rand, host only: every
    position of the first 4000 draws for several seeds (0 is glibc's 1), and
    deep positions reached by stepping glibc itself."""
    L = smj_mod.Library(width)
    libc = ctypes.CDLL(None)
    libc.srand.argtypes = [ctypes.c_uint]
    for seed in (0, 1, 777, 12345, 54321, 2 ** 31 + 5):
        libc.srand(seed)
        ref = [libc.rand() for _ in range(4000)]
        got = [L.glibc_rand(seed, k) for k in range(0, 4000, 7)]
        assert got == ref[::7], seed
    libc.srand(4242)
    for k in range(1_000_000):
        x = libc.rand()
        if k in (65535, 65536, 999_999):
            assert L.glibc_rand(4242, k) == x, k


@pytest.mark.parametrize("width", [8, 16])
def test_c_caller_links(smj_mod, width, tmp_path):
    """tests/compat_check/abi_extras.c (radix_cluster, is_sorted_helper,
    check_sorted through the compat headers) compiles and links against the
    library like a reference driver; tests/test_gpu_abi.py runs it."""
    import subprocess
    src = os.path.join(ROOT, "tests", "compat_check", "abi_extras.c")
    lib = os.path.dirname(smj_mod.lib_path(width))
    name = "smj_hip" if width == 8 else "smj_hip_k8"
    exe = tmp_path / "abi_extras"
    cmd = ["gcc", "-O1", "-std=gnu99", "-I", os.path.join(ROOT, "include", "compat"), src,
           f"-L{lib}", f"-l{name}", "-o", str(exe)] + (["-DKEY_8B"] if width == 16 else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
