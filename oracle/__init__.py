"""CPU checker for the MI355X sort-merge-join library -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  It wraps:

* liboracle{8,16}.so -- the in-repo C restatement of the reference path
  (oracle/smj_oracle.c, every function citing the reference file:line);
* _ref/libref{8,16}.so -- the reference itself compiled from /root/reference
  (oracle/build_ref.sh), available where it was built (this container, and
  the GPU box when the tree was shipped after a build).

Arrays are numpy structured arrays with the reference tuple layout
(payload first, then key): TUPLE8 = (int32 payload, int32 key),
TUPLE16 = (int64 payload, int64 key).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TUPLE8 = np.dtype([("payload", "<i4"), ("key", "<i4")])
TUPLE16 = np.dtype([("payload", "<i8"), ("key", "<i8")])


def tuple_dtype(width: int) -> np.dtype:
    return TUPLE8 if width == 8 else TUPLE16


def build() -> None:
    """(Re)build the restatement and, when /root/reference exists, the reference."""
    subprocess.check_call(["bash", os.path.join(HERE, "build_ref.sh")])


_P = C.c_void_p
_I64 = C.c_int64
_U64 = C.c_uint64


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None else 0


class _Lib:
    def __init__(self, path: str, prefix: str, width: int):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = C.CDLL(path)
        self.prefix = prefix
        self.width = width
        self.dtype = tuple_dtype(width)
        got = getattr(self.lib, prefix + "tuple_bytes")()
        assert got == width, (path, got, width)

    def fn(self, name, restype, *argtypes):
        f = getattr(self.lib, self.prefix + name)
        f.restype = restype
        f.argtypes = list(argtypes)
        return f


class Oracle(_Lib):
    """The C restatement (oracle/smj_oracle.c)."""

    def __init__(self, width: int):
        super().__init__(os.path.join(HERE, f"liboracle{width}.so"), "orc_", width)

    # generators -------------------------------------------------------------
    def seed(self, s: int) -> None:
        self.fn("seed", None, C.c_uint)(s)

    def create_relation_pk(self, n: int) -> np.ndarray:
        t = np.zeros(n, self.dtype)
        self.fn("create_relation_pk", None, _P, _I64)(_ptr(t), n)
        return t

    def create_relation_mway(self, n: int, maxid: int) -> np.ndarray:
        t = np.zeros(n, self.dtype)
        self.fn("create_relation_mway", None, _P, _I64, _I64)(_ptr(t), n, maxid)
        return t

    def create_relation_nonunique(self, n: int, maxid: int) -> np.ndarray:
        t = np.zeros(n, self.dtype)
        self.fn("create_relation_nonunique", None, _P, _I64, _I64)(_ptr(t), n, maxid)
        return t

    def create_relation_fk(self, n: int, maxid: int) -> np.ndarray:
        t = np.zeros(n, self.dtype)
        self.fn("create_relation_fk", None, _P, _I64, _I64)(_ptr(t), n, maxid)
        return t

    def create_relation_zipf(self, n: int, maxid: int, theta: float) -> np.ndarray:
        t = np.zeros(n, self.dtype)
        self.fn("create_relation_zipf", None, _P, _I64, _I64, C.c_double)(
            _ptr(t), n, maxid, theta)
        return t

    # the library's device generators, restated (datagen.hip) ---------------
    def dev_gen_perm(self, n, first, total, maxid, seed, payload=True) -> np.ndarray:
        t = np.zeros(n, self.dtype)
        self.fn("dev_gen_perm", None, _P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                C.c_uint64, C.c_int)(_ptr(t), n, first, total, maxid, seed, int(payload))
        return t

    def dev_gen_zipf(self, n, first, maxid, theta, seed) -> np.ndarray:
        t = np.zeros(n, self.dtype)
        self.fn("dev_gen_zipf", None, _P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_double,
                C.c_uint64)(_ptr(t), n, first, maxid, theta, seed)
        return t

    # path -------------------------------------------------------------------
    def partition(self, t: np.ndarray, nbits: int, shift: int, padded: bool):
        fan = 1 << nbits
        cap = len(t) + (fan * 64 // self.width if padded else 0)
        out = np.zeros(cap, self.dtype)
        cnt = np.zeros(fan, np.int64)
        off = np.zeros(fan, np.int64)
        self.fn("partition", None, _P, _I64, _P, C.c_int, C.c_int, C.c_int, _P, _P)(
            _ptr(t), len(t), _ptr(out), nbits, shift, int(padded), _ptr(cnt), _ptr(off))
        return out, cnt, off

    def sort(self, t: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(t).copy()
        self.fn("sort_tuples", None, _P, _I64)(_ptr(a), len(a))
        return a

    def sort_radix(self, t: np.ndarray) -> np.ndarray:
        """sort()'s order by a stable LSD radix sort (the full-size checker)."""
        a = np.ascontiguousarray(t).copy()
        self.fn("sort_tuples_radix", None, _P, _I64)(_ptr(a), len(a))
        return a

    def sort_int64(self, a: np.ndarray) -> np.ndarray:
        b = np.ascontiguousarray(a, dtype=np.int64).copy()
        self.fn("sort_int64", None, _P, _I64)(_ptr(b), len(b))
        return b

    def sort_int64_fp64(self, a: np.ndarray) -> np.ndarray:
        """avxsort_int64's order: the items compared as IEEE doubles."""
        b = np.ascontiguousarray(a, dtype=np.int64).copy()
        self.fn("sort_int64_fp64", None, _P, _I64)(_ptr(b), len(b))
        return b

    def inregister_sort_keyval32(self, items: np.ndarray) -> np.ndarray:
        """avxsort_core.h:1213-1274 on len(items) / 16 blocks (restated)."""
        a = np.ascontiguousarray(items, dtype=np.int64)
        out = np.zeros_like(a)
        self.fn("inregister_sort_keyval32", None, _P, _P, _I64)(_ptr(a), _ptr(out), len(a) // 16)
        return out

    def merge_int64_fp64(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.int64)
        b = np.ascontiguousarray(b, dtype=np.int64)
        out = np.zeros(len(a) + len(b), np.int64)
        self.fn("merge_int64_fp64", _U64, _P, _P, _P, _U64, _U64)(
            _ptr(a), _ptr(b), _ptr(out), len(a), len(b))
        return out

    def merge(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        out = np.zeros(len(a) + len(b), self.dtype)
        self.fn("merge_tuples", _U64, _P, _P, _P, _U64, _U64)(
            _ptr(a), _ptr(b), _ptr(out), len(a), len(b))
        return out

    def multiway_merge(self, runs) -> np.ndarray:
        k = len(runs)
        runs = [np.ascontiguousarray(r) for r in runs]
        total = sum(len(r) for r in runs)
        out = np.zeros(total, self.dtype)
        ptrs = (C.c_void_p * k)(*[_ptr(r) for r in runs])
        lens = (C.c_uint64 * k)(*[len(r) for r in runs])
        self.fn("multiway_merge", _U64, _P, _P, _P, C.c_uint32)(
            _ptr(out), C.cast(ptrs, _P), C.cast(lens, _P), k)
        return out

    def merge_join(self, r: np.ndarray, s: np.ndarray) -> int:
        return int(self.fn("merge_join", _U64, _P, _P, _U64, _U64)(
            _ptr(r), _ptr(s), len(r), len(s)))

    def merge_join_materialize(self, r: np.ndarray, s: np.ndarray) -> np.ndarray:
        """Output tuples of merge_join with JOIN_MATERIALIZE (sorted r, s)."""
        f = self.fn("merge_join_materialize", _U64, _P, _P, _U64, _U64, _P, _U64)
        n = int(f(_ptr(r), _ptr(s), len(r), len(s), None, 0))
        out = np.zeros(n, self.dtype)
        f(_ptr(r), _ptr(s), len(r), len(s), _ptr(out), n)
        return out

    def sortmergejoin(self, r: np.ndarray, s: np.ndarray):
        sr = np.zeros(len(r), self.dtype)
        ss = np.zeros(len(s), self.dtype)
        c = self.fn("sortmergejoin", _U64, _P, _P, _U64, _U64, _P, _P)(
            _ptr(r), _ptr(s), len(r), len(s), _ptr(sr), _ptr(ss))
        return int(c), sr, ss


class Reference(_Lib):
    """The reference compiled from /root/reference (oracle/_ref/libref*.so)."""

    def __init__(self, width: int):
        super().__init__(os.path.join(HERE, "_ref", f"libref{width}.so"), "ref_", width)

    def seed(self, s: int) -> None:
        self.fn("seed", None, C.c_uint)(s)

    def _gen(self, name, n, *extra, argtypes=()):
        t = np.zeros(n, self.dtype)
        self.fn(name, C.c_int, _P, _I64, *argtypes)(_ptr(t), n, *extra)
        return t

    def create_relation_pk(self, n):
        return self._gen("create_relation_pk", n)

    def create_relation_nonunique(self, n, maxid):
        return self._gen("create_relation_nonunique", n, maxid, argtypes=(_I64,))

    def create_relation_fk(self, n, maxid):
        return self._gen("create_relation_fk", n, maxid, argtypes=(_I64,))

    def create_relation_zipf(self, n, maxid, theta):
        return self._gen("create_relation_zipf", n, maxid, theta,
                         argtypes=(_I64, C.c_double))

    def partition(self, t, nbits, shift, variant):
        fan = 1 << nbits
        inp = self._aligned(len(t))
        inp[:] = t
        # 64-byte aligned: the optimized variants flush 64-byte lines with
        # _mm256_stream_si256 (src/partition/partition.c:59-91)
        out = self._aligned(len(t) + fan * 64 // self.width + 64)
        cnt = np.zeros(fan, np.int64)
        off = np.zeros(fan, np.int64)
        self.fn("partition", None, _P, _I64, _P, C.c_int, C.c_int, C.c_int, _P, _P)(
            _ptr(inp), len(t), _ptr(out), nbits, shift, variant, _ptr(cnt), _ptr(off))
        return out, cnt, off

    def _aligned(self, n):
        # 64-byte aligned buffer (+ slack: AVX kernels read past the end)
        raw = np.zeros(n + 64 + 64 // self.width, self.dtype)
        off = (-raw.ctypes.data % 64) // self.width
        return raw[off:off + n]

    def sort(self, t, fn="avxsort_tuples"):
        a = self._aligned(len(t))
        a[:] = t
        b = self._aligned(len(t))
        res = np.zeros(len(t), self.dtype)
        self.fn(fn, None, _P, _P, _U64, _P)(_ptr(a), _ptr(b), len(t), _ptr(res))
        return res

    def sort_int64(self, v):
        a = np.zeros(len(v) + 16, np.int64)[: len(v)]
        a[:] = v
        b = np.zeros(len(v) + 16, np.int64)[: len(v)]
        res = np.zeros(len(v), np.int64)
        self.fn("avxsort_int64", None, _P, _P, _U64, _P)(_ptr(a), _ptr(b), len(v), _ptr(res))
        return res

    def merge_int64(self, a, b):
        A = np.zeros(len(a) + 16, np.int64)[: len(a)]
        A[:] = a
        B = np.zeros(len(b) + 16, np.int64)[: len(b)]
        B[:] = b
        out = np.zeros(len(a) + len(b) + 16, np.int64)[: len(a) + len(b)]
        self.fn("avx_merge_int64", _U64, _P, _P, _P, _U64, _U64)(
            _ptr(A), _ptr(B), _ptr(out), len(a), len(b))
        return np.array(out)

    def inregister_sort_keyval32(self, items):
        """avxsort_core.h:1213-1274 on len(items) / 16 blocks (the AVX kernel)."""
        a = np.ascontiguousarray(items, dtype=np.int64)
        out = np.zeros_like(a)
        self.fn("inregister_sort_keyval32", None, _P, _P, _I64)(_ptr(a), _ptr(out), len(a) // 16)
        return out

    def merge16_varlen(self, a, b):
        """avxsort_core.h:388-500: (output, A and B as the kernel leaves them --
        its last register is flushed into consumed input slots, :461-475)."""
        A = np.zeros(len(a) + 32, np.int64)
        A[: len(a)] = a
        B = np.zeros(len(b) + 32, np.int64)
        B[: len(b)] = b
        out = np.zeros(len(a) + len(b) + 32, np.int64)
        self.fn("merge16_varlen", None, _P, _P, _P, C.c_uint32, C.c_uint32)(
            _ptr(A), _ptr(B), _ptr(out), len(a), len(b))
        return out[: len(a) + len(b)].copy(), A[: len(a)].copy(), B[: len(b)].copy()

    def merge(self, a, b, fn="avx_merge_tuples"):
        A = self._aligned(len(a))
        A[:] = a
        B = self._aligned(len(b))
        B[:] = b
        out = self._aligned(len(a) + len(b))
        self.fn(fn, _U64, _P, _P, _P, _U64, _U64)(_ptr(A), _ptr(B), _ptr(out), len(a), len(b))
        return np.array(out)

    def multiway_merge(self, runs, bufbytes=4 << 20, scalar=False):
        k = len(runs)
        runs = [np.ascontiguousarray(r) for r in runs]
        total = sum(len(r) for r in runs)
        out = self._aligned(total + 64)
        ptrs = (C.c_void_p * k)(*[_ptr(r) for r in runs])
        lens = (C.c_uint64 * k)(*[len(r) for r in runs])
        n = self.fn("multiway_merge", _U64, _P, _P, _P, C.c_uint32, C.c_uint32, C.c_int)(
            _ptr(out), C.cast(ptrs, _P), C.cast(lens, _P), k, bufbytes, int(scalar))
        return np.array(out[:total]), int(n)

    def merge_join(self, r, s):
        return int(self.fn("merge_join", _U64, _P, _P, _U64, _U64)(
            _ptr(r), _ptr(s), len(r), len(s)))

    def sortmergejoin_multiway(self, r, s, nthreads=1, fanout=128, scalar=None):
        if scalar is None:
            scalar = self.width == 16
        return int(self.fn("sortmergejoin_multiway", _I64, _P, _U64, _P, _U64,
                           C.c_int, C.c_int, C.c_int)(
            _ptr(r), len(r), _ptr(s), len(s), nthreads, fanout, int(scalar)))


def reference_available(width: int = 8) -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", f"libref{width}.so"))
