"""Python binding of the MI355X sort-merge-join C ABI (include/smj.h).

This is plumbing over ctypes, not a second implementation: every call lands in
libsmj_hip.so (8-byte tuples) or libsmj_hip_k8.so (16-byte tuples) and runs on
the GPU.  Loading fails loudly when the library is missing, and the library
itself aborts when no HIP device is present (there is no CPU fallback).

Two views of the same library:

* ``Library.<reference name>`` -- the reference's functions on host numpy
  arrays (structured dtype payload-then-key, like ``tuple_t``), used by the
  parity tests: partition_relation[_optimized], avxsort_tuples,
  avx_merge_tuples, avx_multiway_merge, merge_join, sortmergejoin_multiway.
* ``Library.dev_*`` -- the device-resident asynchronous API on torch tensors
  (shape (n, 2): column 0 payload, column 1 key; int32 or int64), used by
  bench.py and the multi-GPU path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

try:  # torch must own the HIP runtime before our library binds to it
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
# SMJ_LIB_DIR selects an alternative build of the same libraries (kernel
# geometry experiments, tools/); the default is the in-tree lib/.
LIBDIR = os.environ.get("SMJ_LIB_DIR") or os.path.join(ROOT, "lib")
TUPLE8 = np.dtype([("payload", "<i4"), ("key", "<i4")])
TUPLE16 = np.dtype([("payload", "<i8"), ("key", "<i8")])

# Every entry point the C ABI exports (include/smj.h).  The CPU test suite
# checks that both libraries export all of them.
REFERENCE_SYMBOLS = [
    "partition_relation", "partition_relation_optimized",
    "partition_relation_optimized_V2", "histogram_memcpy_bench",
    "avxsort_tuples", "avxsort_int64", "avxsort_int32",
    "avxsortmultiway_tuples", "avxsortmultiway_int64",
    "scalarsort_tuples", "scalarsort_int64", "scalarsort_int32",
    "avx_merge_tuples", "avx_merge_int64", "scalar_merge_tuples",
    "scalar_merge_int64", "avx_multiway_merge", "scalar_multiway_merge",
    "scalar_multiway_merge_modulo", "scalar_multiway_merge_bitand",
    "merge_join", "merge_join_interpolation", "print_timing", "sortmergejoin_multiway",
    "sortmergejoin_multipass", "sortmergejoin_mpsm", "sortmergejoin_initrun",
    "chainedtuplebuffer_init", "chainedtuplebuffer_free", "chainedtuplebuffer_tuples",
    "cb_next_writepos", "write_result_relation", "radix_cluster", "is_sorted_helper",
    "check_sorted",
]
DEVICE_SYMBOLS = [
    "smj_tuple_bytes", "smj_device_name", "smj_workspace_create",
    "smj_workspace_destroy", "smj_dev_partition", "smj_dev_sort",
    "smj_dev_merge2", "smj_dev_multiway_merge_host", "smj_dev_merge_join_count",
    "smj_dev_join", "smj_join_phase_ms", "smj_dev_gen_pk", "smj_dev_gen_fk",
    "smj_dev_gen_zipf", "smj_dev_synchronize", "smj_dev_partition_range",
    "smj_trace_enable", "smj_trace_reset", "smj_trace_only", "smj_trace_read", "smj_dev_join_segmented",
    "smj_dev_partition_range_packed", "smj_dev_materialize", "smj_selfcheck_lds_order",
    "smj_set_materialize", "smj_dev_join_segmented_tables", "smj_dev_partition_range_sampled",
    "smj_sampled_capacity", "smj_sampled_shards", "smj_context_workspace",
    "smj_dev_gen_nonunique", "smj_dev_gen_zipf_ref", "smj_glibc_rand",
    "smj_dev_xsend", "smj_dev_xrecv", "smj_join", "smj_dev_partition_range_planes",
    "smj_dev_join_segmented_planes", "smj_mgpu_join", "smj_mgpu_release",
    "smj_inregister_sort_keyval32", "smj_workspace_set_layouts", "smj_mgpu_unique_id",
    "smj_mgpu_comm_init", "smj_mgpu_rank_join", "smj_mgpu_comm_destroy", "smj_mgpu_rank_sorted",
    "smj_mgpu_comm_workspace", "smj_workspace_last_layout", "smj_mgpu_join_slices",
    "smj_mgpu_last_stats", "smj_mgpu_last_sorted", "smj_mgpu_group_workspace",
    "smj_dev_partition_range_shards",
]


def lib_path(width: int) -> str:
    return os.path.join(LIBDIR, "libsmj_hip.so" if width == 8 else "libsmj_hip_k8.so")


def build(jobs: int = 8) -> None:
    """Compile both libraries for gfx950 (hipcc; cross-compiles without a GPU)."""
    import subprocess
    subprocess.check_call(["make", "-C", ROOT, f"-j{jobs}"])


class Relation(C.Structure):
    _fields_ = [("tuples", C.c_void_p), ("num_tuples", C.c_uint64)]


class JoinConfig(C.Structure):
    _fields_ = [("NTHREADS", C.c_int), ("PARTFANOUT", C.c_int),
                ("SCALARSORT", C.c_int), ("SCALARMERGE", C.c_int),
                ("MWAYMERGEBUFFERSIZE", C.c_int), ("NUMASTRATEGY", C.c_int)]


class ThreadResult(C.Structure):
    _fields_ = [("nresults", C.c_int64), ("results", C.c_void_p),
                ("threadid", C.c_uint32)]


class Result(C.Structure):
    _fields_ = [("totalresults", C.c_int64),
                ("resultlist", C.POINTER(ThreadResult)), ("nthreads", C.c_int)]


class MgpuStats(C.Structure):
    """include/smj.h smj_mgpu_stats."""
    _fields_ = [("layout", C.c_int), ("pbits", C.c_uint32), ("attempts", C.c_int),
                ("replans", C.c_int), ("sent_bytes", C.c_uint64), ("recv_bytes", C.c_uint64),
                ("key_min", C.c_int64), ("key_max", C.c_int64), ("ms", C.c_double),
                # device phases, ms (the five before busy_ms add up to it)
                ("partition_ms", C.c_double), ("tables_ms", C.c_double),
                ("wait_ms", C.c_double), ("join_ms", C.c_double), ("reduce_ms", C.c_double),
                ("busy_ms", C.c_double), ("rows_ms", C.c_double)]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["layout"] = MG_LAYOUTS[d["layout"]]
        return d


# smj_workspace_set_layouts bits (include/smj.h)
LAYOUT_NO_P48, LAYOUT_NO_PACKED, LAYOUT_NO_SAMPLED, LAYOUT_SAMPLE_PLAN = 1, 2, 4, 8
LAYOUT_NO_P32, LAYOUT_NO_P96 = 16, 32
# smj_workspace_last_layout values
LAYOUTS_USED = ("tuples", "words", "p48", "p32", "p96")
# smj_mgpu_join flags (include/smj.h)
MG_COPY, MG_NOPLANES, MG_ONECALL, MG_SAMPLED, MG_EXACT = 1, 2, 4, 8, 16
MG_LAYOUTS = ("tuples", "words", "planes")


class MgpuComm:
    """One rank of a multi-process smj_mgpu_comm (Library.mgpu_comm)."""

    def __init__(self, lib, handle):
        self.lib, self.h = lib, handle

    def join(self, R, S, flags=0, key_range=None, guess_max=0):
        """smj_mgpu_rank_join on this rank's device slices (torch tensors of
        shape (n, 2)): (global count, tuples of the rank's sorted R share and
        S share, stats); sorted() copies the shares out."""
        L = self.lib
        nR, nS = C.c_uint64(), C.c_uint64()
        st = MgpuStats()
        kmin, kmax = key_range if key_range is not None else (1, 0)
        # the library's streams read R and S: torch's writes must be done
        torch.cuda.current_stream(R.device).synchronize()
        c = L.lib.smj_mgpu_rank_join(self.h, R.data_ptr(), R.shape[0], S.data_ptr(),
                                     S.shape[0], flags, kmin, kmax, guess_max, None,
                                     C.byref(nR), None, C.byref(nS), C.byref(st))
        stats = st.as_dict()
        self.n = (nR.value, nS.value)
        return int(c), nR.value, nS.value, stats

    def sorted(self):
        """The rank's sorted shares of the last join, copied into new device
        tensors."""
        sR, sS = self.lib.empty(self.n[0]), self.lib.empty(self.n[1])
        self.lib.lib.smj_mgpu_rank_sorted(self.h, sR.data_ptr() if self.n[0] else None,
                                          sS.data_ptr() if self.n[1] else None)
        return sR, sS

    def close(self):
        if self.h:
            self.lib.lib.smj_mgpu_comm_destroy(self.h)
            self.h = None


class ChainedTupleBuffer(C.Structure):
    """include/smj.h: the library's chainedtuplebuffer_t (one growable array)."""
    _fields_ = [("tuples", C.c_void_p), ("numtuples", C.c_uint64),
                ("capacity", C.c_uint64)]


_P = C.c_void_p
_U64 = C.c_uint64
_I64 = C.c_int64
_U32 = C.c_uint32


_HIP = None


def _hip_copy(dst: int, src: int, nbytes: int) -> None:
    """hipMemcpy(dst, src, nbytes, hipMemcpyDefault) through the HIP runtime
    torch has loaded (device pointers the library hands out)."""
    global _HIP
    if _HIP is None:
        _HIP = C.CDLL("libamdhip64.so")
        _HIP.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _HIP.hipMemcpy.restype = C.c_int
    rc = _HIP.hipMemcpy(dst, src, nbytes, 4)
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed: {rc}")


def _ptr(a):
    return a.ctypes.data


class Library:
    def __init__(self, width: int = 16, path: str | None = None):
        assert width in (8, 16)
        self.width = width
        self.dtype = TUPLE8 if width == 8 else TUPLE16
        self.path = path or lib_path(width)
        if not os.path.exists(self.path):
            raise FileNotFoundError(
                f"{self.path} missing: build it with `make -C {ROOT}` "
                "(there is no CPU fallback)")
        self.lib = C.CDLL(self.path)
        L = self.lib
        sig = {
            "partition_relation": (None, [_P, _P, _P, C.c_int, C.c_int]),
            "partition_relation_optimized": (None, [_P, _P, _P, _U32, _U32]),
            "partition_relation_optimized_V2": (None, [_P, _P, _P, _U32, _U32]),
            "histogram_memcpy_bench": (None, [_P, _P, _P, _U32]),
            "avxsort_tuples": (None, [_P, _P, _U64]),
            "avxsort_int64": (None, [_P, _P, _U64]),
            "avxsort_int32": (None, [_P, _P, _U64]),
            "avxsortmultiway_tuples": (None, [_P, _P, _U64]),
            "avxsortmultiway_int64": (None, [_P, _P, _U64]),
            "scalarsort_tuples": (None, [_P, _P, _U64]),
            "scalarsort_int64": (None, [_P, _P, _U64]),
            "scalarsort_int32": (None, [_P, _P, _U64]),
            "avx_merge_tuples": (_U64, [_P, _P, _P, _U64, _U64]),
            "avx_merge_int64": (_U64, [_P, _P, _P, _U64, _U64]),
            "scalar_merge_tuples": (_U64, [_P, _P, _P, _U64, _U64]),
            "scalar_merge_int64": (_U64, [_P, _P, _P, _U64, _U64]),
            "avx_multiway_merge": (_U64, [_P, _P, _U32, _P, _U32]),
            "scalar_multiway_merge": (_U64, [_P, _P, _U32, _P, _U32]),
            "merge_join": (_U64, [_P, _P, _U64, _U64, _P]),
            "sortmergejoin_multiway": (C.POINTER(Result), [_P, _P, _P]),
            "sortmergejoin_multipass": (C.POINTER(Result), [_P, _P, _P]),
            "sortmergejoin_mpsm": (C.POINTER(Result), [_P, _P, _P]),
            "chainedtuplebuffer_init": (C.POINTER(ChainedTupleBuffer), []),
            "chainedtuplebuffer_free": (None, [_P]),
            "chainedtuplebuffer_tuples": (_U64, [_P]),
            "cb_next_writepos": (_P, [_P]),
            "write_result_relation": (None, [_P, C.c_char_p]),
            "smj_set_materialize": (None, [C.c_int]),
            "smj_join": (C.POINTER(Result), [_P, _P, _P, C.c_int, C.c_int]),
            "radix_cluster": (None, [_P, _P, _P, C.c_int, C.c_int]),
            "is_sorted_helper": (C.c_int, [_P, _U64]),
            "check_sorted": (None, [_P, _P, _U64, _U64, C.c_int]),
            "smj_tuple_bytes": (C.c_int, []),
            "smj_device_name": (C.c_char_p, []),
            "smj_workspace_create": (_P, []),
            "smj_workspace_destroy": (None, [_P]),
            "smj_dev_partition": (None, [_P, _P, _U64, _P, _U32, _U32, C.c_int, _P, _P, _P]),
            "smj_dev_sort": (None, [_P, _P, _U64, _P, _P]),
            "smj_dev_merge2": (None, [_P, _U64, _P, _U64, _P, _P]),
            "smj_dev_multiway_merge_host": (None, [_P, _P, _P, _U32, _P, _P]),
            "smj_dev_merge_join_count": (None, [_P, _U64, _P, _U64, _P, _P]),
            "smj_dev_join": (None, [_P, _P, _U64, _P, _U64, _P, _P, _U32, _I64, _I64, _P, _P]),
            "smj_join_phase_ms": (None, [_P, _P]),
            "smj_dev_gen_pk": (None, [_P, _U64, _U64, _U64, _U64, C.c_int, _P]),
            "smj_dev_gen_fk": (None, [_P, _U64, _U64, _U64, _U64, _U64, _P]),
            "smj_dev_gen_zipf": (None, [_P, _P, _U64, _U64, _U64, C.c_double, _U64, _P]),
            "smj_dev_synchronize": (None, [_P]),
            "smj_dev_partition_range": (None, [_P, _P, _U64, _P, _U32, _I64, _I64, _P, _P]),
            "smj_dev_join_segmented": (None, [_P, _P, _U64, _P, _P, _U64, _P, _U32, _U32,
                                              _I64, _I64, _U32, _P, _P, _P, _P]),
            "smj_dev_partition_range_packed": (C.c_int, [_P, _P, _U64, _P, _U32, _I64, _I64,
                                                         _P, _P, _P]),
            "smj_dev_join_segmented_tables": (None, [_P, _P, _U64, _P, _P, _P, _U64, _P, _P,
                                                     _U32, _U32, _I64, _I64, _U32, _P, _P,
                                                     _P, _P]),
            "smj_dev_partition_range_sampled": (C.c_int, [_P, _P, _U64, _P, _U32, _I64, _I64,
                                                          C.c_int, _P, _P, _P, _P]),
            "smj_dev_partition_range_shards": (C.c_int, [_P, _P, _U64, _P, _U32, _I64, _I64,
                                                         C.c_int, _P, _P, _P, _P]),
            "smj_dev_partition_range_planes": (C.c_int, [_P, _P, _U64, _P, _U64, _U32, _I64,
                                                         _I64, _P, _P, _P, _P]),
            "smj_dev_join_segmented_planes": (None, [_P, _P, _U64, _U64, _P, _P, _P, _U64,
                                                     _U64, _P, _P, _U32, _U32, _I64, _I64,
                                                     _U32, _P, _P, _P, _P]),
            "smj_sampled_capacity": (_U64, [_U64, _U32]),
            "smj_sampled_shards": (_U32, []),
            "smj_dev_materialize": (_U64, [_P, _P, _U64, _P, _U64, _P, _U64, _P]),
            "smj_selfcheck_lds_order": (_U64, [_P, _P]),
            "smj_context_workspace": (_P, []),
            "smj_dev_gen_nonunique": (None, [_P, _P, _U64, _U64, _U64, _I64, _U32, _U64, _P]),
            "smj_dev_gen_zipf_ref": (None, [_P, _P, _U64, _U64, _U64, C.c_double, _U32, _U64,
                                            _P]),
            "smj_glibc_rand": (_U32, [_U32, _U64]),
            "smj_dev_xsend": (None, [_P, _P, _P, _U32, _U32, _U32, _U32, _P, _P, _P]),
            "smj_dev_xrecv": (None, [_P, _P, _U32, _U32, _U32, _U32, _U32, _U64, _P, _P, _P,
                                     _P]),
            "smj_mgpu_join": (_I64, [_P, _U64, _P, _U64, C.c_int, _U32, _I64, _I64, _P, _P,
                                     _P, _P]),
            "smj_mgpu_release": (None, []),
            "smj_mgpu_join_slices": (_I64, [_P, _P, _P, _P, C.c_int, _U32, _I64, _I64, _P, _P]),
            "smj_mgpu_last_stats": (C.c_int, [C.c_int, _P]),
            "smj_mgpu_group_workspace": (_P, [C.c_int]),
            "smj_mgpu_last_sorted": (C.c_int, [C.c_int, _P, _P, _P, _P]),
            "smj_mgpu_unique_id": (C.c_int, [_P, C.c_int]),
            "smj_mgpu_comm_init": (_P, [_P, C.c_int, C.c_int]),
            "smj_mgpu_rank_join": (_I64, [_P, _P, _U64, _P, _U64, _U32, _I64, _I64, _U64,
                                          _P, _P, _P, _P, _P]),
            "smj_mgpu_comm_destroy": (None, [_P]),
            "smj_mgpu_rank_sorted": (None, [_P, _P, _P]),
            "smj_mgpu_comm_workspace": (_P, [_P]),
            "smj_inregister_sort_keyval32": (None, [_P, _P, _U64]),
            "smj_workspace_set_layouts": (None, [_P, _U32]),
            "smj_workspace_last_layout": (C.c_int, [_P]),
            "smj_trace_enable": (None, [_P, C.c_int]),
            "smj_trace_reset": (None, [_P]),
            "smj_trace_only": (None, [_P, C.c_char_p]),
            "smj_trace_read": (C.c_int, [_P, C.c_char_p, C.c_int, _P, _P, C.c_int]),
        }
        for name, (res, args) in sig.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                # an older build loaded for an A/B (SMJ_LIB_DIR): its missing
                # entry points stay unbound; the shipped library has them all
                if os.environ.get("SMJ_LIB_DIR"):
                    continue
                raise
            f.restype = res
            f.argtypes = args
        got = L.smj_tuple_bytes()
        assert got == width, f"{self.path} built for {got}-byte tuples"
        self._ws = None

    # ------------------------------------------------------------------ host
    def _rel(self, a: np.ndarray) -> Relation:
        return Relation(a.ctypes.data, len(a))

    def _parts(self, fan: int):
        rels = (Relation * fan)()
        ptrs = (C.POINTER(Relation) * fan)(*[C.pointer(rels[i]) for i in range(fan)])
        return rels, ptrs

    def partition(self, t: np.ndarray, nbits: int, shift: int, variant: int = 1):
        """variant 0 = partition_relation, 1 = _optimized, 2 = _optimized_V2.
        Returns (output buffer, counts, offsets in tuples)."""
        fan = 1 << nbits
        t = np.ascontiguousarray(t, dtype=self.dtype)
        out = np.zeros(len(t) + fan * 64 // self.width, self.dtype)
        rin, rout = self._rel(t), self._rel(out)
        rout.num_tuples = len(t)
        rels, ptrs = self._parts(fan)
        fn = [self.lib.partition_relation, self.lib.partition_relation_optimized,
              self.lib.partition_relation_optimized_V2][variant]
        fn(C.cast(ptrs, _P), C.byref(rin), C.byref(rout), nbits, shift)
        base = out.ctypes.data
        cnt = np.array([rels[i].num_tuples for i in range(fan)], np.int64)
        off = np.array([(rels[i].tuples - base) // self.width for i in range(fan)], np.int64)
        return out, cnt, off

    def radix_cluster(self, t: np.ndarray, shift: int, bits: int, hist=None):
        """radix_cluster (partition.c:93-149): returns (output, updated int32
        hist).  `hist` (int32, 2^bits) is the caller's histogram the
        reference adds to; zeros by default."""
        t = np.ascontiguousarray(t, dtype=self.dtype)
        h = np.zeros(1 << bits, np.int32) if hist is None else \
            np.ascontiguousarray(hist, dtype=np.int32).copy()
        out = np.zeros(len(t) + int(h.sum()), self.dtype)
        rin, rout = self._rel(t), self._rel(out)
        self.lib.radix_cluster(C.byref(rout), C.byref(rin), _ptr(h), shift, bits)
        return out, h

    def is_sorted_helper(self, t: np.ndarray) -> int:
        t = np.ascontiguousarray(t, dtype=self.dtype)
        return int(self.lib.is_sorted_helper(_ptr(t) if len(t) else None, len(t)))

    def avxsort_tuples(self, t: np.ndarray, fn: str = "avxsort_tuples") -> np.ndarray:
        a = np.ascontiguousarray(t, dtype=self.dtype).copy()
        b = np.zeros_like(a)
        pa, pb = C.c_void_p(a.ctypes.data), C.c_void_p(b.ctypes.data)
        getattr(self.lib, fn)(C.byref(pa), C.byref(pb), len(a))
        res = b if pb.value == b.ctypes.data else a
        return res.copy()

    def sort_int(self, v: np.ndarray, fn: str = "avxsort_int64") -> np.ndarray:
        dt = np.int32 if fn.endswith("int32") else np.int64
        a = np.ascontiguousarray(v, dtype=dt).copy()
        b = np.zeros_like(a)
        pa, pb = C.c_void_p(a.ctypes.data), C.c_void_p(b.ctypes.data)
        getattr(self.lib, fn)(C.byref(pa), C.byref(pb), len(a))
        return (b if pb.value == b.ctypes.data else a).copy()

    def inregister_sort_keyval32(self, items: np.ndarray) -> np.ndarray:
        """smj_inregister_sort_keyval32 on len(items) / 16 blocks."""
        a = np.ascontiguousarray(items, dtype=np.int64)
        out = np.zeros_like(a)
        self.lib.smj_inregister_sort_keyval32(_ptr(a), _ptr(out), len(a) // 16)
        return out

    def merge_int64(self, a, b, fn="avx_merge_int64") -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.int64)
        b = np.ascontiguousarray(b, dtype=np.int64)
        out = np.zeros(len(a) + len(b), np.int64)
        n = getattr(self.lib, fn)(_ptr(a), _ptr(b), _ptr(out), len(a), len(b))
        assert n == len(out)
        return out

    def avx_merge_tuples(self, a, b, fn="avx_merge_tuples") -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=self.dtype)
        b = np.ascontiguousarray(b, dtype=self.dtype)
        out = np.zeros(len(a) + len(b), self.dtype)
        n = getattr(self.lib, fn)(_ptr(a), _ptr(b), _ptr(out), len(a), len(b))
        assert n == len(out)
        return out

    def avx_multiway_merge(self, runs, fn="avx_multiway_merge"):
        runs = [np.ascontiguousarray(r, dtype=self.dtype) for r in runs]
        k = len(runs)
        total = sum(len(r) for r in runs)
        out = np.zeros(total, self.dtype)
        rels = (Relation * k)(*[Relation(r.ctypes.data, len(r)) for r in runs])
        ptrs = (C.POINTER(Relation) * k)(*[C.pointer(rels[i]) for i in range(k)])
        fifo = np.zeros(1 << 16, self.dtype)
        n = getattr(self.lib, fn)(_ptr(out), C.cast(ptrs, _P), k, _ptr(fifo), len(fifo))
        consumed = all(rels[i].num_tuples == 0 and
                       rels[i].tuples == runs[i].ctypes.data + len(runs[i]) * self.width
                       for i in range(k))
        return out, int(n), consumed

    def merge_join(self, r, s) -> int:
        r = np.ascontiguousarray(r, dtype=self.dtype)
        s = np.ascontiguousarray(s, dtype=self.dtype)
        return int(self.lib.merge_join(_ptr(r), _ptr(s), len(r), len(s), None))

    def _take_buffer(self, cb) -> np.ndarray:
        """Copy a chainedtuplebuffer_t's tuples out (the buffer is not freed)."""
        n = int(self.lib.chainedtuplebuffer_tuples(cb))
        if n == 0:
            return np.zeros(0, self.dtype)
        b = C.cast(cb, C.POINTER(ChainedTupleBuffer)).contents
        raw = C.string_at(b.tuples, n * self.width)
        return np.frombuffer(raw, dtype=self.dtype).copy()

    def merge_join_materialize(self, r, s, prefix=None):
        """merge_join with an output buffer (JOIN_MATERIALIZE).  `prefix`:
        tuples written into the buffer with cb_next_writepos first (the
        matches are appended after them).  Returns (count, buffer tuples)."""
        r = np.ascontiguousarray(r, dtype=self.dtype)
        s = np.ascontiguousarray(s, dtype=self.dtype)
        cb = self.lib.chainedtuplebuffer_init()
        try:
            for t in (prefix if prefix is not None else []):
                p = self.lib.cb_next_writepos(cb)
                C.memmove(p, np.array([t], self.dtype).ctypes.data, self.width)
            n = int(self.lib.merge_join(_ptr(r), _ptr(s), len(r), len(s), cb))
            return n, self._take_buffer(cb)
        finally:
            self.lib.chainedtuplebuffer_free(cb)

    def mgpu_join(self, R, S, nranks=0, flags=0, key_range=None, sorted_out=True):
        """smj_mgpu_join: the multi-GPU join of sortmergejoin_mpsm over
        `nranks` ranks (0: one per visible GPU; MG_COPY: ranks may share a
        GPU).  R and S are host numpy arrays or device torch tensors (shape
        (n, 2)).  Returns (count, sorted R, sorted S, per-rank (nR, nS),
        stats dict); the sorted relations are the ranks' shares in rank order
        (None unless sorted_out)."""
        dev = not isinstance(R, np.ndarray)
        if dev:
            # the ranks read device inputs on their own streams, which do not
            # wait for torch's: order the call after every pending write
            for t in (R, S):
                torch.cuda.current_stream(t.device).synchronize()
            nR, nS = R.shape[0], S.shape[0]
            pR, pS = R.data_ptr(), S.data_ptr()
            sR = R.new_empty(R.shape) if sorted_out else None
            sS = S.new_empty(S.shape) if sorted_out else None
            qR = sR.data_ptr() if sorted_out else None
            qS = sS.data_ptr() if sorted_out else None
        else:
            R = np.ascontiguousarray(R, dtype=self.dtype)
            S = np.ascontiguousarray(S, dtype=self.dtype)
            nR, nS = len(R), len(S)
            pR, pS = (_ptr(R) if nR else None), (_ptr(S) if nS else None)
            sR = np.zeros(nR, self.dtype) if sorted_out else None
            sS = np.zeros(nS, self.dtype) if sorted_out else None
            qR = _ptr(sR) if sorted_out and nR else None
            qS = _ptr(sS) if sorted_out and nS else None
        G = nranks
        if G <= 0:
            import torch as _t
            G = _t.cuda.device_count()
        counts = np.zeros(2 * G, np.uint64)
        st = MgpuStats()
        kmin, kmax = key_range if key_range is not None else (1, 0)
        c = self.lib.smj_mgpu_join(pR, nR, pS, nS, G, flags, kmin, kmax, qR, qS,
                                   _ptr(counts), C.byref(st))
        return int(c), sR, sS, counts.reshape(G, 2), st.as_dict()

    def mgpu_join_slices(self, Rs, Ss, flags=0, key_range=None):
        """smj_mgpu_join_slices: rank g joins the slices Rs[g] and Ss[g]
        (device tensors on GPU g, shape (n, 2); read in place) -- a relation
        already sharded over the GPUs' HBM, one host thread per GPU inside
        this process (the reference's T join threads, joincommon.c:118-165).
        Returns (count, per-rank (nR, nS) sorted, [per-rank stats dicts]);
        mgpu_last_sorted(g) copies rank g's sorted shares out."""
        G = len(Rs)
        assert G == len(Ss) and G >= 1
        for t in list(Rs) + list(Ss):
            torch.cuda.current_stream(t.device).synchronize()
        P, U = C.c_void_p * G, C.c_uint64 * G
        pR = P(*[t.data_ptr() if t.shape[0] else None for t in Rs])
        pS = P(*[t.data_ptr() if t.shape[0] else None for t in Ss])
        nR = U(*[t.shape[0] for t in Rs])
        nS = U(*[t.shape[0] for t in Ss])
        counts = np.zeros(2 * G, np.uint64)
        st = MgpuStats()
        kmin, kmax = key_range if key_range is not None else (1, 0)
        c = self.lib.smj_mgpu_join_slices(pR, nR, pS, nS, G, flags, kmin, kmax, _ptr(counts),
                                          C.byref(st))
        return int(c), counts.reshape(G, 2), [self.mgpu_last_stats(g) for g in range(G)]

    def mgpu_last_stats(self, rank):
        """smj_mgpu_last_stats: rank `rank`'s stats of the last smj_mgpu_join /
        _slices call (its device phases)."""
        st = MgpuStats()
        if self.lib.smj_mgpu_last_stats(rank, C.byref(st)) != 0:
            raise IndexError(f"no rank {rank} in the last multi-GPU join")
        return st.as_dict()

    def mgpu_last_sorted(self, rank, device):
        """Rank `rank`'s sorted shares of the last smj_mgpu_join / _slices
        call, copied into new tensors on `device` (the rank's GPU)."""
        pR, pS = C.c_void_p(), C.c_void_p()
        nR, nS = C.c_uint64(), C.c_uint64()
        if self.lib.smj_mgpu_last_sorted(rank, C.byref(pR), C.byref(nR), C.byref(pS),
                                         C.byref(nS)) != 0:
            raise IndexError(f"no rank {rank} in the last multi-GPU join")
        out = []
        for p, n in ((pR, nR.value), (pS, nS.value)):
            t = self.empty(n, device=device)
            if n:
                _hip_copy(t.data_ptr(), p.value, n * self.width)
            out.append(t)
        return tuple(out)

    def mgpu_comm(self, nranks, rank, group=None):
        """smj_mgpu_comm_init for this process's rank of a torch.distributed
        group (one process per GPU): rank 0's id is broadcast over `group`."""
        import torch.distributed as dist
        idb = np.zeros(128, np.uint8)
        if rank == 0:
            n = self.lib.smj_mgpu_unique_id(_ptr(idb), len(idb))
            assert n == 128, n
        if nranks > 1:
            t = torch.from_numpy(idb.astype(np.int64))
            if dist.get_backend(group) == "nccl":
                t = t.cuda()
            dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0,
                           group=group)
            idb = t.cpu().numpy().astype(np.uint8)
        c = self.lib.smj_mgpu_comm_init(_ptr(idb), nranks, rank)
        return MgpuComm(self, c)

    def sortmergejoin_multiway(self, R, S, nthreads=1, fanout=128, mpsm=False,
                               algo=None, materialize=False, persist=None):
        """algo: "m-way" (default), "m-pass" or "mpsm" -- the reference's
        sortmergejoins -a choices (src/main.c:455-466).  materialize: also
        return the output tuples (JOIN_MATERIALIZE); persist: a file name the
        result is appended to with write_result_relation (PERSIST_RELATIONS).
        Returns the count, or (count, output tuples)."""
        R = np.ascontiguousarray(R, dtype=self.dtype)
        S = np.ascontiguousarray(S, dtype=self.dtype)
        cfg = JoinConfig(nthreads, fanout, int(self.width == 16), int(self.width == 16),
                         20 << 20, 2)
        rr, rs = self._rel(R), self._rel(S)
        algo = algo or ("mpsm" if mpsm else "m-way")
        code = {"m-way": 0, "m-pass": 1, "mpsm": 2}[algo]
        # the materialisation is this call's own (smj_join), not the process
        # switch the reference-named functions read
        res = self.lib.smj_join(C.byref(rr), C.byref(rs), C.byref(cfg), code,
                                1 if (materialize or persist) else 0)
        if not res:
            return None
        total = int(res.contents.totalresults)
        out = None
        if materialize or persist:
            if persist:  # main.c:609-614
                self.lib.write_result_relation(C.cast(res, _P), os.fsencode(persist))
            lists = [res.contents.resultlist[i].results for i in range(max(nthreads, 1))]
            out = np.concatenate([self._take_buffer(cb) for cb in lists if cb] or
                                 [np.zeros(0, self.dtype)])
            for cb in lists:  # main.c:621-626
                self.lib.chainedtuplebuffer_free(cb)
        # the caller frees the result (src/main.c:629-632)
        libc = C.CDLL(None)
        libc.free.argtypes = [C.c_void_p]
        libc.free(res.contents.resultlist)
        libc.free(C.cast(res, C.c_void_p))
        return total if out is None else (total, out)

    # ---------------------------------------------------------------- device
    @property
    def ws(self):
        if self._ws is None:
            self._ws = self.lib.smj_workspace_create()
        return self._ws

    def set_layouts(self, off: int = 0):
        """smj_workspace_set_layouts on this Library's workspace (LAYOUT_*
        bits: layouts its device sorts and joins may not use; 0 = all)."""
        self.lib.smj_workspace_set_layouts(self.ws, off)

    def reset_workspace(self):
        """Destroy this Library's workspace (its scratch and its remembered
        layouts); the next device call creates a fresh one."""
        if self._ws is not None:
            import torch
            torch.cuda.synchronize()
            self.lib.smj_workspace_destroy(self._ws)
            self._ws = None

    def last_layout(self, api: bool = False) -> str:
        """The intermediate layout the last device sort or join finished in
        (smj_workspace_last_layout): on this Library's workspace, or (api)
        on the calling thread's, which the reference-named entries use."""
        f = getattr(self.lib, "smj_workspace_last_layout", None)
        if f is None or f.restype is not C.c_int:  # an older A/B build
            return "unknown"
        k = f(None if api else self.ws)
        return LAYOUTS_USED[k] if k >= 0 else "none"

    @staticmethod
    def stream_ptr():
        return torch.cuda.current_stream().cuda_stream

    def empty(self, n: int, device="cuda"):
        dt = torch.int32 if self.width == 8 else torch.int64
        return torch.empty((max(n, 1), 2), dtype=dt, device=device)[:n]

    def to_device(self, a: np.ndarray):
        v = np.ascontiguousarray(a, dtype=self.dtype).view(
            np.int32 if self.width == 8 else np.int64).reshape(-1, 2)
        return torch.from_numpy(v.copy()).cuda()

    def to_host(self, t) -> np.ndarray:
        return t.cpu().numpy().reshape(-1).view(self.dtype).copy()

    def dev_gen_pk(self, out, first, total, seed, with_payload=True):
        self.lib.smj_dev_gen_pk(out.data_ptr(), out.shape[0], first, total, seed,
                                int(with_payload), self.stream_ptr())

    def dev_gen_fk(self, out, first, total, maxid, seed):
        self.lib.smj_dev_gen_fk(out.data_ptr(), out.shape[0], first, total, maxid,
                                seed, self.stream_ptr())

    def dev_gen_zipf(self, out, first, maxid, theta, seed):
        self.lib.smj_dev_gen_zipf(self.ws, out.data_ptr(), out.shape[0], first, maxid,
                                  theta, seed, self.stream_ptr())

    def dev_gen_nonunique(self, out, first, total, maxid, seed, skip=0):
        """create_relation_nonunique after srand(seed) and `skip` rand() calls,
        tuples [first, first + len(out)) of `total` (bit-exact, refgen.hip)."""
        self.lib.smj_dev_gen_nonunique(self.ws, out.data_ptr(), out.shape[0], first, total,
                                       maxid, seed, skip, self.stream_ptr())

    def dev_gen_zipf_ref(self, out, first, maxid, theta, seed, skip=0):
        """create_relation_zipf after srand(seed) and `skip` rand() calls
        (bit-exact; the payload is 0)."""
        self.lib.smj_dev_gen_zipf_ref(self.ws, out.data_ptr(), out.shape[0], first, maxid,
                                      theta, seed, skip, self.stream_ptr())

    def dev_xsend(self, start, cnt, flags, world, msg, chunk, used=0):
        """smj_dev_xsend: start/cnt (F, K) int64, flags int64[2]; `used`: the
        partitions the key range reaches (0 = all)."""
        F, K = start.shape
        self.lib.smj_dev_xsend(start.data_ptr(), cnt.data_ptr(), flags.data_ptr(), F, K, world,
                               used, msg.data_ptr(), chunk.data_ptr(), self.stream_ptr())

    def dev_xrecv(self, msg, chunk, world, rank, mine, K, tstart, tcnt, cap, summary):
        """smj_dev_xrecv: msg (world, 4 + 2 K mine), tstart/tcnt (nb, world K)."""
        self.lib.smj_dev_xrecv(msg.data_ptr(), chunk.data_ptr(), world, rank, mine, K,
                               tstart.shape[0], cap, tstart.data_ptr(), tcnt.data_ptr(),
                               summary.data_ptr(), self.stream_ptr())

    def glibc_rand(self, seed, k):
        return int(self.lib.smj_glibc_rand(seed, k))

    def dev_sort(self, inp, out):
        self.lib.smj_dev_sort(self.ws, inp.data_ptr(), inp.shape[0], out.data_ptr(),
                              self.stream_ptr())

    def dev_partition(self, inp, out, nbits, shift, padded, hist, off):
        self.lib.smj_dev_partition(self.ws, inp.data_ptr(), inp.shape[0], out.data_ptr(),
                                   nbits, shift, int(padded), hist.data_ptr(),
                                   off.data_ptr(), self.stream_ptr())

    def dev_merge2(self, a, b, out):
        self.lib.smj_dev_merge2(a.data_ptr(), a.shape[0], b.data_ptr(), b.shape[0],
                                out.data_ptr(), self.stream_ptr())

    def dev_merge_join_count(self, r, s, count):
        self.lib.smj_dev_merge_join_count(r.data_ptr(), r.shape[0], s.data_ptr(),
                                          s.shape[0], count.data_ptr(), self.stream_ptr())

    @staticmethod
    def run_table(runs):
        """(pointer array, length array, k) of a list of device runs, built
        once for callers that merge the same runs repeatedly."""
        k = len(runs)
        ptrs = (C.c_void_p * k)(*[r.data_ptr() for r in runs])
        lens = (C.c_uint64 * k)(*[r.shape[0] for r in runs])
        return C.cast(ptrs, _P), C.cast(lens, _P), k, (ptrs, lens)

    def dev_multiway_merge(self, runs, out):
        """k-way merge of sorted device runs (list of (n_i, 2) tensors, or a
        run_table of them) into `out` (smj_dev_multiway_merge_host;
        stream-ordered, no host synchronisation for 3..256 runs)."""
        ptrs, lens, k, _keep = runs if isinstance(runs, tuple) else self.run_table(runs)
        self.lib.smj_dev_multiway_merge_host(self.ws, ptrs, lens, k, out.data_ptr(),
                                             self.stream_ptr())

    def dev_materialize(self, sortedR, sortedS, out=None):
        """Materialised merge join (smj_dev_materialize): writes the first
        len(out) output tuples <S.key, S.payload> and returns the total."""
        cap = 0 if out is None else out.shape[0]
        return int(self.lib.smj_dev_materialize(
            self.ws, sortedR.data_ptr(), sortedR.shape[0], sortedS.data_ptr(),
            sortedS.shape[0], out.data_ptr() if cap else None, cap, self.stream_ptr()))

    def dev_join(self, R, S, sortedR, sortedS, count, fanout_bits=10,
                 key_min=1, key_max=0):
        self.lib.smj_dev_join(self.ws, R.data_ptr(), R.shape[0], S.data_ptr(),
                              S.shape[0], sortedR.data_ptr(), sortedS.data_ptr(),
                              fanout_bits, key_min, key_max, count.data_ptr(),
                              self.stream_ptr())

    def dev_join_segmented(self, R, segR, S, segS, bucket_bits, key_lo, key_hi,
                           sortedR, sortedS, count, packed=False):
        """Local join of exchanged range partitions (smj_dev_join_segmented):
        segR/segS are int64 (nseg, 2^bucket_bits) device tensors, row s = the
        partition sizes received from source s.  R and S (tuples, or with
        packed=True int64 words of dev_partition_range_packed) are
        overwritten."""
        assert segR.is_contiguous() and segS.is_contiguous()
        assert segR.shape == segS.shape and segR.shape[1] == 1 << bucket_bits
        self.lib.smj_dev_join_segmented(
            self.ws, R.data_ptr(), R.shape[0], segR.data_ptr(), S.data_ptr(),
            S.shape[0], segS.data_ptr(), segR.shape[0], bucket_bits, key_lo, key_hi,
            1 if packed else 0, sortedR.data_ptr(), sortedS.data_ptr(), count.data_ptr(),
            self.stream_ptr())

    def dev_join_segmented_tables(self, R, nR, startR, cntR, S, nS, startS, cntS, bucket_bits,
                                  key_lo, key_hi, sortedR, sortedS, count, packed=False,
                                  stage=None):
        """smj_dev_join_segmented from explicit segment tables: start/cnt are
        int64 (2^bucket_bits, nseg) device tensors (element offsets into R /
        S and counts); nR / nS count the elements inside the segments.
        stage: None (the whole join), "R" (R's tile stage only) or "REST" (the
        rest, after a "R" call with the same arguments)."""
        for t in (startR, cntR, startS, cntS):
            assert t.is_contiguous() and t.shape == startR.shape
        assert startR.shape[0] == 1 << bucket_bits
        flags = (1 if packed else 0) | {None: 0, "R": 2, "REST": 4}[stage]
        self.lib.smj_dev_join_segmented_tables(
            self.ws, R.data_ptr(), nR, startR.data_ptr(), cntR.data_ptr(), S.data_ptr(), nS,
            startS.data_ptr(), cntS.data_ptr(), startR.shape[1], bucket_bits, key_lo, key_hi,
            flags, sortedR.data_ptr(), sortedS.data_ptr(), count.data_ptr(),
            self.stream_ptr())

    def dev_join_segmented_planes(self, R, strideR, nR, startR, cntR, S, strideS, nS, startS,
                                  cntS, bucket_bits, key_lo, key_hi, sortedR, sortedS, count,
                                  stage=None):
        """smj_dev_join_segmented_tables on 48-bit words in two planes (R / S:
        device buffers of 6 * stride bytes, smj_dev_partition_range_planes'
        layout)."""
        for t in (startR, cntR, startS, cntS):
            assert t.is_contiguous() and t.shape == startR.shape
        assert startR.shape[0] == 1 << bucket_bits
        for X, st in ((R, strideR), (S, strideS)):
            assert X.numel() * X.element_size() >= 6 * st and st % 32 == 0
        flags = {None: 0, "R": 2, "REST": 4}[stage]
        self.lib.smj_dev_join_segmented_planes(
            self.ws, R.data_ptr(), strideR, nR, startR.data_ptr(), cntR.data_ptr(),
            S.data_ptr(), strideS, nS, startS.data_ptr(), cntS.data_ptr(), startR.shape[1],
            bucket_bits, key_lo, key_hi, flags, sortedR.data_ptr(), sortedS.data_ptr(),
            count.data_ptr(), self.stream_ptr())

    def dev_partition_range_planes(self, inp, out, stride, nbits, key_min, key_max, seg_start,
                                   seg_cnt, flags):
        """smj_dev_partition_range_planes: `out` a device buffer of 6 * stride
        bytes; False when the form does not apply (nothing launched)."""
        assert out.numel() * out.element_size() >= 6 * stride
        return bool(self.lib.smj_dev_partition_range_planes(
            self.ws, inp.data_ptr(), inp.shape[0], out.data_ptr(), stride, nbits, key_min,
            key_max, seg_start.data_ptr(), seg_cnt.data_ptr(), flags.data_ptr(),
            self.stream_ptr()))

    def sampled_capacity(self, n, nbits):
        return int(self.lib.smj_sampled_capacity(n, nbits))

    def sampled_shards(self):
        return int(self.lib.smj_sampled_shards())

    def dev_partition_range_sampled(self, inp, out, nbits, key_min, key_max, packed,
                                    seg_start, seg_cnt, flags):
        """smj_dev_partition_range_sampled: seg_start/seg_cnt int64 device
        tensors of 2^nbits * shards, flags int32[2]; False when the form does
        not apply (nothing launched)."""
        return bool(self.lib.smj_dev_partition_range_sampled(
            self.ws, inp.data_ptr(), inp.shape[0], out.data_ptr(), nbits, key_min, key_max,
            1 if packed else 0, seg_start.data_ptr(), seg_cnt.data_ptr(), flags.data_ptr(),
            self.stream_ptr()))

    def dev_partition_range_shards(self, inp, out, nbits, key_min, key_max, packed,
                                   seg_start, seg_cnt, flags):
        """smj_dev_partition_range_shards: the sampled partition's tables with
        exactly sized regions back to back (`out` holds n elements); False when
        the form does not apply (nothing launched)."""
        return bool(self.lib.smj_dev_partition_range_shards(
            self.ws, inp.data_ptr(), inp.shape[0], out.data_ptr(), nbits, key_min, key_max,
            1 if packed else 0, seg_start.data_ptr(), seg_cnt.data_ptr(), flags.data_ptr(),
            self.stream_ptr()))

    def dev_partition_range_packed(self, inp, out_words, nbits, key_min, key_max, hist, bad):
        """smj_dev_partition_range writing packed int64 words; False (nothing
        launched) when the layout does not apply."""
        return bool(self.lib.smj_dev_partition_range_packed(
            self.ws, inp.data_ptr(), inp.shape[0], out_words.data_ptr(), nbits, key_min,
            key_max, hist.data_ptr(), bad.data_ptr(), self.stream_ptr()))

    def dev_partition_range(self, inp, out, nbits, key_min, key_max, hist):
        self.lib.smj_dev_partition_range(self.ws, inp.data_ptr(), inp.shape[0],
                                         out.data_ptr(), nbits, key_min, key_max,
                                         hist.data_ptr(), self.stream_ptr())

    def selfcheck_lds_order(self) -> int:
        """Violations of lane-ordered LDS atomic returns (0 expected)."""
        return int(self.lib.smj_selfcheck_lds_order(self.ws, self.stream_ptr()))

    def trace(self, on: bool, only: str | None = None):
        """Start (reset) or stop the per-kernel event trace; `only` names the
        one kernel to trace."""
        self.lib.smj_trace_enable(self.ws, int(on))
        self.lib.smj_trace_only(self.ws, only.encode() if only else None)
        self.lib.smj_trace_reset(self.ws)

    def trace_read(self):
        """{kernel name: (total ms, launches)} since the last trace(True)."""
        buf = C.create_string_buffer(4096)
        ms = (C.c_float * 64)()
        cnt = (C.c_int * 64)()
        k = self.lib.smj_trace_read(self.ws, buf, 4096, ms, cnt, 64)
        names = buf.value.decode().split("\n")
        return {names[i]: (ms[i], cnt[i]) for i in range(k)}

    def join_phase_ms(self):
        a = (C.c_float * 5)()
        self.lib.smj_join_phase_ms(self.ws, a)
        return list(a)


_LIBS: dict[int, Library] = {}


def load(width: int = 16) -> Library:
    if width not in _LIBS:
        _LIBS[width] = Library(width)
    return _LIBS[width]
