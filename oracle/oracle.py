"""ctypes binding of the C oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this, as the checker or the timed CPU baseline -- never the product path.
See oracle/oracle.h for the reference citations of every function restated.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

KEY_UNIT, KEY_U32, KEY_U64, KEY_BYTES = 0, 1, 2, 3
VAL_UNIT, VAL_U32, VAL_U64, VAL_BYTES = 0, 1, 2, 3
REC_PLAIN, REC_DATED, REC_PROJECTION = 0, 1, 2


class Schema(C.Structure):
    _fields_ = [("key_kind", C.c_int32), ("key_len", C.c_uint32), ("value_kind", C.c_int32),
                ("value_len", C.c_uint32), ("record_kind", C.c_int32), ("reserved", C.c_uint32)]


class Columns(C.Structure):
    _fields_ = [("keys", C.c_void_p), ("phys", C.c_void_p), ("logical", C.c_void_p),
                ("node", C.c_void_p), ("tags", C.c_void_p), ("values", C.c_void_p)]


class Aggregate(C.Structure):
    _fields_ = [("fp", C.c_uint64 * 4), ("size", C.c_uint64)]


_lib: Optional[C.CDLL] = None


def build() -> None:
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.or_blake3.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.or_encode_record.restype = C.c_size_t
        L.or_encode_record.argtypes = [C.POINTER(Schema), C.POINTER(Columns), C.c_size_t, C.c_void_p]
        L.or_lift_records.argtypes = [C.POINTER(Schema), C.POINTER(Columns), C.c_size_t, C.c_void_p, C.c_int]
        L.or_lift_encoded.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_int]
        L.or_range_aggregates.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(Aggregate)]
        L.or_ftm_new.restype = C.c_void_p
        L.or_ftm_new.argtypes = [C.POINTER(Schema), C.POINTER(Columns)]
        L.or_ftm_free.argtypes = [C.c_void_p]
        L.or_ftm_insert.argtypes = [C.c_void_p, C.c_size_t]
        L.or_ftm_insert.restype = C.c_int
        L.or_ftm_fill.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t]
        L.or_ftm_len.argtypes = [C.c_void_p]
        L.or_ftm_len.restype = C.c_size_t
        L.or_ftm_root.argtypes = [C.c_void_p, C.POINTER(Aggregate)]
        L.or_ftm_aggregate.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(Aggregate)]
        L.or_ftm_rank.argtypes = [C.c_void_p, C.c_void_p]
        L.or_ftm_rank.restype = C.c_size_t
        L.or_ftm_select.argtypes = [C.c_void_p, C.c_size_t]
        L.or_ftm_select.restype = C.c_size_t
        L.or_reconcile_fixed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.or_reconcile_fixed.restype = C.c_int
        L.or_ftm_check.argtypes = [C.c_void_p]
        L.or_ftm_check.restype = C.c_int
        L.or_set_simd.argtypes = [C.c_int]
        L.or_set_simd.restype = C.c_int
        L.or_cpu_has_avx512.restype = C.c_int
        L.or_lift_records_x16.argtypes = [C.POINTER(Schema), C.POINTER(Columns), C.c_size_t, C.c_void_p, C.c_int]
        L.or_lift_records_x16.restype = C.c_int
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]) -> Optional[int]:
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def blake3(data: bytes) -> bytes:
    out = (C.c_uint8 * 32)()
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if data else np.zeros(1, np.uint8)
    lib().or_blake3(_ptr(buf), len(data), out)
    return bytes(out)


class Records:
    """Column (SoA) view of a batch of records, the layout the GPU path consumes."""

    def __init__(self, schema: Schema, keys: np.ndarray, values: Optional[np.ndarray] = None,
                 phys: Optional[np.ndarray] = None, logical: Optional[np.ndarray] = None,
                 node: Optional[np.ndarray] = None, tags: Optional[np.ndarray] = None):
        self.schema = schema
        self.keys = np.ascontiguousarray(keys)
        self.values = None if values is None else np.ascontiguousarray(values)
        self.phys = None if phys is None else np.ascontiguousarray(phys, dtype=np.uint64)
        self.logical = None if logical is None else np.ascontiguousarray(logical, dtype=np.uint32)
        self.node = None if node is None else np.ascontiguousarray(node, dtype=np.uint64)
        self.tags = None if tags is None else np.ascontiguousarray(tags, dtype=np.uint8)
        self.n = int(self.keys.shape[0])
        self._cols = Columns(_ptr(self.keys), _ptr(self.phys), _ptr(self.logical), _ptr(self.node),
                             _ptr(self.tags), _ptr(self.values))

    def encode(self, i: int) -> bytes:
        n = lib().or_encode_record(C.byref(self.schema), C.byref(self._cols), i, None)
        buf = np.zeros(max(n, 1), np.uint8)
        lib().or_encode_record(C.byref(self.schema), C.byref(self._cols), i, _ptr(buf))
        return bytes(buf[:n])

    def lift(self, threads: int = 1) -> np.ndarray:
        fps = np.zeros((self.n, 32), np.uint8)
        lib().or_lift_records(C.byref(self.schema), C.byref(self._cols), self.n, _ptr(fps), threads)
        return fps

    def lift_x16(self, threads: int = 1) -> Optional[np.ndarray]:
        """16 records per AVX-512 vector (CPU baseline's best batch lift); None without AVX-512."""
        fps = np.zeros((self.n, 32), np.uint8)
        if lib().or_lift_records_x16(C.byref(self.schema), C.byref(self._cols), self.n, _ptr(fps), threads) != 0:
            return None
        return fps


def set_simd(level: int) -> int:
    """The compression every oracle hash runs: 0 portable (default, what the tests pin), 1 the
    blake3 crate's SSE4.1 row form, 2 its AVX-512VL form.  Returns the level in effect."""
    return int(lib().or_set_simd(level))


def has_avx512() -> bool:
    return bool(lib().or_cpu_has_avx512())


def lift_encoded(blobs: Sequence[bytes], threads: int = 1) -> np.ndarray:
    offsets = np.zeros(len(blobs) + 1, np.uint64)
    offsets[1:] = np.cumsum([len(b) for b in blobs])
    data = np.frombuffer(b"".join(blobs) or b"\0", dtype=np.uint8).copy()
    fps = np.zeros((len(blobs), 32), np.uint8)
    lib().or_lift_encoded(_ptr(data), _ptr(offsets), len(blobs), _ptr(fps), threads)
    return fps


def range_aggregates(fps: np.ndarray, bounds: Sequence[int]):
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.uint64))
    r = len(b) - 1
    out = (Aggregate * max(r, 1))()
    lib().or_range_aggregates(_ptr(np.ascontiguousarray(fps)), fps.shape[0], _ptr(b), r, out)
    return [(list(out[j].fp), int(out[j].size)) for j in range(r)]


class FingerprintTreeMap:
    """The reference's order-6 B-tree restated in C, bound to a Records batch (rows = inserts)."""

    def __init__(self, recs: Records):
        self.recs = recs
        self._h = lib().or_ftm_new(C.byref(recs.schema), C.byref(recs._cols))

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_ftm_free(self._h)
            self._h = None

    def insert(self, i: int) -> bool:
        return bool(lib().or_ftm_insert(self._h, i))

    def fill(self, lo: int, hi: int) -> None:
        lib().or_ftm_fill(self._h, lo, hi)

    def __len__(self) -> int:
        return int(lib().or_ftm_len(self._h))

    def root(self):
        a = Aggregate()
        lib().or_ftm_root(self._h, C.byref(a))
        return list(a.fp), int(a.size)

    def aggregate(self, lo: Optional[bytes], hi: Optional[bytes]):
        a = Aggregate()
        lb = None if lo is None else C.create_string_buffer(lo, len(lo))
        hb = None if hi is None else C.create_string_buffer(hi, len(hi))
        lib().or_ftm_aggregate(self._h, lb, hb, C.byref(a))
        return list(a.fp), int(a.size)

    def rank(self, key: bytes) -> int:
        return int(lib().or_ftm_rank(self._h, C.create_string_buffer(key, len(key))))

    def select(self, index: int) -> int:
        """The record row holding the index-th key (query.rs:142-161); IndexError past the end."""
        row = int(lib().or_ftm_select(self._h, index))
        if row == (1 << 64) - 1:
            raise IndexError("select: index >= len")
        return row

    def check(self) -> bool:
        return lib().or_ftm_check(self._h) == 0


def reconcile_fixed(a: FingerprintTreeMap, b: FingerprintTreeMap, fan_out: int = 16):
    """A whole FixedFanOut reconciliation in C (oracle.c or_reconcile_fixed):
    (rounds, segments answered, IDLIST segments)."""
    out = (C.c_uint64 * 3)()
    if lib().or_reconcile_fixed(a._h, b._h, fan_out, out) != 0:
        raise ValueError("keys longer than 32 bytes")
    return int(out[0]), int(out[1]), int(out[2])
