"""GpuFingerprintStore -- an rsos::Rsos<K> realisation resident on one MI355X.

Mirrors rsos/src/rsos_trait.rs:39-90 (method names, argument meaning, panics-as-errors):

  size()                 -> |X|
  aggregate(range)       -> Aggregate over X ∩ range   (summary-folds-lift: computed with lift)
  rank(z)                -> number of keys strictly below z
  select(r)              -> r-th key; IndexError if r >= size()  (the reference panics)
  enumerate(range)       -> (key, record index) pairs in key order
  insert(k, v) / delete(k)

Keys and fingerprints are held in rank order in HBM with the block / super-block sums; rank,
select and range bounds are answered on the device.  Record payloads are lifted on ingest and
not kept on the device (the caller owns K and V, as the reference's map does).  Keys are
fixed-width: bytes of schema.key_len for byte keys (memcmp order = Ord of [u8; L]), ints for
u32/u64 keys.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Iterator, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _abi as A
from .fingerprint import Aggregate
from .schema import RecordSchema

Key = Union[bytes, int]
HOST_COLS = ("keys", "phys", "logical", "node", "tags", "values")


def _torch_stream() -> int:
    """The stream torch queued the device columns on: the store waits for it before reading."""
    import torch
    return torch.cuda.current_stream().cuda_stream


def _np_ptr(a: Optional[np.ndarray]) -> Optional[int]:
    return None if a is None else a.ctypes.data


class KeyRange:
    """std::ops range with Bound semantics: kinds 'unbounded' | 'included' | 'excluded'."""

    _K = {"unbounded": 0, "included": 1, "excluded": 2}

    def __init__(self, start: Optional[Key] = None, end: Optional[Key] = None,
                 start_kind: str = "included", end_kind: str = "excluded"):
        self.start, self.end = start, end
        self.start_kind = "unbounded" if start is None else start_kind
        self.end_kind = "unbounded" if end is None else end_kind

    @staticmethod
    def full() -> "KeyRange":  # `..`
        return KeyRange()


# stores created with host_tier=None follow this (tests run the same suites with the tier on)
DEFAULT_HOST_TIER = False


class GpuFingerprintStore:
    _P = "rh_store_"  # the entry points' prefix (the sharded store's are rh_sstore_*)

    def _f(self, name: str):
        return getattr(A.lib(), self._P + name)

    def __init__(self, schema: RecordSchema, device: int = 0, host_tier: Optional[bool] = None):
        self.schema = schema
        self._s = schema.c()
        h = C.c_void_p()
        A.check(A.lib().rh_store_create(device, C.byref(self._s), C.byref(h)), "rh_store_create")
        self._h = h
        if DEFAULT_HOST_TIER if host_tier is None else host_tier:
            self.set_host_tier(True)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._f("destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- key encoding --------------------------------------------------------------------
    def _key_bytes(self, k: Key) -> bytes:
        s = self.schema
        if s.key_kind == A.KEY_U32:
            return int(k).to_bytes(4, "little")
        if s.key_kind == A.KEY_U64:
            return int(k).to_bytes(8, "little")
        b = bytes(k)
        if len(b) != s.key_row:
            raise ValueError(f"key must be {s.key_row} bytes")
        return b

    def _key_out(self, b: bytes) -> Key:
        if self.schema.key_kind in (A.KEY_U32, A.KEY_U64):
            return int.from_bytes(b, "little")
        return b

    @staticmethod
    def _columns(cols: Dict[str, np.ndarray]) -> Tuple[A.Columns, Dict[str, np.ndarray]]:
        held = {k: np.ascontiguousarray(v) for k, v in cols.items() if v is not None}
        for k in held:
            if k not in HOST_COLS:
                raise ValueError(f"unknown column {k!r}")
        return A.Columns(*[_np_ptr(held.get(k)) for k in HOST_COLS]), held

    # ---- fill ----------------------------------------------------------------------------
    def load_bulk(self, cols: Dict[str, np.ndarray]) -> None:
        """Replace the contents with records sorted by key, without duplicates."""
        c, held = self._columns(cols)
        n = len(held["keys"]) if "keys" in held else len(held["values"])
        A.check(self._f("load")(self._h, C.byref(c), n), "rh_store_load")

    def load_bulk_device(self, cols) -> None:
        """load_bulk from device (torch) columns already resident in HBM."""
        from .device import _check_cols, _columns
        n = _check_cols(self.schema, cols)
        c = _columns(cols)
        A.check(self._f("load_device")(self._h, C.byref(c), n, _torch_stream()), "rh_store_load_device")

    def apply_device(self, cols, ops=None) -> Tuple[int, int, int]:
        """apply() with device (torch) columns / ops; returns (new, overwritten, deleted)."""
        from .device import _check_cols, _columns
        m = _check_cols(self.schema, cols)
        if ops is not None and (ops.numel() != m or not ops.is_cuda):
            raise ValueError("ops must be m device bytes")
        c = _columns(cols)
        a, b, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
        A.check(self._f("apply_device")(self._h, C.byref(c), None if ops is None else ops.data_ptr(), m,
                                              C.byref(a), C.byref(b), C.byref(d), _torch_stream()),
                "rh_store_apply_device")
        return int(a.value), int(b.value), int(d.value)

    def apply_device_many(self, batches, ops=None) -> List[Tuple[int, int, int]]:
        """apply_device over several device batches in order, in one call: batch i + 1 is
        key-sorted while the host waits for batch i's result (rh_store_apply_device_many).  ops: None or one
        entry (None or m device bytes) per batch.  Returns (new, overwritten, deleted) per batch."""
        from .device import _check_cols, _columns
        k = len(batches)
        if ops is not None and len(ops) != k:
            raise ValueError("ops must have one entry per batch")
        cols = (A.Columns * max(k, 1))()
        ns = (C.c_size_t * max(k, 1))()
        optr = (C.c_void_p * max(k, 1))()
        for i, b in enumerate(batches):
            ns[i] = _check_cols(self.schema, b)
            cols[i] = _columns(b)
            o = None if ops is None else ops[i]
            if o is not None and (o.numel() != ns[i] or not o.is_cuda):
                raise ValueError("ops must be m device bytes")
            optr[i] = None if o is None else o.data_ptr()
        out = (C.c_uint64 * (3 * max(k, 1)))()
        A.check(self._f("apply_device_many")(self._h, cols, None if ops is None else optr, ns, k, out,
                                                   _torch_stream()), "rh_store_apply_device_many")
        return [(int(out[3 * i]), int(out[3 * i + 1]), int(out[3 * i + 2])) for i in range(k)]

    def compact(self) -> None:
        A.check(self._f("compact")(self._h), "rh_store_compact")

    def set_host_tier(self, enable: bool = True, round_max: int = 0) -> None:
        """Answer rank / select / aggregate and protocol rounds of at most `round_max` segments
        (0: the default, 128) from a host copy of the keys and fingerprint prefix sums plus a tree
        of every later batch's signed deltas (rh_store_set_host_tier): a batch updates it in
        O(batch log n); the base is copied again only after a load or a delta grown past base / 8."""
        A.check(self._f("set_host_tier")(self._h, 1 if enable else 0, round_max), "rh_store_set_host_tier")

    def set_compaction(self, divisor: int, min_rows: int) -> None:
        A.check(self._f("set_compaction")(self._h, divisor, min_rows), "rh_store_set_compaction")

    def reserve(self, rows: int, batch_rows: int) -> None:
        """Size every device buffer for `rows` resident rows and batches of up to `batch_rows`
        (compacts first; contents unchanged), so later batches never reallocate."""
        A.check(self._f("reserve")(self._h, rows, batch_rows), "rh_store_reserve")

    def stats(self) -> Dict[str, int]:
        b, d, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        A.check(self._f("stats")(self._h, C.byref(b), C.byref(d), C.byref(c)), "rh_store_stats")
        return {"base_rows": int(b.value), "delta_rows": int(d.value), "compactions": int(c.value)}

    def tier_sync(self) -> None:
        """Wait until the host tier is fresh (its background refresh landed): rh_store_tier_sync."""
        A.check(self._f("tier_sync")(self._h), "rh_store_tier_sync")

    def set_tier_policy(self, keep_fresh: bool) -> None:
        """Whether writes keep the host tier fresh (wait for the copies they cause; the default)
        or never wait (questions go to the device meanwhile): rh_store_set_tier_policy."""
        A.check(self._f("set_tier_policy")(self._h, 1 if keep_fresh else 0), "rh_store_set_tier_policy")

    def batch_stats(self) -> Dict[str, int]:
        """Batches applied by the small-batch path and by the large-batch path (rh_store_batch_stats)."""
        a, b = C.c_uint64(), C.c_uint64()
        A.check(self._f("batch_stats")(self._h, C.byref(a), C.byref(b)), "rh_store_batch_stats")
        return {"small": int(a.value), "large": int(b.value)}

    def stage(self, cols: Dict[str, np.ndarray], ops: np.ndarray) -> None:
        """Queue host rows (rh_store_stage): applied as one batch by the next call that reads the
        store; a key staged more than once keeps its last operation."""
        c, held = self._columns(cols)
        ops_a = np.ascontiguousarray(ops, dtype=np.uint8)
        A.check(self._f("stage")(self._h, C.byref(c), _np_ptr(ops_a), len(ops_a)), "rh_store_stage")

    def tier_stats(self) -> Dict[str, int]:
        """The host tier's bookkeeping (rh_store_tier_stats): rows of its base copy and its delta
        entries (tree + run copy) while fresh, copies taken from the device (base refreshes and run
        copies) and batch folds so far."""
        b, d, r, f = C.c_uint64(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        A.check(self._f("tier_stats")(self._h, C.byref(b), C.byref(d), C.byref(r), C.byref(f)),
                "rh_store_tier_stats")
        return {"base_rows": int(b.value), "delta_entries": int(d.value), "refreshes": int(r.value),
                "folds": int(f.value)}

    # ---- Rsos<K> -------------------------------------------------------------------------
    def size(self) -> int:
        out = C.c_uint64()
        A.check(self._f("len")(self._h, C.byref(out)), "rh_store_len")
        return int(out.value)

    __len__ = size

    def aggregate(self, rng: Optional[KeyRange] = None) -> Aggregate:
        rng = rng or KeyRange.full()
        lo = None if rng.start is None else C.create_string_buffer(self._key_bytes(rng.start))
        hi = None if rng.end is None else C.create_string_buffer(self._key_bytes(rng.end))
        out = A.Aggregate()
        A.check(self._f("aggregate_keys")(self._h, KeyRange._K[rng.start_kind], lo,
                                                KeyRange._K[rng.end_kind], hi, C.byref(out)),
                "rh_store_aggregate_keys")
        return Aggregate.from_c(out)

    def aggregate_ranks(self, lo: int, hi: int) -> Aggregate:
        out = A.Aggregate()
        A.check(self._f("aggregates")(self._h, _np_ptr(np.array([lo], np.uint64)), _np_ptr(np.array([hi], np.uint64)), 1, C.byref(out)),
                self._P + "aggregates")
        return Aggregate.from_c(out)

    def aggregates_ranks(self, lo: Sequence[int], hi: Sequence[int]):
        lo_a = np.ascontiguousarray(lo, dtype=np.uint64)
        hi_a = np.ascontiguousarray(hi, dtype=np.uint64)
        r = len(lo_a)
        out = (A.Aggregate * max(r, 1))()
        A.check(self._f("aggregates")(self._h, _np_ptr(lo_a), _np_ptr(hi_a), r, out),
                "rh_store_aggregates")
        return [Aggregate.from_c(out[j]) for j in range(r)]

    def rank(self, z: Key) -> int:
        out = C.c_uint64()
        A.check(self._f("rank")(self._h, C.create_string_buffer(self._key_bytes(z)), C.byref(out)),
                "rh_store_rank")
        return int(out.value)

    def select(self, r: int) -> Key:
        if r < 0 or r >= self.size():
            raise IndexError("select: r >= size()")
        buf = C.create_string_buffer(max(self.schema.key_row, 1))
        A.check(self._f("select")(self._h, r, buf), "rh_store_select")
        return self._key_out(buf.raw[: self.schema.key_row])

    def enumerate(self, rng: Optional[KeyRange] = None) -> Iterator[Tuple[Key, int]]:
        """Keys in X ∩ range with their ranks, in key order (Rsos::enumerate's key half)."""
        rng = rng or KeyRange.full()
        n = self.size()
        lo = 0 if rng.start is None else self.rank(rng.start)
        if rng.start is not None and rng.start_kind == "excluded" and lo < n and self.select(lo) == rng.start:
            lo += 1
        hi = n if rng.end is None else self.rank(rng.end)
        if rng.end is not None and rng.end_kind == "included" and hi < n and self.select(hi) == rng.end:
            hi += 1
        if hi <= lo:
            return
        kl = self.schema.key_row
        buf = np.zeros((hi - lo) * kl, np.uint8)
        A.check(self._f("keys")(self._h, lo, hi, _np_ptr(buf)), "rh_store_keys")
        for r in range(lo, hi):
            yield self._key_out(buf[(r - lo) * kl:(r - lo + 1) * kl].tobytes()), r

    def ranks(self, keys: np.ndarray) -> np.ndarray:
        """Rank of each of m keys (rows of key_len bytes) in one device search."""
        k = np.ascontiguousarray(keys, dtype=np.uint8).reshape(-1, self.schema.key_row)
        out = np.zeros(k.shape[0], np.uint64)
        A.check(self._f("ranks")(self._h, _np_ptr(k), k.shape[0], _np_ptr(out)), "rh_store_ranks")
        return out

    def fingerprints(self, lo: int = 0, hi: Optional[int] = None) -> np.ndarray:
        hi = self.size() if hi is None else hi
        out = np.zeros((max(hi - lo, 0), 32), np.uint8)
        A.check(self._f("fingerprints")(self._h, lo, hi, _np_ptr(out) if hi > lo else None),
                "rh_store_fingerprints")
        return out

    # ---- rbsr protocol round, batched (rh_store_resolve_segments / rh_store_split_segments) ----
    def resolve_segments(self, segments: Sequence) -> Tuple[np.ndarray, np.ndarray, list]:
        """For r segments (objects with .start / .end: None = Unbounded, else Included(start) /
        Excluded(end)): raw start / end ranks (Unbounded -> 0 / size) and the local aggregate
        over each key range (ZERO if inverted), in one device round trip."""
        r, kl = len(segments), self.schema.key_row
        sk, ek = np.zeros(max(r, 1), np.uint8), np.zeros(max(r, 1), np.uint8)
        skeys, ekeys = np.zeros((max(r, 1), kl), np.uint8), np.zeros((max(r, 1), kl), np.uint8)
        for j, seg in enumerate(segments):
            if seg.start is not None:
                sk[j] = 1
                skeys[j] = np.frombuffer(self._key_bytes(seg.start), np.uint8)
            if seg.end is not None:
                ek[j] = 1
                ekeys[j] = np.frombuffer(self._key_bytes(seg.end), np.uint8)
        lo, hi = np.zeros(max(r, 1), np.uint64), np.zeros(max(r, 1), np.uint64)
        out = (A.Aggregate * max(r, 1))()
        A.check(self._f("resolve_segments")(self._h, r, _np_ptr(sk), _np_ptr(skeys), _np_ptr(ek),
                                                  _np_ptr(ekeys), _np_ptr(lo), _np_ptr(hi), out),
                "rh_store_resolve_segments")
        return lo[:r], hi[:r], [Aggregate.from_c(out[j]) for j in range(r)]

    def split_segments(self, select_ranks: Sequence[int], lo: Sequence[int], hi: Sequence[int]):
        """select() at every rank of `select_ranks` and the aggregates of the rank ranges
        [lo[i], hi[i]), in one device round trip: (keys, aggregates)."""
        kl = self.schema.key_row
        sel = np.ascontiguousarray(select_ranks, dtype=np.uint64)
        lo_a = np.ascontiguousarray(lo, dtype=np.uint64)
        hi_a = np.ascontiguousarray(hi, dtype=np.uint64)
        m, q = len(sel), len(lo_a)
        keys = np.zeros((max(m, 1), kl), np.uint8)
        out = (A.Aggregate * max(q, 1))()
        A.check(self._f("split_segments")(self._h, m, _np_ptr(sel), _np_ptr(keys), q, _np_ptr(lo_a),
                                                _np_ptr(hi_a), out), "rh_store_split_segments")
        return [self._key_out(keys[i].tobytes()) for i in range(m)], [Aggregate.from_c(out[j]) for j in range(q)]

    def apply(self, cols: Dict[str, np.ndarray], ops: np.ndarray) -> Tuple[int, int, int]:
        """Batched insert (op 0) / delete (op 1); returns (new, overwritten, deleted)."""
        c, held = self._columns(cols)
        ops_a = np.ascontiguousarray(ops, dtype=np.uint8)
        a, b, d = C.c_uint64(), C.c_uint64(), C.c_uint64()
        A.check(self._f("apply")(self._h, C.byref(c), _np_ptr(ops_a), len(ops_a), C.byref(a), C.byref(b),
                                       C.byref(d)), "rh_store_apply")
        return int(a.value), int(b.value), int(d.value)

    def insert(self, key: Key, value: bytes = b"", phys: int = 0, logical: int = 0, node: int = 0,
               tombstone: bool = False) -> bool:
        """Insert-or-overwrite one record; True if the key was new (Rsos::insert returns the old V)."""
        s = self.schema
        cols = {"keys": np.frombuffer(self._key_bytes(key), np.uint8).copy()}
        if s.value_row:
            v = value if isinstance(value, (bytes, bytearray)) else int(value).to_bytes(s.value_row, "little")
            if len(v) != s.value_row:
                raise ValueError(f"value must be {s.value_row} bytes")
            cols["values"] = np.frombuffer(bytes(v), np.uint8).copy()
        if s.dated_kind:
            cols["phys"] = np.array([phys], np.uint64)
            cols["logical"] = np.array([logical], np.uint32)
            cols["node"] = np.array([node], np.uint64)
        if s.record_kind != A.REC_PLAIN:
            cols["tags"] = np.array([1 if tombstone else 0], np.uint8)
        new, _, _ = self.apply(cols, np.zeros(1, np.uint8))
        return new == 1

    def delete(self, key: Key) -> bool:
        cols = {"keys": np.frombuffer(self._key_bytes(key), np.uint8).copy()}
        _, _, d = self.apply(cols, np.ones(1, np.uint8))
        return d == 1
