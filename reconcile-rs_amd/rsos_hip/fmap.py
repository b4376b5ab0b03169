"""FingerprintMap -- Rsos<K> with the host owning K and V, updates staged into device batches.

The Python twin of the Rust binding's `HipFingerprintMap` (rust/rsos-hip/src/lib.rs), so its
logic is tested here where no Rust toolchain exists:

* **Ownership** (rsos/src/rsos_trait.rs:66-80): keys and values live in host memory -- a sorted
  key index (`sortedcontainers.SortedList`: O(log n) insert, rank and select) and a dict of
  values -- so `select` / `enumerate` hand back the caller's objects, and `insert` / `delete`
  return the displaced value as FingerprintTreeMap::insert / remove do (mutate.rs:23-154).
* **Staged updates**: `insert` / `delete` append one row to a host buffer; rows go to the
  library in chunks (rh_store_stage), and the library applies everything staged as ONE device
  batch before any question reads the store.  A bulk seed through single inserts
  (ReplicatedMap::insert_bulk -> just_insert_bulk, src/replica/write.rs:107-121) is therefore
  O(log n) host work per record plus one device batch, not one device round trip per record.
* **Wrong-length values are errors**: a value whose encoding does not fill the schema's value
  column exactly raises ValueError -- never padded or truncated, which would hash some other
  record and reconcile silently wrongly (rsos_trait.rs:54-56).
* rank / select / size / enumerate come from the host index; aggregate from the store (its host
  tier by default: no device round trip once the staged batch is applied).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Iterator, Optional, Tuple, Union

import numpy as np
from sortedcontainers import SortedList

from . import _abi as A
from .fingerprint import Aggregate
from .schema import RecordSchema
from .store import GpuFingerprintStore, KeyRange

Key = Union[bytes, int]


@dataclass(frozen=True)
class Entry:
    """Entry<Timestamp, V> (lww-register/src/entry.rs:88-94) for DATED maps, State<V> (:24-29)
    for PROJECTION maps (stamp ignored): value bytes (or an int for u32 / u64 values), the HLC
    stamp, and whether the state is State::Tombstone."""
    value: Union[bytes, int] = b""
    phys: int = 0
    logical: int = 0
    node: int = 0
    tombstone: bool = False


def encode_row(schema: RecordSchema, value) -> Tuple[bytes, int, int, int, int]:
    """(value column bytes, phys, logical, node, tag) of one record.  ValueError when the value
    does not fill the value column exactly (a tombstone carries no value bytes)."""
    e = value if isinstance(value, Entry) else Entry(value)
    if schema.record_kind == A.REC_PLAIN and (e.tombstone or e.phys or e.logical or e.node):
        raise ValueError("a plain map's values carry no stamp or state")
    vr = schema.value_row
    if e.tombstone:
        if e.value not in (b"", 0, None):
            raise ValueError("a tombstone carries no value bytes")
        vb = bytes(vr)
    elif isinstance(e.value, int):
        if schema.value_kind not in (A.VAL_U32, A.VAL_U64):
            raise ValueError("an integer value needs a u32 / u64 value column")
        vb = int(e.value).to_bytes(vr, "little")
    else:
        vb = bytes(e.value)
        if len(vb) != vr:
            raise ValueError(f"value encodes to {len(vb)} bytes; the value column holds exactly {vr}")
    return vb, e.phys, e.logical, e.node, 1 if e.tombstone else 0


class _Rows:
    """Staged rows not yet handed to the library (appends into bytes buffers, ~1 us a row)."""

    def __init__(self, schema: RecordSchema):
        self.s = schema
        self.clear()

    def clear(self):
        self.keys, self.vals, self.tags, self.ops = bytearray(), bytearray(), bytearray(), bytearray()
        self.phys, self.logical, self.node = [], [], []
        self.n = 0

    def add(self, kb: bytes, row, op: int):
        vb, ph, lg, nd, tag = row
        self.keys += kb
        self.vals += vb
        self.tags.append(tag)
        self.ops.append(op)
        if self.s.dated_kind:
            self.phys.append(ph)
            self.logical.append(lg)
            self.node.append(nd)
        self.n += 1

    def stage(self, store: GpuFingerprintStore):
        if not self.n:
            return
        s, n = self.s, self.n
        held = {"keys": np.frombuffer(bytes(self.keys), np.uint8),
                "values": np.frombuffer(bytes(self.vals), np.uint8) if s.value_row else None,
                "tags": np.frombuffer(bytes(self.tags), np.uint8) if s.record_kind != A.REC_PLAIN else None}
        if s.dated_kind:
            held["phys"] = np.array(self.phys, np.uint64)
            held["logical"] = np.array(self.logical, np.uint32)
            held["node"] = np.array(self.node, np.uint64)
        ops = np.frombuffer(bytes(self.ops), np.uint8)
        ptr = lambda k: None if held.get(k) is None else held[k].ctypes.data  # noqa: E731
        cols = A.Columns(*[ptr(k) for k in ("keys", "phys", "logical", "node", "tags", "values")])
        A.check(A.lib().rh_store_stage(store._h, C.byref(cols), ops.ctypes.data, n), "rh_store_stage")
        self.clear()


class FingerprintMap:
    """Rsos<K> (rsos/src/rsos_trait.rs:39-90) over a GPU store, the host owning K and V."""

    def __init__(self, schema: RecordSchema, device: int = 0, host_tier: bool = True, chunk: int = 1 << 16):
        self.schema = schema
        self.store = GpuFingerprintStore(schema, device, host_tier=host_tier)
        self._index = SortedList()
        self._vals = {}
        self._rows = _Rows(schema)
        self._chunk = chunk

    def close(self):
        self.store.close()

    def _key(self, k: Key) -> bytes:
        return self.store._key_bytes(k)

    def _stage(self):
        self._rows.stage(self.store)

    # ---- updates ----------------------------------------------------------------------------
    def insert(self, key: Key, value) -> Optional[object]:
        """Insert or overwrite; returns the displaced value (None if the key was new)."""
        kb, row = self._key(key), encode_row(self.schema, value)
        old = self._vals.get(key)
        if old is None:
            self._index.add(key)
        self._vals[key] = value
        self._rows.add(kb, row, 0)
        if self._rows.n >= self._chunk:
            self._stage()
        return old

    def delete(self, key: Key) -> Optional[object]:
        old = self._vals.pop(key, None)
        if old is None:
            return None
        self._index.remove(key)
        self._rows.add(self._key(key), (bytes(self.schema.value_row), 0, 0, 0, 0), 1)
        if self._rows.n >= self._chunk:
            self._stage()
        return old

    # ---- questions ---------------------------------------------------------------------------
    def size(self) -> int:
        return len(self._index)

    __len__ = size

    def get(self, key: Key):
        return self._vals.get(key)

    def rank(self, z: Key) -> int:
        return self._index.bisect_left(z)

    def select(self, r: int) -> Key:
        if r < 0 or r >= len(self._index):
            raise IndexError("select: r >= size()")  # the reference panics
        return self._index[r]

    def enumerate(self, rng: Optional[KeyRange] = None) -> Iterator[Tuple[Key, object]]:
        rng = rng or KeyRange.full()
        inc = (rng.start_kind != "excluded", rng.end_kind == "included")
        for k in self._index.irange(rng.start, rng.end, inclusive=inc):
            yield k, self._vals[k]

    def aggregate(self, rng: Optional[KeyRange] = None) -> Aggregate:
        """Σ lift over the range: every staged row is applied first (one device batch)."""
        self._stage()
        return self.store.aggregate(rng)

    def flush(self) -> None:
        """Apply everything staged now (the next question would do it anyway)."""
        self._stage()
        self.store.size()
