"""EncodedFingerprintMap -- Rsos<K> for any serde K / V over the encoded store (rh_estore_*).

What `ReplicatedMap<String, String>` (the reference's own example, examples/k8s/main.rs:53) needs:
keys and values without a fixed-width column form.  Every record goes to the device as its
canonical bytes -- encode(K) then encode(V) (rsos_hip.encoding; the Rust binding uses
rsos::encoding::encode_to_vec) -- and is hashed there (lift = BLAKE3 of that concatenation,
rsos/src/fingerprint.rs:270-275); the device keeps the fingerprints in rank order with the block
sums, and (host tier) their prefix sums.  The keys and their order -- the key type's Ord, which for
String / Vec<u8> is not the order of their length-prefixed encodings -- stay here, in a sorted
index; the device is addressed by rank.

Updates are staged like FingerprintMap's: insert / delete return the displaced value at once and
queue the operation; the next question applies every queued operation as ONE rank-addressed
device batch (rh_estore_apply), a key queued twice keeping its last operation.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Iterator, List, Optional, Tuple

import numpy as np
from sortedcontainers import SortedList

from . import _abi as A
from .encoding import encode
from .fingerprint import Aggregate
from .store import KeyRange

_DELETE = object()


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64)


class EncodedFingerprintMap:
    def __init__(self, key_type: Any, value_type: Any, device: int = 0, host_tier: bool = True):
        self.key_type, self.value_type = key_type, value_type
        h = C.c_void_p()
        A.check(A.lib().rh_estore_create(device, C.byref(h)), "rh_estore_create")
        self._h = h
        if host_tier:
            A.check(A.lib().rh_estore_set_host_tier(self._h, 1), "rh_estore_set_host_tier")
        self._vals = {}                 # key -> value, current (returns displaced values at once)
        self._dev = SortedList()        # the keys on the device, in rank order
        self._pending = {}              # key -> value | _DELETE, not yet on the device

    def close(self) -> None:
        if getattr(self, "_h", None):
            A.lib().rh_estore_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def record(self, key, value) -> bytes:
        """The record's canonical bytes: encode(K) ‖ encode(V) (what lift hashes)."""
        return encode(self.key_type, key) + encode(self.value_type, value)

    @staticmethod
    def _pack(records: List[bytes]) -> Tuple[np.ndarray, np.ndarray]:
        offs = np.zeros(len(records) + 1, np.uint64)
        if records:
            offs[1:] = np.cumsum([len(r) for r in records], dtype=np.uint64)
        data = np.frombuffer(b"".join(records) or b"\0", np.uint8)
        return data, offs

    # ---- fill ----------------------------------------------------------------------------------
    def load_bulk(self, items) -> None:
        """Replace the contents (FromIterator / load_bulk): the last value of a repeated key wins."""
        vals = {}
        for k, v in items:
            vals[k] = v
        keys = sorted(vals)
        recs = [self.record(k, vals[k]) for k in keys]
        data, offs = self._pack(recs)
        A.check(A.lib().rh_estore_load(self._h, data.ctypes.data, offs.ctypes.data, len(keys)), "rh_estore_load")
        self._vals, self._dev, self._pending = vals, SortedList(keys), {}

    # ---- staged updates --------------------------------------------------------------------------
    def insert(self, key, value) -> Optional[Any]:
        self.record(key, value)  # encodes, or raises before anything changes
        old = self._vals.get(key)
        self._vals[key] = value
        self._pending[key] = value
        return old

    def delete(self, key) -> Optional[Any]:
        old = self._vals.pop(key, None)
        if old is not None:
            self._pending[key] = _DELETE
        return old

    def flush(self) -> None:
        """Apply every staged operation as one rank-addressed device batch."""
        if not self._pending:
            return
        pos, kinds, recs, adds, dels = [], [], [], [], []
        for k in sorted(self._pending):
            v = self._pending[k]
            p = self._dev.bisect_left(k)
            present = p < len(self._dev) and self._dev[p] == k
            if v is _DELETE:
                if present:
                    pos.append(p), kinds.append(2), dels.append(k)
                continue
            pos.append(p)
            kinds.append(1 if present else 0)
            recs.append(self.record(k, v))
            if not present:
                adds.append(k)
        self._pending = {}
        if not pos:
            return
        p_a, k_a = _u64(pos), np.asarray(kinds, np.uint8)
        data, offs = self._pack(recs)
        A.check(A.lib().rh_estore_apply(self._h, p_a.ctypes.data, k_a.ctypes.data, len(pos), data.ctypes.data,
                                        offs.ctypes.data, len(recs)), "rh_estore_apply")
        for k in dels:
            self._dev.remove(k)
        self._dev.update(adds)

    # ---- the inherent FingerprintTreeMap surface (public-api/rsos.txt:129-194) ---------------------
    def contains_key(self, key) -> bool:
        return key in self._vals

    def remove(self, key):
        return self.delete(key)

    def retain(self, f) -> None:
        """Keep the entries f(key, value) accepts; the others are deleted (one staged batch)."""
        for k in [k for k, v in self._vals.items() if not f(k, v)]:
            self.delete(k)

    def with_mut(self, key, f):
        """In-place edit (FingerprintTreeMap::with_mut + Relift, access.rs:46-76): f receives the
        value (or None) and returns (result, new_value); the new value's fingerprint replaces the
        old one through the staged batch (the `new - old` delta)."""
        old = self._vals.get(key)
        result, new = f(old)
        if old is not None:
            self.record(key, new)
            self._vals[key] = new
            self._pending[key] = new
        return result

    def or_insert(self, key, value):
        """entry(key).or_insert(value) (rsos::Entry, public-api/rsos.txt:118-121)."""
        if key not in self._vals:
            self.insert(key, value)
        return self._vals[key]

    def range(self, rng: Optional[KeyRange] = None):
        return self.enumerate(rng)

    def first_key_value(self):
        self.flush()
        return (self._dev[0], self._vals[self._dev[0]]) if self._dev else None

    def last_key_value(self):
        self.flush()
        return (self._dev[-1], self._vals[self._dev[-1]]) if self._dev else None

    def position(self, key) -> Optional[int]:
        self.flush()
        r = self._dev.bisect_left(key)
        return r if r < len(self._dev) and self._dev[r] == key else None

    # ---- Rsos<K> -----------------------------------------------------------------------------------
    def size(self) -> int:
        self.flush()
        return len(self._dev)

    __len__ = size

    def get(self, key):
        return self._vals.get(key)

    def rank(self, z) -> int:
        self.flush()
        return self._dev.bisect_left(z)

    def select(self, r: int):
        self.flush()
        if r < 0 or r >= len(self._dev):
            raise IndexError("select: r >= size()")  # the reference panics
        return self._dev[r]

    def _bounds(self, rng: Optional[KeyRange]) -> Tuple[int, int]:
        rng = rng or KeyRange.full()
        n = len(self._dev)
        lo = 0 if rng.start is None else (self._dev.bisect_left(rng.start) if rng.start_kind != "excluded"
                                          else self._dev.bisect_right(rng.start))
        hi = n if rng.end is None else (self._dev.bisect_right(rng.end) if rng.end_kind == "included"
                                        else self._dev.bisect_left(rng.end))
        return lo, max(lo, hi)  # inverted -> ZERO (rbsr/src/protocol.rs:230-232)

    def enumerate(self, rng: Optional[KeyRange] = None) -> Iterator[Tuple[Any, Any]]:
        self.flush()
        lo, hi = self._bounds(rng)
        for r in range(lo, hi):
            k = self._dev[r]
            yield k, self._vals[k]

    def aggregate(self, rng: Optional[KeyRange] = None) -> Aggregate:
        self.flush()
        lo, hi = self._bounds(rng)
        return self.aggregates_ranks([lo], [hi])[0]

    def aggregates_ranks(self, lo, hi) -> List[Aggregate]:
        self.flush()
        lo_a, hi_a = _u64(lo), _u64(hi)
        r = len(lo_a)
        out = (A.Aggregate * max(r, 1))()
        A.check(A.lib().rh_estore_aggregates(self._h, lo_a.ctypes.data, hi_a.ctypes.data, r, out),
                "rh_estore_aggregates")
        return [Aggregate.from_c(out[j]) for j in range(r)]

    def root(self) -> Aggregate:
        self.flush()
        out = A.Aggregate()
        A.check(A.lib().rh_estore_root(self._h, C.byref(out)), "rh_estore_root")
        return Aggregate.from_c(out)

    def fingerprints(self, lo: int = 0, hi: Optional[int] = None) -> np.ndarray:
        self.flush()
        hi = len(self._dev) if hi is None else hi
        out = np.zeros((max(hi - lo, 0), 32), np.uint8)
        A.check(A.lib().rh_estore_fingerprints(self._h, lo, hi, out.ctypes.data if hi > lo else None),
                "rh_estore_fingerprints")
        return out
