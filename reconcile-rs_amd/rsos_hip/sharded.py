"""ShardedStore -- one replica's map over several GPUs inside one process.

The benchmark scales with one process per GPU (torch.distributed); a replica is one process, so
here the same key-range partitioning is a list of GpuFingerprintStore shards,
one per device, each owning a contiguous key range cut at equal counts when loaded.  Every
question of the Rsos<K> surface (rsos/src/rsos_trait.rs:39-90) and of a protocol round
(rbsr/src/protocol.rs:212-317) decomposes with no device-to-device traffic:

  size / rank(z)        sums over shards: rank(z) = Σ_s #(keys of shard s below z)
  aggregate(range)      Σ_s aggregate(range ∩ shard s) with Aggregate's Add
                        (rsos/src/aggregate.rs:79-89: commutative and associative)
  select(r)             the shard whose rank interval holds r
  apply(batch)          rows routed to their key's shard by the load-time splitters
  resolve_segments      element-wise sums of the shards' answers (ranks and aggregates add)
  split_segments        select per cut; each rank range cut into per-shard rank ranges, summed

Shards are queried concurrently from host threads (each store has its own stream and lock; the
library releases the GIL inside every call).  rsos_hip.rbsr's two-call protocol path runs on it
unchanged.
"""
from __future__ import annotations

import bisect
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .fingerprint import Aggregate
from .schema import RecordSchema
from .store import GpuFingerprintStore, KeyRange, Key


class ShardedStore:
    def __init__(self, schema: RecordSchema, devices: Sequence[int]):
        if not devices:
            raise ValueError("at least one device")
        self.schema = schema
        self.shards = [GpuFingerprintStore(schema, device=d) for d in devices]
        self.splitters: List[Key] = []  # first key of shards 1..G-1
        self._pool = ThreadPoolExecutor(max_workers=len(devices))

    def close(self) -> None:
        for s in self.shards:
            s.close()
        self._pool.shutdown()

    def _all(self, fn):
        return list(self._pool.map(fn, self.shards))

    def _shard_of(self, key: Key) -> int:
        return bisect.bisect_right(self.splitters, key)

    def _order_view(self, rows: np.ndarray) -> np.ndarray:
        """Key rows (n x key_row bytes) as a numpy array that sorts as the keys' Ord: numeric for
        u32 / u64 keys (stored little-endian), memcmp for byte keys ('S' compares equal-length
        rows in byte order; stripping trailing NULs keeps that order)."""
        from . import _abi as A
        rows = np.ascontiguousarray(rows, dtype=np.uint8).reshape(-1, self.schema.key_row)
        if self.schema.key_kind == A.KEY_U32:
            return rows.view("<u4").ravel()
        if self.schema.key_kind == A.KEY_U64:
            return rows.view("<u8").ravel()
        return rows.view(f"S{self.schema.key_row}").ravel()

    def _owners(self, keys: np.ndarray) -> np.ndarray:
        """_shard_of for every key row at once (np.searchsorted, side='right' = bisect_right)."""
        n = len(keys) // max(self.schema.key_row, 1) if keys.ndim == 1 else len(keys)
        if not self.splitters:
            return np.zeros(n, np.int64)
        if self.schema.key_row == 0:  # unit keys: every row is the one key
            return np.full(n, self._shard_of(self.shards[0]._key_out(b"")), np.int64)
        split = self._order_view(np.frombuffer(b"".join(self.shards[0]._key_bytes(k) for k in self.splitters),
                                               np.uint8))
        return np.searchsorted(split, self._order_view(keys), side="right").astype(np.int64)

    # ---- fill ----------------------------------------------------------------------------
    def load_bulk(self, cols: Dict[str, np.ndarray]) -> None:
        """Records sorted by key, without duplicates: cut into equal-count contiguous shards."""
        n = len(cols["keys"])
        g = len(self.shards)
        cuts = [n * j // g for j in range(g + 1)]
        parts = [{k: np.ascontiguousarray(v[cuts[j]:cuts[j + 1]]) for k, v in cols.items() if v is not None}
                 for j in range(g)]
        list(self._pool.map(lambda a: a[0].load_bulk(a[1]), zip(self.shards, parts)))
        key_out = self.shards[0]._key_out
        self.splitters = [key_out(np.ascontiguousarray(cols["keys"][cuts[j]]).tobytes()) for j in range(1, g)
                          if cuts[j] < n]
        # a shard left empty by a small load still owns the range above the last splitter
        while len(self.splitters) < g - 1:
            self.splitters.append(self.splitters[-1] if self.splitters else key_out(b"\xff" * self.schema.key_row))

    def apply(self, cols: Dict[str, np.ndarray], ops: np.ndarray) -> Tuple[int, int, int]:
        """Batched insert (op 0) / delete (op 1), each row applied on its key's shard."""
        owner = self._owners(np.ascontiguousarray(cols["keys"]).reshape(len(ops), self.schema.key_row))
        jobs = []
        for s, st in enumerate(self.shards):
            rows = np.nonzero(owner == s)[0]
            if len(rows):
                jobs.append((st, {k: np.ascontiguousarray(v[rows]) for k, v in cols.items() if v is not None},
                             np.ascontiguousarray(ops[rows])))
        out = list(self._pool.map(lambda j: j[0].apply(j[1], j[2]), jobs))
        return tuple(int(sum(c[i] for c in out)) for i in range(3))  # type: ignore[return-value]

    # ---- Rsos<K> -------------------------------------------------------------------------
    def sizes(self) -> List[int]:
        return [s.size() for s in self.shards]

    def size(self) -> int:
        return sum(self.sizes())

    __len__ = size

    def aggregate(self, rng: Optional[KeyRange] = None) -> Aggregate:
        total = Aggregate.ZERO
        for a in self._all(lambda s: s.aggregate(rng)):
            total = total + a
        return total

    def rank(self, z: Key) -> int:
        return sum(self._all(lambda s: s.rank(z)))

    def select(self, r: int) -> Key:
        if r < 0:
            raise IndexError("select: r < 0")
        for s, n in zip(self.shards, self.sizes()):
            if r < n:
                return s.select(r)
            r -= n
        raise IndexError("select: r >= size()")

    # ---- the two protocol-round questions (rsos_hip.rbsr, native=False) ---------------------
    def resolve_segments(self, segments: Sequence):
        parts = self._all(lambda s: s.resolve_segments(segments))
        lo = sum(p[0] for p in parts)
        hi = sum(p[1] for p in parts)
        aggs = [Aggregate.ZERO] * len(segments)
        for _, _, a in parts:
            aggs = [x + y for x, y in zip(aggs, a)]
        return lo, hi, aggs

    def split_segments(self, select_ranks: Sequence[int], lo: Sequence[int], hi: Sequence[int]):
        sizes = self.sizes()
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        keys = [self.select(int(r)) for r in select_ranks]  # few per round: one per SPLIT cut
        lo_a, hi_a = np.asarray(lo, np.int64), np.asarray(hi, np.int64)

        def part(j):
            s = self.shards[j]
            l = np.clip(lo_a - offs[j], 0, sizes[j])
            h = np.clip(hi_a - offs[j], 0, sizes[j])
            h = np.maximum(h, l)
            return s.aggregates_ranks(l, h) if len(l) else []
        aggs = [Aggregate.ZERO] * len(lo_a)
        for p in self._pool.map(part, range(len(self.shards))):
            aggs = [x + y for x, y in zip(aggs, p)]
        return keys, aggs
