"""ShardedStore -- one replica's map over several GPUs inside one process (rh_sstore_*).

The benchmark scales with one process per GPU (torch.distributed); a replica is one process
(src/replica.rs:68-74), so inside it the same key-range partitioning is the
library's sharded store: one column store per device, each owning a contiguous key range
[split[s - 1], split[s]), cut at equal counts by a load (before the first load the key space is
cut evenly).  The library answers every question of the Rsos<K> surface (rsos/src/rsos_trait.rs:39-90)
and whole protocol rounds (rbsr/src/protocol.rs:212-317) by decomposing them over the shards, with
no device-to-device traffic and one host thread per shard (include/rsos_hip.h, csrc/sharded_store.hip):

  size / rank(z)        sums over shards: rank(z) = rows of the shards below z's + rank in z's shard
  aggregate(range)      the shards inside the range give their roots, <= 2 boundary shards are asked
                        (Aggregate's Add, rsos/src/aggregate.rs:79-89)
  select(r)             the shard whose rank interval holds r
  apply / stage         rows routed to their key's shard by the splitters
  protocol round        a run of segments inside one shard is that shard's own round; a segment
                        straddling a boundary is resolved from its two boundary shards, decided on
                        the host and cut by routed selects and rank-range aggregates

ShardedStore has GpuFingerprintStore's interface (the same methods, on rh_sstore_* entry points), so
rsos_hip.rbsr's native and two-call round paths run on it unchanged.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _abi as A
from .schema import RecordSchema
from .store import GpuFingerprintStore, Key, _np_ptr, DEFAULT_HOST_TIER


class _Shard(GpuFingerprintStore):
    """One shard's store, borrowed from the sharded store (destroyed with it)."""

    def __init__(self, schema: RecordSchema, handle: C.c_void_p):
        self.schema = schema
        self._s = schema.c()
        self._h = handle

    def close(self) -> None:
        self._h = None  # borrowed: the sharded store destroys it

    def _f(self, name):
        if self._h is None:
            raise ValueError("shard of a closed ShardedStore")
        return GpuFingerprintStore._f(self, name)


class ShardedStore(GpuFingerprintStore):
    _P = "rh_sstore_"

    def __init__(self, schema: RecordSchema, devices: Sequence[int], host_tier: Optional[bool] = None):
        if not devices:
            raise ValueError("at least one device")
        self.schema = schema
        self._s = schema.c()
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        A.check(A.lib().rh_sstore_create(devs, len(devices), C.byref(self._s), C.byref(h)), "rh_sstore_create")
        self._h = h
        self.shards = []
        for i in range(len(devices)):
            sh = C.c_void_p()
            A.check(A.lib().rh_sstore_shard(self._h, i, C.byref(sh)), "rh_sstore_shard")
            self.shards.append(_Shard(schema, sh))
        if DEFAULT_HOST_TIER if host_tier is None else host_tier:
            self.set_host_tier(True)

    def close(self) -> None:
        """Destroy the sharded store and every shard's store: the _Shard views (and any the caller
        kept) are detached first, so a later call on one raises instead of reaching freed memory."""
        for sh in getattr(self, "shards", []):
            sh.close()
        GpuFingerprintStore.close(self)

    # ---- the partition -------------------------------------------------------------------
    @property
    def splitters(self) -> List[Key]:
        kl = self.schema.key_row
        g = len(self.shards)
        buf = np.zeros(max((g - 1) * kl, 1), np.uint8)
        A.check(A.lib().rh_sstore_splitters(self._h, _np_ptr(buf)), "rh_sstore_splitters")
        return [self._key_out(buf[j * kl:(j + 1) * kl].tobytes()) for j in range(g - 1)]

    def set_splitters(self, keys: Sequence[Key]) -> None:
        """Cut an empty map's key space at `keys` (len(shards) - 1 of them, non-decreasing)."""
        if len(keys) != len(self.shards) - 1:
            raise ValueError("one splitter per shard boundary")
        buf = np.frombuffer(b"".join(self._key_bytes(k) for k in keys) or b"\0", np.uint8).copy()
        A.check(A.lib().rh_sstore_set_splitters(self._h, _np_ptr(buf)), "rh_sstore_set_splitters")

    def sizes(self) -> List[int]:
        return [s.size() for s in self.shards]

    # ---- per-shard bookkeeping (the shards' own counters) --------------------------------
    def stats(self) -> Dict[str, int]:
        out = {"base_rows": 0, "delta_rows": 0, "compactions": 0}
        for s in self.shards:
            for k, v in s.stats().items():
                out[k] += v
        return out

    def tier_stats(self) -> Dict[str, int]:
        out = {"base_rows": 0, "delta_entries": 0, "refreshes": 0, "folds": 0}
        for s in self.shards:
            for k, v in s.tier_stats().items():
                out[k] += v
        return out

    def batch_stats(self) -> Dict[str, int]:
        out = {"small": 0, "large": 0}
        for s in self.shards:
            for k, v in s.batch_stats().items():
                out[k] += v
        return out

    def tier_sync(self) -> None:
        for s in self.shards:
            s.tier_sync()

    def set_compaction(self, divisor: int, min_rows: int) -> None:
        for s in self.shards:
            s.set_compaction(divisor, min_rows)

    def load_bulk_device(self, cols) -> None:
        raise NotImplementedError("the sharded store takes host columns (load_bulk)")

    def apply_device(self, cols, ops=None):
        raise NotImplementedError("the sharded store takes host columns (apply / stage)")

    def apply_device_many(self, batches, ops=None):
        raise NotImplementedError("the sharded store takes host columns (apply / stage)")

    def _key_bytes(self, k: Key) -> bytes:
        return GpuFingerprintStore._key_bytes(self, k)
