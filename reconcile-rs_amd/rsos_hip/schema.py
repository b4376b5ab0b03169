"""Record schemas: which (K, V) the kernels synthesise the canonical encoding for.

rsos::encoding (rsos/src/encoding.rs:17-35) is generic over serde; the GPU path is
specialised per fixed-width record shape.  Shapes without a specialised
kernel are hashed through the encoded-bytes path (`lift_encoded`).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _abi as A


@dataclass(frozen=True)
class RecordSchema:
    key_kind: int      # A.KEY_*
    key_len: int
    value_kind: int    # A.VAL_*
    value_len: int
    record_kind: int   # A.REC_PLAIN / REC_DATED / REC_PROJECTION

    # ---- constructors for the reference's record types -------------------------------
    @staticmethod
    def plain(key: str, value: str) -> "RecordSchema":
        """FingerprintTreeMap<K, V>: lift(k, v).  key/value: 'u32', 'u64', 'bytesN'."""
        kk, kl = _kind(key, True)
        vk, vl = _kind(value, False)
        return RecordSchema(kk, kl, vk, vl, A.REC_PLAIN)

    @staticmethod
    def dated(key: str, value: str) -> "RecordSchema":
        """Replica.map: FingerprintTreeMap<K, Entry<Timestamp, V>> (src/replica.rs:69)."""
        kk, kl = _kind(key, True)
        vk, vl = _kind(value, False)
        return RecordSchema(kk, kl, vk, vl, A.REC_DATED)

    @staticmethod
    def projection(key: str, value: str) -> "RecordSchema":
        """Replica.projection: FingerprintTreeMap<K, State<V>> (src/replica.rs:74)."""
        kk, kl = _kind(key, True)
        vk, vl = _kind(value, False)
        return RecordSchema(kk, kl, vk, vl, A.REC_PROJECTION)

    # ---- derived -------------------------------------------------------------------------
    def c(self) -> A.Schema:
        return A.Schema(self.key_kind, self.key_len, self.value_kind, self.value_len, self.record_kind, 0)

    @property
    def key_row(self) -> int:
        return {A.KEY_UNIT: 0, A.KEY_U32: 4, A.KEY_U64: 8}.get(self.key_kind, self.key_len)

    @property
    def value_row(self) -> int:
        return {A.VAL_UNIT: 0, A.VAL_U32: 4, A.VAL_U64: 8}.get(self.value_kind, self.value_len)

    @property
    def dated_kind(self) -> bool:
        return self.record_kind == A.REC_DATED

    def record_len(self, tombstone: bool = False) -> int:
        s = self.c()
        return int(A.check(A.lib().rh_schema_record_len(C.byref(s), int(tombstone)), "rh_schema_record_len"))

    def supported(self) -> bool:
        s = self.c()
        return A.check(A.lib().rh_schema_supported(C.byref(s)), "rh_schema_supported") == 1

    def with_kind(self, record_kind: int) -> "RecordSchema":
        return RecordSchema(self.key_kind, self.key_len, self.value_kind, self.value_len, record_kind)


def _kind(name: str, key: bool):
    if name == "unit":
        return (A.KEY_UNIT if key else A.VAL_UNIT), 0
    if name == "u32":
        return (A.KEY_U32 if key else A.VAL_U32), 4
    if name == "u64":
        return (A.KEY_U64 if key else A.VAL_U64), 8
    if name.startswith("bytes"):
        return (A.KEY_BYTES if key else A.VAL_BYTES), int(name[5:])
    raise ValueError(f"unknown field kind {name!r}")
