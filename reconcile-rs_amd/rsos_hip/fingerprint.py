"""Fingerprint / Aggregate value types (rsos/src/fingerprint.rs:62-228, rsos/src/aggregate.rs:38-89).

Plain value types: combining two already-computed fingerprints (a 256-bit add) is host
arithmetic in the reference too (Aggregate's Add); no hashing happens here.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import ClassVar, Iterable, Tuple

_MOD = 1 << 256


@dataclass(frozen=True)
class Fingerprint:
    """256-bit fingerprint: four little-endian u64 limbs, limb 0 least significant.

    An abelian group under addition mod 2^256 (`+` = combine, `-` = remove, `ZERO`)."""

    limbs: Tuple[int, int, int, int]

    ZERO: ClassVar["Fingerprint"]

    @staticmethod
    def from_int(x: int) -> "Fingerprint":
        x %= _MOD
        return Fingerprint(tuple((x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)))  # type: ignore[arg-type]

    @staticmethod
    def from_le_bytes(b: bytes) -> "Fingerprint":  # fingerprint.rs:106-124
        if len(b) != 32:
            raise ValueError("a fingerprint is 32 bytes")
        return Fingerprint(struct.unpack("<4Q", bytes(b)))

    def to_le_bytes(self) -> bytes:  # fingerprint.rs:131-141
        return struct.pack("<4Q", *self.limbs)

    def to_int(self) -> int:
        return sum(l << (64 * i) for i, l in enumerate(self.limbs))

    def combine(self, other: "Fingerprint") -> "Fingerprint":  # fingerprint.rs:145-154
        return Fingerprint.from_int(self.to_int() + other.to_int())

    def remove(self, other: "Fingerprint") -> "Fingerprint":  # fingerprint.rs:159-173
        return Fingerprint.from_int(self.to_int() - other.to_int())

    __add__ = combine
    __sub__ = remove

    def __neg__(self) -> "Fingerprint":  # fingerprint.rs:202-207
        return Fingerprint.ZERO.remove(self)

    def __str__(self) -> str:  # most-significant limb first, fingerprint.rs:220-228
        return "".join(f"{l:016x}" for l in reversed(self.limbs))

    def __repr__(self) -> str:
        return f"Fingerprint({self})"

    @staticmethod
    def sum(fps: Iterable["Fingerprint"]) -> "Fingerprint":
        return Fingerprint.from_int(sum(f.to_int() for f in fps))


Fingerprint.ZERO = Fingerprint((0, 0, 0, 0))


@dataclass(frozen=True)
class Aggregate:
    """(size, fingerprint) monoid; emptiness is decided on size, never the fingerprint."""

    size: int
    fingerprint: Fingerprint

    ZERO: ClassVar["Aggregate"]

    @staticmethod
    def new(size: int, fingerprint: Fingerprint) -> "Aggregate":  # aggregate.rs:53
        return Aggregate(size, fingerprint)

    def is_empty(self) -> bool:
        return self.size == 0

    def __add__(self, other: "Aggregate") -> "Aggregate":  # aggregate.rs:79-89
        return Aggregate(self.size + other.size, self.fingerprint + other.fingerprint)

    @staticmethod
    def from_c(agg) -> "Aggregate":
        return Aggregate(int(agg.size), Fingerprint(tuple(int(x) for x in agg.fingerprint)))


Aggregate.ZERO = Aggregate(0, Fingerprint.ZERO)
