"""Pure-Python restatement of the fingerprint-hash path -- the SECOND, independent oracle.

TEST INFRASTRUCTURE ONLY: imported by tests/ and tests/golden/make_golden.py, never by the
product package.  It exists so the C oracle (oracle/oracle.c) is cross-checked by code
written separately, for the multi-block (65..1024 B) and multi-chunk (>1024 B) BLAKE3
inputs that the reference's own golden vectors do not reach.

Restates:
  * BLAKE3 (crate `blake3` 1.8.5, Cargo.lock:197-200) from the published specification,
    structured as "split into chunks, hash each chunk, fold the binary tree whose left
    subtree holds the largest power-of-two number of chunks" (the spec's recursive form),
    unlike the C oracle's incremental CV stack.
  * the canonical serializer, rsos/src/encoding.rs:17-35 + encoding/serializer.rs:40-212,
    over a small typed value model (U8(..), U32(..), Str(..), Seq(..), Struct(..), ...).
  * lift / digest (rsos/src/fingerprint.rs:270-292) and the 2^256 group (:145-173).
Small cases only: it is slow (pure-Python loops).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Any, List, Sequence

MASK = 0xFFFFFFFF
IV = (0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19)
SCHEDULE: List[List[int]] = []
_p = list(range(16))
for _ in range(7):
    SCHEDULE.append(_p)
    _p = [_p[i] for i in (2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8)]
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8


def _rot(x: int, n: int) -> int:
    return ((x >> n) | (x << (32 - n))) & MASK


def _compress(cv: Sequence[int], words: Sequence[int], counter: int, blen: int, flags: int) -> List[int]:
    s = list(cv) + list(IV[:4]) + [counter & MASK, (counter >> 32) & MASK, blen, flags]
    lanes = ((0, 4, 8, 12), (1, 5, 9, 13), (2, 6, 10, 14), (3, 7, 11, 15),
             (0, 5, 10, 15), (1, 6, 11, 12), (2, 7, 8, 13), (3, 4, 9, 14))
    for rnd in range(7):
        m = [words[j] for j in SCHEDULE[rnd]]
        for gi, (a, b, c, d) in enumerate(lanes):
            s[a] = (s[a] + s[b] + m[2 * gi]) & MASK
            s[d] = _rot(s[d] ^ s[a], 16)
            s[c] = (s[c] + s[d]) & MASK
            s[b] = _rot(s[b] ^ s[c], 12)
            s[a] = (s[a] + s[b] + m[2 * gi + 1]) & MASK
            s[d] = _rot(s[d] ^ s[a], 8)
            s[c] = (s[c] + s[d]) & MASK
            s[b] = _rot(s[b] ^ s[c], 7)
    return [s[i] ^ s[i + 8] for i in range(8)] + [s[i + 8] ^ cv[i] for i in range(8)]


def _words(block: bytes) -> List[int]:
    return list(struct.unpack("<16I", block.ljust(64, b"\0")))


def _chunk_cv(chunk: bytes, index: int, root: bool) -> List[int]:
    blocks = [chunk[i:i + 64] for i in range(0, len(chunk), 64)] or [b""]
    cv = list(IV)
    for bi, blk in enumerate(blocks):
        flags = (CHUNK_START if bi == 0 else 0) | (CHUNK_END if bi == len(blocks) - 1 else 0)
        if root and bi == len(blocks) - 1:
            flags |= ROOT
        cv = _compress(cv, _words(blk), index, len(blk), flags)[:8]
    return cv


def _subtree(data: bytes, first_chunk: int, root: bool) -> List[int]:
    n_chunks = max(1, -(-len(data) // 1024))
    if n_chunks == 1:
        return _chunk_cv(data, first_chunk, root)
    left_chunks = 1 << ((n_chunks - 1).bit_length() - 1)  # largest power of 2 < n_chunks
    split = left_chunks * 1024
    left = _subtree(data[:split], first_chunk, False)
    right = _subtree(data[split:], first_chunk + left_chunks, False)
    return _compress(IV, left + right, 0, 64, PARENT | (ROOT if root else 0))[:8]


def blake3(data: bytes) -> bytes:
    return struct.pack("<8I", *_subtree(bytes(data), 0, True))


# ---- canonical encoding over a typed value model -------------------------------------

@dataclass(frozen=True)
class Int:
    value: int
    width: int  # bytes: 1, 2, 4, 8, 16


def U8(v: int) -> Int: return Int(v & 0xFF, 1)
def U32(v: int) -> Int: return Int(v & MASK, 4)
def U64(v: int) -> Int: return Int(v & (2**64 - 1), 8)


@dataclass(frozen=True)
class Str:
    value: bytes  # str / bytes / Vec<u8> encode identically (serializer.rs:105-113,162-174)


@dataclass(frozen=True)
class Seq:
    items: tuple  # Vec<T>, [T; N] (serde tuple), tuples: u64 count then elements


@dataclass(frozen=True)
class Struct:
    fields: tuple  # declaration order, no names, no count (serializer.rs:210-212)


@dataclass(frozen=True)
class Unit:
    pass


@dataclass(frozen=True)
class Variant:
    index: int
    payload: Any = None  # None -> unit variant, else newtype variant payload


@dataclass(frozen=True)
class Opt:
    value: Any = None  # None -> 0 ; Some(v) -> 1, v


def encode(v: Any) -> bytes:
    if isinstance(v, Int):
        return (v.value % (1 << (8 * v.width))).to_bytes(v.width, "little")
    if isinstance(v, Str):
        return struct.pack("<Q", len(v.value)) + bytes(v.value)
    if isinstance(v, Seq):
        return struct.pack("<Q", len(v.items)) + b"".join(encode(x) for x in v.items)
    if isinstance(v, Struct):
        return b"".join(encode(x) for x in v.fields)
    if isinstance(v, Unit):
        return b""
    if isinstance(v, Variant):
        head = struct.pack("<I", v.index)
        return head if v.payload is None else head + encode(v.payload)
    if isinstance(v, Opt):
        return b"\0" if v.value is None else b"\1" + encode(v.value)
    raise TypeError(f"no canonical form for {v!r}")


def timestamp(physical: int, logical: int, node_id: int) -> Struct:
    """Timestamp { hlc: Hlc { physical, logical }, node_id } (lww-register/src/clock.rs:143-181)."""
    return Struct((Struct((U64(physical), U32(logical))), U64(node_id)))


def present(v: Any) -> Variant:  # State::Present(v), lww-register/src/entry.rs:24-29
    return Variant(0, v)


TOMBSTONE = Variant(1)


def entry(stamp: Struct, state: Variant) -> Struct:  # Entry { stamp, state }, entry.rs:88-94
    return Struct((stamp, state))


def lift(key: Any, value: Any) -> bytes:
    return blake3(encode(key) + encode(value))


def digest(value: Any) -> bytes:
    return blake3(encode(value))


def fp_limbs(b: bytes) -> List[int]:
    return list(struct.unpack("<4Q", b))


def fp_int(b: bytes) -> int:
    return int.from_bytes(b, "little")


def fp_add(*fps: bytes) -> bytes:
    return (sum(fp_int(f) for f in fps) % (1 << 256)).to_bytes(32, "little")


def fp_sub(a: bytes, b: bytes) -> bytes:
    return ((fp_int(a) - fp_int(b)) % (1 << 256)).to_bytes(32, "little")
