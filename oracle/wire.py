"""CPU restatement of the gossip wire codec for RangeAggregate (TEST INFRASTRUCTURE ONLY).

Only tests/ import this, as the checker of librsos_hip.so's rh_wire_* codec.

The gossip codec is bincode 1.3.3 with `DefaultOptions` (gossip/src/bincode.rs:65-100):
varint integers, little-endian, no framing on structs / tuples.  bincode's VarintEncoding:
v < 251 -> the byte v; v < 2^16 -> 251 + u16 LE; v < 2^32 -> 252 + u32 LE; else 253 + u64 LE
(254 + u128 LE for u128, not used here).  u8 is written raw.  Enum variants are u32 varints.

Restated items:
  RangeAggregate<K> = KeyRange(StartBound<K>, EndBound<K>), Aggregate     rbsr/src/protocol.rs:47-88
  StartBound: 0 Unbounded | 1 Included(K);  EndBound: 0 Unbounded | 1 Excluded(K)
  Aggregate = fingerprint ([u8; 32] raw, rsos/src/fingerprint.rs:74-83), size (usize -> u64)
                                                                        rsos/src/aggregate.rs:24-42
  Timestamp = physical u64, logical u32, node_id u64                    lww-register/src/clock.rs:141-181
  Entry<Timestamp, V> = stamp, State<V> (0 Present(V) | 1 Tombstone)    lww-register/src/entry.rs:24-29,88-94
  Message<K, V, P> variant tags                                          src/replica.rs:184-210
Pinned by the reference's golden vectors: tests/wire_format.rs:37-62 (RangeAggregate<u32>) and
tests/timestamp_wire_format.rs:59-100 (Timestamp, Entry<Timestamp, u32>) -- tests/test_wire.py.
decode_stream follows gossip::bincode::decode_stream: an end of input anywhere is a clean end
of the stream (the partial item is dropped), any other error rejects the input.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple


class Eof(Exception):
    pass


class Bad(ValueError):
    pass


def varint(v: int) -> bytes:
    if v < 0:
        raise ValueError("unsigned only")
    if v < 251:
        return bytes([v])
    if v < 1 << 16:
        return b"\xfb" + struct.pack("<H", v)
    if v < 1 << 32:
        return b"\xfc" + struct.pack("<I", v)
    if v < 1 << 64:
        return b"\xfd" + struct.pack("<Q", v)
    raise ValueError("u128 not used")


class Reader:
    def __init__(self, data: bytes):
        self.d, self.p = bytes(data), 0

    def take(self, n: int) -> bytes:
        if len(self.d) - self.p < n:
            raise Eof()
        b = self.d[self.p:self.p + n]
        self.p += n
        return b

    def varint(self, max_value: int = (1 << 64) - 1) -> int:
        m = self.take(1)[0]
        if m < 251:
            v = m
        elif m == 251:
            v = struct.unpack("<H", self.take(2))[0]
        elif m == 252:
            v = struct.unpack("<I", self.take(4))[0]
        elif m == 253:
            v = struct.unpack("<Q", self.take(8))[0]
        else:
            raise Bad(f"invalid varint marker {m}")
        if v > max_value:
            raise Bad(f"varint {v} out of range")
        return v


# ---- key codecs: (encode, decode) ------------------------------------------------------------
def key_codec(kind: str, key_len: int = 0) -> Tuple[Callable[[object], bytes], Callable[[Reader], object]]:
    """kind: 'u32' | 'u64' (ints), 'array' ([u8; L]: raw bytes), 'vec' (Vec<u8>/String)."""
    if kind == "u32":
        return (lambda k: varint(int(k))), (lambda r: r.varint((1 << 32) - 1))
    if kind == "u64":
        return (lambda k: varint(int(k))), (lambda r: r.varint())
    if kind == "array":
        return (lambda k: bytes(k)), (lambda r: r.take(key_len))

    def dec_vec(r: Reader) -> bytes:
        n = r.varint()
        if n != key_len:
            raise Bad(f"key length {n} != {key_len}")
        return r.take(n)
    return (lambda k: varint(len(bytes(k))) + bytes(k)), dec_vec


@dataclass(frozen=True)
class RangeAggregate:
    start: Optional[object]   # None = Unbounded, else Included(start)
    end: Optional[object]     # None = Unbounded, else Excluded(end)
    fingerprint: Tuple[int, int, int, int]
    size: int


def encode_range_aggregate(ra: RangeAggregate, enc_key, msg_tag: Optional[int] = None) -> bytes:
    out = b"" if msg_tag is None else varint(msg_tag)
    out += varint(0) if ra.start is None else varint(1) + enc_key(ra.start)
    out += varint(0) if ra.end is None else varint(1) + enc_key(ra.end)
    out += b"".join(struct.pack("<Q", l) for l in ra.fingerprint)
    return out + varint(ra.size)


def decode_range_aggregate(r: Reader, dec_key, msg_tag: Optional[int] = None) -> RangeAggregate:
    if msg_tag is not None:
        t = r.varint((1 << 32) - 1)
        if t != msg_tag:
            raise Bad(f"message tag {t}")
    sv = r.varint((1 << 32) - 1)
    if sv > 1:
        raise Bad(f"invalid start bound variant {sv}")
    start = dec_key(r) if sv else None
    ev = r.varint((1 << 32) - 1)
    if ev > 1:
        raise Bad(f"invalid end bound variant {ev}")
    end = dec_key(r) if ev else None
    fp = struct.unpack("<4Q", r.take(32))
    return RangeAggregate(start, end, fp, r.varint())


def decode_stream(data: bytes, dec_key, max_items: int, msg_tag: Optional[int] = None
                  ) -> Tuple[List[RangeAggregate], int]:
    """Items and the bytes they span; Bad propagates (the whole input is rejected)."""
    r, out, done = Reader(data), [], 0
    while len(out) < max_items:
        try:
            out.append(decode_range_aggregate(r, dec_key, msg_tag))
        except Eof:
            break
        done = r.p
    return out, done


# ---- Timestamp / Entry (the goldens that pin the varint layer) --------------------------------
def encode_timestamp(phys: int, logical: int, node: int) -> bytes:
    return varint(phys) + varint(logical) + varint(node)


def encode_entry_u32(phys: int, logical: int, node: int, value: Optional[int]) -> bytes:
    state = varint(1) if value is None else varint(0) + varint(value)
    return encode_timestamp(phys, logical, node) + state
