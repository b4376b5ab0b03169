"""CPU restatement of the RCNL v1 snapshot file (TEST INFRASTRUCTURE ONLY).

Only tests/ and bench.py's cpu_baseline leg import this: it writes the snapshots the GPU decoder
is tested on and decodes small ones independently as the checker.

File (src/snapshot.rs:30-58): b"RCNL" | u32 LE format version (1) | bincode::serialize(state).
decode_snapshot's checks and messages: src/snapshot.rs:60-98.
bincode 1.3.3's top-level serialize / deserialize use fixint encoding, little-endian, trailing
bytes allowed: ints fixed-width LE, seq / map lengths u64, enum variants u32, tuples / structs /
newtypes without framing ([u8; L] is a tuple: the raw bytes), Vec<u8> / String = u64 length + bytes.
state = PersistedState<K, V> (lww-register/src/persistence.rs:62-70):
    entries:        Vec<(K, Entry<Timestamp, V>)>                (:32)
    members:        HashSet<IpAddr>
    tombstone_acks: HashMap<K, HashMap<IpAddr, u64>>
Entry<Timestamp, V> = stamp, State<V> (lww-register/src/entry.rs:24-29,88-94);
Timestamp = physical u64 (ms), logical u32, node_id u64 (lww-register/src/clock.rs:141-181,
newtypes add nothing); State: variant 0 Present(V), 1 Tombstone.
IpAddr (serde, non-human-readable): variant u32 0 V4 / 1 V6, then the octets as a tuple.

Parity: the field order and widths of Timestamp / Entry are pinned by the reference's golden
vectors (tests/timestamp_wire_format.rs, varint form; tests/test_wire.py), the header by
src/snapshot.rs's own tests (reproduced in tests/test_snapshot.py); the fixint layer is bincode
1.3.3's published encoding (Cargo.lock:167-170) -- no byte-level fixint snapshot vector exists
in the reference, so that layer is restated, not pinned.
"""
from __future__ import annotations

import ipaddress
import struct
from typing import Dict, Optional, Sequence

import numpy as np

MAGIC = b"RCNL"
VERSION = 1
HEADER_LEN = 8


def _widths(key_kind: str, key_len: int, value_kind: str, value_len: int):
    """(key_pre, key_row, val_pre, val_row); key_kind u32|u64|array|vec, value_kind unit|u32|u64|bytes."""
    kr = {"u32": 4, "u64": 8}.get(key_kind, key_len)
    vr = {"unit": 0, "u32": 4, "u64": 8}.get(value_kind, value_len)
    return (8 if key_kind == "vec" else 0), kr, (8 if value_kind == "bytes" else 0), vr


def _ip(a) -> bytes:
    a = ipaddress.ip_address(a)
    return struct.pack("<I", 0 if a.version == 4 else 1) + a.packed


def encode_snapshot(keys: np.ndarray, phys: np.ndarray, logical: np.ndarray, node: np.ndarray,
                    tags: np.ndarray, values: Optional[np.ndarray], key_kind: str, value_kind: str,
                    members: Sequence = (), acks: Optional[Dict[bytes, Dict[object, int]]] = None,
                    magic: bytes = MAGIC, version: int = VERSION) -> bytes:
    """keys (n, key_row) u8 (LE bytes for int keys), values (n, value_row) u8; tags 1 = tombstone."""
    n = int(keys.shape[0])
    kp, kr, vp, vr = _widths(key_kind, keys.shape[1] if keys.ndim == 2 else 0, value_kind,
                             0 if values is None else values.shape[1])
    lt = kp + kr + 24
    lp = lt + vp + vr
    tags = np.asarray(tags, np.uint8)
    lens = np.where(tags == 1, lt, lp).astype(np.int64)
    offs = np.zeros(n, np.int64)
    if n:
        offs[1:] = np.cumsum(lens)[:-1]
    offs += 16
    body_end = 16 + int(lens.sum())
    buf = np.zeros(body_end, np.uint8)
    buf[:4] = np.frombuffer(magic, np.uint8)
    buf[4:8] = np.frombuffer(struct.pack("<I", version), np.uint8)
    buf[8:16] = np.frombuffer(struct.pack("<Q", n), np.uint8)

    def col(a, w):
        return np.ascontiguousarray(a).view(np.uint8).reshape(n, w)

    fields = []
    if kp:
        fields.append((0, np.tile(np.frombuffer(struct.pack("<Q", kr), np.uint8), (n, 1)), None))
    if kr:
        fields.append((kp, np.ascontiguousarray(keys, np.uint8).reshape(n, kr), None))
    fields.append((kp + kr, col(np.asarray(phys, np.uint64), 8), None))
    fields.append((kp + kr + 8, col(np.asarray(logical, np.uint32), 4), None))
    fields.append((kp + kr + 12, col(np.asarray(node, np.uint64), 8), None))
    fields.append((kp + kr + 20, col(tags.astype(np.uint32), 4), None))
    present = tags == 0
    if vp:
        fields.append((lt, np.tile(np.frombuffer(struct.pack("<Q", vr), np.uint8), (n, 1)), present))
    if vr:
        fields.append((lt + vp, np.ascontiguousarray(values, np.uint8).reshape(n, vr), present))
    for lo in range(0, n, 1 << 16):  # bounded index arrays
        hi = min(n, lo + (1 << 16))
        for rel, arr, mask in fields:
            w = arr.shape[1]
            rows = np.arange(lo, hi) if mask is None else lo + np.nonzero(mask[lo:hi])[0]
            if rows.size:
                buf[(offs[rows] + rel)[:, None] + np.arange(w)] = arr[rows]
    tail = bytearray(struct.pack("<Q", len(members)))
    for m in members:
        tail += _ip(m)
    acks = acks or {}
    tail += struct.pack("<Q", len(acks))
    for k, peers in acks.items():
        kb = bytes(k)
        tail += (struct.pack("<Q", len(kb)) if key_kind == "vec" else b"") + kb
        tail += struct.pack("<Q", len(peers))
        for ip, ver in peers.items():
            tail += _ip(ip) + struct.pack("<Q", ver)
    return buf.tobytes() + bytes(tail)


class _R:
    def __init__(self, d: bytes, p: int):
        self.d, self.p = d, p

    def take(self, k: int) -> bytes:
        if len(self.d) - self.p < k:
            raise ValueError("io error: unexpected end of file")
        b = self.d[self.p:self.p + k]
        self.p += k
        return b

    def u32(self) -> int:
        return struct.unpack("<I", self.take(4))[0]

    def u64(self) -> int:
        return struct.unpack("<Q", self.take(8))[0]

    def ip(self):
        v = self.u32()
        if v > 1:
            raise ValueError(f"invalid value: integer `{v}`, expected variant index 0 <= i < 2")
        return ipaddress.ip_address(self.take(4 if v == 0 else 16))


def check_header(data: bytes) -> None:
    """src/snapshot.rs:66-97."""
    if len(data) < HEADER_LEN:
        raise ValueError(f"snapshot is {len(data)} bytes, shorter than the {HEADER_LEN}-byte format header "
                         "(truncated, or a pre-Entry/State snapshot without the versioned header)")
    if data[:4] != MAGIC:
        raise ValueError("snapshot magic does not match; the file is not a reconcile snapshot, "
                         "or predates the versioned format")
    version = struct.unpack("<I", data[4:8])[0]
    if version != VERSION:
        raise ValueError(f"snapshot format version {version} is not supported by this build "
                         f"(expected {VERSION})")


def decode_snapshot(data: bytes, key_kind: str, key_len: int, value_kind: str, value_len: int):
    """Pure-Python decode (small files): (columns dict, members, acks, entries_end)."""
    data = bytes(data)
    check_header(data)
    kp, kr, vp, vr = _widths(key_kind, key_len, value_kind, value_len)
    r = _R(data, HEADER_LEN)
    n = r.u64()
    keys, phys, logical, node, tags, vals = [], [], [], [], [], []

    def key(rr: _R) -> bytes:
        if kp and rr.u64() != kr:
            raise ValueError("key length differs from the schema's")
        return rr.take(kr)

    for _ in range(n):
        keys.append(key(r))
        phys.append(r.u64())
        logical.append(r.u32())
        node.append(r.u64())
        v = r.u32()
        if v > 1:
            raise ValueError(f"invalid value: integer `{v}`, expected variant index 0 <= i < 2")
        tags.append(v)
        if v == 0:
            if vp and r.u64() != vr:
                raise ValueError("value length differs from the schema's")
            vals.append(r.take(vr))
        else:
            vals.append(bytes(vr))
    entries_end = r.p
    members = [r.ip() for _ in range(r.u64())]
    acks = {}
    for _ in range(r.u64()):
        k = key(r)
        acks[k] = {}
        for _ in range(r.u64()):
            ip = r.ip()
            acks[k][ip] = r.u64()
    cols = {
        "keys": np.frombuffer(b"".join(keys), np.uint8).reshape(n, kr).copy() if kr else np.zeros((n, 0), np.uint8),
        "phys": np.array(phys, np.uint64), "logical": np.array(logical, np.uint32),
        "node": np.array(node, np.uint64), "tags": np.array(tags, np.uint8),
        "values": np.frombuffer(b"".join(vals), np.uint8).reshape(n, vr).copy() if vr else np.zeros((n, 0), np.uint8),
    }
    return cols, members, acks, entries_end


def last_wins(cols: Dict[str, np.ndarray], int_keys: bool = False) -> np.ndarray:
    """Row indices the sequential replay keeps, in key order: the last row of every key
    (just_insert_bulk inserts in file order, src/replica/write.rs:117-120).  Byte keys order
    by memcmp ([u8; L] Ord), int keys (LE bytes) numerically."""
    k = cols["keys"]
    last = {}
    for i in range(k.shape[0]):
        last[k[i].tobytes()] = i
    order = sorted(last, key=(lambda b: int.from_bytes(b, "little")) if int_keys else None)
    return np.array([last[b] for b in order], np.int64)
