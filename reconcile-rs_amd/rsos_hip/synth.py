"""Seeded synthetic records of the BASELINE shapes, generated directly in HBM.

Follows SURVEY.md §8(d): SplitMix64 streams (counter-based: every byte is a function of the
seed and the global row index), keys unique and sorted by memcmp (the Ord of [u8; L]); stamps
follow benches/bench.rs:286-293's pattern (physical = 1_700_000_000_000 + i, logical 0,
node_id 1); values are random bytes; optional tombstones at a given fraction.  Keys: the
first 8 bytes are the big-endian u64 i * stride + r (r < stride) -- strictly increasing, hence
unique and memcmp-sorted -- and the remaining key bytes are random.
"""
from __future__ import annotations

from typing import Dict

import torch

from .schema import RecordSchema
from . import _abi as A


_M64 = (1 << 64) - 1


def _s64(c: int) -> int:
    """An unsigned 64-bit constant as the int64 torch computes with (two's complement)."""
    c &= _M64
    return c - (1 << 64) if c >> 63 else c


_GOLD, _C1, _C2 = _s64(0x9E3779B97F4A7C15), _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB)


def _srl(z: torch.Tensor, k: int) -> torch.Tensor:
    """Logical right shift of int64 bit patterns."""
    return (z >> k) & ((1 << (64 - k)) - 1)


def splitmix64(seed: int, ctr: torch.Tensor) -> torch.Tensor:
    """Counter-based SplitMix64: the ctr-th output of the stream seeded `seed`,
    as int64 bit patterns.  Element i depends only on (seed, ctr[i]), so any row range of a data
    set is generated identically whatever shard or chunk asks for it."""
    z = (ctr + 1) * _GOLD + _s64(seed * 0xD1B54A32D192ED03)
    z = (z ^ _srl(z, 30)) * _C1
    z = (z ^ _srl(z, 27)) * _C2
    return z ^ _srl(z, 31)


def _row_bytes(seed: int, idx: torch.Tensor, width: int, chunk_words: int = 1 << 25) -> torch.Tensor:
    """(n, width) bytes: row i = the words idx[i] * W .. idx[i] * W + W - 1 of the stream, W =
    ceil(width / 8); generated in row chunks so temporaries stay ~chunk_words words."""
    n, w8 = idx.shape[0], (width + 7) // 8
    out = torch.empty((n, w8 * 8), dtype=torch.uint8, device=idx.device)
    step = max(1, chunk_words // max(w8, 1))
    lane = torch.arange(w8, device=idx.device, dtype=torch.int64)
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        ctr = idx[lo:hi, None] * w8 + lane[None, :]
        out[lo:hi] = splitmix64(seed, ctr).view(torch.uint8).view(hi - lo, w8 * 8)
    return out[:, :width] if width != w8 * 8 else out


def make_records(schema: RecordSchema, n: int, seed: int = 42, device="cuda",
                 tombstone_fraction: float = 0.0, first_index: int = 0,
                 random_keys: bool = False, key_space: int = 0,
                 indices: torch.Tensor = None) -> Dict[str, torch.Tensor]:
    """Rows [first_index, first_index + n) of a key-sorted set of `key_space` records
    (default first_index + n) whose keys spread evenly over the whole key space: row i's
    first 8 key bytes are the big-endian u64 i * stride + r, r < stride = 2^64 / key_space.
    Every byte is a counter-based SplitMix64 function of (seed, global row index), so a shard
    [a, b) of the set is the same rows whether it is generated alone or as part of the whole
    (strong-scaling runs at any GPU count hash the same data set).
    random_keys: uniformly random byte keys instead (unsorted; update batches that land
    anywhere in an existing key range).
    indices: the global row indices to generate (int64, n of them) instead of
    [first_index, first_index + n) -- rows picked from a set without gathering its columns
    (bench.py's overwrites of resident keys); key_space must then be given."""
    dev = torch.device(device)
    cols: Dict[str, torch.Tensor] = {}
    if indices is not None:
        if not key_space or indices.shape[0] != n:
            raise ValueError("indices: n of them, and the set's key_space")
        idx = indices.to(device=dev, dtype=torch.int64).contiguous()
    else:
        idx = torch.arange(first_index, first_index + n, device=dev, dtype=torch.int64)
    sk, sv, st = seed * 4 + 1, seed * 4 + 2, seed * 4 + 3  # key / value / tag streams
    if schema.key_kind == A.KEY_BYTES:
        kl = schema.key_len
        keys = _row_bytes(sk, idx, kl).contiguous()
        space = max(key_space or (first_index + n), 2)
        stride = min((1 << 64) // space, (1 << 63) - 1)
        if kl >= 8 and not random_keys:
            r = _srl(splitmix64(st + (1 << 32), idx), 1) % stride
            head = idx * stride + r  # wraps in int64; the bit pattern is the unsigned value
            shifts = torch.arange(56, -8, -8, device=dev, dtype=torch.int64)  # big-endian bytes
            keys[:, :8] = ((head[:, None] >> shifts[None, :]) & 0xFF).to(torch.uint8)  # arithmetic >> ok: & 0xFF
        cols["keys"] = keys.contiguous()
    elif schema.key_kind == A.KEY_U64:  # integer keys stay sorted (random_keys applies to byte keys)
        r = _srl(splitmix64(sk, idx), 44)  # < 2^20
        cols["keys"] = ((idx << 20) | r).contiguous().view(torch.uint8).view(n, 8)
    elif schema.key_kind == A.KEY_U32:
        cols["keys"] = idx.to(torch.int32).contiguous().view(torch.uint8).view(n, 4)
    if schema.value_row:
        cols["values"] = _row_bytes(sv, idx, schema.value_row).contiguous()
    if schema.record_kind == A.REC_DATED:
        cols["phys"] = (1_700_000_000_000 + idx).contiguous()
        cols["logical"] = torch.zeros(n, dtype=torch.int32, device=dev)
        cols["node"] = torch.ones(n, dtype=torch.int64, device=dev)
    if schema.record_kind != A.REC_PLAIN and tombstone_fraction > 0:
        u = _srl(splitmix64(st, idx), 11).to(torch.float64) * (1.0 / (1 << 53))
        cols["tags"] = (u < tombstone_fraction).to(torch.uint8)
    return cols


def to_host(cols: Dict[str, torch.Tensor], lo: int = 0, hi=None):
    """numpy copies of rows [lo, hi) with the dtypes the oracle binding expects."""
    import numpy as np
    out = {}
    for k, t in cols.items():
        a = t[lo:hi].cpu().numpy()
        if k in ("phys", "node"):
            a = a.view(np.uint64)
        elif k == "logical":
            a = a.view(np.uint32)
        out[k] = np.ascontiguousarray(a)
    return out


def make_snapshot(cols: Dict[str, torch.Tensor], schema: RecordSchema, key_form: str = "array",
                  chunk: int = 1 << 20) -> torch.Tensor:
    """The RCNL v1 file (src/snapshot.rs:30-58) of a PersistedState whose entries are the rows
    of `cols` (dated records; tags 1 = tombstone) and whose members / tombstone_acks are empty,
    built on the device as bench / test input: b"RCNL", u32 1, then bincode fixint of
    Vec<(K, Entry<Timestamp, V>)> (lww-register/src/persistence.rs:32,62-70)."""
    dev = cols["keys"].device if "keys" in cols else cols["values"].device
    n = (cols["keys"] if "keys" in cols else cols["values"]).shape[0]
    kr, vr = schema.key_row, schema.value_row
    kp = 8 if key_form == "vec" else 0
    vp = 8 if schema.value_kind == A.VAL_BYTES else 0
    lt = kp + kr + 24
    lp = lt + vp + vr
    tags = cols.get("tags")
    tags = torch.zeros(n, dtype=torch.uint8, device=dev) if tags is None else tags
    lens = torch.where(tags == 1, lt, lp).to(torch.int64)
    offs = torch.cumsum(lens, 0) - lens + 16
    body = 16 + int(lens.sum().item())
    buf = torch.zeros(body + 16, dtype=torch.uint8, device=dev)  # + empty members, empty acks
    head = b"RCNL" + (1).to_bytes(4, "little") + int(n).to_bytes(8, "little")
    buf[:16] = torch.tensor(list(head), dtype=torch.uint8, device=dev)

    def u8(t: torch.Tensor, w: int) -> torch.Tensor:
        return t.contiguous().view(torch.uint8).view(-1, w)

    def const(v: int, w: int, m: int) -> torch.Tensor:
        return torch.tensor(list(v.to_bytes(w, "little")), dtype=torch.uint8, device=dev).expand(m, w)

    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        o = offs[lo:hi]
        present = tags[lo:hi] == 0
        fields = []
        if kp:
            fields.append((0, const(kr, 8, hi - lo), None))
        if kr:
            fields.append((kp, cols["keys"][lo:hi], None))
        fields += [(kp + kr, u8(cols["phys"][lo:hi], 8), None), (kp + kr + 8, u8(cols["logical"][lo:hi], 4), None),
                   (kp + kr + 12, u8(cols["node"][lo:hi], 8), None),
                   (kp + kr + 20, u8(tags[lo:hi].to(torch.int32), 4), None)]
        if vp:
            fields.append((lt, const(vr, 8, hi - lo), present))
        if vr:
            fields.append((lt + vp, cols["values"][lo:hi], present))
        for rel, data, mask in fields:
            w = data.shape[1]
            oo, dd = (o, data) if mask is None else (o[mask], data[mask])
            idx = (oo + rel)[:, None] + torch.arange(w, device=dev)[None, :]
            buf[idx.reshape(-1)] = dd.reshape(-1)
    return buf


def encode_rows(schema: RecordSchema, cols: Dict[str, torch.Tensor]) -> torch.Tensor:
    """(n, L) uint8: the canonical bytes lift hashes for every record of `cols` (present records
    only), built on the device -- what rsos::encoding::encode_to_vec of the key then the value gives
    (rsos/src/encoding.rs:17-35): a byte key [u8; L] is a serde tuple (u64 length L, then the bytes),
    u32 / u64 keys and values are fixed LE, Vec<u8> values are u64 length + bytes, a dated record
    is Timestamp (u64 physical, u32 logical, u64 node) then State::Present (u32 0) then the value,
    a projection State::Present then the value.  The drop-in encoded map's input for the
    fixed-width shapes (bench.py --config encoded, tests)."""
    if cols.get("tags") is not None and bool((cols["tags"] != 0).any()):
        raise ValueError("encode_rows: present records only (a tombstone's encoding is shorter)")
    n = (cols["keys"] if "keys" in cols else cols["values"]).shape[0]
    dev = (cols["keys"] if "keys" in cols else cols["values"]).device

    def const(v: int, w: int) -> torch.Tensor:
        return torch.tensor(list(v.to_bytes(w, "little")), dtype=torch.uint8, device=dev).expand(n, w)

    def u8(t: torch.Tensor, w: int) -> torch.Tensor:
        return t.contiguous().view(torch.uint8).view(n, w)

    parts = []
    if schema.key_kind == A.KEY_BYTES:
        parts += [const(schema.key_len, 8), cols["keys"]]
    elif schema.key_kind != A.KEY_UNIT:
        parts.append(cols["keys"])
    if schema.record_kind == A.REC_DATED:
        parts += [u8(cols["phys"], 8), u8(cols["logical"], 4), u8(cols["node"], 8)]
    if schema.record_kind != A.REC_PLAIN:
        parts.append(const(0, 4))
    if schema.value_kind == A.VAL_BYTES:
        parts.append(const(schema.value_row, 8))
    if schema.value_row:
        parts.append(cols["values"])
    return torch.cat(parts, dim=1).contiguous()
