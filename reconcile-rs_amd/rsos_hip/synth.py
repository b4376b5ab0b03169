"""Seeded synthetic records of the BASELINE shapes, generated directly in HBM.

Follows SURVEY.md §8(d): keys are unique and sorted by memcmp (the Ord of [u8; L]); stamps
follow benches/bench.rs:286-293's pattern (physical = 1_700_000_000_000 + i, logical 0,
node_id 1); values are random bytes; optional tombstones at a given fraction.  Keys: the
first 8 bytes are the big-endian u64 (i << 24 | r24) -- strictly increasing, hence unique
and memcmp-sorted -- and the remaining key bytes are random.
"""
from __future__ import annotations

from typing import Dict

import torch

from .schema import RecordSchema
from . import _abi as A


def _rand_bytes(gen: torch.Generator, shape, device) -> torch.Tensor:
    # int64 random words viewed as bytes (fast on device)
    n = 1
    for s in shape:
        n *= s
    words = (n + 7) // 8
    w = torch.randint(-2**63, 2**63 - 1, (words,), generator=gen, device=device, dtype=torch.int64)
    return w.view(torch.uint8)[:n].view(*shape)


def make_records(schema: RecordSchema, n: int, seed: int = 42, device="cuda",
                 tombstone_fraction: float = 0.0, first_index: int = 0,
                 random_keys: bool = False, key_space: int = 0) -> Dict[str, torch.Tensor]:
    """Rows [first_index, first_index + n) of a key-sorted set of `key_space` records
    (default first_index + n) whose keys spread evenly over the whole key space: row i's
    first 8 key bytes are the big-endian u64 i * stride + r, r < stride = 2^64 / key_space.
    random_keys: uniformly random keys instead (unsorted; update batches that land anywhere
    in an existing key range)."""
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    cols: Dict[str, torch.Tensor] = {}
    idx = torch.arange(first_index, first_index + n, device=dev, dtype=torch.int64)
    if schema.key_kind == A.KEY_BYTES:
        kl = schema.key_len
        keys = _rand_bytes(gen, (n, kl), dev).clone()
        space = max(key_space or (first_index + n), 2)
        stride = min((1 << 64) // space, (1 << 63) - 1)
        r = torch.randint(0, stride, (n,), generator=gen, device=dev, dtype=torch.int64)
        head = idx * stride + r  # wraps in int64; the bit pattern is the unsigned value
        # big-endian bytes of head into keys[:, :8]
        shifts = torch.arange(56, -8, -8, device=dev, dtype=torch.int64)
        if kl >= 8 and not random_keys:
            keys[:, :8] = ((head[:, None] >> shifts[None, :]) & 0xFF).to(torch.uint8)  # arithmetic >> ok: & 0xFF
        cols["keys"] = keys.contiguous()
    elif schema.key_kind == A.KEY_U64:
        r = torch.randint(0, 1 << 20, (n,), generator=gen, device=dev, dtype=torch.int64)
        cols["keys"] = ((idx << 20) | r).contiguous().view(torch.uint8).view(n, 8)
    elif schema.key_kind == A.KEY_U32:
        cols["keys"] = idx.to(torch.int32).contiguous().view(torch.uint8).view(n, 4)
    if schema.value_row:
        cols["values"] = _rand_bytes(gen, (n, schema.value_row), dev).contiguous()
    if schema.record_kind == A.REC_DATED:
        cols["phys"] = (1_700_000_000_000 + idx).contiguous()
        cols["logical"] = torch.zeros(n, dtype=torch.int32, device=dev)
        cols["node"] = torch.ones(n, dtype=torch.int64, device=dev)
    if schema.record_kind != A.REC_PLAIN and tombstone_fraction > 0:
        u = torch.rand(n, generator=gen, device=dev)
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
