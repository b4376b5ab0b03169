"""RangeAggregate on the wire, over librsos_hip.so's rh_wire_* codec.

RangeAggregate<K> (rbsr/src/protocol.rs:63-88) is what one rbsr protocol round sends for every
active child range: the range's bounds and the Aggregate computed over it.  The gossip codec
serialises it with bincode 1.3.3 DefaultOptions (varint integers; gossip/src/bincode.rs:65-100),
inside Message::ComparisonItem (tag 0) or ValueComparisonItem (tag 3) (src/replica.rs:184-199).
The byte layout is pinned by tests/wire_format.rs:37-62 (checked in tests/test_wire.py).

`child_ranges_wire` is the GPU producer: the aggregates of consecutive child ranges come from
a GpuFingerprintStore, and the encoded bytes are ready to be packed into datagrams.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _abi as A
from .fingerprint import Aggregate
from .schema import RecordSchema

Key = Union[bytes, int]
COMPARISON_ITEM, VALUE_COMPARISON_ITEM = 0, 3
_FORMS = {"array": A.FORM_ARRAY, "vec": A.FORM_VEC}


@dataclass(frozen=True)
class RangeAggregate:
    """RangeAggregate::new(start, end, aggregate) (rbsr/src/protocol/range_aggregate.rs:28):
    start None = Unbounded, else Included(start); end None = Unbounded, else Excluded(end)."""
    start: Optional[Key]
    end: Optional[Key]
    aggregate: Aggregate


def _key_bytes(schema: RecordSchema, k: Key) -> bytes:
    if schema.key_kind == A.KEY_U32:
        return int(k).to_bytes(4, "little")
    if schema.key_kind == A.KEY_U64:
        return int(k).to_bytes(8, "little")
    b = bytes(k)
    if len(b) != schema.key_row:
        raise ValueError(f"key must be {schema.key_row} bytes")
    return b


def _key_out(schema: RecordSchema, b: bytes) -> Key:
    return int.from_bytes(b, "little") if schema.key_kind in (A.KEY_U32, A.KEY_U64) else b


def _arrays(schema: RecordSchema, items: Sequence[RangeAggregate]):
    r, kl = len(items), schema.key_row
    sk = np.zeros(max(r, 1), np.uint8)
    ek = np.zeros(max(r, 1), np.uint8)
    skeys = np.zeros((max(r, 1), kl), np.uint8)
    ekeys = np.zeros((max(r, 1), kl), np.uint8)
    aggs = (A.Aggregate * max(r, 1))()
    for i, it in enumerate(items):
        if it.start is not None:
            sk[i] = 1
            skeys[i] = np.frombuffer(_key_bytes(schema, it.start), np.uint8)
        if it.end is not None:
            ek[i] = 1
            ekeys[i] = np.frombuffer(_key_bytes(schema, it.end), np.uint8)
        aggs[i].fingerprint[:] = list(it.aggregate.fingerprint.limbs)
        aggs[i].size = it.aggregate.size
    return sk, skeys, ek, ekeys, aggs


def encode(schema: RecordSchema, items: Sequence[RangeAggregate], key_form: str = "array",
           msg_tag: Optional[int] = None) -> bytes:
    s = schema.c()
    sk, skeys, ek, ekeys, aggs = _arrays(schema, items)
    n = C.c_size_t()
    tag = -1 if msg_tag is None else msg_tag
    args = (C.byref(s), _FORMS[key_form], tag, sk.ctypes.data, skeys.ctypes.data, ek.ctypes.data, ekeys.ctypes.data,
            aggs, len(items))
    A.check(A.lib().rh_wire_encode_range_aggregates(*args, None, 0, C.byref(n)), "rh_wire_encode_range_aggregates")
    out = C.create_string_buffer(max(n.value, 1))
    A.check(A.lib().rh_wire_encode_range_aggregates(*args, out, n.value, C.byref(n)),
            "rh_wire_encode_range_aggregates")
    return out.raw[:n.value]


def decode_stream(schema: RecordSchema, data: bytes, max_items: int, key_form: str = "array",
                  msg_tag: Optional[int] = None) -> Tuple[List[RangeAggregate], int]:
    """gossip::bincode::decode_stream for RangeAggregate items: (items, bytes consumed)."""
    s = schema.c()
    kl, cap = schema.key_row, max(max_items, 1)
    sk, ek = np.zeros(cap, np.uint8), np.zeros(cap, np.uint8)
    skeys, ekeys = np.zeros((cap, kl), np.uint8), np.zeros((cap, kl), np.uint8)
    aggs = (A.Aggregate * cap)()
    buf = np.frombuffer(bytes(data) or b"\0", np.uint8)
    r, used = C.c_size_t(), C.c_size_t()
    A.check(A.lib().rh_wire_decode_range_aggregates(C.byref(s), _FORMS[key_form], -1 if msg_tag is None else msg_tag,
                                                    buf.ctypes.data, len(data), max_items, sk.ctypes.data,
                                                    skeys.ctypes.data, ek.ctypes.data, ekeys.ctypes.data, aggs,
                                                    C.byref(r), C.byref(used)), "rh_wire_decode_range_aggregates")
    out = []
    for i in range(r.value):
        out.append(RangeAggregate(_key_out(schema, skeys[i].tobytes()) if sk[i] else None,
                                  _key_out(schema, ekeys[i].tobytes()) if ek[i] else None,
                                  Aggregate.from_c(aggs[i])))
    return out, int(used.value)


def child_ranges_wire(store, cuts: Sequence[Optional[Key]], key_form: str = "array",
                      msg_tag: Optional[int] = COMPARISON_ITEM) -> Tuple[List[RangeAggregate], bytes]:
    """The child ranges [cuts[i], cuts[i+1]) of one SPLIT (rbsr/src/protocol.rs:299-307), each
    with its aggregate from the GPU store, and their wire bytes.  cuts[0] / cuts[-1] may be
    None (Unbounded)."""
    from .store import KeyRange
    items = []
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        agg = store.aggregate(KeyRange(lo, hi, "included", "excluded"))
        items.append(RangeAggregate(lo, hi, agg))
    return items, encode(store.schema, items, key_form, msg_tag)
