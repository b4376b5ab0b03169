"""RangeAggregate wire codec: librsos_hip.so's rh_wire_* (host code, no GPU) against the
reference's golden vectors and the oracle restatement (oracle/wire.py).

Golden vectors: tests/wire_format.rs:37-62 (RangeAggregate<u32>), tests/timestamp_wire_format.rs:
59-100 (Timestamp and Entry<Timestamp, u32>, which pin the varint layer the codec shares).
Stream semantics: gossip/src/bincode.rs:79-100 (an end of input ends the stream cleanly).
"""
import random
import struct

import pytest

# tests/wire_format.rs:41-44
GOLDEN_RANGE_AGGREGATE = bytes([
    1, 7, 1, 42, 239, 205, 171, 137, 103, 69, 35, 1, 16, 50, 84, 118, 152, 186, 220, 254, 1, 0,
    0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0, 0, 0, 0, 251, 44, 1,
])
# tests/timestamp_wire_format.rs:63-66 and :83-86 (sample_stamp: 0x0123456789abcdef, 0x11223344,
# 0xfeedfacedeadbeef)
GOLDEN_TIMESTAMP = bytes([
    253, 239, 205, 171, 137, 103, 69, 35, 1, 252, 68, 51, 34, 17, 253, 239, 190, 173, 222, 206,
    250, 237, 254,
])
GOLDEN_ENTRY = GOLDEN_TIMESTAMP + bytes([0, 251, 57, 48])
STAMP = (0x0123456789ABCDEF, 0x11223344, 0xFEEDFACEDEADBEEF)
FP = (0x0123456789ABCDEF, 0xFEDCBA9876543210, 1, 2)


def schema(kind):
    from rsos_hip import RecordSchema
    return {"u32": RecordSchema.plain("u32", "u32"), "u64": RecordSchema.plain("u64", "u32"),
            "b16": RecordSchema.plain("bytes16", "u32"), "b32": RecordSchema.plain("bytes32", "u32")}[kind]


def test_oracle_varint_matches_reference_goldens():
    import wire as W
    assert W.encode_timestamp(*STAMP) == GOLDEN_TIMESTAMP
    assert W.encode_entry_u32(*STAMP, 12345) == GOLDEN_ENTRY
    enc, _ = W.key_codec("u32")
    ra = W.RangeAggregate(7, 42, FP, 300)
    assert W.encode_range_aggregate(ra, enc) == GOLDEN_RANGE_AGGREGATE


def test_codec_golden_range_aggregate(rsos_hip_lib):
    from rsos_hip.fingerprint import Aggregate, Fingerprint
    from rsos_hip import wire
    item = wire.RangeAggregate(7, 42, Aggregate(300, Fingerprint(FP)))
    s = schema("u32")
    assert wire.encode(s, [item]) == GOLDEN_RANGE_AGGREGATE
    back, used = wire.decode_stream(s, GOLDEN_RANGE_AGGREGATE, 16)
    assert back == [item] and used == len(GOLDEN_RANGE_AGGREGATE)
    # the fingerprint is always 32 raw bytes (#382: the worst case for a varint limb encoding)
    big = wire.RangeAggregate(7, 42, Aggregate(300, Fingerprint((2**64 - 1,) * 4)))
    assert len(wire.encode(s, [big])) == len(GOLDEN_RANGE_AGGREGATE)


def _random_items(kind, form, r, rng):
    from rsos_hip.fingerprint import Aggregate, Fingerprint
    from rsos_hip import wire
    import wire as W
    out, ref = [], []
    for _ in range(r):
        def key():
            if kind == "u32":
                return rng.choice([0, 1, 250, 251, 65535, 65536, 2**32 - 1, rng.randrange(2**32)])
            if kind == "u64":
                return rng.choice([0, 250, 2**16, 2**32 - 1, 2**32, 2**64 - 1, rng.randrange(2**64)])
            return bytes(rng.randrange(256) for _ in range(16 if kind == "b16" else 32))
        start = None if rng.random() < 0.2 else key()
        end = None if rng.random() < 0.2 else key()
        fp = tuple(rng.randrange(2**64) for _ in range(4))
        size = rng.choice([0, 1, 250, 251, 300, 65536, 2**32, rng.randrange(2**64)])
        out.append(wire.RangeAggregate(start, end, Aggregate(size, Fingerprint(fp))))
        ref.append(W.RangeAggregate(start, end, fp, size))
    return out, ref


@pytest.mark.parametrize("kind,form", [("u32", "array"), ("u64", "array"), ("b16", "array"), ("b16", "vec"),
                                       ("b32", "array"), ("b32", "vec")])
@pytest.mark.parametrize("msg_tag", [None, 0, 3])
def test_codec_matches_oracle(rsos_hip_lib, kind, form, msg_tag):
    from rsos_hip import wire
    import wire as W
    rng = random.Random(hash((kind, form, msg_tag)) & 0xFFFF)
    items, ref = _random_items(kind, form, 40, rng)
    s = schema(kind)
    okind = kind if kind in ("u32", "u64") else form
    enc, dec = W.key_codec(okind, s.key_row)
    want = b"".join(W.encode_range_aggregate(x, enc, msg_tag) for x in ref)
    got = wire.encode(s, items, form, msg_tag)
    assert got == want
    back, used = wire.decode_stream(s, got, 100, form, msg_tag)
    assert back == items and used == len(got)
    # a truncated last item ends the stream cleanly (gossip/src/bincode.rs:90-95)
    cut = got[:-3]
    back, used = wire.decode_stream(s, cut, 100, form, msg_tag)
    oback, oused = W.decode_stream(cut, dec, 100, msg_tag)
    assert len(back) == len(oback) == len(items) - 1 and used == oused
    # max_items caps the count
    back, used = wire.decode_stream(s, got, 5, form, msg_tag)
    assert back == items[:5]


def test_codec_rejects_malformed(rsos_hip_lib):
    from rsos_hip import wire, _abi as A
    s = schema("u32")
    bad_variant = bytes([2]) + GOLDEN_RANGE_AGGREGATE[1:]
    with pytest.raises(A.RsosHipError) as e:
        wire.decode_stream(s, bad_variant, 4)
    assert e.value.code == A.ERR_DATA and "variant" in str(e.value)
    bad_marker = bytes([1, 254]) + GOLDEN_RANGE_AGGREGATE[2:]
    with pytest.raises(A.RsosHipError):
        wire.decode_stream(s, bad_marker, 4)
    with pytest.raises(A.RsosHipError):  # a u32 key wider than u32
        wire.decode_stream(s, bytes([1, 253]) + struct.pack("<Q", 2**40) + GOLDEN_RANGE_AGGREGATE[2:], 4)
    with pytest.raises(A.RsosHipError):  # wrong Message tag
        wire.decode_stream(s, bytes([1]) + GOLDEN_RANGE_AGGREGATE, 4, msg_tag=0)
    sv = schema("b16")
    with pytest.raises(A.RsosHipError):  # Vec key of the wrong length
        wire.decode_stream(sv, bytes([1, 15]) + bytes(15) + bytes([0]) + bytes(32) + bytes([0]), 4, "vec")
    assert wire.decode_stream(s, b"", 4) == ([], 0)


def test_codec_encode_capacity(rsos_hip_lib):
    import ctypes as C
    from rsos_hip import _abi as A
    s = schema("u32").c()
    n = C.c_size_t()
    k = (C.c_uint8 * 1)(1)
    keys = (C.c_uint32 * 1)(7)
    agg = (A.Aggregate * 1)()
    rc = A.lib().rh_wire_encode_range_aggregates(C.byref(s), 0, -1, k, keys, k, keys, agg, 1, None, 0, C.byref(n))
    assert rc == 0 and n.value == 1 + 1 + 1 + 1 + 32 + 1
    small = C.create_string_buffer(4)
    rc = A.lib().rh_wire_encode_range_aggregates(C.byref(s), 0, -1, k, keys, k, keys, agg, 1, small, 4, C.byref(n))
    assert rc == A.ERR_ARG


@pytest.mark.gpu
def test_child_ranges_from_gpu_store(gpu):
    """A SPLIT's child ranges (rbsr/src/protocol.rs:299-307) aggregated on the GPU store and
    encoded: decoding gives back the same bounds and aggregates, and the children partition
    the parent (Aggregate's Add, rsos/src/aggregate.rs:79-89)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, wire
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records
    s = RecordSchema.dated("bytes16", "bytes64")
    store = GpuFingerprintStore(s)
    store.load_bulk_device(make_records(s, 50000, seed=8))
    keys = [k for k, _ in store.enumerate()]
    cuts = [None] + [keys[i] for i in range(3125, 50000, 3125)] + [None]
    items, data = wire.child_ranges_wire(store, cuts, msg_tag=wire.COMPARISON_ITEM)
    back, used = wire.decode_stream(s, data, 64, msg_tag=wire.COMPARISON_ITEM)
    assert back == items and used == len(data) and len(items) == 16
    total = items[0].aggregate
    for it in items[1:]:
        total = total + it.aggregate
    assert total == store.aggregate() and all(it.aggregate.size == 3125 for it in items)
    assert items[3].aggregate == store.aggregate(KeyRange(cuts[3], cuts[4]))
