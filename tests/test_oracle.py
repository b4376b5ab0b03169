"""CPU tests: the oracle (C restatement + pure-Python restatement) pinned against the
reference's golden vectors and the BLAKE3 specification vectors, and the reference-
faithful FingerprintTreeMap restatement against the fold-of-lift laws the reference tests.

Mirrors: rsos/src/fingerprint/tests.rs, rsos/src/encoding/tests.rs,
rsos/src/fingerprint_tree_map/tests/aggregate.rs:59-78, tests/basic.rs:90-200,
tests/proptest_fingerprint_tree_map/btreemap_oracle.rs:132-231.
"""
import struct

import numpy as np
import pytest

import pyref as P


def limbs(b: bytes):
    return [f"0x{x:016x}" for x in struct.unpack("<4Q", b)]


def to_int(hexlimbs):
    return sum(int(x, 16) << (64 * i) for i, x in enumerate(hexlimbs))


# ---- reference golden vectors ----------------------------------------------------------

def test_golden_element_hash(golden, oracle_lib):
    v = golden["reference"]["vectors"][0]
    enc = bytes.fromhex(v["encoded_hex"])
    assert enc == P.encode(P.U64(50)) + P.encode(P.Str(b"Hello"))
    assert limbs(P.blake3(enc)) == v["limbs"]
    assert limbs(oracle_lib.blake3(enc)) == v["limbs"]


def test_golden_combined_fingerprint(golden, oracle_lib):
    v = golden["reference"]["vectors"][1]
    parts = [oracle_lib.blake3(bytes.fromhex(h)) for h in v["encoded_hex_parts"]]
    assert limbs(P.fp_add(*parts)) == v["limbs"]


def test_golden_entry_fingerprint(golden, oracle_lib):
    v = golden["reference"]["vectors"][2]
    r = v["record"]
    schema = oracle_lib.Schema(oracle_lib.KEY_U32, 4, oracle_lib.VAL_U32, 4, oracle_lib.REC_DATED, 0)
    recs = oracle_lib.Records(schema, np.array([r["key_u32"]], np.uint32).view(np.uint8).reshape(1, 4),
                              np.array([r["value_u32"]], np.uint32).view(np.uint8).reshape(1, 4),
                              np.array([int(r["phys"], 16)], np.uint64), np.array([int(r["logical"], 16)], np.uint32),
                              np.array([int(r["node"], 16)], np.uint64))
    assert recs.encode(0).hex() == v["encoded_hex"]
    assert limbs(recs.lift()[0].tobytes()) == v["limbs"]


def test_carry_borrow_kats(golden):
    for kat in golden["reference"]["carry_borrow"]:
        a, b, out = to_int(kat["a"]), to_int(kat["b"]), to_int(kat["out"])
        got = (a + b) % (1 << 256) if kat["op"] == "add" else (a - b) % (1 << 256)
        assert got == out


def test_encoding_kats(golden):
    enc = {
        "1u32": P.encode(P.U32(1)), "1u64": P.encode(P.U64(1)), "\"ab\"": P.encode(P.Str(b"ab")),
        "None::<u8>": P.encode(P.Opt(None)), "Some(0u8)": P.encode(P.Opt(P.U8(0))),
        "E::A(1) (newtype variant 0)": P.encode(P.Variant(0, P.U32(1))),
        "U::B (unit variant 1)": P.encode(P.Variant(1)),
        "Pair(1u32, 2u32) (tuple struct)": P.encode(P.Seq((P.U32(1), P.U32(2)))),
    }
    for kat in golden["reference"]["encodings"]:
        assert enc[kat["what"]].hex() == kat["hex"], kat["what"]


def test_framing_is_unambiguous():
    # rsos/src/fingerprint/tests.rs:97-107
    assert P.lift(P.Str(b"ab"), P.Str(b"c")) != P.lift(P.Str(b"a"), P.Str(b"bc"))
    assert P.digest(P.Str(b"Hello")) == P.lift(P.Unit(), P.Str(b"Hello"))


# ---- BLAKE3 specification vectors (multi-block / multi-chunk) ---------------------------

def test_blake3_spec_vectors(golden, oracle_lib):
    for v in golden["blake3_spec"]["vectors"]:
        data = bytes(i % 251 for i in range(v["len"]))
        assert oracle_lib.blake3(data).hex() == v["hash"], v["len"]
        assert P.blake3(data).hex() == v["hash"], v["len"]
    assert oracle_lib.blake3(b"abc").hex() == golden["blake3_spec"]["abc"]


def test_c_and_python_restatements_agree(oracle_lib):
    rng = np.random.default_rng(1)
    for n in [0, 1, 55, 56, 64, 65, 119, 120, 121, 1079, 1080, 2047, 2048, 2049, 3100, 8193]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle_lib.blake3(d) == P.blake3(d), n


def test_shape_vectors_reproduce(golden, oracle_lib):
    O = oracle_lib
    for s in golden["shapes"]:
        n = s["n"]
        schema = O.Schema(s["key_kind"], s["key_len"], s["value_kind"], s["value_len"], s["record_kind"], 0)
        keys = np.frombuffer(bytes.fromhex(s["keys"]), np.uint8).reshape(n, s["key_len"])
        vals = np.frombuffer(bytes.fromhex(s["values"]), np.uint8).reshape(n, s["value_len"])
        dated = s["record_kind"] == O.REC_DATED
        recs = O.Records(schema, keys, vals,
                         np.array(s["phys"], np.uint64) if dated else None,
                         np.array(s["logical"], np.uint32) if dated else None,
                         np.array(s["node"], np.uint64) if dated else None,
                         np.array(s["tags"], np.uint8) if s["tags"] is not None else None)
        fps = recs.lift(threads=2)
        assert [f.tobytes().hex() for f in fps] == s["fps"], s["name"]


def test_encoded_vectors_reproduce(golden, oracle_lib):
    blobs = [bytes.fromhex(r["hex"]) for r in golden["encoded"]]
    fps = oracle_lib.lift_encoded(blobs, threads=3)
    assert [f.tobytes().hex() for f in fps] == [r["fp"] for r in golden["encoded"]]


def test_record_lengths_match_survey(oracle_lib):
    """SURVEY.md §8a byte counts: 16B/64B dated 120, projection 100, tombstone 48, 1 KiB 1080."""
    O = oracle_lib
    cases = [((O.KEY_BYTES, 16, O.VAL_BYTES, 64, O.REC_DATED), 0, 120),
             ((O.KEY_BYTES, 16, O.VAL_BYTES, 64, O.REC_PROJECTION), 0, 100),
             ((O.KEY_BYTES, 16, O.VAL_BYTES, 64, O.REC_DATED), 1, 48),
             ((O.KEY_BYTES, 16, O.VAL_BYTES, 1024, O.REC_DATED), 0, 1080),
             ((O.KEY_U64, 8, O.VAL_BYTES, 64, O.REC_PLAIN), 0, 80),
             ((O.KEY_U32, 4, O.VAL_U32, 4, O.REC_PLAIN), 0, 8)]
    for sch, tomb, want in cases:
        schema = O.Schema(*sch, 0)
        kl, vl = sch[1], sch[3]
        recs = O.Records(schema, np.zeros((1, kl), np.uint8), np.zeros((1, vl), np.uint8),
                         np.zeros(1, np.uint64), np.zeros(1, np.uint32), np.zeros(1, np.uint64),
                         np.array([tomb], np.uint8))
        assert len(recs.encode(0)) == want


# ---- FingerprintTreeMap restatement (the CPU baseline) -----------------------------------

def _u64_records(O, n, seed, dup_every=0):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 2**63, n, dtype=np.uint64)
    if dup_every:
        keys[dup_every::dup_every] = keys[: len(keys[dup_every::dup_every])]
    vals = rng.integers(0, 2**63, n, dtype=np.uint64)
    schema = O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0)
    return O.Records(schema, keys.view(np.uint8).reshape(n, 8), vals.view(np.uint8).reshape(n, 8)), keys


def test_ftm_big_test_invariants(oracle_lib):
    """tests/basic.rs:90-200: 1000 random inserts, invariants after each, partition additivity."""
    O = oracle_lib
    recs, keys = _u64_records(O, 1000, 3)
    t = O.FingerprintTreeMap(recs)
    for i in range(1000):
        t.insert(i)
        if i % 97 == 0:
            assert t.check()
    assert t.check()
    assert len(t) == len(set(keys.tolist()))
    root = t.root()
    # fold of lift over the final contents
    fps = recs.lift()
    last = {}
    for i, k in enumerate(keys.tolist()):
        last[k] = i
    s = sum(int.from_bytes(fps[i].tobytes(), "little") for i in last.values()) % (1 << 256)
    assert sum(x << (64 * j) for j, x in enumerate(root[0])) == s
    # partition additivity agg(..mid) + agg(mid..) == agg(..)
    mid = np.uint64(2**62).tobytes()
    a, b = t.aggregate(None, mid), t.aggregate(mid, None)
    tot = (sum(x << (64 * j) for j, x in enumerate(a[0])) + sum(x << (64 * j) for j, x in enumerate(b[0]))) % (1 << 256)
    assert tot == s and a[1] + b[1] == root[1]


def test_ftm_overwrite_is_a_delta(oracle_lib):
    """Duplicate delivery / overwrite keeps the fold single (btreemap_oracle.rs:195-231)."""
    O = oracle_lib
    recs, keys = _u64_records(O, 400, 5, dup_every=4)
    t = O.FingerprintTreeMap(recs)
    t.fill(0, 400)
    assert t.check()
    fps = recs.lift()
    last = {}
    for i, k in enumerate(keys.tolist()):
        last[k] = i
    s = sum(int.from_bytes(fps[i].tobytes(), "little") for i in last.values()) % (1 << 256)
    root = t.root()
    assert root[1] == len(last)
    assert sum(x << (64 * j) for j, x in enumerate(root[0])) == s


def test_ftm_aggregate_brute_force_every_boundary_pair(oracle_lib):
    """rsos/src/fingerprint_tree_map/tests/aggregate.rs:59-78: 100 keys x all (lo, hi)."""
    O = oracle_lib
    n = 100
    keys = np.arange(0, 2 * n, 2, dtype=np.uint64)
    vals = (keys * 7 + 1).astype(np.uint64)
    schema = O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0)
    recs = O.Records(schema, keys.view(np.uint8).reshape(n, 8), vals.view(np.uint8).reshape(n, 8))
    t = O.FingerprintTreeMap(recs)
    t.fill(0, n)
    fps = [int.from_bytes(f.tobytes(), "little") for f in recs.lift()]
    probes = list(range(-1, 2 * n + 1, 3))
    for lo in probes:
        for hi in probes:
            lob = np.uint64(max(lo, 0)).tobytes()
            hib = np.uint64(max(hi, 0)).tobytes()
            fp, size = t.aggregate(lob, hib)
            sel = [i for i in range(n) if max(lo, 0) <= keys[i] < max(hi, 0)]
            assert size == len(sel)
            assert sum(x << (64 * j) for j, x in enumerate(fp)) == sum(fps[i] for i in sel) % (1 << 256)
            assert t.rank(lob) == sum(1 for k in keys if k < max(lo, 0))


@pytest.mark.parametrize("shape", [("u32", "u32", 0), ("u64", "bytes64", 1), ("bytes16", "bytes64", 1),
                                   ("bytes16", "bytes1024", 1), ("bytes16", "bytes1024", 2)])
def test_simd_backends_equal_portable(oracle_lib, shape):
    """The CPU baseline's SIMD BLAKE3 (the crate's SSE4.1 / AVX-512VL row-form compress and the
    16-records-per-vector AVX-512 batch lift) give the portable restatement's fingerprints bit for
    bit, on ragged counts, tombstones and multi-chunk records."""
    import rsos_hip  # noqa: F401  (path setup)
    from rsos_hip import RecordSchema
    from rsos_hip.synth import make_records, to_host
    O = oracle_lib
    k, v, kind = shape
    s = [RecordSchema.plain, RecordSchema.dated, RecordSchema.projection][kind](k, v)
    n = 1001
    h = to_host(make_records(s, n, seed=5, device="cpu", tombstone_fraction=0.1 if kind else 0.0))
    sc = O.Schema(s.key_kind, s.key_len, s.value_kind, s.value_len, s.record_kind, 0)
    recs = O.Records(sc, h["keys"], h.get("values"), h.get("phys"), h.get("logical"), h.get("node"), h.get("tags"))
    want = recs.lift(threads=2)
    try:
        for level in (1, 2):
            got_level = O.set_simd(level)
            assert got_level <= level
            assert np.array_equal(recs.lift(threads=3), want), level
    finally:
        assert O.set_simd(0) == 0
    if O.has_avx512():
        for threads in (1, 5):
            assert np.array_equal(recs.lift_x16(threads=threads), want)
