"""The encoded store (rh_estore_*) and EncodedFingerprintMap: Rsos<K> for any serde K / V.

CPU: the product's canonical encoder (rsos_hip.encoding) against the oracle's independent typed
restatement (oracle/pyref.py) and the reference's golden inputs.
GPU: a String -> String map (ragged lengths, values past one 1 KiB chunk), staged inserts /
overwrites / deletes, checked by a fold of the oracle's lift over the expected contents in the
key type's order (the reference's btreemap_oracle.rs:132-162 strategy) on random key ranges, plus
rank / select / size; the reference's golden lift(&50u64, &"Hello") through the map's root."""
import numpy as np
import pytest

import pyref as P

M256 = 1 << 256


def test_encoder_matches_oracle_restatement():
    from rsos_hip.encoding import encode
    from rsos_hip.fmap import Entry
    rng = np.random.default_rng(1)
    for _ in range(300):
        s = "".join(chr(int(c)) for c in rng.integers(32, 0x2FFF, rng.integers(0, 40)))
        b = rng.bytes(int(rng.integers(0, 3000)))
        u = int(rng.integers(0, 2**63))
        assert encode("str", s) == P.encode(P.Str(s.encode()))
        assert encode("bytes", b) == P.encode(P.Str(b)) == encode(("vec", "u8"), b)
        assert encode("u64", u) == P.encode(P.U64(u))
        assert encode(("array", "u8", 16), b[:16].ljust(16, b"\0")) == P.encode(P.Seq(tuple(P.U8(x) for x in b[:16].ljust(16, b"\0"))))
        e = Entry(s, u, int(rng.integers(0, 2**32)), u ^ 7)
        assert encode(("entry", "str"), e) == P.encode(P.entry(P.timestamp(e.phys, e.logical, e.node),
                                                              P.present(P.Str(s.encode()))))
        t = Entry(b"", u, 3, 9, tombstone=True)
        assert encode(("entry", "bytes"), t) == P.encode(P.entry(P.timestamp(u, 3, 9), P.TOMBSTONE))
        assert encode(("state", "str"), e) == P.encode(P.present(P.Str(s.encode())))
        assert encode(("option", "u32"), None) == b"\0" and encode(("option", "u32"), 5) == b"\1\5\0\0\0"
        assert encode(("tuple", "u32", "str"), (7, s)) == P.encode(P.Seq((P.U32(7), P.Str(s.encode()))))


def _oracle_root(O, recs):
    """Σ oracle lift over records (bytes) mod 2^256"""
    if not recs:
        return 0
    fps = O.lift_encoded(recs, threads=8)
    return sum(int.from_bytes(f.tobytes(), "little") for f in fps) % M256


@pytest.mark.gpu
def test_string_map_against_fold_of_oracle_lift(gpu, oracle_lib):
    from rsos_hip.emap import EncodedFingerprintMap
    from rsos_hip.store import KeyRange
    O = oracle_lib
    rng = np.random.default_rng(7)

    def word(lo, hi):
        return "".join(chr(int(c)) for c in rng.integers(0x20, 0x7F, int(rng.integers(lo, hi))))

    def lift_rec(k, v):  # the oracle's own encoding of (String, String)
        return P.encode(P.Str(k.encode())) + P.encode(P.Str(v.encode()))

    for tier in (False, True):
        m = EncodedFingerprintMap("str", "str", host_tier=tier)
        want = {}
        seed = {word(0, 30): word(0, 2600) for _ in range(3000)}
        m.load_bulk(seed.items())
        want.update(seed)
        for step in range(4):
            keys = list(want)
            for _ in range(700):
                r = rng.random()
                if r < 0.5:  # new key (some multi-chunk values)
                    k, v = word(0, 30), word(0, 3100 if rng.random() < 0.1 else 200)
                    assert m.insert(k, v) == want.get(k)
                    want[k] = v
                elif r < 0.8:  # overwrite
                    k = keys[int(rng.integers(len(keys)))]
                    v = word(0, 100)
                    assert m.insert(k, v) == want.get(k)
                    want[k] = v
                else:  # delete (sometimes of a key already gone)
                    k = keys[int(rng.integers(len(keys)))]
                    assert m.delete(k) == want.pop(k, None)
            order = sorted(want)  # String's Ord: UTF-8 byte order = code point order
            assert m.size() == len(order)
            assert m.root().size == len(order)
            assert m.root().fingerprint.to_int() == _oracle_root(O, [lift_rec(k, want[k]) for k in order])
            for _ in range(40):
                a, b = sorted(rng.integers(0, len(order), 2))
                lo, hi = order[a], order[b]
                rg = KeyRange(lo, hi, "included", "excluded")
                agg = m.aggregate(rg)
                exp = order[a:b]
                assert agg.size == len(exp)
                assert agg.fingerprint.to_int() == _oracle_root(O, [lift_rec(k, want[k]) for k in exp])
            for r in (0, len(order) // 3, len(order) - 1):
                assert m.select(r) == order[r] and m.rank(order[r]) == r
            assert m.rank("\x7f" * 40) == len(order)
            assert [k for k, _ in m.enumerate(KeyRange(order[5], order[9]))] == order[5:9]
        m.close()


@pytest.mark.gpu
def test_encoded_map_reference_golden(gpu, golden):
    """lift(&50u64, &"Hello") and the 3-element sum (rsos/src/fingerprint/tests.rs:68-93) as the
    roots of FingerprintTreeMap<u64, &str>-shaped encoded maps."""
    from rsos_hip.emap import EncodedFingerprintMap
    v0, v1 = golden["reference"]["vectors"][0], golden["reference"]["vectors"][1]
    m = EncodedFingerprintMap("u64", "str")
    m.insert(50, "Hello")
    assert [f"0x{x:016x}" for x in m.root().fingerprint.limbs] == v0["limbs"]
    m.insert(25, "World!")
    m.insert(75, "Everyone!")
    assert [f"0x{x:016x}" for x in m.root().fingerprint.limbs] == v1["limbs"]
    assert m.select(0) == 25 and m.size() == 3
    m.close()


@pytest.mark.gpu
def test_estore_rejects_bad_batches_unchanged(gpu):
    import ctypes as C
    from rsos_hip import _abi as A
    from rsos_hip.emap import EncodedFingerprintMap
    m = EncodedFingerprintMap("u64", "u64", host_tier=False)
    m.load_bulk([(k, k * 3) for k in range(100)])
    root = m.root()
    L = A.lib()
    pos = np.array([5, 3], np.uint64)  # not sorted
    kinds = np.array([1, 1], np.uint8)
    data = np.zeros(32, np.uint8)
    offs = np.array([0, 16, 32], np.uint64)
    assert L.rh_estore_apply(m._h, pos.ctypes.data, kinds.ctypes.data, 2, data.ctypes.data, offs.ctypes.data, 2) == A.ERR_ARG
    pos = np.array([100], np.uint64)  # overwrite past the end
    assert L.rh_estore_apply(m._h, pos.ctypes.data, kinds.ctypes.data, 1, data.ctypes.data, offs.ctypes.data, 1) == A.ERR_ARG
    pos = np.array([4, 4], np.uint64)  # two overwrites of one row
    assert L.rh_estore_apply(m._h, pos.ctypes.data, kinds.ctypes.data, 2, data.ctypes.data, offs.ctypes.data, 2) == A.ERR_ARG
    assert m.root() == root
    m.close()


@pytest.mark.gpu
def test_inherent_surface_with_mut_retain_entry(gpu, oracle_lib):
    """The FingerprintTreeMap methods the facade calls beyond Rsos (with_mut, retain, entry's
    or_insert, contains_key, range, first / last_key_value, position): every edit re-lifts the
    record through the staged batch, so the root always equals the fold of the oracle's lift
    over the map's current contents."""
    from rsos_hip.emap import EncodedFingerprintMap
    from rsos_hip.store import KeyRange
    O = oracle_lib
    m = EncodedFingerprintMap("str", "u64")
    for i in range(500):
        m.insert(f"k{i:04d}", i)

    def check():
        items = sorted(m._vals.items())
        recs = [P.encode(P.Str(k.encode())) + P.encode(P.U64(v)) for k, v in items]
        assert m.root().fingerprint.to_int() == _oracle_root(O, recs)
        assert m.size() == len(items)

    check()
    assert m.with_mut("k0007", lambda v: (v, v + 1000)) == 7 and m.get("k0007") == 1007
    assert m.with_mut("nope", lambda v: (v, 1)) is None and not m.contains_key("nope")
    check()
    m.retain(lambda k, v: v % 3 != 0)
    assert not m.contains_key("k0003") and m.contains_key("k0004")
    check()
    assert m.or_insert("k0004", 99) == 4 and m.or_insert("zzz", 99) == 99
    check()
    assert m.first_key_value() == ("k0001", 1) and m.last_key_value() == ("zzz", 99)
    assert m.position("k0002") == 1 and m.position("k0003") is None
    assert [k for k, _ in m.range(KeyRange("k0010", "k0016"))] == ["k0010", "k0011", "k0013", "k0014"]
    assert m.remove("k0010") == 10 and m.remove("k0010") is None
    check()
    m.close()


@pytest.mark.gpu
def test_fixed_length_records_take_fixed_kernel(gpu, oracle_lib):
    """A map whose records all encode to one length -- u64 keys with Entry<Timestamp, Vec<u8>> values
    of 64 bytes, 104 B each, the shape the fixed-length kernels (k_lift_fixed_ct) take -- loaded and
    updated through the encoded store: the root and random rank-range aggregates equal a fold of the
    oracle's lift, with the host tier on and off; a batch mixing lengths (a tombstone, 32 B) takes
    the offsets kernel and stays equal too."""
    from rsos_hip.emap import EncodedFingerprintMap
    from rsos_hip.fmap import Entry
    O = oracle_lib
    rng = np.random.default_rng(11)

    def rec(k, e):
        return P.encode(P.U64(k)) + (P.encode(P.entry(P.timestamp(e.phys, e.logical, e.node), P.TOMBSTONE))
                                     if e.tombstone else
                                     P.encode(P.entry(P.timestamp(e.phys, e.logical, e.node), P.present(P.Str(e.value)))))

    for tier in (False, True):
        m = EncodedFingerprintMap("u64", ("entry", "bytes"), host_tier=tier)
        want = {int(k): Entry(rng.bytes(64), int(k) + 5, 0, 1) for k in rng.integers(0, 2**62, 5_000)}
        m.load_bulk(want.items())
        for step in range(3):
            for _ in range(400):
                k = int(rng.integers(0, 2**62))
                e = Entry(rng.bytes(64), k, step, 2, tombstone=(step == 2 and rng.random() < 0.3))
                m.insert(k, e)
                want[k] = e
            keys = sorted(want)
            recs = [rec(k, want[k]) for k in keys]
            assert m.root().fingerprint.to_int() == _oracle_root(O, recs) and m.size() == len(keys)
            fps = O.lift_encoded(recs, threads=8)
            for _ in range(20):
                lo = int(rng.integers(0, len(keys)))
                hi = int(rng.integers(lo, len(keys) + 1))
                a = m.aggregates_ranks([lo], [hi])[0]
                assert a.size == hi - lo
                assert a.fingerprint.to_int() == sum(int.from_bytes(f.tobytes(), "little") for f in fps[lo:hi]) % M256
        m.close()
