"""FingerprintMap: Rsos<K> with host-owned K / V and single-record updates staged into one device
batch (rh_store_stage) -- the logic of the Rust binding's HipFingerprintMap, testable here.

The reference fills through one insert per record under one write lock (src/replica/write.rs:
107-121, :44-45); these inserts must cost host work per record and one device batch, and the
map's root must equal the oracle FingerprintTreeMap's over the same inserts, in order."""
import time

import numpy as np
import pytest


def test_wrong_length_value_is_an_error_not_a_pad(rsos_hip_lib):
    """A value that does not fill the value column exactly is rejected (the Rust binding
    panics); padding or truncating would hash another record (rsos_trait.rs:54-56)."""
    from rsos_hip import RecordSchema
    from rsos_hip.fmap import Entry, encode_row
    s = RecordSchema.dated("bytes16", "bytes64")
    assert encode_row(s, Entry(bytes(64), 1, 2, 3))[0] == bytes(64)
    for bad in (bytes(63), bytes(65), b""):
        with pytest.raises(ValueError):
            encode_row(s, Entry(bad, 1, 2, 3))
    assert encode_row(s, Entry(b"", 1, 2, 3, tombstone=True))[4] == 1
    with pytest.raises(ValueError):
        encode_row(s, Entry(bytes(64), 1, 2, 3, tombstone=True))
    p = RecordSchema.plain("u64", "u64")
    assert encode_row(p, 7)[0] == (7).to_bytes(8, "little")
    with pytest.raises(ValueError):
        encode_row(p, b"\x01" * 7)


@pytest.mark.gpu
def test_million_single_inserts_staged(gpu, oracle_lib):
    """10^6 single-record inserts (2 % of them overwrites, then 1 % deletes) through the staged
    path: seconds, one device batch per question, and the root / sizes / ranks / selects equal
    the oracle FTM's after the same operations in order."""
    from rsos_hip import Entry, FingerprintMap, RecordSchema
    O = oracle_lib
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 1_000_000
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    keys = np.unique(keys.view("V16")).view(np.uint8).reshape(-1, 16)
    rng.shuffle(keys)
    n = len(keys)
    vals = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    fm = FingerprintMap(s)
    kb = [k.tobytes() for k in keys]
    vb = [v.tobytes() for v in vals]
    t0 = time.perf_counter()
    for i in range(n):
        assert fm.insert(kb[i], Entry(vb[i], 1_700_000_000_000 + i, 0, 1)) is None
    ov = rng.choice(n, n // 50, replace=False)
    for i in ov:  # overwrite: a new stamp, the old value returned
        old = fm.insert(kb[i], Entry(vb[i], 1_800_000_000_000 + int(i), 1, 2))
        assert old.phys == 1_700_000_000_000 + int(i)
    dl = rng.choice(n, n // 100, replace=False)
    for i in dl:
        assert fm.delete(kb[i]) is not None
    root = fm.aggregate()  # the one device batch
    elapsed = time.perf_counter() - t0
    assert elapsed < 120, elapsed  # seconds of host work, not 10^6 device round trips
    # the oracle: the final contents in key order (overwrites restamped, deletes gone)
    phys = 1_700_000_000_000 + np.arange(n, dtype=np.uint64)
    logical = np.zeros(n, np.uint32)
    node = np.ones(n, np.uint64)
    phys[ov] = 1_800_000_000_000 + ov.astype(np.uint64)
    logical[ov] = 1
    node[ov] = 2
    live = np.ones(n, bool)
    live[dl] = False
    order = np.argsort(keys[live].view("V16").ravel(), kind="stable")
    sc = O.Schema(s.key_kind, s.key_len, s.value_kind, s.value_len, s.record_kind, 0)
    sel = np.nonzero(live)[0][order]
    recs = O.Records(sc, np.ascontiguousarray(keys[sel]), np.ascontiguousarray(vals[sel]), phys[sel],
                     logical[sel], node[sel], np.zeros(len(sel), np.uint8))
    t = O.FingerprintTreeMap(recs)
    t.fill(0, recs.n)
    fp, size = t.aggregate(None, None)
    assert root.size == size == fm.size() == int(live.sum())
    assert list(root.fingerprint.limbs) == [int(x) for x in fp]
    for r in (0, 1, size // 2, size - 1):
        assert fm.select(r) == keys[sel[r]].tobytes()
        assert fm.rank(fm.select(r)) == r
    print(f"{n} staged inserts + {len(ov)} overwrites + {len(dl)} deletes: {elapsed:.2f} s")
    fm.close()


@pytest.mark.gpu
def test_staged_rows_last_write_wins_and_loads_drop_them(gpu, oracle_lib):
    """A key staged several times keeps its last operation (insert, overwrite, delete, insert
    again); the store's own size / aggregate calls flush first; a load drops staged rows."""
    import ctypes as C
    from rsos_hip import FingerprintMap, GpuFingerprintStore, RecordSchema, _abi as A
    O = oracle_lib
    s = RecordSchema.plain("u64", "u64")
    fm = FingerprintMap(s, host_tier=False, chunk=3)
    for k in range(10):
        fm.insert(k, k * 7)
    fm.insert(4, 99)
    fm.delete(5)
    fm.insert(5, 55)
    fm.delete(6)
    fm.insert(11, 1)
    want = {k: k * 7 for k in range(10)}
    want.update({4: 99, 5: 55, 11: 1})
    del want[6]
    ks = np.array(sorted(want), np.uint64)
    vs = np.array([want[int(k)] for k in ks], np.uint64)
    sc = O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0)
    t = O.FingerprintTreeMap(O.Records(sc, ks.view(np.uint8).reshape(-1, 8), vs.view(np.uint8).reshape(-1, 8)))
    t.fill(0, len(ks))
    fp, size = t.aggregate(None, None)
    agg = fm.aggregate()
    assert agg.size == size == fm.size() and list(agg.fingerprint.limbs) == [int(x) for x in fp]
    # staged rows are visible to the store's own questions (they flush first) ...
    st = GpuFingerprintStore(s)
    cols = A.Columns(C.addressof((C.c_uint64 * 1)(3)), None, None, None, None, C.addressof((C.c_uint64 * 1)(4)))
    assert A.lib().rh_store_stage(st._h, C.byref(cols), (C.c_uint8 * 1)(0), 1) == 0
    assert st.size() == 1
    # ... and a load replaces them
    assert A.lib().rh_store_stage(st._h, C.byref(cols), (C.c_uint8 * 1)(1), 1) == 0
    st.load_bulk({"keys": np.array([8, 9], np.uint64).view(np.uint8).reshape(2, 8),
                  "values": np.array([1, 2], np.uint64).view(np.uint8).reshape(2, 8)})
    assert st.size() == 2
    st.close()
    fm.close()
