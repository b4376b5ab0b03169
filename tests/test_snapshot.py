"""Snapshot reload: the RCNL v1 file (src/snapshot.rs:30-98) decoded on the GPU and replayed
into the dated map and its projection (src/replicated_map/persistence.rs:108-143,
src/replica/write.rs:107-121).

CPU tests: the header checks of rh_snapshot_header against src/snapshot.rs's own tests (short
file, legacy header-less file, unknown version), the oracle's encode / decode round trip
(persisted_state_bincode_roundtrip, src/snapshot.rs:243-249), and the host-side tail decoder.
GPU tests: decoded columns equal the columns the file was written from; both stores equal the
oracle's lift + FingerprintTreeMap of the replayed entries (including repeated keys: the last
entry wins), through host and device bytes; corrupt files are rejected as InvalidData.
"""
import ipaddress

import numpy as np
import pytest

import snapshot as OS  # oracle/snapshot.py

SHAPES = {  # name -> (key, value, oracle key kind, key form)
    "b16_b64": ("bytes16", "bytes64", "array", "array"),
    "b16v_b64": ("bytes16", "bytes64", "vec", "vec"),
    "u64_u64": ("u64", "u64", "u64", "array"),
    "u32_u32": ("u32", "u32", "u32", "array"),
    "b16_b1024": ("bytes16", "bytes1024", "array", "array"),
    "b32_b64": ("bytes32", "bytes64", "array", "array"),
}


def make_cols(key, value, n, seed, tomb=0.0, shuffle=False, dup=0.0):
    """numpy columns of n entries sorted by key (unless shuffled), unique keys unless dup > 0."""
    rng = np.random.default_rng(seed)
    if key == "u32":
        k = np.unique(rng.integers(0, 2**32, n + n // 8 + 8, dtype=np.uint64))[:n]
        k = k.astype(np.uint32).view(np.uint8).reshape(n, 4)
    elif key == "u64":
        k = (np.arange(n, dtype=np.uint64) * np.uint64(1 << 40) + rng.integers(0, 1 << 40, n, dtype=np.uint64)
             ).view(np.uint8).reshape(n, 8)
    else:
        kl = int(key[5:])
        k = rng.integers(0, 256, (n, kl), dtype=np.uint8)
        k = k[np.lexsort(k.T[::-1])]
    vl = {"u32": 4, "u64": 8}.get(value, int(value[5:]) if value.startswith("bytes") else 0)
    v = rng.integers(0, 256, (n, vl), dtype=np.uint8)
    tags = (rng.random(n) < tomb).astype(np.uint8)
    v[tags == 1] = 0
    cols = {"keys": np.ascontiguousarray(k), "values": v, "tags": tags,
            "phys": (1_700_000_000_000 + rng.integers(0, 1 << 30, n)).astype(np.uint64),
            "logical": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
            "node": rng.integers(0, 2**63, n, dtype=np.uint64)}
    if dup and n > 1:
        src = rng.integers(0, n, int(n * dup))
        dst = rng.integers(0, n, int(n * dup))
        cols["keys"][dst] = cols["keys"][src]
    if shuffle:
        perm = rng.permutation(n)
        cols = {c: np.ascontiguousarray(a[perm]) for c, a in cols.items()}
    return cols


def encode(shape, cols, members=(), acks=None, **kw):
    key, value, okind, _ = SHAPES[shape]
    vkind = {"u32": "u32", "u64": "u64"}.get(value, "bytes")
    return OS.encode_snapshot(cols["keys"], cols["phys"], cols["logical"], cols["node"], cols["tags"],
                              cols["values"], okind, vkind, members, acks, **kw)


# ---- CPU ----------------------------------------------------------------------------------------

def test_header_checks(rsos_hip_lib):
    """src/snapshot.rs: headerless_legacy_snapshot_is_rejected, unknown_format_version_is_rejected,
    truncated-below-header; all io::ErrorKind::InvalidData."""
    from rsos_hip import _abi as A
    from rsos_hip.snapshot import read_header
    good = encode("u32_u32", make_cols("u32", "u32", 3, 1))
    assert read_header(good) == 3
    for data, needle in [(good[:5], "shorter than the 8-byte format header"),
                         (good[8:], "magic"),
                         (good[:4] + (2).to_bytes(4, "little") + good[8:], "format version 2"),
                         (good[:12], "truncated")]:
        with pytest.raises(A.RsosHipError) as e:
            read_header(data)
        assert e.value.code == A.ERR_DATA and needle in str(e.value)
        with pytest.raises(ValueError):
            OS.decode_snapshot(data, "u32", 4, "u32", 4)


@pytest.mark.parametrize("shape", ["b16_b64", "b16v_b64", "u32_u32"])
def test_oracle_round_trip(shape):
    key, value, okind, _ = SHAPES[shape]
    cols = make_cols(key, value, 300, 7, tomb=0.3)
    members = ["10.0.0.1", "::1", "192.168.1.20"]
    acks = {cols["keys"][5].tobytes(): {ipaddress.ip_address("10.0.0.1"): 77},
            cols["keys"][9].tobytes(): {ipaddress.ip_address("::1"): 2**40, ipaddress.ip_address("10.0.0.2"): 1}}
    data = encode(shape, cols, members, acks)
    vkind = {"u32": "u32", "u64": "u64"}.get(value, "bytes")
    got, mem, ak, end = OS.decode_snapshot(data, okind, cols["keys"].shape[1], vkind, cols["values"].shape[1])
    for c in cols:
        assert np.array_equal(got[c], cols[c]), c
    assert mem == [ipaddress.ip_address(m) for m in members] and ak == acks


def test_host_tail_decoder(rsos_hip_lib):
    from rsos_hip import RecordSchema
    from rsos_hip.snapshot import decode_tail
    cols = make_cols("bytes16", "bytes64", 50, 3, tomb=0.5)
    members = ["10.1.2.3", "fe80::1"]
    acks = {cols["keys"][1].tobytes(): {ipaddress.ip_address("10.1.2.3"): 5}}
    for shape, form in [("b16_b64", "array"), ("b16v_b64", "vec")]:
        data = encode(shape, cols, members, acks)
        _, mem, ak, end = OS.decode_snapshot(data, SHAPES[shape][2], 16, "bytes", 64)
        m2, a2 = decode_tail(data, end, RecordSchema.dated("bytes16", "bytes64"), form)
        assert m2 == mem and a2 == ak


# ---- GPU ----------------------------------------------------------------------------------------

def _schemas(shape):
    from rsos_hip import RecordSchema
    key, value, _, form = SHAPES[shape]
    return RecordSchema.dated(key, value), RecordSchema.projection(key, value), form


def _oracle_lift(O, schema, cols, rows):
    sch = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
    h = {c: np.ascontiguousarray(a[rows]) for c, a in cols.items()}
    dated = schema.record_kind == O.REC_DATED
    return O.Records(sch, h["keys"], h["values"] if schema.value_row else None,
                     h["phys"] if dated else None, h["logical"] if dated else None, h["node"] if dated else None,
                     h["tags"]).lift(threads=8)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("n,tomb", [(0, 0.0), (1, 0.0), (1, 1.0), (777, 0.25), (20000, 0.1), (5000, 1.0)])
def test_decode_matches_source(gpu, shape, n, tomb):
    import torch
    from rsos_hip.snapshot import decode_entries_device
    key, value, okind, form = SHAPES[shape]
    if value == "bytes1024" and n > 5000:
        n = 3000
    cols = make_cols(key, value, n, 11 + n, tomb=tomb)
    data = encode(shape, cols, ["10.0.0.9"], {})
    dev = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    d, _, _ = _schemas(shape)
    got, info = decode_entries_device(d, dev, form)
    assert info.entries == n and info.tombstones == int(cols["tags"].sum())
    vkind = {"u32": "u32", "u64": "u64"}.get(value, "bytes")
    if n <= 1000:
        _, _, _, end = OS.decode_snapshot(data, okind, cols["keys"].shape[1], vkind, cols["values"].shape[1])
    else:  # entries end where the tail (u64 member count ...) starts
        end = len(data) - (8 + 8) - (4 + 4)
    assert info.entries_end == end
    host = {c: t.cpu().numpy() for c, t in got.items()}
    assert np.array_equal(host["keys"], cols["keys"])
    assert np.array_equal(host["values"], cols["values"])
    assert np.array_equal(host["tags"], cols["tags"])
    assert np.array_equal(host["phys"].view(np.uint64), cols["phys"])
    assert np.array_equal(host["logical"].view(np.uint32), cols["logical"])
    assert np.array_equal(host["node"].view(np.uint64), cols["node"])


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["b16_b64", "b16v_b64", "u64_u64", "u32_u32", "b16_b1024"])
@pytest.mark.parametrize("order", ["sorted", "shuffled", "repeats"])
def test_reload_matches_oracle(gpu, oracle_lib, shape, order):
    """Both stores after reload == the oracle's lifts of the replayed entries, in key order,
    and FingerprintTreeMap's root over the same inserts."""
    import torch
    from rsos_hip import GpuFingerprintStore
    from rsos_hip.snapshot import load_snapshot
    O = oracle_lib
    key, value, okind, form = SHAPES[shape]
    n = 2000 if value == "bytes1024" else 30000
    cols = make_cols(key, value, n, 5, tomb=0.2, shuffle=order != "sorted", dup=0.05 if order == "repeats" else 0)
    data = encode(shape, cols, ["10.0.0.1"], {})
    sd, sp, _ = _schemas(shape)
    dated, proj = GpuFingerprintStore(sd), GpuFingerprintStore(sp)
    via_device = order == "shuffled"
    src = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda() if via_device else data
    info = load_snapshot(src, dated, proj, form)
    rows = OS.last_wins(cols, int_keys=key in ("u32", "u64"))
    assert info.entries == n and info.keys == len(rows) == dated.size() == proj.size()
    for store, schema in [(dated, sd), (proj, sp)]:
        want = _oracle_lift(O, schema, cols, rows)
        assert np.array_equal(store.fingerprints(), want), schema
        ks = np.zeros((len(rows), schema.key_row), np.uint8)
        assert np.array_equal(np.stack([np.frombuffer(k if isinstance(k, bytes) else
                                                       int(k).to_bytes(schema.key_row, "little"), np.uint8)
                                        for k, _ in store.enumerate()]), cols["keys"][rows])
    # FingerprintTreeMap over the inserts in file order (overwrites included)
    sch = O.Schema(sd.key_kind, sd.key_len, sd.value_kind, sd.value_len, sd.record_kind, 0)
    recs = O.Records(sch, cols["keys"], cols["values"], cols["phys"], cols["logical"], cols["node"], cols["tags"])
    ftm = O.FingerprintTreeMap(recs)
    ftm.fill(0, n)
    fp, size = ftm.root()
    agg = dated.aggregate()
    assert size == agg.size and tuple(fp) == agg.fingerprint.limbs


@pytest.mark.gpu
def test_reload_rejects_corrupt_files(gpu):
    from rsos_hip import GpuFingerprintStore, _abi as A
    from rsos_hip.snapshot import load_snapshot
    cols = make_cols("bytes16", "bytes64", 5000, 9, tomb=0.3)
    data = bytearray(encode("b16_b64", cols))
    sd, sp, _ = _schemas("b16_b64")
    dated = GpuFingerprintStore(sd)
    # a State variant of 7 in the middle of the entries
    bad = bytearray(data)
    off = 16
    for i in range(2500):
        off += 40 if cols["tags"][i] else 112
    bad[off + 36] = 7
    cases = [(bytes(bad), "entries parse"), (bytes(data[: len(data) // 2]), "entries"),
             (bytes(data[:8]) + (10**9).to_bytes(8, "little") + bytes(data[16:]), "exceeds"),
             (bytes(data[:4]) + (3).to_bytes(4, "little") + bytes(data[8:]), "format version 3")]
    for blob, needle in cases:
        with pytest.raises(A.RsosHipError) as e:
            load_snapshot(blob, dated, None, "array")
        assert e.value.code == A.ERR_DATA and needle in str(e.value), str(e.value)
    # the store is usable afterwards
    info = load_snapshot(bytes(data), dated, None, "array")
    assert info.keys == 5000 == dated.size()


@pytest.mark.gpu
def test_reload_full_size_properties(gpu):
    """1M entries (16 B / 64 B dated, 10 % tombstones): decoded columns equal the source, and
    the root aggregate equals the sum of the GPU lifts of the source columns."""
    import torch
    from rsos_hip import GpuFingerprintStore, lift_records
    from rsos_hip.snapshot import load_snapshot, decode_entries_device
    from rsos_hip.synth import make_records, to_host
    sd, sp, _ = _schemas("b16_b64")
    n = 1_000_000
    src = make_records(sd, n, seed=3, tombstone_fraction=0.1)
    h = to_host(src)
    h["values"][h["tags"] == 1] = 0
    data = OS.encode_snapshot(h["keys"], h["phys"], h["logical"], h["node"], h["tags"], h["values"], "array", "bytes")
    dev = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).cuda()
    got, info = decode_entries_device(sd, dev, "array")
    for c in ("keys", "values", "tags", "phys", "logical", "node"):
        want = torch.from_numpy(np.ascontiguousarray(h[c]).view({"phys": np.int64, "node": np.int64,
                                                                  "logical": np.int32}.get(c, h[c].dtype))).cuda()
        assert torch.equal(got[c].view(want.dtype).reshape(want.shape), want), c
    dated, proj = GpuFingerprintStore(sd), GpuFingerprintStore(sp)
    info = load_snapshot(dev, dated, proj, "array")
    assert info.keys == n and info.tombstones == int(h["tags"].sum())
    fps, _ = lift_records(sd, src, block_sums=False)
    limbs = fps.view(torch.int64).view(n, 4).cpu().numpy().view(np.uint64)
    total = sum(int(x) << (64 * i) for i, x in enumerate([int(limbs[:, j].astype(object).sum()) for j in range(4)]))
    total %= 1 << 256
    agg = dated.aggregate()
    assert agg.size == n and agg.fingerprint.to_int() == total


@pytest.mark.parametrize("kv,form", [(("bytes16", "bytes64"), "array"), (("bytes16", "bytes64"), "vec"),
                                     (("u32", "u32"), "array"), (("u64", "u64"), "array")])
def test_device_snapshot_builder_matches_oracle(rsos_hip_lib, kv, form):
    """synth.make_snapshot (the bench's input builder, torch) writes the oracle's bytes."""
    from rsos_hip import RecordSchema
    from rsos_hip.synth import make_records, make_snapshot, to_host
    s = RecordSchema.dated(*kv)
    c = make_records(s, 3000, seed=1, device="cpu", tombstone_fraction=0.3)
    got = make_snapshot(c, s, form, chunk=1000).numpy().tobytes()
    h = to_host(c)
    ints = {"u32": "u32", "u64": "u64"}
    want = OS.encode_snapshot(h["keys"], h["phys"], h["logical"], h["node"], h["tags"], h["values"],
                              ints.get(kv[0], form), ints.get(kv[1], "bytes"))
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("point", ["snapshot.load_begin", "snapshot.load_finish"])
def test_reload_failure_leaves_both_stores_empty(gpu, point):
    """A reload that fails after the first store has begun loading (an injected allocation
    failure in the projection's load_begin, or in the dated store's load_finish) leaves BOTH
    stores empty and consistent -- size 0 and the zero root -- never the new size beside the old
    root; the stores reload normally afterwards."""
    import torch
    from rsos_hip import GpuFingerprintStore, _abi as A
    from rsos_hip.snapshot import load_snapshot
    from rsos_hip.synth import make_records, make_snapshot
    sd, sp, _ = _schemas("b16_b64")
    old = make_records(sd, 3000, seed=11)
    new = make_records(sd, 5000, seed=12, tombstone_fraction=0.1)
    dated, proj = GpuFingerprintStore(sd), GpuFingerprintStore(sp)
    load_snapshot(make_snapshot(old, sd), dated, proj)
    assert dated.size() == proj.size() == 3000
    blob = make_snapshot(new, sd)
    A.lib().rh_debug_fail_point(point.encode())
    with pytest.raises(A.RsosHipError) as e:
        load_snapshot(blob, dated, proj)
    assert e.value.code == A.ERR_OOM and "injected" in str(e.value)
    for st in (dated, proj):
        agg = st.aggregate()
        assert st.size() == 0 and agg.size == 0 and agg.fingerprint.to_int() == 0
    info = load_snapshot(blob, dated, proj)
    assert info.keys == 5000 == dated.size() == proj.size()
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["b16_b64", "u32_u32", "b32_b64", "b16v_b64"])
@pytest.mark.parametrize("which", ["dated", "projection"])
def test_reload_into_one_store(gpu, oracle_lib, shape, which):
    """The fused pass for a single store (dated-only and projection-only reloads; candidate-word
    strides 2 (g = 8, 24) and 1 (u32 / u32: g = 4)): fingerprints, keys, root, ranks and sampled
    searches equal the oracle's."""
    from rsos_hip import GpuFingerprintStore
    from rsos_hip.snapshot import load_snapshot
    O = oracle_lib
    key, value, okind, form = SHAPES[shape]
    n = 25_000
    cols = make_cols(key, value, n, 17, tomb=0.15)
    data = encode(shape, cols, [], {})
    sd, sp, _ = _schemas(shape)
    schema = sd if which == "dated" else sp
    st = GpuFingerprintStore(schema)
    info = load_snapshot(data, st if which == "dated" else None, st if which == "projection" else None, form)
    assert info.entries == info.keys == n == st.size() and info.tombstones == int(cols["tags"].sum())
    rows = np.arange(n)
    want = _oracle_lift(O, schema, cols, rows)
    assert np.array_equal(st.fingerprints(), want)
    # ranks through the search samples the fused pass wrote, for present keys and their successors
    probe = np.linspace(0, n - 1, 97).astype(np.int64)
    assert np.array_equal(st.ranks(np.ascontiguousarray(cols["keys"][probe])), probe)
    limbs = want.view(np.uint64).reshape(n, 4)
    total = sum(int(limbs[:, j].astype(object).sum()) << (64 * j) for j in range(4)) % (1 << 256)
    assert st.aggregate().fingerprint.to_int() == total


@pytest.mark.gpu
def test_corrupt_reload_leaves_stores_unchanged(gpu):
    """A corrupt file fails the fused reload before either store changes (Replica::load_snapshot
    decodes the whole file first, src/snapshot.rs:76-98): with a batch pending in the delta run,
    sizes, roots and key-range aggregates are what they were, and the rank-order contents equal a
    twin pair of stores that never saw the file; both stores keep working."""
    from rsos_hip import GpuFingerprintStore, _abi as A
    from rsos_hip.store import KeyRange
    from rsos_hip.snapshot import load_snapshot
    cols = make_cols("bytes16", "bytes64", 20_000, 23, tomb=0.1)
    batch = make_cols("bytes16", "bytes64", 3000, 29)
    batch_cols = {c: batch[c] for c in ("keys", "values", "phys", "logical", "node", "tags")}
    sd, sp, _ = _schemas("b16_b64")
    pairs = []
    for _ in range(2):  # the stores under test, and their twins
        dated, proj = GpuFingerprintStore(sd), GpuFingerprintStore(sp)
        load_snapshot(encode("b16_b64", cols, [], {}), dated, proj)
        for st in (dated, proj):
            st.apply(batch_cols, np.zeros(3000, np.uint8))
        pairs.append((dated, proj))
    (dated, proj), twins = pairs
    cuts = [bytes(cols["keys"][i]) for i in range(0, 20_000, 1999)]

    def state(st):  # no rank-order question: the delta run stays pending
        aggs = [st.aggregate(KeyRange(lo, hi)) for lo, hi in zip(cuts, cuts[1:])]
        return st.size(), st.aggregate().fingerprint.to_int(), [(a.size, a.fingerprint.to_int()) for a in aggs]
    before = [state(dated), state(proj)]
    bad_cols = make_cols("bytes16", "bytes64", 30_000, 31, tomb=0.1)
    off = 16 + int(np.sum(np.where(bad_cols["tags"][:20_000] == 1, 40, 112)))
    bad = bytearray(encode("b16_b64", bad_cols, [], {}))
    bad[off + 36] = 5  # a State variant of 5 at entry 20,000
    for blob in (bytes(bad), bytes(bad[: len(bad) // 3])):
        with pytest.raises(A.RsosHipError) as e:
            load_snapshot(blob, dated, proj)
        assert e.value.code == A.ERR_DATA
        assert [state(dated), state(proj)] == before
    for st, twin in zip((dated, proj), twins):
        assert np.array_equal(st.fingerprints(), twin.fingerprints())
        assert [k for k, _ in st.enumerate()] == [k for k, _ in twin.enumerate()]
    info = load_snapshot(encode("b16_b64", bad_cols, [], {}), dated, proj)
    assert info.keys == 30_000 == dated.size() == proj.size()
