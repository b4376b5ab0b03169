"""GPU parity: the HIP path (librsos_hip.so, through its C ABI) against the oracle.

Bit-exact for everything (integer / byte work).  Golden fixtures first, then seeded random
batches against the C oracle, then size-independent properties at full size.
Mirrors the reference's own strategy: golden vectors (rsos/src/fingerprint/tests.rs:68-93,
tests/timestamp_wire_format.rs:105-121), fold-of-lift oracles
(tests/proptest_fingerprint_tree_map/btreemap_oracle.rs:132-162,
rsos/src/fingerprint_tree_map/tests/aggregate.rs:59-78), duplicate delivery (:195-231).
"""
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M256 = 1 << 256


def fp_int(b) -> int:
    return int.from_bytes(bytes(b), "little")


def limbs_int(l) -> int:
    return sum(int(x) << (64 * i) for i, x in enumerate(l))


def agg_int(row) -> int:
    """row of an (r, 5) int64 aggregate tensor -> fingerprint as int"""
    return sum((int(x) & (2**64 - 1)) << (64 * i) for i, x in enumerate(row[:4]))


def dev_cols(torch, schema_d, n, keys, values, phys=None, logical=None, node=None, tags=None):
    cols = {"keys": torch.from_numpy(np.ascontiguousarray(keys).copy()).cuda()} if schema_d["key_len"] else {}
    if values is not None and schema_d["value_len"]:
        cols["values"] = torch.from_numpy(np.ascontiguousarray(values).copy()).cuda()
    if phys is not None:
        cols["phys"] = torch.from_numpy(np.asarray(phys, np.uint64).view(np.int64)).cuda()
        cols["logical"] = torch.from_numpy(np.asarray(logical, np.uint32).view(np.int32)).cuda()
        cols["node"] = torch.from_numpy(np.asarray(node, np.uint64).view(np.int64)).cuda()
    if tags is not None:
        cols["tags"] = torch.from_numpy(np.asarray(tags, np.uint8)).cuda()
    return cols


def schema_of(s):
    from rsos_hip import RecordSchema
    return RecordSchema(s["key_kind"], s["key_len"], s["value_kind"], s["value_len"], s["record_kind"])


# ---- golden fixtures -------------------------------------------------------------------------

def test_reference_golden_entry_fingerprint_on_gpu(gpu, golden):
    """lift(&7u32, &Entry::present(stamp, 12345u32)) == tests/timestamp_wire_format.rs:105-121"""
    import torch
    from rsos_hip import RecordSchema, lift_records
    v = golden["reference"]["vectors"][2]
    r = v["record"]
    s = RecordSchema.dated("u32", "u32")
    cols = {"keys": torch.tensor([r["key_u32"]], dtype=torch.int32).view(torch.uint8).view(1, 4).cuda(),
            "values": torch.tensor([r["value_u32"]], dtype=torch.int32).view(torch.uint8).view(1, 4).cuda(),
            "phys": torch.tensor([int(r["phys"], 16)], dtype=torch.int64).cuda(),
            "logical": torch.tensor([int(r["logical"], 16)], dtype=torch.int32).cuda(),
            "node": torch.from_numpy(np.array([int(r["node"], 16)], np.uint64).view(np.int64)).cuda()}
    fps, bs = lift_records(s, cols)
    torch.cuda.synchronize()
    got = [f"0x{x:016x}" for x in np.frombuffer(fps.cpu().numpy().tobytes(), np.uint64)]
    assert got == v["limbs"]
    assert bytes(bs.cpu().numpy()[0]) == bytes(fps.cpu().numpy()[0])


def test_reference_golden_u64_str_via_encoded_path(gpu, golden):
    """lift(&50u64, &"Hello") and the 3-element sum through the generic encoded-bytes kernel."""
    import torch
    from rsos_hip import lift_encoded
    v0, v1 = golden["reference"]["vectors"][0], golden["reference"]["vectors"][1]
    blobs = [bytes.fromhex(v0["encoded_hex"])] + [bytes.fromhex(h) for h in v1["encoded_hex_parts"]]
    offs = np.zeros(len(blobs) + 1, np.int64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    data = torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8).cuda()
    fps, _ = lift_encoded(data, torch.from_numpy(offs).cuda())
    fps = fps.cpu().numpy()
    assert [f"0x{x:016x}" for x in np.frombuffer(fps[0].tobytes(), np.uint64)] == v0["limbs"]
    s = sum(fp_int(fps[i]) for i in (1, 2, 3)) % M256
    assert s == limbs_int([int(x, 16) for x in v1["limbs"]])


def _n_shapes():
    import json, os
    with open(os.path.join(os.path.dirname(__file__), "golden", "vectors.json")) as f:
        return len(json.load(f)["shapes"])


@pytest.mark.parametrize("idx", range(_n_shapes()))
def test_shape_golden_vectors(gpu, golden, idx):
    import torch
    from rsos_hip import lift_records
    s = golden["shapes"][idx]
    n = s["n"]
    keys = np.frombuffer(bytes.fromhex(s["keys"]), np.uint8).reshape(n, s["key_len"])
    vals = np.frombuffer(bytes.fromhex(s["values"]), np.uint8).reshape(n, s["value_len"])
    dated = s["record_kind"] == 1
    cols = dev_cols(torch, s, n, keys, vals, s["phys"] if dated else None, s["logical"] if dated else None,
                    s["node"] if dated else None, s["tags"])
    fps, bs = lift_records(schema_of(s), cols)
    torch.cuda.synchronize()
    assert [bytes(f).hex() for f in fps.cpu().numpy()] == s["fps"], s["name"]
    assert bytes(bs.cpu().numpy()[0]).hex() == s["sum"]


def test_encoded_golden_ragged(gpu, golden):
    import torch
    from rsos_hip import lift_encoded
    blobs = [bytes.fromhex(r["hex"]) for r in golden["encoded"]]
    offs = np.zeros(len(blobs) + 1, np.int64)
    offs[1:] = np.cumsum([len(b) for b in blobs])
    data = torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8).cuda()
    fps, bs = lift_encoded(data, torch.from_numpy(offs).cuda())
    got = [bytes(f).hex() for f in fps.cpu().numpy()]
    assert got == [r["fp"] for r in golden["encoded"]]
    assert fp_int(bs.cpu().numpy()[0]) == sum(fp_int(bytes.fromhex(r["fp"])) for r in golden["encoded"]) % M256


# ---- seeded random batches vs the C oracle ---------------------------------------------------

SHAPES = [("u32", "u32"), ("u64", "u64"), ("u64", "bytes64"), ("bytes16", "bytes64"),
          ("bytes16", "bytes1024"), ("bytes16", "u64"), ("bytes32", "bytes64"), ("bytes16", "unit"),
          ("u64", "unit")]


def oracle_records(O, schema, h):
    sch = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
    return O.Records(sch, h["keys"], h.get("values"), h.get("phys"), h.get("logical"), h.get("node"), h.get("tags"))


@pytest.mark.parametrize("kind", ["plain", "dated", "projection"])
@pytest.mark.parametrize("shape", SHAPES)
def test_random_batches_bit_exact(gpu, oracle_lib, shape, kind):
    import torch
    from rsos_hip import RecordSchema, lift_records
    from rsos_hip.synth import make_records, to_host
    schema = getattr(RecordSchema, kind)(*shape)
    n = 3001 if shape[1] != "bytes1024" else 1201  # ragged last block
    cols = make_records(schema, n, seed=11, tombstone_fraction=0.2 if kind != "plain" else 0.0)
    fps, bs = lift_records(schema, cols)
    torch.cuda.synchronize()
    want = oracle_records(oracle_lib, schema, to_host(cols)).lift(threads=8)
    got = fps.cpu().numpy()
    bad = np.nonzero((got != want).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatching rows, first {bad[:5]}"
    bsn = bs.cpu().numpy()
    for g in range(bsn.shape[0]):
        s = sum(fp_int(want[i]) for i in range(256 * g, min(n, 256 * g + 256))) % M256
        assert fp_int(bsn[g]) == s, g


def test_dual_lift_equals_two_lifts(gpu):
    import torch
    from rsos_hip import RecordSchema, lift_dual, lift_records
    from rsos_hip.synth import make_records
    for vshape in ("bytes64", "bytes1024"):
        d = RecordSchema.dated("bytes16", vshape)
        cols = make_records(d, 2000, seed=3, tombstone_fraction=0.3)
        fd, bd, fpj, bpj = lift_dual(d, cols)
        a, ab = lift_records(d, cols)
        b, bb = lift_records(d.with_kind(2), cols)
        torch.cuda.synchronize()
        assert torch.equal(fd, a) and torch.equal(fpj, b) and torch.equal(bd, ab) and torch.equal(bpj, bb)


def test_encoded_random_ragged(gpu, oracle_lib):
    import torch
    from rsos_hip import lift_encoded
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 3000, 1500)
    lens[:6] = [0, 0, 1, 1024, 1025, 2048]
    blobs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    offs = np.zeros(len(blobs) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    data = torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8).cuda()
    fps, _ = lift_encoded(data, torch.from_numpy(offs).cuda())
    want = oracle_lib.lift_encoded(blobs, threads=8)
    assert np.array_equal(fps.cpu().numpy(), want)


def test_encoded_short_mix(gpu, oracle_lib):
    """Mostly one-chunk records (the lane-refill kernel) with a few multi-chunk ones scattered
    in (left to the long kernel), over many waves; the last record ends at the buffer's end."""
    import torch
    from rsos_hip import lift_encoded
    rng = np.random.default_rng(11)
    n = 20_011
    lens = rng.integers(0, 200, n)
    lens[rng.integers(0, n, 40)] = rng.integers(1025, 4000, 40)
    lens[rng.integers(0, n, 40)] = 1024
    lens[-1] = 67
    blobs = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lens]
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    data = torch.frombuffer(bytearray(b"".join(blobs)), dtype=torch.uint8).cuda()
    fps, bs = lift_encoded(data, torch.from_numpy(offs).cuda())
    want = oracle_lib.lift_encoded(blobs, threads=8)
    assert np.array_equal(fps.cpu().numpy(), want)
    tot = sum(int.from_bytes(f.tobytes(), "little") for f in want[:256]) % (1 << 256)
    assert int.from_bytes(bs.cpu().numpy()[0].tobytes(), "little") == tot


def test_encoded_word_aligned_ragged(gpu, oracle_lib):
    """Ragged records whose lengths are all multiples of 4 (every block address dword-aligned:
    the loader's no-funnel-shift branch, partial blocks ending on a word boundary), then one odd
    length in the middle, which sends its wave down the funnel-shift branch."""
    import torch
    from rsos_hip import lift_encoded
    rng = np.random.default_rng(17)
    n = 3000
    lens = 4 * rng.integers(0, 70, n)
    lens[:4] = [0, 4, 60, 64]
    for odd in (False, True):
        if odd:
            lens[1500] = 61
        blobs = [rng.integers(0, 256, int(x), dtype=np.uint8).tobytes() for x in lens]
        offs = np.zeros(n + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        data = torch.frombuffer(bytearray(b"".join(blobs) + bytes(8)), dtype=torch.uint8).cuda()
        fps, _ = lift_encoded(data, torch.from_numpy(offs).cuda())
        want = oracle_lib.lift_encoded(blobs, threads=8)
        assert np.array_equal(fps.cpu().numpy(), want), odd


@pytest.mark.parametrize("length,offset", [(L, 0) for L in (0, 1, 4, 63, 64, 65, 120, 128, 1023, 1024, 1025, 2048,
                                                              3000)] +
                         [(L, o) for L in (48, 80, 100, 104, 120) for o in (0, 4)])
def test_fixed_length_records(gpu, oracle_lib, length, offset):
    """rh_lift_fixed_async: one length for every record (one chunk, exact blocks, multi-chunk),
    several workgroups and a ragged last one; block sums over the fingerprints.  The lengths with
    a compile-time kernel (k_lift_fixed_ct: 48, 80, 100, 104, 120) also from a buffer 4 bytes off
    its alignment, which takes the runtime-length kernel instead."""
    import torch
    from rsos_hip import lift_fixed
    rng = np.random.default_rng(length)
    n = 700
    raw = rng.integers(0, 256, n * length + 3, dtype=np.uint8)  # + bytes past the last record
    blobs = [raw[i * length:(i + 1) * length].tobytes() for i in range(n)]
    dev = torch.zeros(raw.size + 16, dtype=torch.uint8, device="cuda")
    dev[offset:offset + raw.size] = torch.from_numpy(raw).cuda()
    fps, bs = lift_fixed(dev[offset:offset + raw.size], length, n=n)
    want = oracle_lib.lift_encoded(blobs, threads=8)
    assert np.array_equal(fps.cpu().numpy(), want)
    tot = sum(int.from_bytes(f.tobytes(), "little") for f in want[256:512]) % (1 << 256)
    assert int.from_bytes(bs.cpu().numpy()[1].tobytes(), "little") == tot


def test_encoded_rows_lift_equals_schema_kernel(gpu):
    """The north_star record's canonical bytes (rsos_hip.synth.encode_rows) hashed by the fixed-length
    kernels -- compile-time (aligned) and runtime (4 bytes off) -- and by the offsets kernel equal the
    schema kernel's lift from the columns, for 16 B / 64 B dated and projection and u64 / 64 B
    dated and plain records (120, 100, 104, 80 B)."""
    import torch
    from rsos_hip import RecordSchema, lift_encoded, lift_fixed, lift_records
    from rsos_hip.synth import encode_rows, make_records
    for s in (RecordSchema.dated("bytes16", "bytes64"), RecordSchema.projection("bytes16", "bytes64"),
              RecordSchema.dated("u64", "bytes64"), RecordSchema.plain("u64", "bytes64")):
        n = 300_001
        cols = make_records(s, n, seed=8)
        rows = encode_rows(s, cols)
        assert rows.shape == (n, s.record_len())
        flat = rows.view(-1)
        ref, rb = lift_records(s, cols)
        mis = torch.zeros(flat.numel() + 16, dtype=torch.uint8, device="cuda")
        mis[4:4 + flat.numel()] = flat
        offs = torch.arange(0, n + 1, dtype=torch.int64, device="cuda") * rows.shape[1]
        for got, gb in (lift_fixed(flat, rows.shape[1]), lift_fixed(mis[4:4 + flat.numel()], rows.shape[1]),
                        lift_encoded(flat, offs)):
            assert torch.equal(got, ref) and torch.equal(gb, rb)


def test_fixed_equals_encoded_full_size(gpu, oracle_lib):
    """10 M records of 120 B: the fixed-length path equals the offsets path everywhere and the
    oracle on a sample."""
    import torch
    from rsos_hip import lift_encoded, lift_fixed
    n, L = 10_000_000, 120
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device="cuda", generator=g)
    a, ba = lift_fixed(data, L)
    b, bb = lift_encoded(data, torch.arange(0, n + 1, dtype=torch.int64, device="cuda") * L)
    assert torch.equal(a, b) and torch.equal(ba, bb)
    idx = np.random.default_rng(1).integers(0, n, 300)
    host = data.view(n, L)[torch.from_numpy(idx).cuda()].cpu().numpy()
    want = oracle_lib.lift_encoded([r.tobytes() for r in host], threads=8)
    assert np.array_equal(a[torch.from_numpy(idx).cuda()].cpu().numpy(), want)


def test_encoded_malformed_offsets_are_bounded(gpu, oracle_lib):
    """Offsets that decrease or run past the buffer: no fault, no runaway loop; well-formed
    records in the same launch still hash correctly."""
    import torch
    from rsos_hip import lift_encoded
    blobs = [b"abc", b"x" * 70, b"", b"hello world"]
    data = bytearray(b"".join(blobs))
    offs = [0]
    for b in blobs:
        offs.append(offs[-1] + len(b))
    good = len(offs) - 1
    offs += [offs[-1] - 5, 1 << 40, 3, (1 << 64) - 1 - (1 << 63)]  # decreasing, far past the end, ...
    t = torch.frombuffer(data, dtype=torch.uint8).cuda()
    fps, _ = lift_encoded(t, torch.tensor(offs, dtype=torch.int64).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(fps.cpu().numpy()[:good], oracle_lib.lift_encoded(blobs))


def test_empty_batches(gpu):
    import torch
    from rsos_hip import RecordSchema, lift_records, range_aggregates
    from rsos_hip.synth import make_records
    s = RecordSchema.dated("bytes16", "bytes64")
    cols = make_records(s, 0)
    fps, bs = lift_records(s, cols)
    assert fps.shape == (0, 32) and bs.shape == (0, 32)
    lo = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = range_aggregates(fps, bs, None, lo, lo)
    torch.cuda.synchronize()
    assert out.cpu().tolist() == [[0, 0, 0, 0, 0]]


# ---- range aggregates -------------------------------------------------------------------------

def test_range_aggregates_match_prefix_sums(gpu, oracle_lib):
    import torch
    from rsos_hip import RecordSchema, lift_records, range_aggregates, reduce_blocks
    from rsos_hip.synth import make_records, to_host
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 300_007  # > 4 super-blocks, ragged
    cols = make_records(s, n, seed=9)
    fps, bs = lift_records(s, cols)
    ss = reduce_blocks(bs)
    want = oracle_records(oracle_lib, s, to_host(cols)).lift(threads=8)
    assert np.array_equal(fps.cpu().numpy(), want)
    pref = [0]
    for f in want:
        pref.append(pref[-1] + fp_int(f))
    rng = np.random.default_rng(2)
    short = rng.integers(0, n - 700, 300)  # a protocol round's many short ranges (one wave each)
    width = rng.integers(0, 700, 300)
    lo = list(rng.integers(0, n, 200)) + [0, 0, 5, n - 1, 65536, 65535, 256, 100, n] + list(short)
    hi = list(rng.integers(0, n + 50, 200)) + [n, 0, 5, n, 3 * 65536 + 7, 65536 * 4, 512, 50, n] + list(short + width)
    lo_t = torch.tensor(lo, dtype=torch.int64, device="cuda")
    hi_t = torch.tensor(hi, dtype=torch.int64, device="cuda")
    for b, sup in ((bs, ss), (bs, None), (None, None)):
        out = range_aggregates(fps, b, sup, lo_t, hi_t).cpu().numpy()
        for j, (l, h) in enumerate(zip(lo, hi)):
            h2 = min(int(h), n)
            l2 = min(int(l), h2)
            assert int(out[j][4]) == h2 - l2
            assert agg_int(out[j]) == (pref[h2] - pref[l2]) % M256, (j, l, h)


def test_combine_aggregates(gpu):
    import torch
    from rsos_hip import combine_aggregates
    rng = np.random.default_rng(4)
    parts = rng.integers(-2**63, 2**63 - 1, (8, 16, 5), dtype=np.int64)
    parts[..., 4] = rng.integers(0, 10**9, (8, 16))
    parts[0, 0, :4] = -1  # all-ones limbs: carries everywhere
    parts[1, 0, :4] = [1, 0, 0, 0]
    out = combine_aggregates(torch.from_numpy(parts).cuda()).cpu().numpy()
    for j in range(16):
        want = sum(agg_int(parts[p, j]) for p in range(8)) % M256
        assert agg_int(out[j]) == want
        assert int(out[j][4]) == int(parts[:, j, 4].sum())


# ---- the store (Rsos<K> realisation) -----------------------------------------------------

def _store_fixture(oracle_lib, n=5000, seed=1):
    from rsos_hip import GpuFingerprintStore, RecordSchema
    rng = np.random.default_rng(seed)
    keys = np.unique(rng.integers(0, 2**40, n, dtype=np.uint64))
    n = len(keys)
    vals = rng.integers(0, 2**63, n, dtype=np.uint64)
    schema = RecordSchema.plain("u64", "u64")
    st = GpuFingerprintStore(schema)
    st.load_bulk({"keys": keys.view(np.uint8).reshape(n, 8), "values": vals.view(np.uint8).reshape(n, 8)})
    O = oracle_lib
    recs = O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0), keys.view(np.uint8).reshape(n, 8),
                     vals.view(np.uint8).reshape(n, 8))
    return st, keys, vals, recs


def test_store_rsos_surface(gpu, oracle_lib):
    from rsos_hip.store import KeyRange
    st, keys, vals, recs = _store_fixture(oracle_lib)
    n = len(keys)
    t = oracle_lib.FingerprintTreeMap(recs)
    t.fill(0, n)
    root = st.aggregate()
    assert root.size == n == st.size()
    assert root.fingerprint.to_int() == limbs_int(t.root()[0])
    assert np.array_equal(st.fingerprints(), recs.lift())
    rng = np.random.default_rng(3)
    for _ in range(300):
        a, b = (int(x) for x in rng.integers(0, 2**40, 2))
        got = st.aggregate(KeyRange(a, b))
        fp, size = t.aggregate(np.uint64(a).tobytes(), np.uint64(b).tobytes())
        assert got.size == size and got.fingerprint.to_int() == limbs_int(fp)
        assert st.rank(a) == t.rank(np.uint64(a).tobytes())
    # count-agreement and rank/select inverse laws (rbsr/src/rsos_view.rs:30-36)
    for r in rng.integers(0, n, 50):
        k = st.select(int(r))
        assert k == int(keys[r]) and st.rank(k) == r
    with pytest.raises(IndexError):
        st.select(n)
    k0, k1 = int(keys[10]), int(keys[20])
    assert st.aggregate(KeyRange(k0, k1)).size == st.rank(k1) - st.rank(k0) == 10
    assert st.aggregate(KeyRange(k0, k1, "included", "included")).size == 11
    assert st.aggregate(KeyRange(k0, k1, "excluded", "excluded")).size == 9
    assert st.aggregate(KeyRange(k1, k0)).is_empty()  # inverted -> ZERO
    assert [k for k, _ in st.enumerate(KeyRange(k0, k1))] == [int(x) for x in keys[10:20]]
    st.close()


def test_store_apply_insert_overwrite_delete(gpu, oracle_lib):
    st, keys, vals, recs = _store_fixture(oracle_lib, n=3000, seed=8)
    O = oracle_lib
    content = {int(k): int(v) for k, v in zip(keys, vals)}
    rng = np.random.default_rng(12)
    for rnd in range(3):
        new_keys = rng.integers(0, 2**40, 300, dtype=np.uint64)
        over = rng.choice(np.array(list(content.keys()), np.uint64), 100, replace=False)
        dels = rng.choice(np.array(list(content.keys()), np.uint64), 50, replace=False)
        bk = np.unique(np.concatenate([new_keys, over]))
        bk = np.setdiff1d(bk, dels)
        bv = rng.integers(0, 2**63, len(bk), dtype=np.uint64)
        allk = np.concatenate([bk, dels])
        allv = np.concatenate([bv, np.zeros(len(dels), np.uint64)])
        ops = np.concatenate([np.zeros(len(bk), np.uint8), np.ones(len(dels), np.uint8)])
        n_new, n_over, n_del = st.apply({"keys": allk.view(np.uint8).reshape(-1, 8),
                                         "values": allv.view(np.uint8).reshape(-1, 8)}, ops)
        exp_new = sum(1 for k in bk if int(k) not in content)
        assert (n_new, n_over, n_del) == (exp_new, len(bk) - exp_new, len(dels))
        for k, v in zip(bk, bv):
            content[int(k)] = int(v)
        for k in dels:
            content.pop(int(k))
        ks = np.array(sorted(content), np.uint64)
        vs = np.array([content[int(k)] for k in ks], np.uint64)
        r2 = O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0), ks.view(np.uint8).reshape(-1, 8),
                       vs.view(np.uint8).reshape(-1, 8))
        want = sum(fp_int(f) for f in r2.lift()) % M256
        root = st.aggregate()
        assert root.size == len(content) and root.fingerprint.to_int() == want
    # duplicate delivery moves the aggregate by 0 (btreemap_oracle.rs:195-231)
    before = st.aggregate()
    k = int(ks[7]); v = content[k]
    assert st.insert(k, v.to_bytes(8, "little")) is False
    assert st.aggregate() == before
    assert st.delete(k) is True and st.aggregate().size == before.size - 1
    assert st.insert(k, v.to_bytes(8, "little")) is True and st.aggregate() == before
    st.close()


@pytest.mark.parametrize("value,n,pinned", [("bytes64", 4000, False), ("bytes1024", 500_000, True)])
def test_lift_host_end_to_end(gpu, oracle_lib, value, n, pinned):
    """rh_lift_host: one chunk from pageable buffers, and (1 KiB values: ~126 k records per
    chunk) four chunks through the three-deep pipeline into a pinned rh_host_alloc buffer."""
    import ctypes as C
    from rsos_hip import RecordSchema, _abi as A
    from rsos_hip.synth import make_records, to_host
    s = RecordSchema.dated("bytes16", value)
    h = to_host(make_records(s, n, seed=21, tombstone_fraction=0.1))
    cols = A.Columns(*[None if h.get(k) is None else h[k].ctypes.data for k in
                       ("keys", "phys", "logical", "node", "tags", "values")])
    sc = s.c()
    ptr = C.c_void_p()
    if pinned:
        A.check(A.lib().rh_host_alloc(n * 32, C.byref(ptr)), "rh_host_alloc")
        out = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(n, 32))
    else:
        out = np.zeros((n, 32), np.uint8)
    try:
        A.check(A.lib().rh_lift_host(0, C.byref(sc), C.byref(cols), n, out.ctypes.data), "rh_lift_host")
        assert np.array_equal(out, oracle_records(oracle_lib, s, h).lift(threads=16))
    finally:
        if pinned:
            A.check(A.lib().rh_host_free(ptr), "rh_host_free")


# ---- full size: size-independent properties ------------------------------------------------------

def test_full_size_config2_properties(gpu, oracle_lib):
    """10 M records, 16 B key / 64 B value, dated (BASELINE config 2): sampled bit-exactness,
    block sums == an independent torch reduction, partition additivity of range aggregates."""
    import torch
    from rsos_hip import RecordSchema, lift_records, range_aggregates, reduce_blocks
    from rsos_hip.synth import make_records, to_host
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 10_000_000
    cols = make_records(s, n, seed=42)
    fps, bs = lift_records(s, cols)
    ss = reduce_blocks(bs)
    # sampled rows vs the oracle: a contiguous window at each end + the middle
    for lo in (0, n // 2 - 1000, n - 3000):
        want = oracle_records(oracle_lib, s, to_host(cols, lo, lo + 3000)).lift(threads=8)
        assert np.array_equal(fps[lo:lo + 3000].cpu().numpy(), want)
    # root via the kernels vs an independent torch reduction over u16 limbs
    limbs16 = fps.view(torch.int16).to(torch.int64) & 0xFFFF  # (n, 16)
    col = limbs16.sum(dim=0).cpu().tolist()
    want_root = sum(int(c) << (16 * i) for i, c in enumerate(col)) % M256
    lo_t = torch.tensor([0, 0, 1234567], dtype=torch.int64, device="cuda")
    hi_t = torch.tensor([n, 1234567, n], dtype=torch.int64, device="cuda")
    out = range_aggregates(fps, bs, ss, lo_t, hi_t).cpu().numpy()
    assert agg_int(out[0]) == want_root and int(out[0][4]) == n
    assert (agg_int(out[1]) + agg_int(out[2])) % M256 == want_root


@pytest.mark.parametrize("value,n", [("bytes64", 100_000_000), ("bytes1024", 100_000_000)],
                         ids=["north_star_100M_x_64B", "config3_full_100M_x_1KiB"])
def test_full_size_100m_properties(gpu, oracle_lib, value, n):
    """The north_star's 100 M x 16 B / 64 B dated set (bench.py's default config4 at N = 1) and
    BASELINE configs[2]'s 100 M x 16 B / 1 KiB: oracle-checked windows at both ends and the
    middle, the root aggregate against an independent torch reduction of the kernel's
    fingerprints (u16 limbs), and partition additivity of range aggregates over the 16 equal
    count ranges the bench queries."""
    import torch
    from rsos_hip import RecordSchema, lift_records, range_aggregates, reduce_blocks
    from rsos_hip.synth import make_records, to_host
    s = RecordSchema.dated("bytes16", value)
    cols = make_records(s, n, seed=42, key_space=n)
    fps, bs = lift_records(s, cols)
    ss = reduce_blocks(bs)
    w = 2048
    for lo in (0, n // 2 - w // 2, n - w):
        want = oracle_records(oracle_lib, s, to_host(cols, lo, lo + w)).lift(threads=8)
        assert np.array_equal(fps[lo:lo + w].cpu().numpy(), want), lo
    # a strided sample across the whole set (one row in ~50 k)
    rows = torch.arange(12345, n, 48_611, device="cuda")
    sub = {k: v[rows] for k, v in cols.items()}
    want = oracle_records(oracle_lib, s, to_host(sub)).lift(threads=8)
    assert np.array_equal(fps[rows].cpu().numpy(), want)
    del cols, sub
    want_root = 0
    for lo in range(0, n, 25_000_000):  # the u16-limb reduction in chunks (bounded temporaries)
        want_root += _torch_root(torch, fps[lo:lo + 25_000_000])
    want_root %= M256
    cuts = [n * j // 16 for j in range(17)]
    lo_t = torch.tensor([0] + cuts[:-1], dtype=torch.int64, device="cuda")
    hi_t = torch.tensor([n] + cuts[1:], dtype=torch.int64, device="cuda")
    out = range_aggregates(fps, bs, ss, lo_t, hi_t).cpu().numpy()
    assert agg_int(out[0]) == want_root and int(out[0][4]) == n
    assert sum(agg_int(r) for r in out[1:]) % M256 == want_root
    assert [int(r[4]) for r in out[1:]] == [b - a for a, b in zip(cuts, cuts[1:])]


def test_store_device_batches_bytes16_dated(gpu, oracle_lib):
    """Batched insert / overwrite / delete on the device merge path (16 B keys, dated records),
    checked against a fold of the oracle's lift over the expected contents after each batch."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records, to_host
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 200_000
    base = make_records(s, n, seed=5)
    st = GpuFingerprintStore(s)
    st.load_bulk_device(base)
    hb = to_host(base)
    content = {}  # key bytes -> record row (dict of numpy rows)

    def rows(h, i):
        return {k: h[k][i] for k in h}
    for i in range(n):
        content[hb["keys"][i].tobytes()] = rows(hb, i)
    O = oracle_lib
    sc = O.Schema(s.key_kind, s.key_len, s.value_kind, s.value_len, s.record_kind, 0)

    def expected_root():
        ks = sorted(content)
        cols = {c: np.stack([content[k][c] for k in ks]) for c in hb}
        fps = O.Records(sc, cols["keys"], cols["values"], cols["phys"], cols["logical"], cols["node"]).lift(threads=8)
        return len(ks), sum(int.from_bytes(f.tobytes(), "little") for f in fps) % M256, ks

    rng = np.random.default_rng(77)
    for rnd in range(3):
        m = 20_000
        fresh = make_records(s, m, seed=100 + rnd)  # keys interleave with the stored ones
        hf = to_host(fresh)
        existing = list(content)
        pick = rng.choice(len(existing), 6000, replace=False)
        over_keys, del_keys = [existing[i] for i in pick[:4000]], [existing[i] for i in pick[4000:]]
        # batch = fresh inserts + overwrites (new values/stamps) + deletes, shuffled
        keys = np.concatenate([hf["keys"], np.frombuffer(b"".join(over_keys + del_keys), np.uint8).reshape(-1, 16)])
        tot = len(keys)
        vals = rng.integers(0, 256, (tot, 64), dtype=np.uint8)
        phys = rng.integers(0, 2**62, tot, dtype=np.uint64)
        logical = rng.integers(0, 2**31, tot, dtype=np.uint32)
        node = rng.integers(0, 2**62, tot, dtype=np.uint64)
        ops = np.zeros(tot, np.uint8)
        ops[m + 4000:] = 1
        perm = rng.permutation(tot)
        keys, vals, phys, logical, node, ops = keys[perm], vals[perm], phys[perm], logical[perm], node[perm], ops[perm]
        dev = {"keys": torch.from_numpy(keys.copy()).cuda(), "values": torch.from_numpy(vals.copy()).cuda(),
               "phys": torch.from_numpy(phys.view(np.int64).copy()).cuda(),
               "logical": torch.from_numpy(logical.view(np.int32).copy()).cuda(),
               "node": torch.from_numpy(node.view(np.int64).copy()).cuda()}
        exp_new = sum(1 for k in hf["keys"] if k.tobytes() not in content)
        got = st.apply_device(dev, torch.from_numpy(ops).cuda())
        assert got == (exp_new, 4000 + (m - exp_new), 2000)
        for j in range(tot):
            k = keys[j].tobytes()
            if ops[j]:
                content.pop(k, None)
            else:
                content[k] = {"keys": keys[j], "values": vals[j], "phys": phys[j], "logical": logical[j],
                              "node": node[j]}
        size, root, ks = expected_root()
        agg = st.aggregate()
        assert agg.size == size == st.size()
        assert agg.fingerprint.to_int() == root
        # rank / select / enumerate against the expected key order
        for r in rng.integers(0, size, 20):
            assert st.select(int(r)) == ks[r] and st.rank(ks[r]) == r
        lo_k, hi_k = ks[1000], ks[1100]
        assert [k for k, _ in st.enumerate(KeyRange(lo_k, hi_k))] == ks[1000:1100]
    st.close()


def test_store_rejects_bad_batches_unchanged(gpu):
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema, RsosHipError
    from rsos_hip.synth import make_records
    s = RecordSchema.plain("bytes16", "bytes64")
    st = GpuFingerprintStore(s)
    base = make_records(s, 5000, seed=1)
    st.load_bulk_device(base)
    before = st.aggregate()
    batch = make_records(s, 10, seed=2)
    batch["keys"][3] = batch["keys"][7]  # duplicate within one batch
    with pytest.raises(RsosHipError):
        st.apply_device(batch)
    assert st.aggregate() == before
    # deleting absent keys is a no-op; an empty batch is a no-op
    absent = make_records(s, 10, seed=3)
    assert st.apply_device(absent, torch.ones(10, dtype=torch.uint8, device="cuda")) == (0, 0, 0)
    assert st.aggregate() == before
    # unsorted load is refused
    bad = make_records(s, 100, seed=4)
    bad["keys"] = bad["keys"].flip(0).contiguous()
    with pytest.raises(RsosHipError):
        st.load_bulk_device(bad)
    st.close()


def test_store_lsm_policies_agree(gpu, oracle_lib):
    """The LSM store answers identically whether the delta run is compacted after every batch
    or never, or with its capacity reserved up front (rh_store_reserve, twice, the second time
    over a pending delta run): key-range aggregates, ranks and sizes over base + delta equal the
    compacted base, and all equal a fold of the oracle's lift over the expected contents."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    s = RecordSchema.plain("u64", "u64")
    O = oracle_lib
    rng = np.random.default_rng(31)
    keys = np.unique(rng.integers(0, 2**40, 50_000, dtype=np.uint64))
    vals = rng.integers(0, 2**63, len(keys), dtype=np.uint64)
    content = {int(k): int(v) for k, v in zip(keys, vals)}
    lazy, eager, res = GpuFingerprintStore(s), GpuFingerprintStore(s), GpuFingerprintStore(s)
    lazy.set_compaction(1, 1 << 40)         # threshold max(base / 1, 2^40): never on its own
    eager.set_compaction(1 << 40, 0)        # threshold max(base / 2^40, 0) = 0: after every batch
    res.set_compaction(8, 4096)             # the default ratio, with capacity reserved up front
    for st in (lazy, eager, res):
        st.load_bulk({"keys": keys.view(np.uint8).reshape(-1, 8), "values": vals.view(np.uint8).reshape(-1, 8)})
    res.reserve(len(keys) + 10_000, 6000)
    sc = O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0)
    inserted = []
    for rnd in range(6):
        present = np.array(list(content.keys()), np.uint64)
        new = rng.integers(0, 2**40, 3000, dtype=np.uint64)
        over = rng.choice(present, 1000, replace=False)
        dele = rng.choice(np.setdiff1d(present, over), 800, replace=False)
        if inserted:  # delete some keys that only ever lived in the delta run
            dele = np.unique(np.concatenate([dele, np.array(inserted[-300:], np.uint64)]))
        bk = np.setdiff1d(np.unique(np.concatenate([new, over])), dele)
        bv = rng.integers(0, 2**63, len(bk), dtype=np.uint64)
        allk = np.concatenate([bk, dele])
        allv = np.concatenate([bv, np.zeros(len(dele), np.uint64)])
        ops = np.concatenate([np.zeros(len(bk), np.uint8), np.ones(len(dele), np.uint8)])
        perm = rng.permutation(len(allk))
        cols = {"keys": allk[perm].view(np.uint8).reshape(-1, 8), "values": allv[perm].view(np.uint8).reshape(-1, 8)}
        exp = (sum(1 for k in bk if int(k) not in content), sum(1 for k in bk if int(k) in content),
               sum(1 for k in dele if int(k) in content))
        assert lazy.apply(cols, ops[perm]) == exp
        assert eager.apply(cols, ops[perm]) == exp
        assert res.apply(cols, ops[perm]) == exp
        if rnd == 2:  # grow again with a pending delta run and a live base (kept across the move)
            res.reserve(4 * len(keys), 8000)
        for k, v in zip(bk, bv):
            if int(k) not in content:
                inserted.append(int(k))
            content[int(k)] = int(v)
        for k in dele:
            content.pop(int(k), None)
        assert lazy.stats()["delta_rows"] > 0 and eager.stats()["delta_rows"] == 0
        ks = np.array(sorted(content), np.uint64)
        fps = O.Records(sc, ks.view(np.uint8).reshape(-1, 8),
                        np.array([content[int(k)] for k in ks], np.uint64).view(np.uint8).reshape(-1, 8)).lift(threads=8)
        pref = [0]
        for f in fps:
            pref.append(pref[-1] + fp_int(f))
        assert lazy.size() == eager.size() == res.size() == len(ks)
        assert lazy.aggregate().fingerprint.to_int() == eager.aggregate().fingerprint.to_int() == pref[-1] % M256
        assert res.aggregate().fingerprint.to_int() == pref[-1] % M256
        for _ in range(25):
            a, b = sorted(int(x) for x in rng.integers(0, 2**40, 2))
            ra, rb = np.searchsorted(ks, a), np.searchsorted(ks, b)
            for st in (lazy, eager, res):
                agg = st.aggregate(KeyRange(a, b))
                assert agg.size == rb - ra and agg.fingerprint.to_int() == (pref[rb] - pref[ra]) % M256
        probes = rng.integers(0, 2**40, 64, dtype=np.uint64)
        want = np.searchsorted(ks, probes)
        assert (lazy.ranks(probes.view(np.uint8).reshape(-1, 8)) == want).all()
        assert (eager.ranks(probes.view(np.uint8).reshape(-1, 8)) == want).all()
        assert (res.ranks(probes.view(np.uint8).reshape(-1, 8)) == want).all()
        # rank-order reads over base + delta run as they stand (select over both, no compaction):
        # select, key dumps, rank-range aggregates (inverted and beyond-the-end ones too) and the
        # two-call round's steps
        nl = len(ks)
        sel = sorted({0, nl - 1} | {int(x) for x in rng.integers(0, nl, 40)})
        lo_r, hi_r = rng.integers(0, nl + 3, 40), rng.integers(0, nl + 3, 40)

        def want_agg(a, b):
            b = min(int(b), nl)
            a = min(int(a), b)
            return b - a, (pref[b] - pref[a]) % M256
        ka, kb = sorted(int(x) for x in rng.integers(0, 2**40, 2))
        segs = [types.SimpleNamespace(start=ka, end=kb), types.SimpleNamespace(start=kb, end=ka),
                types.SimpleNamespace(start=None, end=ka), types.SimpleNamespace(start=kb, end=None)]
        for st in (lazy, res):
            assert [st.select(r) for r in sel[:8]] == [int(ks[r]) for r in sel[:8]]
            got = st.aggregates_ranks(lo_r, hi_r)
            assert [(g.size, g.fingerprint.to_int()) for g in got] == [want_agg(a, b) for a, b in zip(lo_r, hi_r)]
            ra, rb = int(np.searchsorted(ks, ka)), int(np.searchsorted(ks, kb))
            assert [k for k, _ in st.enumerate(KeyRange(ka, kb))] == [int(k) for k in ks[ra:rb]]
            keys_out, aggs = st.split_segments(sel, lo_r, hi_r)
            assert keys_out == [int(ks[r]) for r in sel]
            assert [(g.size, g.fingerprint.to_int()) for g in aggs] == [want_agg(a, b) for a, b in zip(lo_r, hi_r)]
            lo, hi, la = st.resolve_segments(segs)
            assert list(lo) == [ra, rb, 0, rb] and list(hi) == [rb, ra, ra, nl]
            assert [(g.size, g.fingerprint.to_int()) for g in la] == \
                [want_agg(ra, rb), (0, 0), want_agg(0, ra), want_agg(rb, nl)]
        assert lazy.stats()["delta_rows"] > 0 and lazy.stats()["compactions"] == 0
    # the reads left the lazy store's delta run in place; the fingerprint dump compacts it, and
    # afterwards the stores agree row for row
    assert lazy.select(100) == int(ks[100])
    assert lazy.stats()["delta_rows"] > 0
    assert np.array_equal(lazy.fingerprints(), eager.fingerprints())
    assert lazy.stats()["delta_rows"] == 0
    assert np.array_equal(res.fingerprints(), eager.fingerprints())
    lazy.close()
    eager.close()
    res.close()


def test_store_batch_keys_sharing_leading_bytes(gpu, oracle_lib):
    """16 B keys whose first 8 bytes repeat (the batch sort's most-significant-digit pass alone
    cannot order them, so it falls back to the full sort): applied batches, and a reload with
    repeated keys, still give the oracle's key order and fingerprints."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    O = oracle_lib
    s = RecordSchema.plain("bytes16", "bytes64")
    rng = np.random.default_rng(21)
    heads = rng.integers(0, 256, (40, 8), dtype=np.uint8)
    n = 4000
    keys = np.concatenate([heads[rng.integers(0, 40, n)], rng.integers(0, 256, (n, 8), dtype=np.uint8)], axis=1)
    keys = np.unique(keys.view("V16"), axis=0).view(np.uint8).reshape(-1, 16)
    keys = keys[rng.permutation(len(keys))]
    vals = rng.integers(0, 256, (len(keys), 64), dtype=np.uint8)
    st = GpuFingerprintStore(s)
    half = len(keys) // 2
    for lo, hi in [(0, half), (half, len(keys))]:
        st.apply({"keys": keys[lo:hi], "values": vals[lo:hi]}, np.zeros(hi - lo, np.uint8))
    order = np.lexsort(keys.T[::-1])
    sch = O.Schema(O.KEY_BYTES, 16, O.VAL_BYTES, 64, O.REC_PLAIN, 0)
    want = O.Records(sch, np.ascontiguousarray(keys[order]), np.ascontiguousarray(vals[order])).lift()
    assert np.array_equal(st.fingerprints(), want)
    assert [k for k, _ in st.enumerate()] == [keys[i].tobytes() for i in order]
    st.close()


@pytest.mark.gpu
def test_store_batch_sort_skewed_and_dense(gpu, oracle_lib):
    """The update batches' bucket sort: a tight cluster of 3000 u64 keys plus far outliers (one
    bucket overflows: the full radix sort takes over), then a dense arithmetic run and a
    random batch (the bucket path) -- the store's key order and fingerprints match the oracle's."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    O = oracle_lib
    s = RecordSchema.plain("u64", "bytes64")
    rng = np.random.default_rng(33)
    batches = [
        np.concatenate([10**12 + np.arange(3000, dtype=np.uint64), np.array([5, 2**63, 2**64 - 7], np.uint64)]),
        np.arange(20000, dtype=np.uint64) * 3 + 7,
        rng.integers(0, 2**63, 50000, dtype=np.uint64) * 2 + 1,
    ]
    st = GpuFingerprintStore(s)
    all_keys, all_vals = [], []
    for b in batches:
        b = b[rng.permutation(len(b))]
        v = rng.integers(0, 256, (len(b), 64), dtype=np.uint8)
        st.apply({"keys": b.view(np.uint8).reshape(-1, 8), "values": v}, np.zeros(len(b), np.uint8))
        all_keys.append(b)
        all_vals.append(v)
    keys, vals = np.concatenate(all_keys), np.concatenate(all_vals)
    keys, first = np.unique(keys, return_index=True)
    assert len(keys) == st.size()
    sch = O.Schema(O.KEY_U64, 8, O.VAL_BYTES, 64, O.REC_PLAIN, 0)
    want = O.Records(sch, np.ascontiguousarray(keys.view(np.uint8).reshape(-1, 8)),
                     np.ascontiguousarray(vals[first])).lift()
    assert np.array_equal(st.fingerprints(), want)
    assert [k for k, _ in st.enumerate()] == [int(k) for k in keys]
    st.close()


def _torch_root(torch, fps) -> int:
    """Σ fingerprints mod 2^256 by an independent torch reduction over u16 limbs."""
    limbs16 = fps.view(torch.int16).to(torch.int64) & 0xFFFF
    col = limbs16.sum(dim=0).cpu().tolist()
    return sum(int(c) << (16 * i) for i, c in enumerate(col)) % M256


def test_full_size_incremental_properties(gpu):
    """config5's shape at a tenth of the size: 10 M resident records, then 1 M-record random-key
    batches (inserts, then a batch that overwrites 100 k and deletes 100 k existing keys).  After
    each batch the store's root equals an independent torch reduction over the lifts of exactly
    the records that should be live, and rank / size agree (count-agreement law)."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema, lift_records
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records
    s = RecordSchema.dated("bytes16", "bytes64")
    n, m = 10_000_000, 1_000_000
    base = make_records(s, n, seed=5)
    st = GpuFingerprintStore(s)
    st.load_bulk_device(base)
    live = [lift_records(s, base, block_sums=False)[0]]
    for k in range(2):
        b = make_records(s, m, seed=600 + k, random_keys=True)
        assert st.apply_device(b) == (m, 0, 0)
        live.append(lift_records(s, b, block_sums=False)[0])
        root = st.aggregate()
        assert root.size == n + (k + 1) * m
        assert root.fingerprint.to_int() == (sum(_torch_root(torch, f) for f in live)) % M256
    # overwrite rows [0, 100k) of the base with new values, delete rows [100k, 200k)
    ov = {c: t[:200_000].clone() for c, t in base.items()}
    ov["values"][:100_000] ^= 0x5A
    ops = torch.zeros(200_000, dtype=torch.uint8, device="cuda")
    ops[100_000:] = 1
    assert st.apply_device(ov, ops) == (0, 100_000, 100_000)
    new_fps, _ = lift_records(s, {c: t[:100_000] for c, t in ov.items()}, block_sums=False)
    want = (sum(_torch_root(torch, f) for f in live) - _torch_root(torch, live[0][:200_000])
            + _torch_root(torch, new_fps)) % M256
    root = st.aggregate()
    assert root.size == n + 2 * m - 100_000 and root.fingerprint.to_int() == want
    # count agreement over a key range spanning base and delta rows
    lo_key, hi_key = base["keys"][50_000].cpu().numpy().tobytes(), base["keys"][5_000_000].cpu().numpy().tobytes()
    agg = st.aggregate(KeyRange(lo_key, hi_key))
    assert agg.size == st.rank(hi_key) - st.rank(lo_key)
    st.compact()
    assert st.aggregate() == root and st.stats()["delta_rows"] == 0
    st.close()


def test_store_load_refuses_2_pow_31_rows(gpu):
    """Ranks are 32-bit on the device: a load of >= 2^31 rows is an argument error before any
    column is read (host or device path), and the store keeps its contents."""
    import ctypes as C
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema, _abi as A
    from rsos_hip.synth import make_records
    s = RecordSchema.plain("u32", "u32")
    st = GpuFingerprintStore(s)
    st.load_bulk_device(make_records(s, 1000, seed=1))
    root = st.aggregate()
    tiny = torch.zeros(64, dtype=torch.uint8, device="cuda")
    cols = A.Columns(tiny.data_ptr(), None, None, None, None, tiny.data_ptr())
    assert A.lib().rh_store_load_device(st._h, C.byref(cols), 1 << 31, None) == A.ERR_ARG
    assert b"2^31" in A.lib().rh_last_error()
    host = (C.c_uint8 * 64)()
    hcols = A.Columns(C.addressof(host), None, None, None, None, C.addressof(host))
    assert A.lib().rh_store_load(st._h, C.byref(hcols), (1 << 31) + 5) == A.ERR_ARG
    assert st.aggregate() == root and st.size() == 1000
    st.close()


def test_host_tier_equals_device_answers(gpu, oracle_lib):
    """The host tier (rh_store_set_host_tier) against the device path on the same store, before
    and after batches (a load or a moved buffer refreshes the tier in the background, the device
    answering meanwhile; batches fold into it): ranks of
    present and absent keys, select, key-range aggregates with every bound kind (inverted ones
    give ZERO), rank-range aggregates, and the root against the oracle FTM's."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records, to_host
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 300_000
    base = make_records(s, n, seed=21)
    dev, tier = GpuFingerprintStore(s, host_tier=False), GpuFingerprintStore(s, host_tier=True)
    for st in (dev, tier):
        st.load_bulk_device(base)
    rng = np.random.default_rng(5)
    keys_h = to_host(base)["keys"]

    def probe():
        assert tier.size() == dev.size() and tier.aggregate() == dev.aggregate()
        ks = [keys_h[i].tobytes() for i in rng.integers(0, n, 200)] + [rng.bytes(16) for _ in range(200)]
        ks += [b"\x00" * 16, b"\xff" * 16]
        karr = np.frombuffer(b"".join(ks), np.uint8).reshape(-1, 16)
        assert np.array_equal(tier.ranks(karr), dev.ranks(karr))
        assert [tier.rank(k) for k in ks[:20]] == [int(x) for x in dev.ranks(karr[:20])]
        for r in [0, 1, tier.size() - 1] + list(rng.integers(0, tier.size(), 50)):
            assert tier.select(int(r)) == dev.select(int(r))
        for _ in range(100):
            a, b = ks[rng.integers(len(ks))], ks[rng.integers(len(ks))]
            sk, ek = ["included", "excluded"][rng.integers(2)], ["included", "excluded"][rng.integers(2)]
            rg = KeyRange(a if rng.random() > 0.1 else None, b if rng.random() > 0.1 else None, sk, ek)
            assert tier.aggregate(rg) == dev.aggregate(rg)
        lo = rng.integers(0, tier.size(), 64)
        hi = lo + rng.integers(0, 70_000, 64)
        assert tier.aggregates_ranks(list(lo), list(hi)) == dev.aggregates_ranks(list(lo), list(hi))

    probe()  # answered by the device or the tier, whichever holds the copy by then
    tier.tier_sync()
    assert tier.tier_stats()["refreshes"] == 1
    for k in range(3):  # inserts, then overwrites + deletes of existing keys
        b = make_records(s, 20_000, seed=300 + k, random_keys=True)
        ops = None
        if k == 2:
            b = {c: t[1000:21000].clone() for c, t in base.items()}
            b["values"][:10_000] ^= 0x33
            ops = torch.zeros(20_000, dtype=torch.uint8, device="cuda")
            ops[10_000:] = 1
        assert tier.apply_device(b, ops) == dev.apply_device(b, ops)
        probe()
    # the batches were folded into the tier's delta tree: no second copy of the base
    st = tier.tier_stats()
    assert st["refreshes"] == 1 and st["folds"] == 3 and st["base_rows"] == n
    assert st["delta_entries"] == tier.stats()["delta_rows"]
    # deletes of keys inserted since the base copy drop their entries; a key inserted and deleted
    # and inserted again; a compaction between batches (the next fold forms its deltas against the
    # tier's own base, not the device's new one)
    ins = make_records(s, 3_000, seed=400, random_keys=True)
    gone = {c: t[:1_000].clone() for c, t in ins.items()}
    dels = torch.ones(1_000, dtype=torch.uint8, device="cuda")
    for st_ in (dev, tier):
        assert st_.apply_device(ins) == (3_000, 0, 0)
        assert st_.apply_device(gone, dels) == (0, 0, 1_000)
        st_.compact()
    probe()
    again = {c: t[:500].clone() for c, t in ins.items()}
    again["values"] ^= 0x5A
    for st_ in (dev, tier):
        assert st_.apply_device(again) == (500, 0, 0)
        assert st_.apply_device(gone, dels) == (0, 0, 500)
    probe()
    assert tier.tier_stats()["refreshes"] == 1
    # a larger reservation moves the tier's page-locked buffers: the next question copies the base
    # again instead of reading the old ones (a use-after-free before)
    tier.reserve(4 * n, 20_000)
    probe()
    tier.tier_sync()
    assert tier.tier_stats()["refreshes"] == 2
    # small batches (the staged-insert shape): one row, then 1,000 rows
    one = make_records(s, 1, seed=501, random_keys=True)
    thousand = make_records(s, 1_000, seed=502, random_keys=True)
    for b in (one, thousand):
        assert tier.apply_device(b) == dev.apply_device(b)
        probe()
    assert tier.tier_stats()["refreshes"] == 2
    dev.close()
    tier.close()


@pytest.mark.gpu
def test_keys_checked_after_staged_rows(gpu):
    """rh_store_keys / select check the rank range against the size the staged rows leave (the
    batch is applied first): ranks past the end after staged deletes are refused, ranks made valid
    by staged inserts are answered -- with and without the host tier."""
    import ctypes as C
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip import _abi as A
    s = RecordSchema.plain("u64", "u64")
    for tier in (False, True):
        st = GpuFingerprintStore(s, host_tier=tier)
        keys = np.arange(0, 2_000, 2, dtype=np.uint64)
        st.load_bulk({"keys": keys.view(np.uint8).reshape(-1, 8), "values": (keys * 3).view(np.uint8).reshape(-1, 8)})
        assert st.size() == 1_000 and st.select(999) == 1998
        # stage 10 deletes of the top keys: rank 995 is now past the end
        dk = keys[-10:].copy()
        cols = A.Columns(dk.ctypes.data, None, None, None, None, dk.ctypes.data)
        ops = np.ones(10, np.uint8)
        A.check(A.lib().rh_store_stage(st._h, C.byref(cols), ops.ctypes.data, 10), "stage")
        buf = np.zeros(8, np.uint8)
        assert A.lib().rh_store_keys(st._h, 995, 996, buf.ctypes.data) == A.ERR_ARG
        assert st.size() == 990
        # stage 20 inserts above the top: ranks up to 1,009 answer
        ik = np.arange(5_001, 5_041, 2, dtype=np.uint64)
        cols = A.Columns(ik.ctypes.data, None, None, None, None, ik.ctypes.data)
        A.check(A.lib().rh_store_stage(st._h, C.byref(cols), np.zeros(20, np.uint8).ctypes.data, 20), "stage")
        out = np.zeros(20, np.uint64)
        A.check(A.lib().rh_store_keys(st._h, 990, 1_010, out.ctypes.data), "keys")
        assert np.array_equal(out, ik)
        assert st.select(1_009) == 5_039
        st.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind,m", [("u32", 1), ("u32", 1025), ("u64", 8193), ("bytes16", 2), ("bytes16", 70_000),
                                    ("bytes32", 8192), ("bytes16", 1_500_000)])
def test_store_batch_sort_sizes(gpu, kind, m):
    """The update batches' bucket sort (store_kernels.hip k_cs_*) across key kinds and the sizes
    at its tile and bucket-count boundaries (1, 1,025 and 8,193 keys; 1.5 M keys = 2,048 coarse
    buckets): a shuffled batch applied to an empty store leaves the fingerprints of the batch's
    rows in key order -- the GPU lift of the key-sorted columns, sorted on the host."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema, lift_records
    from rsos_hip.synth import make_records
    s = RecordSchema.plain(kind, "u32" if kind == "u32" else "bytes64")  # schemas with a store lift kernel
    cols = make_records(s, m, seed=71 + m, random_keys=True)
    perm = torch.randperm(m, generator=torch.Generator().manual_seed(m)).cuda()
    cols = {c: t[perm].contiguous() for c, t in cols.items()}  # integer keys come sorted
    st = GpuFingerprintStore(s)
    assert st.apply_device(cols) == (m, 0, 0)
    keys = cols["keys"].cpu().numpy().reshape(m, -1)
    if kind == "u32":
        order = np.argsort(keys.copy().view(np.uint32).ravel(), kind="stable")
    elif kind == "u64":
        order = np.argsort(keys.copy().view(np.uint64).ravel(), kind="stable")
    else:
        order = np.lexsort(keys.T[::-1])
    o = torch.from_numpy(order).cuda()
    want = lift_records(s, {c: t[o].contiguous() for c, t in cols.items()}, block_sums=False)[0].cpu().numpy()
    st.compact()
    assert np.array_equal(st.fingerprints(), want)
    st.close()


@pytest.mark.gpu
def test_store_batch_sort_duplicate_in_large_batch(gpu):
    """A repeated key in a 1 M batch (bucket path, full-key ties inside a fine bucket) is refused
    and the store is left as it was; the same keys with the duplicate's leading 8 bytes kept but
    its last byte changed are accepted."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema, RsosHipError
    from rsos_hip.synth import make_records
    s = RecordSchema.plain("bytes16", "bytes64")
    st = GpuFingerprintStore(s)
    st.load_bulk_device(make_records(s, 100_000, seed=5))
    before = st.aggregate()
    b = make_records(s, 1_000_000, seed=6, random_keys=True)
    b["keys"][777_777] = b["keys"][123]
    with pytest.raises(RsosHipError):
        st.apply_device(b)
    assert st.aggregate() == before
    b["keys"][777_777, 15] ^= 0x01  # same leading digit as row 123, different key
    assert st.apply_device(b) == (1_000_000, 0, 0)
    assert st.size() == 1_100_000
    st.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["clustered", "narrow", "tiny"])
def test_store_device_ranks_skewed_keys(gpu, layout):
    """The base run's searches (bucket table over the second-level samples, then one sample line
    and one key line) on key sets whose leading 8 bytes are far from uniform: three clusters of
    equal leading digits plus outliers at both ends ("clustered"), every key inside a range of
    2^20 digits ("narrow"), and a 5-row store ("tiny").  Device ranks of present and absent
    keys equal numpy's searchsorted over the sorted keys, before and after a batch that lands
    in the delta run."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    s = RecordSchema.plain("bytes16", "bytes64")
    rng = np.random.default_rng(97)
    if layout == "clustered":
        heads = np.array([[0x10] * 8, [0x80] + [0] * 7, [0x80] + [0] * 6 + [1]], np.uint8)
        keys = np.concatenate([heads[rng.integers(0, 3, 200_000)], rng.integers(0, 256, (200_000, 8), dtype=np.uint8)],
                              axis=1)
        keys = np.concatenate([keys, np.array([[0] * 16, [255] * 16], np.uint8)])
    elif layout == "narrow":
        d = (np.uint64(0x123456789ABC0000) + rng.integers(0, 1 << 20, 300_000).astype(np.uint64)).astype(">u8")
        keys = np.concatenate([d.view(np.uint8).reshape(-1, 8), rng.integers(0, 256, (300_000, 8), dtype=np.uint8)],
                              axis=1)
    else:
        keys = rng.integers(0, 256, (5, 16), dtype=np.uint8)
    keys = np.unique(keys.view("V16"), axis=0).view(np.uint8).reshape(-1, 16)  # sorted by memcmp
    vals = rng.integers(0, 256, (len(keys), 64), dtype=np.uint8)
    st = GpuFingerprintStore(s, host_tier=False)
    st.load_bulk({"keys": keys, "values": vals})

    def check(all_keys):
        sk = np.unique(all_keys.view("V16"), axis=0)
        probes = np.concatenate([all_keys[rng.integers(0, len(all_keys), 500)],
                                 rng.integers(0, 256, (300, 16), dtype=np.uint8),
                                 all_keys[rng.integers(0, len(all_keys), 200)] ^ np.eye(16, dtype=np.uint8)[15],
                                 np.array([[0] * 16, [255] * 16, [0x80] + [0] * 15], np.uint8)])
        want = np.searchsorted(sk.ravel(), probes.view("V16").ravel(), side="left")
        assert np.array_equal(st.ranks(np.ascontiguousarray(probes)), want)

    check(keys)
    extra = rng.integers(0, 256, (1000, 16), dtype=np.uint8)
    extra[:500, :8] = keys[rng.integers(0, len(keys), 500), :8]  # same leading digits as base keys
    extra = np.unique(extra.view("V16"), axis=0).view(np.uint8).reshape(-1, 16)
    extra = extra[~np.isin(extra.view("V16").ravel(), keys.view("V16").ravel())]
    st.apply({"keys": extra, "values": rng.integers(0, 256, (len(extra), 64), dtype=np.uint8)},
             np.zeros(len(extra), np.uint8))
    check(np.concatenate([keys, extra]))
    st.close()


@pytest.mark.gpu
def test_store_apply_device_many_equals_one_by_one(gpu, oracle_lib):
    """rh_store_apply_device_many (batch i + 1 lifted while batch i's result returns) leaves the
    store exactly as applying the same batches one call at a time: per-batch counts, root,
    ranks, selects and every fingerprint, across inserts, overwrites, deletes, an empty batch,
    a batch whose keys share their leading 8 bytes (the full-sort re-run, with the next batch
    already lifted), and compactions between batches.  A duplicate key in batch 3 of 5 leaves
    batches 0-2 applied and the rest not."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema, RsosHipError
    from rsos_hip.synth import make_records
    s = RecordSchema.dated("bytes16", "bytes64")
    base = make_records(s, 300_000, seed=5)
    g = torch.Generator(device="cuda")
    g.manual_seed(9)

    def batches():
        out, ops = [], []
        for k in range(7):
            if k == 3:  # empty
                b = {c: t[:0].contiguous() for c, t in make_records(s, 1, seed=50).items()}
                out.append(b)
                ops.append(None)
                continue
            b = make_records(s, 40_000, seed=100 + k, random_keys=True)
            if k == 4:  # leading 8 bytes shared by many keys
                heads = torch.randint(0, 256, (16, 8), dtype=torch.uint8, device="cuda", generator=g)
                b["keys"][:, :8] = heads[torch.randint(0, 16, (40_000,), device="cuda", generator=g)]
            rows = torch.randperm(300_000, device="cuda", generator=g)[:5_000]
            b["keys"][:5_000] = base["keys"][rows]  # overwrites / deletes of resident keys
            b["phys"][:5_000] = base["phys"][rows] + 7
            o = torch.zeros(40_000, dtype=torch.uint8, device="cuda")
            o[:2_000] = 1
            out.append(b)
            ops.append(o)
        return out, ops

    bs, ops = batches()
    one, many = GpuFingerprintStore(s), GpuFingerprintStore(s)
    for st in (one, many):
        st.set_compaction(4, 50_000)  # a compaction every few batches
        st.load_bulk_device(base)
    want = [one.apply_device(b, o) for b, o in zip(bs, ops)]
    got = many.apply_device_many(bs, ops)
    assert got == want and got[3] == (0, 0, 0)
    assert many.stats()["compactions"] == one.stats()["compactions"] > 0
    assert many.size() == one.size() and many.aggregate() == one.aggregate()
    assert np.array_equal(many.fingerprints(), one.fingerprints())
    n = one.size()
    for r in range(0, n, n // 37):
        k = one.select(r)
        assert many.select(r) == k and many.rank(k) == r
    # a duplicate inside batch 3 of 5: 0-2 applied, 3-4 not
    bs2 = [make_records(s, 20_000, seed=300 + k, random_keys=True) for k in range(5)]
    bs2[3]["keys"][11] = bs2[3]["keys"][12]
    ref = GpuFingerprintStore(s)
    ref.load_bulk_device(base)
    for b in bs2[:3]:
        ref.apply_device(b)
    part = GpuFingerprintStore(s)
    part.load_bulk_device(base)
    with pytest.raises(RsosHipError):
        part.apply_device_many(bs2)
    assert part.aggregate() == ref.aggregate() and part.size() == ref.size()
    for st in (one, many, ref, part):
        st.close()


def test_batch_path_variants_agree(gpu, oracle_lib, monkeypatch):
    """The batch path's fused lift + search launch (k_lift_search) against the lift and the two
    searches as separate launches (RSOS_HIP_UNFUSED=1, read when a store is created), the next
    batch's digit min / max formed by that launch against the sort's own pass
    (RSOS_HIP_PRE_MINMAX=0, read when a store is created), and the merges' precomputed tile bounds
    (k_tile_bounds) against each tile searching its own (RSOS_HIP_TILE_SEARCH=1, read per
    merge), and the small-batch path (one workgroup + the merge, small_batch.hpp) against the
    large-batch path for the batches of <= 1,024 rows (RSOS_HIP_SMALL_MAX=0, read when a store is
    created): the same batches -- 30,000, 700 and 1 rows of fresh keys, overwrites, deletes,
    through apply_device and apply_device_many, across compactions -- leave every store with the
    same counts, fingerprints, ranks and root, and that root equals the oracle's fold of the live
    records' lifts."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.synth import make_records
    O = oracle_lib
    s = RecordSchema.dated("bytes16", "bytes64")
    base = make_records(s, 200_000, seed=71)
    g = torch.Generator(device="cuda")
    g.manual_seed(72)
    bs, ops = [], []
    for k in range(6):
        b = make_records(s, 30_000, seed=700 + k, random_keys=True)
        rows = torch.randperm(200_000, device="cuda", generator=g)[:4_000]
        b["keys"][:4_000] = base["keys"][rows]  # overwrites / deletes of resident keys
        b["phys"][:4_000] = base["phys"][rows] + 3
        o = torch.zeros(30_000, dtype=torch.uint8, device="cuda")
        o[:1_500] = 1
        bs.append(b)
        ops.append(o)
        # two batches the small path takes: 700 rows (200 overwrites and 60 deletes of resident
        # keys) and one fresh row
        b2 = make_records(s, 700, seed=800 + k, random_keys=True)
        rows = torch.randperm(200_000, device="cuda", generator=g)[:200]
        b2["keys"][:200] = base["keys"][rows]
        b2["phys"][:200] = base["phys"][rows] + 5
        o2 = torch.zeros(700, dtype=torch.uint8, device="cuda")
        o2[:60] = 1
        bs += [b2, make_records(s, 1, seed=900 + k, random_keys=True)]
        ops += [o2, torch.zeros(1, dtype=torch.uint8, device="cuda")]

    def run(unfused, tile_search, many, pre_minmax=True, small=True):
        monkeypatch.setenv("RSOS_HIP_UNFUSED", "1" if unfused else "")
        monkeypatch.setenv("RSOS_HIP_TILE_SEARCH", "1" if tile_search else "0")
        monkeypatch.setenv("RSOS_HIP_PRE_MINMAX", "1" if pre_minmax else "0")
        if small:
            monkeypatch.delenv("RSOS_HIP_SMALL_MAX", raising=False)
        else:
            monkeypatch.setenv("RSOS_HIP_SMALL_MAX", "0")
        st = GpuFingerprintStore(s)
        st.set_compaction(4, 40_000)
        st.load_bulk_device(base)
        counts = st.apply_device_many(bs, ops) if many else [st.apply_device(b, o) for b, o in zip(bs, ops)]
        out = (counts, st.size(), st.aggregate(), st.fingerprints(), st.stats()["compactions"],
               [st.select(r) for r in range(0, st.size(), 9_973)], st.batch_stats())
        st.close()
        return out

    ref = run(False, False, True)
    assert ref[4] > 0  # compactions happened
    for variant in [(True, False, True), (False, True, True), (True, True, False), (False, False, False),
                    (False, False, True, False), (False, False, False, True, False)]:
        got = run(*variant)
        assert got[0] == ref[0] and got[1] == ref[1] and got[2] == ref[2] and got[4] == ref[4], variant
        assert np.array_equal(got[3], ref[3]) and got[5] == ref[5], variant
        if variant[2] is False:  # one call per batch: the 12 small batches took the small path, or none did
            assert got[6]["small"] == (0 if variant[4:] == (False,) else 12), (variant, got[6])
    # the root against the oracle: Σ lift over the live records (last write wins, deletes removed)
    live = {}
    cols = {c: t.cpu().numpy() for c, t in base.items()}
    for i in range(len(cols["keys"])):
        live[cols["keys"][i].tobytes()] = (0, i)
    for bi, (b, o) in enumerate(zip(bs, ops)):
        bc = {c: t.cpu().numpy() for c, t in b.items()}
        oc = o.cpu().numpy()
        for i in range(len(bc["keys"])):
            k = bc["keys"][i].tobytes()
            if oc[i]:
                live.pop(k, None)
            else:
                live[k] = (bi + 1, i)
    src = [cols] + [{c: t.cpu().numpy() for c, t in b.items()} for b in bs]
    keys = sorted(live)
    assert len(keys) == ref[1]
    sch = O.Schema(O.KEY_BYTES, 16, O.VAL_BYTES, 64, O.REC_DATED, 0)
    pick = lambda name: np.stack([src[live[k][0]][name][live[k][1]] for k in keys])
    recs = O.Records(sch, np.ascontiguousarray(pick("keys")), np.ascontiguousarray(pick("values")),
                     np.ascontiguousarray(pick("phys")), np.ascontiguousarray(pick("logical")),
                     np.ascontiguousarray(pick("node")), None)
    want = recs.lift()
    assert np.array_equal(ref[3], want)


@pytest.mark.parametrize("n", [10_000_000, 100_000_000], ids=["10m", "100m"])
def test_full_size_config5_100m(gpu, oracle_lib, n):
    """config5 at its stated size (BASELINE configs[4]): 100 M resident 16 B / 64 B dated records,
    then 18 batches of 1 M rows -- 900 k fresh random keys, 50 k overwrites and 50 k deletes of
    resident keys each -- so the delta run passes the compaction threshold at this size (a
    111 M-row base is merged at least once).  Afterwards, against exactly the records that should be
    live (assembled and key-sorted on the host with numpy; torch's gathers with 10^8 output rows
    return wrong rows on this image: profiles/r04_torch_large_ops_repro.log): the root and size (an independent torch reduction of
    their lifts); the store's whole rank order dumped -- every key and fingerprint, row for row;
    select at 200 ranks; rank of present and absent keys; 20 rank-range and key-range aggregates;
    and the fingerprints at 20 sampled ranks against the oracle's lift of those records
    (mutate.rs:23-154 semantics)."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema, lift_records
    from rsos_hip import _abi as A
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records, to_host
    O = oracle_lib
    s = RecordSchema.dated("bytes16", "bytes64")
    m, K, touch = 1_000_000, 18, 50_000
    base = make_records(s, n, seed=5)

    def lift_host(cols):  # (rows, 32) uint8 lifts on the host, lifted in 16 M-row chunks
        rows = cols["keys"].shape[0]
        out = np.empty((rows, 32), np.uint8)
        for i in range(0, rows, 16_000_000):
            f = lift_records(s, {c: t[i:i + 16_000_000] for c, t in cols.items()}, block_sums=False)[0]
            out[i:i + 16_000_000] = f.cpu().numpy()
        return out

    bf = lift_host(base)
    st = GpuFingerprintStore(s)
    st.load_bulk_device(base)
    st.reserve(n + K * m, m)
    perm = np.random.default_rng(9).permutation(n)[:K * 2 * touch]
    batches, ops = [], []
    for k in range(K):
        ins = make_records(s, m - 2 * touch, seed=700 + k, random_keys=True)
        rows = torch.from_numpy(perm[k * 2 * touch:(k + 1) * 2 * touch]).cuda()
        ex = {c: t[rows].clone() for c, t in base.items()}
        ex["values"][:touch] ^= 0x3C  # overwrites: new values for existing keys
        ex["phys"][:touch] += 7
        b = {c: torch.cat([ins[c], ex[c]]).contiguous() for c in ins}
        o = torch.zeros(m, dtype=torch.uint8, device="cuda")
        o[m - touch:] = 1  # the last 50 k rows delete their (existing) keys
        batches.append(b)
        ops.append(o)
    comp0 = st.stats()["compactions"]
    counts = st.apply_device_many(batches, ops)
    assert counts == [(m - 2 * touch, touch, touch)] * K
    assert st.stats()["compactions"] - comp0 >= 1
    # the live set on the host: resident rows not touched, the overwritten rows' new records, the
    # inserted rows; origin r < n: base row r, n + k * m + j: row j of batch k
    keep = np.ones(n, bool)
    keep[perm] = False
    ek = [base["keys"].cpu().numpy()[keep]]
    ef = [bf[keep]]
    origin = [np.nonzero(keep)[0]]
    del bf
    for k, b in enumerate(batches):
        part = {c: t[:m - touch] for c, t in b.items()}  # inserts + overwrites
        ek.append(part["keys"].cpu().numpy())
        ef.append(lift_host(part))
        origin.append(n + k * m + np.arange(m - touch))
    ek, ef, origin = np.concatenate(ek), np.concatenate(ef), np.concatenate(origin)
    N = ek.shape[0]
    assert N == n + K * (m - 3 * touch)
    root = st.aggregate()
    assert root.size == N == st.size()
    want_root = sum(_torch_root(torch, torch.from_numpy(ef[i:i + 8_000_000]).cuda()) for i in range(0, N, 8_000_000))
    assert root.fingerprint.to_int() == want_root % M256
    # memcmp order: the big-endian leading u64 (unique across these keys), then the rest
    hi = ek[:, :8].copy().view(">u8").ravel().astype(np.uint64)
    lo = ek[:, 8:].copy().view(">u8").ravel().astype(np.uint64)
    order = np.lexsort((lo, hi))
    ek, ef, origin, hi, lo = ek[order], ef[order], origin[order], hi[order], lo[order]
    # the store's whole rank order, row for row
    dk = np.zeros(N * 16, np.uint8)
    A.check(A.lib().rh_store_keys(st._h, 0, N, dk.ctypes.data), "rh_store_keys")
    assert np.array_equal(dk.reshape(N, 16), ek)
    del dk
    assert np.array_equal(st.fingerprints(), ef)
    rng = np.random.default_rng(17)
    rs = [0, N - 1] + [int(x) for x in rng.integers(0, N, 198)]
    for r in rs:
        assert st.select(r) == ek[r].tobytes()
    for r in rs[:40]:  # present keys: their own rank; a key with its last bit flipped: counted
        assert st.rank(ek[r].tobytes()) == r
        k2 = bytearray(ek[r].tobytes())
        k2[15] ^= 1
        khi, klo = int.from_bytes(k2[:8], "big"), int.from_bytes(k2[8:], "big")
        i = int(np.searchsorted(hi, np.uint64(khi), "left"))
        while i < N and int(hi[i]) == khi and int(lo[i]) < klo:
            i += 1
        assert st.rank(bytes(k2)) == i
    for _ in range(20):
        a = int(rng.integers(0, N))
        b = min(N, a + int(rng.integers(0, 2_000_000)))
        g = st.aggregates_ranks([a], [b])[0]
        assert g.size == b - a and g.fingerprint.to_int() == _torch_root(torch, torch.from_numpy(ef[a:b]).cuda())
        g2 = st.aggregate(KeyRange(ek[a].tobytes(), ek[b].tobytes() if b < N else None))
        assert g2.size == b - a and g2.fingerprint.to_int() == g.fingerprint.to_int()
    # the fingerprints at sampled ranks against the oracle's lift of the same source records
    pick = sorted(rs[:20])
    recs = []
    for r in pick:
        o = int(origin[r])
        src, row = (base, o) if o < n else (batches[(o - n) // m], (o - n) % m)
        recs.append(to_host({c: t[row:row + 1] for c, t in src.items()}))
    h = {c: np.concatenate([x[c] for x in recs]) for c in recs[0]}
    sc = O.Schema(s.key_kind, s.key_len, s.value_kind, s.value_len, s.record_kind, 0)
    want = O.Records(sc, h["keys"], h["values"], h["phys"], h["logical"], h["node"], None).lift()
    assert np.array_equal(ef[pick], want)
    st.close()


@pytest.mark.gpu
def test_host_tier_nowait_run_refresh_equals_device_answers(gpu, monkeypatch):
    """Writes that never wait (RSOS_HIP_TIER_SYNC=0, read at store creation): a batch too large for
    the tier's tree leaves the tier stale and starts a copy of the device's delta run alone on the
    copy engines (rsos_hip_abi.hip start_run_refresh: no compaction), into the spare run set; it
    lands only if nothing was written meanwhile.  While it is in flight the device answers; once it
    has landed (tier_sync) the tier -- base copy + run copy, then the tree of later small batches
    over them -- answers ranks, selects, key-bound and rank-range aggregates and key dumps exactly
    as the device does, and no write compacted for it."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records, to_host
    monkeypatch.setenv("RSOS_HIP_TIER_TREE", "2000")
    monkeypatch.setenv("RSOS_HIP_TIER_SYNC", "0")
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 200_000
    base = make_records(s, n, seed=41)
    dev, tier = GpuFingerprintStore(s, host_tier=False), GpuFingerprintStore(s, host_tier=True)
    for st in (dev, tier):
        st.load_bulk_device(base)
    tier.tier_sync()
    rng = np.random.default_rng(19)
    seen = [to_host(base)["keys"]]

    def probe():
        assert tier.size() == dev.size() and tier.aggregate() == dev.aggregate()
        pool = np.concatenate(seen)
        ks = [pool[i].tobytes() for i in rng.integers(0, len(pool), 200)] + [rng.bytes(16) for _ in range(50)]
        karr = np.frombuffer(b"".join(ks), np.uint8).reshape(-1, 16)
        assert np.array_equal(tier.ranks(karr), dev.ranks(karr))
        size = tier.size()
        for r in [0, 1, size - 1] + list(rng.integers(0, size, 100)):
            assert tier.select(int(r)) == dev.select(int(r))
        for _ in range(80):
            a, b = ks[rng.integers(len(ks))], ks[rng.integers(len(ks))]
            rg = KeyRange(a, b, ["included", "excluded"][rng.integers(2)], ["included", "excluded"][rng.integers(2)])
            assert tier.aggregate(rg) == dev.aggregate(rg)
        lo = rng.integers(0, size, 32)
        hi = lo + rng.integers(0, 30_000, 32)
        assert tier.aggregates_ranks(list(lo), list(hi)) == dev.aggregates_ranks(list(lo), list(hi))
        lo0 = int(rng.integers(0, size - 2000))
        a0, b0 = tier.select(lo0), tier.select(lo0 + 2000)
        assert list(tier.enumerate(KeyRange(a0, b0))) == list(dev.enumerate(KeyRange(a0, b0)))

    def both(b, ops=None):
        assert tier.apply_device(b, ops) == dev.apply_device(b, ops)
        seen.append(to_host(b)["keys"])

    c0 = tier.stats()["compactions"]
    r0 = tier.tier_stats()["refreshes"]
    for k in range(3):
        b = make_records(s, 6_000, seed=700 + k, random_keys=True)
        ops = torch.zeros(6_000, dtype=torch.uint8, device="cuda")
        if k:  # overwrite base rows and delete some
            b["keys"][:400] = base["keys"][torch.from_numpy(rng.choice(n, 400, replace=False)).cuda()]
            ops[200:400] = 1
        both(b, ops)
        probe()  # the run copy in flight or landed: either way the answers are the device's
        tier.tier_sync()
        st = tier.tier_stats()
        assert st["base_rows"] == n and st["delta_entries"] == tier.stats()["delta_rows"] > 0, st
        probe()
    assert tier.stats()["compactions"] == c0  # run copies: no write compacted for the tier
    assert tier.tier_stats()["refreshes"] >= r0 + 3
    both(make_records(s, 100, seed=710, random_keys=True))  # small: folded over base + run copy
    assert tier.tier_stats()["base_rows"] == n
    probe()
    # a compaction while a run copy is in flight: the copy is relative to the tier's base and the
    # contents did not change, so it lands; the next large batch then refreshes the base
    both(make_records(s, 6_000, seed=720, random_keys=True))
    for st_ in (dev, tier):
        st_.compact()
    probe()
    tier.tier_sync()
    probe()
    both(make_records(s, 6_000, seed=721, random_keys=True))
    probe()
    tier.tier_sync()
    assert tier.tier_stats()["delta_entries"] == tier.stats()["delta_rows"]
    probe()
    # the policy switched, and the store closed, with a run copy in flight
    both(make_records(s, 6_000, seed=722, random_keys=True))
    tier.set_tier_policy(True)
    probe()
    tier.set_tier_policy(False)
    both(make_records(s, 6_000, seed=723, random_keys=True))
    tier.close()


@pytest.mark.gpu
def test_host_tier_nowait_steady_write_stream(gpu, monkeypatch):
    """Writes that never wait, back to back with no question between them: a run copy
    a write lands on is discarded, and after RUN_DISCARD_MAX such discards in a row the next write
    takes a base refresh instead (its batches logged and replayed: rsos_hip_abi.hip refresh_now).
    Whatever landed, every answer during and after the stream is the device's, and the tier is
    fresh again once the stream stops (tier_sync)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records, to_host
    monkeypatch.setenv("RSOS_HIP_TIER_TREE", "2000")
    monkeypatch.setenv("RSOS_HIP_TIER_SYNC", "0")
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 300_000
    base = make_records(s, n, seed=43)
    dev, tier = GpuFingerprintStore(s, host_tier=False), GpuFingerprintStore(s, host_tier=True)
    for st in (dev, tier):
        st.load_bulk_device(base)
    tier.tier_sync()
    rng = np.random.default_rng(23)
    keys = [to_host(base)["keys"]]
    for k in range(24):
        b = make_records(s, 8_000 + 500 * k, seed=800 + k, random_keys=True)
        assert tier.apply_device(b) == dev.apply_device(b)
        keys.append(to_host(b)["keys"])
        if k % 6 == 5:  # now and then a few questions mid-stream (stale or fresh: the device's answers)
            pool = np.concatenate(keys)
            ks = np.ascontiguousarray(pool[rng.integers(0, len(pool), 64)])
            assert np.array_equal(tier.ranks(ks), dev.ranks(ks))
            assert tier.aggregate() == dev.aggregate()
    tier.tier_sync()
    st = tier.tier_stats()
    assert st["base_rows"] > 0, st  # fresh (a stale tier reports 0)
    assert tier.size() == dev.size() and tier.aggregate() == dev.aggregate()
    for _ in range(40):
        r = int(rng.integers(0, dev.size()))
        assert tier.select(r) == dev.select(r)
        a, b2 = dev.select(int(rng.integers(0, dev.size()))), dev.select(int(rng.integers(0, dev.size())))
        assert tier.aggregate(KeyRange(a, b2)) == dev.aggregate(KeyRange(a, b2))
    for st_ in (dev, tier):
        st_.close()


@pytest.mark.gpu
def test_host_tier_run_copy_equals_device_answers(gpu, monkeypatch):
    """Batches too large for the tier's tree (RSOS_HIP_TIER_TREE=2000 here, read at store creation)
    take a copy of the device's delta run instead of a refresh of the whole base
    (rsos_hip_abi.hip tier_run_snapshot, host_tier.hpp HostTier::Run): inserts, overwrites and
    deletes of base keys, deletes of keys a previous batch inserted, re-inserts.  After each, the
    tier -- base copy + run copy, and the tree of the small batches folded over them -- answers
    ranks of present and absent keys, select at every kind of rank, key-bound aggregates of every
    bound kind, rank-range aggregates and key dumps exactly as the device does; small batches
    after a run copy fold into the tree (no copy), a large batch after a compaction refreshes the
    base instead."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records, to_host
    monkeypatch.setenv("RSOS_HIP_TIER_TREE", "2000")
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 200_000
    base = make_records(s, n, seed=31)
    dev, tier = GpuFingerprintStore(s, host_tier=False), GpuFingerprintStore(s, host_tier=True)
    for st in (dev, tier):
        st.load_bulk_device(base)
    rng = np.random.default_rng(9)
    keys_h = to_host(base)["keys"]
    seen, fresh = [keys_h], []

    def probe():
        assert tier.size() == dev.size() and tier.aggregate() == dev.aggregate()
        pool = np.concatenate(seen)
        ks = [pool[i].tobytes() for i in rng.integers(0, len(pool), 300)] + [rng.bytes(16) for _ in range(100)]
        ks += [b"\x00" * 16, b"\xff" * 16]
        karr = np.frombuffer(b"".join(ks), np.uint8).reshape(-1, 16)
        assert np.array_equal(tier.ranks(karr), dev.ranks(karr))
        size = tier.size()
        for r in [0, 1, size - 1] + list(rng.integers(0, size, 200)):
            assert tier.select(int(r)) == dev.select(int(r))
        for _ in range(150):
            a, b = ks[rng.integers(len(ks))], ks[rng.integers(len(ks))]
            sk, ek = ["included", "excluded"][rng.integers(2)], ["included", "excluded"][rng.integers(2)]
            rg = KeyRange(a if rng.random() > 0.1 else None, b if rng.random() > 0.1 else None, sk, ek)
            assert tier.aggregate(rg) == dev.aggregate(rg)
        lo = rng.integers(0, size, 64)
        hi = lo + rng.integers(0, 30_000, 64)
        assert tier.aggregates_ranks(list(lo), list(hi)) == dev.aggregates_ranks(list(lo), list(hi))
        lo0 = int(rng.integers(0, size - 3000))
        a0, b0 = tier.select(lo0), tier.select(lo0 + 3000)
        assert list(tier.enumerate(KeyRange(a0, b0))) == list(dev.enumerate(KeyRange(a0, b0)))  # rh_store_keys

    def both(b, ops=None):
        assert tier.apply_device(b, ops) == dev.apply_device(b, ops)

    def large(seed, over=0):
        b = make_records(s, 6_000, seed=seed, random_keys=True)
        ops = torch.zeros(6_000, dtype=torch.uint8, device="cuda")
        if over:  # overwrite and delete resident keys, delete keys an earlier batch inserted
            rows = torch.from_numpy(rng.choice(n, 2 * over, replace=False)).cuda()
            b["keys"][:2 * over] = base["keys"][rows]
            b["phys"][:2 * over] = base["phys"][rows] + 7
            ops[over:2 * over] = 1
            prev = torch.from_numpy(fresh[-1][:over].copy()).cuda()  # keys the last large batch inserted
            b["keys"][2 * over:3 * over] = prev
            ops[2 * over:3 * over] = 1
        kh = to_host(b)["keys"]
        seen.append(kh)
        fresh.append(kh[3 * over:])
        return b, ops

    probe()
    r0 = tier.tier_stats()["refreshes"]
    b, o = large(600)
    both(b, o)
    st = tier.tier_stats()
    # (the tier's own device delta run: the device-only store compacts for its selects)
    assert st["refreshes"] == r0 + 1 and st["delta_entries"] == tier.stats()["delta_rows"] and st["base_rows"] == n
    probe()
    b, o = large(601, over=800)  # a second run copy over the first's keys
    both(b, o)
    assert tier.tier_stats()["delta_entries"] == tier.stats()["delta_rows"]
    probe()
    st0 = tier.tier_stats()
    small = make_records(s, 100, seed=602, random_keys=True)
    both(small)  # after a run copy: folded into the tree over base + run copy (no copy)
    ov = {c: t[:300].clone() for c, t in base.items()}  # overwrites of base rows the run holds or not
    ov["values"] ^= 0x21
    dl = torch.ones(300, dtype=torch.uint8, device="cuda")
    both({c: t[300:600].clone() for c, t in base.items()}, dl)  # deletes of base rows
    both(ov)
    both({c: t[:50].clone() for c, t in b.items()}, torch.ones(50, dtype=torch.uint8, device="cuda"))  # run keys deleted
    st = tier.tier_stats()
    assert st["refreshes"] == st0["refreshes"] and st["folds"] == st0["folds"] + 4
    probe()
    b, o = large(603, over=500)
    both(b, o)
    assert tier.tier_stats()["delta_entries"] == tier.stats()["delta_rows"] > 0
    probe()
    for st_ in (dev, tier):
        st_.compact()
    b, o = large(604, over=300)  # after a compaction the run would not match the tier's base
    both(b, o)
    assert tier.tier_stats()["delta_entries"] == 0
    probe()
    # a run copy that fails for want of host memory: the batch still commits, the tier goes stale
    # (the device answers), and the next write brings it back
    from rsos_hip import _abi as A
    b, o = large(605, over=200)
    A.lib().rh_debug_fail_point(b"tier.run_copy")
    both(b, o)
    A.lib().rh_debug_fail_point(b"")
    assert tier.tier_stats()["base_rows"] == 0  # stale
    probe()
    both(make_records(s, 10, seed=606, random_keys=True))
    assert tier.tier_stats()["base_rows"] > 0
    probe()
    dev.close()
    tier.close()


@pytest.mark.gpu
def test_search_table_with_bunched_keys(gpu):
    """Keys bunched in one corner of their digit range (the leading 8 bytes below 2^40), then a
    batch of uniformly random keys: the search tables' buckets are almost all one long gap
    (k_search_table leaves it to k_search_table_gaps).  Ranks of present and absent keys, selects
    and the key dump equal numpy's sort of the same set, before and after a compaction."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.synth import make_records
    s = RecordSchema.plain("bytes16", "u64")
    n = 300_000
    rng = np.random.default_rng(17)
    hi8 = np.sort(rng.choice(1 << 40, n, replace=False)).astype(">u8")
    keys = np.zeros((n, 16), np.uint8)
    keys[:, :8] = hi8.view(np.uint8).reshape(n, 8)
    keys[:, 8:] = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    base = {"keys": torch.from_numpy(keys).cuda(), "values": torch.from_numpy(rng.integers(0, 256, (n, 8), dtype=np.uint8)).cuda()}
    st = GpuFingerprintStore(s, host_tier=False)
    st.load_bulk_device(base)
    b = make_records(s, 50_000, seed=5, random_keys=True)
    st.apply_device(b)
    allk = np.concatenate([keys, b["keys"].cpu().numpy()])
    srt = allk[np.lexsort(allk.T[::-1])]
    view = srt.view("S16").ravel()

    def check():
        probes = np.concatenate([allk[rng.integers(0, len(allk), 2000)], rng.integers(0, 256, (2000, 16), dtype=np.uint8)])
        want = np.searchsorted(view, probes.view("S16").ravel(), side="left")
        assert np.array_equal(st.ranks(probes).astype(np.int64), want)
        for r in rng.integers(0, len(srt), 100):
            assert st.select(int(r)) == srt[r].tobytes()

    check()
    st.compact()
    check()
    st.close()


@pytest.mark.gpu
def test_tier_policy_switch(gpu):
    """rh_store_set_tier_policy: with writes never waiting, a batch past the tier's tree returns at
    once and questions may go to the device while the copy is in flight; switched back, the next
    such batch leaves the tier fresh (base copy or run copy).  Answers equal the device path's
    either way."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.synth import make_records, to_host
    s = RecordSchema.dated("bytes16", "bytes64")
    n = 100_000
    base = make_records(s, n, seed=41)
    dev, tier = GpuFingerprintStore(s, host_tier=False), GpuFingerprintStore(s, host_tier=True)
    for st in (dev, tier):
        st.load_bulk_device(base)
    rng = np.random.default_rng(3)
    pool = to_host(base)["keys"]

    def same():
        ks = np.concatenate([pool[rng.integers(0, n, 300)], rng.integers(0, 256, (100, 16), dtype=np.uint8)])
        assert np.array_equal(tier.ranks(ks), dev.ranks(ks))
        assert tier.aggregate() == dev.aggregate()
        for r in rng.integers(0, dev.size(), 50):
            assert tier.select(int(r)) == dev.select(int(r))

    tier.set_tier_policy(False)
    b = make_records(s, 70_000, seed=42, random_keys=True)
    assert tier.apply_device(b) == dev.apply_device(b)
    same()
    tier.set_tier_policy(True)
    b = make_records(s, 70_000, seed=43, random_keys=True)
    assert tier.apply_device(b) == dev.apply_device(b)
    assert tier.tier_stats()["base_rows"] > 0  # fresh right after the write
    same()
    dev.close()
    tier.close()


@pytest.mark.gpu
def test_waited_launches_ignore_a_stale_sequence_word(gpu):
    """The one-launch device paths -- a tiny protocol round (k_round_tiny), a tiny rank / select /
    aggregate (k_query_tiny), a small batch (k_small_batch) -- return when the kernel's sequence
    word lands in page-locked memory.  That memory may already hold the very number the next
    launch will store: a larger round's header is copied over the round buffer, and page-locked
    memory the runtime reuses after a store is destroyed keeps its last owner's words (a sharded
    round once read a shard's previous answer this way).  So the word is cleared before every such
    launch.  The fail points put the next number there first; every answer must still equal an
    identical store's (host tiers off: the device answers)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R, _abi as A
    from rsos_hip.store import KeyRange
    sch = RecordSchema.plain("u64", "u64")
    rng = np.random.default_rng(77)
    keys = np.unique(rng.integers(0, 1 << 40, 50000, dtype=np.uint64))
    cols = {"keys": keys.view(np.uint8).reshape(-1, 8), "values": (keys * 3).view(np.uint8).reshape(-1, 8)}
    a = GpuFingerprintStore(sch, host_tier=False)
    b = GpuFingerprintStore(sch, host_tier=False)
    peer = GpuFingerprintStore(sch, host_tier=False)
    for st in (a, b):
        st.load_bulk(cols)
    pv = cols["values"].copy()
    pv[rng.random(len(keys)) < 0.02] ^= 5
    peer.load_bulk({"keys": cols["keys"], "values": pv})

    def rounds_equal(segs, point):
        ch_b, en_b = [], []
        ob = R.protocol_round_with_policy(b, R.FixedFanOut(16), segs, ch_b, en_b)
        ch_a, en_a = [], []
        if point:
            A.check(A.lib().rh_debug_fail_point(point), "fail point")
        try:
            oa = R.protocol_round_with_policy(a, R.FixedFanOut(16), segs, ch_a, en_a)
        finally:
            A.lib().rh_debug_fail_point(b"")
        assert oa == ob
        assert [(c.start, c.end, c.aggregate) for c in ch_a] == [(c.start, c.end, c.aggregate) for c in ch_b]
        assert en_a == en_b
        return ch_b

    # the peer's children of the whole range, then of those: hundreds of segments
    active = R.initial_ranges(a)
    for side in (peer, b):
        ch, en = [], []
        R.protocol_round_with_policy(side, R.FixedFanOut(16), active, ch, en)
        active = ch
    assert len(active) > 100
    for t in range(12):
        if t % 3 == 0:
            rounds_equal(active, None)  # a large round: its header lands in the round buffer
        m = int(rng.integers(1, 13))
        rounds_equal([active[i] for i in rng.permutation(len(active))[:m]], b"round.stale_seq")
    # tiny questions
    for t in range(8):
        z = int(keys[int(rng.integers(0, len(keys)))]) + int(rng.integers(0, 2))
        A.check(A.lib().rh_debug_fail_point(b"query.stale_seq"), "fail point")
        assert a.rank(z) == b.rank(z)
        r = int(rng.integers(0, len(keys)))
        A.check(A.lib().rh_debug_fail_point(b"query.stale_seq"), "fail point")
        assert a.select(r) == b.select(r)
        lo, hi = sorted(int(x) for x in rng.integers(0, 1 << 40, 2))
        A.check(A.lib().rh_debug_fail_point(b"query.stale_seq"), "fail point")
        assert a.aggregate(KeyRange(lo, hi)) == b.aggregate(KeyRange(lo, hi))
    A.lib().rh_debug_fail_point(b"")
    # small batches
    for t in range(6):
        k = rng.integers(0, 1 << 40, 3, dtype=np.uint64)
        one = {"keys": k.view(np.uint8).reshape(-1, 8), "values": (k * 11).view(np.uint8).reshape(-1, 8)}
        ops = np.zeros(3, np.uint8)
        counts_b = b.apply(one, ops)
        A.check(A.lib().rh_debug_fail_point(b"small_batch.stale_seq"), "fail point")
        try:
            counts_a = a.apply(one, ops)
        finally:
            A.lib().rh_debug_fail_point(b"")
        assert counts_a == counts_b
        assert a.size() == b.size() and a.aggregate() == b.aggregate()
    assert a.batch_stats()["small"] >= 6
    for st in (a, b, peer):
        st.close()
