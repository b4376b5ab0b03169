"""The sharded store (rh_sstore_*, csrc/sharded_store.hip): one map over key-range shards, here 4
shards on device 0 (the GPU box has one GPU; the shards' streams, threads and decomposition are
the same whatever device each sits on).

Against one rh_store holding the same records and against the oracle's fold (FingerprintTreeMap's
semantics over oracle.c's lifts, rsos/src/fingerprint_tree_map/mutate.rs:23-154): the root, sizes,
ranks, selects, key-range aggregates with every bound kind, rank-range aggregates across shard
boundaries, key and fingerprint dumps, and whole FixedFanOut / SqrtFanOut reconciliations
(rbsr/src/protocol.rs:212-317) round by round -- after a load and after routed batches (rh_sstore_apply)
and staged rows (rh_sstore_stage), with the shards' host tiers off and on; plus the edge cases: an
empty map, fewer rows than shards, even splitters before the first load, a rejected batch leaving
every shard unchanged, an unsorted load leaving the map empty."""
import ctypes as C

import numpy as np
import pytest

from test_small_batch import M256, Model, _batch, _gen

G = 4


def _sorted_unique(sch, cols):
    k = cols["keys"]
    if sch.key_kind in (1, 2):
        order = np.argsort(k.copy().view("<u4" if sch.key_row == 4 else "<u8").ravel(), kind="stable")
    else:
        order = np.lexsort(k.T[::-1])
    cols = {c: v[order] for c, v in cols.items()}
    _, first = np.unique(cols["keys"], axis=0, return_index=True)
    keep = np.sort(first)
    return {c: v[keep] for c, v in cols.items()}


def _fp_int(agg):
    return sum(int(x) << (64 * i) for i, x in enumerate(agg.fingerprint.limbs))


def _want_range(model, sch, lo, lk, hi, hk):
    """the oracle fold over keys in the range (bound kinds 'included' / 'excluded' / 'unbounded')"""
    from test_small_batch import _order
    tot, n = 0, 0
    for k, f in model.d.items():
        o = _order(sch, k)
        if lk == "included" and o < lo or lk == "excluded" and o <= lo:
            continue
        if hk == "excluded" and o >= hi or hk == "included" and o > hi:
            continue
        tot += int.from_bytes(f, "little")
        n += 1
    return tot % M256, n


def _drive(a, b, policy):
    """a whole reconciliation between two maps, native rounds: every round's output"""
    from rsos_hip import rbsr as R
    out, active, sides, k = [], R.initial_ranges(a), [b, a], 0
    while active and k < 64:
        ch, en = [], []
        o = R.protocol_round_with_policy(sides[k % 2], policy, active, ch, en)
        out.append(([(c.start, c.end, c.aggregate) for c in ch], en,
                    (o.skipped, o.enumerated, o.split, o.children, o.dropped_malformed)))
        active, k = ch, k + 1
    return out


def _check_same(sh, one, model, sch, rng):
    from rsos_hip.store import KeyRange
    n = one.size()
    assert sh.size() == n == len(model.d)
    assert sum(sh.sizes()) == n
    root = sh.aggregate()
    assert root == one.aggregate()
    assert (_fp_int(root), root.size) == model.root()
    keys = model.sorted_keys()
    key_out = one._key_out
    # every shard holds exactly its splitter range
    spl = sh.splitters
    from test_small_batch import _order
    ok = lambda k: _order(sch, one._key_bytes(k))  # noqa: E731
    r0 = 0
    for s, size in enumerate(sh.sizes()):
        for r in (r0, r0 + size - 1) if size else ():
            k = ok(one.select(r))
            if s > 0:
                assert k >= ok(spl[s - 1])
            if s < len(sh.sizes()) - 1:
                assert k < ok(spl[s])
        r0 += size
    # ranks: random probes, the stored keys, the splitters
    probes = [key_out(rng.integers(0, 256, sch.key_row, dtype=np.uint8).tobytes()) for _ in range(60)]
    probes += [key_out(keys[i]) for i in rng.integers(0, max(n, 1), 40)] if n else []
    probes += list(spl)
    for z in probes:
        assert sh.rank(z) == one.rank(z)
    pk = np.stack([np.frombuffer(one._key_bytes(z), np.uint8) for z in probes])
    assert (sh.ranks(pk) == one.ranks(pk)).all()
    # selects, including both sides of every shard boundary
    offs = np.cumsum([0] + sh.sizes())
    rs = sorted(set([int(x) for x in rng.integers(0, max(n, 1), 60)] +
                    [int(o) + d for o in offs[1:-1] for d in (-1, 0)] + [0, n - 1]))
    for r in rs:
        if 0 <= r < n:
            assert sh.select(r) == one.select(r) == key_out(keys[r])
    with pytest.raises(IndexError):
        sh.select(n)
    # key-range aggregates with every bound kind
    kinds = ["included", "excluded"]
    for i in range(40):
        i0, i1 = (int(x) for x in rng.integers(0, len(probes), 2))
        a, b = sorted((probes[i0], probes[i1]), key=ok)
        if i % 5 == 0:
            a, b = b, a  # inverted: ZERO
        lk, hk = kinds[i % 2], kinds[(i // 2) % 2]
        for rng_ in (KeyRange(a, b, lk, hk), KeyRange(None, b, end_kind=hk), KeyRange(a, None, start_kind=lk)):
            got = sh.aggregate(rng_)
            assert got == one.aggregate(rng_)
            want = _want_range(model, sch, ok(a) if rng_.start is not None else None, rng_.start_kind,
                               ok(b) if rng_.end is not None else None, rng_.end_kind)
            assert (_fp_int(got), got.size) == want
    # rank-range aggregates: across boundaries, inverted, past the end
    lo = [int(x) for x in rng.integers(0, n + 5, 50)] + [int(o) - 3 for o in offs[1:-1]] + [n - 1, 5]
    hi = [int(x) for x in rng.integers(0, n + 5, 50)] + [int(o) + 3 for o in offs[1:-1]] + [n + 10, 2]
    lo = [max(x, 0) for x in lo]
    assert sh.aggregates_ranks(lo, hi) == one.aggregates_ranks(lo, hi)
    # dumps across the boundaries
    if n:
        a, b = max(int(offs[1]) - 7, 0), min(int(offs[-2]) + 7, n)
        kd1 = np.zeros((b - a) * sch.key_row, np.uint8)
        kd2 = np.zeros_like(kd1)
        from rsos_hip import _abi as A
        A.check(A.lib().rh_sstore_keys(sh._h, a, b, kd1.ctypes.data), "keys")
        A.check(A.lib().rh_store_keys(one._h, a, b, kd2.ctypes.data), "keys")
        assert (kd1 == kd2).all()
        assert (sh.fingerprints(a, b) == one.fingerprints(a, b)).all()


SHARD_SCHEMAS = [("dated", "bytes16", "bytes64", True), ("plain", "u64", "u64", False)]


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [G, 8])
@pytest.mark.parametrize("tier", [False, True], ids=["device", "host_tier"])
@pytest.mark.parametrize("spec", SHARD_SCHEMAS, ids=lambda s: f"{s[0]}-{s[1]}-{s[2]}")
def test_sharded_equals_single_store_and_oracle(gpu, oracle_lib, spec, tier, shards):
    """Everything the map answers, against one store and the oracle fold; with 8 shards on the one
    device two share an issuing thread (at most 4 per device)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    from rsos_hip.sharded import ShardedStore
    kind, kk, vk, tomb = spec
    sch = getattr(RecordSchema, kind)(kk, vk)
    rng = np.random.default_rng(11)
    model = Model(oracle_lib, sch)
    cols = _sorted_unique(sch, _gen(rng, sch, 30000, tomb))
    one = GpuFingerprintStore(sch, host_tier=tier)
    sh = ShardedStore(sch, [0] * shards, host_tier=tier)
    peer = GpuFingerprintStore(sch, host_tier=tier)
    one.load_bulk(cols)
    sh.load_bulk(cols)
    model.apply(cols, np.zeros(len(cols["keys"]), np.uint8))
    n = len(model.d)
    assert sh.sizes() == [n * (s + 1) // shards - n * s // shards for s in range(shards)]  # equal-count cuts
    _check_same(sh, one, model, sch, rng)
    # the peer: the same records with some missing and some re-stamped
    pc = {c: v.copy() for c, v in cols.items()}
    drop = rng.random(n) < 0.002
    pc["values"][rng.random(n) < 0.002] ^= 1
    peer.load_bulk({c: v[~drop] for c, v in pc.items()})
    for policy in (R.FixedFanOut(16), R.SqrtFanOut()):
        assert _drive(sh, peer, policy) == _drive(one, peer, policy)
    # routed batches (distinct keys) and staged rows (repeats keep the last operation)
    for step in range(4):
        b, ops = _batch(rng, sch, model, [3000, 700, 40, 5000][step], tomb)
        assert sh.apply(b, ops) == one.apply(b, ops) == model.apply(b, ops)
        b, ops = _batch(rng, sch, model, [1, 300, 2000, 9][step], tomb, repeats=True)
        for st in (sh, one):
            if step == 0:  # one row at a time, as Rsos::insert stages it
                for i in range(len(ops)):
                    st.stage({c: v[i:i + 1] for c, v in b.items()}, ops[i:i + 1])
            else:
                st.stage(b, ops)
        model.apply(b, ops)
        _check_same(sh, one, model, sch, rng)
        assert _drive(sh, peer, R.FixedFanOut(16)) == _drive(one, peer, R.FixedFanOut(16))
    # the two-call path over the sharded map (any policy)
    got = []
    a = R.initial_ranges(sh)
    while a:
        ch, en = [], []
        R.protocol_round_with_policy(peer, R.FixedFanOut(4), a, ch, en, native=False)
        ch2, en2 = [], []
        R.protocol_round_with_policy(sh, R.FixedFanOut(4), ch, ch2, en2, native=False)
        ch3, en3 = [], []
        R.protocol_round_with_policy(one, R.FixedFanOut(4), ch, ch3, en3, native=False)
        assert [(c.start, c.end, c.aggregate) for c in ch2] == [(c.start, c.end, c.aggregate) for c in ch3]
        assert en2 == en3
        got.append(len(ch2))
        a = ch2
    assert len(got) >= 2
    for s in (one, peer, sh):
        s.close()


@pytest.mark.gpu
def test_sharded_edge_cases(gpu, oracle_lib):
    from rsos_hip import GpuFingerprintStore, RecordSchema, _abi as A, rbsr as R
    from rsos_hip.sharded import ShardedStore
    from rsos_hip.store import KeyRange
    sch = RecordSchema.plain("u64", "u64")
    rng = np.random.default_rng(5)
    sh = ShardedStore(sch, [0] * G)
    # empty: even splitters over the u64 key space
    assert sh.size() == 0 and sh.aggregate().size == 0
    assert sh.splitters == [(2**64 * j) // G for j in range(1, G)]
    assert sh.rank(12345) == 0
    with pytest.raises(IndexError):
        sh.select(0)
    # single inserts into the empty map spread over every shard by the even cut
    model = Model(oracle_lib, sch)
    b = _gen(rng, sch, 400, False)
    for i in range(400):
        sh.stage({c: v[i:i + 1] for c, v in b.items()}, np.zeros(1, np.uint8))
    model.apply(b, np.zeros(400, np.uint8))
    assert sh.size() == 400 and all(s > 50 for s in sh.sizes())
    assert (_fp_int(sh.aggregate()), sh.size()) == model.root()
    # splitters are only settable while empty
    with pytest.raises(A.RsosHipError):
        sh.set_splitters([1, 2, 3])
    # fewer rows than shards
    few = _sorted_unique(sch, _gen(rng, sch, 2, False))
    sh.load_bulk(few)
    one = GpuFingerprintStore(sch)
    one.load_bulk(few)
    assert sh.size() == 2 and sh.aggregate() == one.aggregate() and sum(1 for s in sh.sizes() if s) == 2
    assert [sh.select(r) for r in range(2)] == [one.select(r) for r in range(2)]
    peer = GpuFingerprintStore(sch)
    peer.load_bulk(_sorted_unique(sch, _gen(rng, sch, 50, False)))
    assert _drive(sh, peer, R.FixedFanOut(16)) == _drive(one, peer, R.FixedFanOut(16))
    # a batch with a repeated key changes no shard
    cols = _sorted_unique(sch, _gen(rng, sch, 5000, False))
    sh.load_bulk(cols)
    before = (sh.aggregate(), sh.sizes())
    bad = _gen(rng, sch, 100, False)
    bad["keys"][7] = bad["keys"][60]
    with pytest.raises(A.RsosHipError) as e:
        sh.apply(bad, np.zeros(100, np.uint8))
    assert e.value.code == A.ERR_ARG and (sh.aggregate(), sh.sizes()) == before
    # an unsorted load is refused and leaves the map empty (as one store's)
    un = {c: v[::-1].copy() for c, v in cols.items()}
    with pytest.raises(A.RsosHipError):
        sh.load_bulk(un)
    assert sh.size() == 0 and sh.aggregate().size == 0
    # an empty load, then set_splitters, then routed rows
    sh.load_bulk({c: v[:0] for c, v in cols.items()})
    sh.set_splitters([10, 20, 30])
    assert sh.splitters == [10, 20, 30]
    keys = np.arange(40, dtype=np.uint64)
    vals = keys * 7
    sh.apply({"keys": keys.view(np.uint8).reshape(-1, 8), "values": vals.view(np.uint8).reshape(-1, 8)},
             np.zeros(40, np.uint8))
    assert sh.sizes() == [10, 10, 10, 10]
    assert sh.aggregate(KeyRange(10, 30)).size == 20 and sh.rank(25) == 25 and sh.select(31) == 31
    # a bad op anywhere in a batch spanning every shard is refused before any shard changes
    before = (sh.aggregate(), sh.sizes())
    ops = np.zeros(40, np.uint8)
    ops[33] = 2
    with pytest.raises(A.RsosHipError) as e:
        sh.apply({"keys": keys.view(np.uint8).reshape(-1, 8), "values": (vals + 1).view(np.uint8).reshape(-1, 8)}, ops)
    assert e.value.code == A.ERR_ARG and (sh.aggregate(), sh.sizes()) == before
    for s in (one, peer, sh):
        s.close()


@pytest.mark.gpu
def test_sharded_failed_apply_is_sticky_until_a_load(gpu):
    """A device or allocation failure in one shard's part of a batch, after the batch's checks, may
    leave the other shards' parts committed: the sharded store then refuses every call with
    RH_ERR_STATE (never a half-applied answer) until a load replaces the contents.  Closing the
    store detaches the shard views."""
    from rsos_hip import RecordSchema, _abi as A
    from rsos_hip.sharded import ShardedStore
    sch = RecordSchema.plain("u64", "u64")
    sh = ShardedStore(sch, [0] * G)
    keys = np.arange(4000, dtype=np.uint64)
    cols = {"keys": keys.view(np.uint8).reshape(-1, 8), "values": (keys * 3).view(np.uint8).reshape(-1, 8)}
    sh.load_bulk(cols)
    root = sh.aggregate()
    batch = {"keys": keys[::7].copy().view(np.uint8).reshape(-1, 8),
             "values": (keys[::7] * 5).view(np.uint8).reshape(-1, 8)}
    A.lib().rh_debug_fail_point(b"sstore.apply_last_shard")
    with pytest.raises(A.RsosHipError) as e:
        sh.apply(batch, np.zeros(len(keys[::7]), np.uint8))
    A.lib().rh_debug_fail_point(b"")
    assert e.value.code == A.ERR_OOM
    for call in (sh.size, sh.aggregate, lambda: sh.rank(5), lambda: sh.select(0)):
        with pytest.raises(A.RsosHipError) as e:
            call()
        assert e.value.code == A.ERR_STATE and "load to recover" in str(e.value)
    sh.load_bulk(cols)
    assert sh.size() == 4000 and sh.aggregate() == root
    shard0 = sh.shards[0]
    assert shard0.size() == 1000
    sh.close()
    with pytest.raises(ValueError):
        shard0.size()


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [4, 8])
@pytest.mark.parametrize("tier", [False, True], ids=["device", "host_tier"])
def test_sharded_rounds_any_segment_order(gpu, tier, shards):
    """A round's segments normally arrive in key order (a peer's children), which the sharded store
    routes by 2 (G - 1) binary searches and then verifies (csrc/sharded_store.hip route_sorted).  Out
    of order -- shuffled children, overlapping and inverted segments, unbounded ones in the middle,
    as a malformed or hostile peer may send -- the verification fails and every segment is routed on
    its own (route_each); either way the round equals one store's segment for segment, in the input
    order, for rounds small enough for the host tier and large enough for the device.  With 8
    shards on the one device a thread drives two of them (at most 4 threads per device), issuing
    both device rounds before completing either."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    from rsos_hip.sharded import ShardedStore
    sch = RecordSchema.plain("u64", "u64")
    rng = np.random.default_rng(31)
    keys = np.unique(rng.integers(0, 1 << 40, 60000, dtype=np.uint64))
    cols = {"keys": keys.view(np.uint8).reshape(-1, 8), "values": (keys * 7).view(np.uint8).reshape(-1, 8)}
    one = GpuFingerprintStore(sch, host_tier=tier)
    sh = ShardedStore(sch, [0] * shards, host_tier=tier)
    peer = GpuFingerprintStore(sch, host_tier=tier)
    for st in (one, sh):
        st.load_bulk(cols)
    pv = cols["values"].copy()
    pv[rng.random(len(keys)) < 0.01] ^= 3
    peer.load_bulk({"keys": cols["keys"], "values": pv})
    # three rounds in (peer, one, peer): hundreds of key-ordered children from the peer
    active = R.initial_ranges(sh)
    for side in (peer, one, peer):
        ch, en = [], []
        R.protocol_round_with_policy(side, R.FixedFanOut(16), active, ch, en)
        active = ch
    assert len(active) > 200

    def same(segs):
        a_ch, a_en, b_ch, b_en = [], [], [], []
        oa = R.protocol_round_with_policy(sh, R.FixedFanOut(16), segs, a_ch, a_en)
        ob = R.protocol_round_with_policy(one, R.FixedFanOut(16), segs, b_ch, b_en)
        assert oa == ob
        assert [(c.start, c.end, c.aggregate) for c in a_ch] == [(c.start, c.end, c.aggregate) for c in b_ch]
        assert a_en == b_en

    same(active)  # key-ordered: the fast routing
    for m in (12, 100, len(active)):  # host-tier sized and device sized
        segs = [active[i] for i in rng.permutation(len(active))[:m]]
        same(segs)
        # overlapping, inverted and unbounded segments mixed in
        extra = []
        for s in segs[:5]:
            extra.append(R.RangeAggregate(s.end, s.start, s.aggregate) if s.start is not None and s.end is not None
                         else s)
            extra.append(R.RangeAggregate(None, s.end, s.aggregate))
            extra.append(R.RangeAggregate(s.start, None, s.aggregate))
        same(segs[: m // 2] + extra + segs[m // 2:])
    for st in (one, sh, peer):
        st.close()
