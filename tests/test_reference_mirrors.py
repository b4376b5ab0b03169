"""The reference's own tests of this path, restated against the GPU store.

  aggregate_matches_brute_force_for_every_boundary_pair
      rsos/src/fingerprint_tree_map/tests/aggregate.rs:59-78 (100 u32/u32 keys, every lo..hi)
  big_test          tests/basic.rs: 1,000 random u64/u64 inserts, the root checked
                    after each, partition additivity, rank / select
  test_compare / diff / reconcile
      tests/diff.rs:12-108: the two-tree diff driver over rbsr, its expected ranges, and
      reconcile() bringing both trees to the same content

The reference's trees hold `&str` values in test_compare; the ranges the diff reports depend only
on which keys differ, so the restatement uses u32 values (the store needs fixed-width values).
"""
import numpy as np
import pytest

import oracle as O
import rbsr as OR  # oracle/rbsr.py


@pytest.fixture(autouse=True, params=["device", "host_tier"])
def store_tier(request):
    """Every GPU store of this module answers from the device, then from the host tier
    (rh_store_set_host_tier): the answers must be identical."""
    import rsos_hip.store as S
    old = S.DEFAULT_HOST_TIER
    S.DEFAULT_HOST_TIER = request.param == "host_tier"
    yield request.param
    S.DEFAULT_HOST_TIER = old


def _u32_recs(pairs):
    pairs = sorted(pairs)
    k = np.array([a for a, _ in pairs], np.uint32)
    v = np.array([b for _, b in pairs], np.uint32)
    n = len(pairs)
    return O.Records(O.Schema(O.KEY_U32, 4, O.VAL_U32, 4, O.REC_PLAIN, 0), k.view(np.uint8).reshape(n, 4),
                     v.view(np.uint8).reshape(n, 4))


def _ftm(recs):
    t = O.FingerprintTreeMap(recs)
    t.fill(0, recs.n)
    return t


def oracle_diff(a, b):
    """tests/diff.rs:12-37 over the oracle: (ranges a owes b, ranges b owes a)."""
    da, db = [], []
    seg_a = OR.initial_ranges(a)
    while seg_a:
        seg_b = []
        OR.protocol_round(b, OR.fixed_fan_out(16), seg_a, seg_b, db)
        seg_a = []
        OR.protocol_round(a, OR.fixed_fan_out(16), seg_b, seg_a, da)
    return da, db


def gpu_diff(a, b):
    """The same driver on two GPU stores (rsos_hip.rbsr, the library's native round)."""
    from rsos_hip import rbsr as R
    da, db = [], []
    seg_a = R.initial_ranges(a)
    while seg_a:
        seg_b = []
        R.protocol_round(b, seg_a, seg_b, db)
        seg_a = []
        R.protocol_round(a, seg_b, seg_a, da)
    return da, db


def _u32_store(pairs):
    from rsos_hip import GpuFingerprintStore, RecordSchema
    pairs = sorted(pairs)
    st = GpuFingerprintStore(RecordSchema.plain("u32", "u32"))
    k = np.array([a for a, _ in pairs], np.uint32).view(np.uint8).reshape(-1, 4)
    v = np.array([b for _, b in pairs], np.uint32).view(np.uint8).reshape(-1, 4)
    st.load_bulk({"keys": k, "values": v})
    return st


TREES = {
    1: [(25, 1), (50, 2), (75, 3)],
    4: [(75, 3), (25, 1), (40, 2)],
    5: [(25, 1), (50, 2), (75, 4)],
}
EXPECT = {  # tests/diff.rs:79-95
    1: ([], []),
    4: ([(40, 75)], [(40, 75)]),
    5: ([(75, None)], [(75, None)]),
}


def test_compare_oracle(oracle_lib):
    t1 = OR.FtmView(_ftm(_u32_recs(TREES[1])), True)
    for j in (1, 4, 5):
        tj = OR.FtmView(_ftm(_u32_recs(TREES[j])), True)
        assert oracle_diff(t1, tj) == EXPECT[j]


@pytest.mark.gpu
def test_compare_gpu(gpu):
    s1 = _u32_store(TREES[1])
    for j in (1, 4, 5):
        sj = _u32_store(TREES[j])
        assert (s1.aggregate() == sj.aggregate()) == (j == 1)
        assert gpu_diff(s1, sj) == EXPECT[j]
        sj.close()
    s1.close()


@pytest.mark.gpu
def test_aggregate_every_boundary_pair(gpu, oracle_lib):
    """aggregate.rs:59-78: 100 u32/u32 keys (k, 7k), every range lo..hi for 0 <= lo <= hi <= 100,
    against a fold of lift -- all 5,151 key ranges in one batched device call."""
    from rsos_hip.wire import RangeAggregate
    from rsos_hip import Aggregate
    entries = [(k, 7 * k) for k in range(100)]
    st = _u32_store(entries)
    fps = _u32_recs(entries).lift()
    fold = [0]
    for f in fps:
        fold.append(fold[-1] + int.from_bytes(f.tobytes(), "little"))
    pairs = [(lo, hi) for lo in range(101) for hi in range(lo, 101)]
    segs = [RangeAggregate(lo, hi, Aggregate.ZERO) for lo, hi in pairs]
    raw_lo, raw_hi, aggs = st.resolve_segments(segs)
    for (lo, hi), a, rl, rh in zip(pairs, aggs, raw_lo, raw_hi):
        assert (int(rl), int(rh)) == (lo, hi)
        assert a.size == hi - lo
        assert a.fingerprint.to_int() == (fold[hi] - fold[lo]) % (1 << 256), (lo, hi)
    st.close()


@pytest.mark.gpu
def test_big_test_mirror(gpu, oracle_lib):
    """tests/basic.rs big_test: 1,000 random u64/u64 inserts one at a time; after each the root
    equals the FTM's; at the end partition additivity agg(..mid) + agg(mid..) == agg(..) for
    every 50th key and the rank / select inverse."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    rng = np.random.default_rng(90)
    m = 1000
    keys = rng.integers(0, 1 << 20, m, dtype=np.uint64)  # repeats: overwrites
    vals = rng.integers(0, 1 << 62, m, dtype=np.uint64)
    recs = O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0), keys.view(np.uint8).reshape(m, 8),
                     vals.view(np.uint8).reshape(m, 8))
    t = O.FingerprintTreeMap(recs)
    st = GpuFingerprintStore(RecordSchema.plain("u64", "u64"))
    st.load_bulk({"keys": np.zeros((0, 8), np.uint8), "values": np.zeros((0, 8), np.uint8)})
    for i in range(m):
        st.insert(int(keys[i]), int(vals[i]).to_bytes(8, "little"))
        t.insert(i)
        fp, size = t.root()
        root = st.aggregate()
        assert root.size == size == len(t)
        assert root.fingerprint.limbs == tuple(int(x) for x in fp), i
    uniq = np.unique(keys)
    whole = st.aggregate()
    for mid in uniq[::50]:
        lo = st.aggregate(KeyRange(None, int(mid)))
        hi = st.aggregate(KeyRange(int(mid), None))
        assert lo + hi == whole
    for r in range(0, len(uniq), 37):
        k = st.select(r)
        assert k == int(uniq[r]) and st.rank(k) == r
    st.close()


@pytest.mark.gpu
def test_reconcile_to_convergence(gpu, oracle_lib):
    """tests/diff.rs reconcile(): the ranges each side owes are sent as records and inserted by
    the other side (the sender's value wins, local first); afterwards both stores hold the same
    content -- equal roots, and the root is the FTM fold of the merged content."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    rng = np.random.default_rng(17)
    common = rng.choice(1 << 30, 6000, replace=False).astype(np.uint64)
    a = {int(k): int(k) * 3 for k in common[:5800]}
    b = dict(a)
    for k in common[5800:5900]:
        a[int(k)] = 11
    for k in common[5900:]:
        b[int(k)] = 22
    for k in common[:40]:
        b[int(k)] += 1

    def store(d):
        ks = np.array(sorted(d), np.uint64)
        vs = np.array([d[int(k)] for k in ks], np.uint64)
        st = GpuFingerprintStore(RecordSchema.plain("u64", "u64"))
        st.load_bulk({"keys": ks.view(np.uint8).reshape(-1, 8), "values": vs.view(np.uint8).reshape(-1, 8)})
        return st

    sa, sb = store(a), store(b)
    owed_a, owed_b = gpu_diff(sa, sb)
    assert owed_a and owed_b

    def send(src_store, src, dst_store, dst, ranges):
        keys = []
        for s, e in ranges:
            keys += [k for k, _ in src_store.enumerate(KeyRange(s, e))]
        if not keys:
            return
        ks = np.array(keys, np.uint64)
        vs = np.array([src[int(k)] for k in ks], np.uint64)
        dst_store.apply({"keys": ks.view(np.uint8).reshape(-1, 8), "values": vs.view(np.uint8).reshape(-1, 8)},
                        np.zeros(len(ks), np.uint8))
        for k in keys:
            dst[int(k)] = src[int(k)]

    send(sa, a, sb, b, owed_a)
    send(sb, b, sa, a, owed_b)
    assert a == b
    ra, rb = sa.aggregate(), sb.aggregate()
    assert ra == rb and ra.size == len(a)
    ks = np.array(sorted(a), np.uint64)
    vs = np.array([a[int(k)] for k in ks], np.uint64)
    t = O.FingerprintTreeMap(O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0),
                                       ks.view(np.uint8).reshape(-1, 8), vs.view(np.uint8).reshape(-1, 8)))
    t.fill(0, len(ks))
    assert ra.fingerprint.limbs == tuple(int(x) for x in t.root()[0])
    assert gpu_diff(sa, sb) == ([], [])
    sa.close()
    sb.close()


@pytest.mark.gpu
def test_concurrent_readers_one_store(gpu, oracle_lib):
    """§8b threading: the store is shared by readers under the replica's read lock
    (src/replica.rs:69,74); the library serialises calls on one store with its own mutex.
    8 host threads (ctypes releases the GIL inside each call) query one store at once; every
    answer equals the single-threaded one."""
    import threading
    from rsos_hip.store import KeyRange
    entries = [(k * 3, k) for k in range(20_000)]
    st = _u32_store(entries)
    rng = np.random.default_rng(5)
    queries = [tuple(sorted(int(x) for x in rng.integers(0, 60_000, 2))) for _ in range(300)]
    want = [(st.aggregate(KeyRange(a, b)), st.rank(a)) for a, b in queries]
    errors = []

    def reader(seed):
        order = np.random.default_rng(seed).permutation(len(queries))
        for j in order:
            a, b = queries[j]
            got = (st.aggregate(KeyRange(a, b)), st.rank(a))
            if got != want[j]:
                errors.append((j, got, want[j]))

    threads = [threading.Thread(target=reader, args=(s,)) for s in range(8)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors[:3]
    st.close()


@pytest.mark.gpu
def test_u64_keys_full_range_order(gpu, oracle_lib):
    """u64 keys across the whole range (top bit set included) order numerically, as Ord of u64
    does: ranks, selects, key-range aggregates and an update batch agree with the FTM."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    rng = np.random.default_rng(64)
    keys = np.unique(np.concatenate([rng.integers(0, 2**64 - 1, 3000, dtype=np.uint64, endpoint=True),
                                     np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 1], np.uint64)]))
    n = len(keys)
    vals = rng.integers(0, 2**63, n, dtype=np.uint64)
    st = GpuFingerprintStore(RecordSchema.plain("u64", "u64"))
    st.load_bulk({"keys": keys.view(np.uint8).reshape(n, 8), "values": vals.view(np.uint8).reshape(n, 8)})
    recs = O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0), keys.view(np.uint8).reshape(n, 8),
                     vals.view(np.uint8).reshape(n, 8))
    t = _ftm(recs)
    assert st.aggregate().fingerprint.limbs == tuple(int(x) for x in t.root()[0])
    probes = [0, 1, 2**63 - 1, 2**63, 2**63 + 1, 2**64 - 1] + [int(x) for x in rng.integers(0, 2**64 - 1, 200,
                                                                                              dtype=np.uint64)]
    for z in probes:
        assert st.rank(z) == t.rank(np.uint64(z).tobytes()), z
    for r in range(0, n, 97):
        assert st.select(r) == int(keys[r])
    for a, b in zip(probes[::2], probes[1::2]):
        lo, hi = min(a, b), max(a, b)
        got = st.aggregate(KeyRange(lo, hi))
        fp, size = t.aggregate(np.uint64(lo).tobytes(), np.uint64(hi).tobytes())
        assert got.size == size and got.fingerprint.limbs == tuple(int(x) for x in fp), (lo, hi)
    st.close()


@pytest.mark.gpu
def test_sharded_store_matches_single(gpu, oracle_lib):
    """rsos_hip.sharded: one map over several stores (here 3 shards on device 0), answering the
    Rsos surface and protocol rounds by decomposition, equals one store -- before and after a
    routed update batch -- and reconciles round by round like the FTM driver."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    from rsos_hip.sharded import ShardedStore
    from rsos_hip.store import KeyRange
    rng = np.random.default_rng(33)
    schema = RecordSchema.plain("u64", "u64")
    keys = np.unique(rng.integers(0, 2**63, 9000, dtype=np.uint64))
    n = len(keys)
    vals = rng.integers(0, 2**62, n, dtype=np.uint64)
    cols = {"keys": keys.view(np.uint8).reshape(n, 8), "values": vals.view(np.uint8).reshape(n, 8)}
    one = GpuFingerprintStore(schema)
    one.load_bulk(cols)
    sh = ShardedStore(schema, [0, 0, 0])
    sh.load_bulk(cols)
    assert sh.size() == one.size() and sh.aggregate() == one.aggregate()
    probes = [int(x) for x in rng.integers(0, 2**63, 60, dtype=np.uint64)] + [int(keys[0]), int(keys[-1])]
    for a, b in zip(probes[::2], probes[1::2]):
        lo, hi = min(a, b), max(a, b)
        assert sh.aggregate(KeyRange(lo, hi)) == one.aggregate(KeyRange(lo, hi))
        assert sh.rank(lo) == one.rank(lo)
    for r in range(0, n, 401):
        assert sh.select(r) == one.select(r)
    # a routed batch: new keys everywhere, overwrites, deletes
    newk = rng.integers(0, 2**63, 700, dtype=np.uint64)
    bk = np.unique(np.concatenate([newk, keys[::37]]))
    bv = rng.integers(0, 2**62, len(bk), dtype=np.uint64)
    ops = (rng.random(len(bk)) < 0.2).astype(np.uint8)
    batch = {"keys": bk.view(np.uint8).reshape(-1, 8), "values": bv.view(np.uint8).reshape(-1, 8)}
    assert sh.apply(batch, ops) == one.apply(batch, ops)
    assert sh.size() == one.size() and sh.aggregate() == one.aggregate()
    for r in range(0, one.size(), 389):
        assert sh.select(r) == one.select(r)
    # protocol rounds: the sharded map against a single store holding different content
    other = GpuFingerprintStore(schema)
    other.load_bulk(cols)
    got = _rounds(sh, other)
    want = _rounds(one, other)
    assert got == want and len(got) > 2
    for s in (one, other):
        s.close()
    sh.close()


def _rounds(a, b):
    from rsos_hip import rbsr as R
    out, active, sides, k = [], R.initial_ranges(a), [b, a], 0
    while active:
        ch, en = [], []
        o = R.protocol_round_with_policy(sides[k % 2], R.DEFAULT_POLICY, active, ch, en, native=False)
        out.append(([(c.start, c.end, c.aggregate) for c in ch], en, (o.skipped, o.enumerated, o.split)))
        active, k = ch, k + 1
    return out
