"""rbsr protocol rounds (rbsr/src/protocol.rs:212-317) served by the GPU store.

rsos_hip.rbsr answers a round in two batched store calls; oracle/rbsr.py is the literal,
one-question-at-a-time restatement over the oracle's FingerprintTreeMap.  The CPU tests pin the
oracle driver to the reference's own doc examples (protocol.rs:114-133, :190-210) and run the
product driver's host logic against it through a batched adapter over the same FTM; the GPU
tests run both drivers through whole two-replica reconciliations and require identical rounds.
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


# ---- helpers ---------------------------------------------------------------------------------

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


def _agg_t(a):
    """rsos_hip Aggregate -> the oracle's (fp limbs, size)."""
    return tuple(int(x) for x in a.fingerprint.limbs), int(a.size)


def _norm(children):
    out = []
    for c in children:
        if isinstance(c, tuple):
            out.append(c)
        else:
            out.append((c.start, c.end, _agg_t(c.aggregate)))
    return out


class BatchedFtm:
    """The two batched questions of rsos_hip.rbsr answered by the oracle FTM (host-logic check)."""

    def __init__(self, view):
        self.v = view

    def size(self):
        return self.v.size()

    def aggregate(self):
        from rsos_hip import Aggregate, Fingerprint
        fp, size = self.v.aggregate(None, None)
        return Aggregate(size, Fingerprint(fp))

    def resolve_segments(self, segs):
        from rsos_hip import Aggregate, Fingerprint
        n = self.v.size()
        lo = np.array([0 if s.start is None else self.v.rank(s.start) for s in segs], np.uint64)
        hi = np.array([n if s.end is None else self.v.rank(s.end) for s in segs], np.uint64)
        aggs = []
        for s in segs:
            fp, size = self.v.aggregate(s.start, s.end)
            aggs.append(Aggregate(size, Fingerprint(fp)))
        return lo, hi, aggs

    def split_segments(self, sel, lo, hi):
        from rsos_hip import Aggregate, Fingerprint
        keys = [self.v.select(int(r)) for r in sel]
        aggs = []
        for a, b in zip(lo, hi):
            ka = None if a == 0 else self.v.select(int(a))
            kb = None if b >= self.v.size() else self.v.select(int(b))
            fp, size = self.v.aggregate(ka, kb)
            aggs.append(Aggregate(size, Fingerprint(fp)))
        return keys, aggs


def _to_product(segs):
    from rsos_hip import Aggregate, Fingerprint
    from rsos_hip.wire import RangeAggregate
    return [RangeAggregate(s, e, Aggregate(a[1], Fingerprint(tuple(a[0])))) for s, e, a in segs]


def reconcile(a, b, round_fn, init, max_rounds=200):
    """Ping-pong rounds starting from a's root at b; per round: (children, enumerations, outcome)."""
    active = init(a)
    sides = [b, a]
    log, enums = [], {id(a): [], id(b): []}
    for k in range(max_rounds):
        if not active:
            return log, enums[id(a)], enums[id(b)]
        side = sides[k % 2]
        children, en = [], []
        outcome = round_fn(side, active, children, en)
        log.append((_norm(children), list(en), outcome))
        enums[id(side)].extend(en)
        active = children
    raise AssertionError("reconciliation did not terminate")


def _covered(k, ranges, lt):
    return any((s is None or not lt(k, s)) and (e is None or lt(k, e)) for s, e in ranges)


# ---- CPU: the oracle driver against the reference's doc examples -------------------------------

def test_oracle_round_doc_example_three_outcomes(oracle_lib):
    """protocol.rs:114-133: SKIP, IDLIST and SPLIT in one round against the same responder."""
    b = OR.FtmView(_ftm(_u32_recs([(i, i) for i in range(40)])), True)
    empty = OR.FtmView(_ftm(_u32_recs([])), True)
    c = OR.FtmView(_ftm(_u32_recs([(i + 1000, i) for i in range(40)])), True)
    active = OR.initial_ranges(b) + OR.initial_ranges(empty) + OR.initial_ranges(c)
    children, enums = [], []
    sk, en, sp, ch, dr = OR.protocol_round(b, OR.fixed_fan_out(16), active, children, enums)
    assert (sk, en, sp, dr) == (1, 1, 1, 0)
    assert ch == len(children)


def test_oracle_round_doc_example_sqrt(oracle_lib):
    """protocol.rs:190-210: SqrtFanOut cuts a 400-element span into 20 children."""
    a = OR.FtmView(_ftm(_u32_recs([(i, i) for i in range(400)])), True)
    b = OR.FtmView(_ftm(_u32_recs([(i, i) for i in range(400)] + [(999, 999)])), True)
    children, enums = [], []
    OR.protocol_round(a, OR.sqrt_fan_out, OR.initial_ranges(b), children, enums)
    assert len(children) == 20 and enums == []


def test_policy_params():
    """params.rs doc examples: ceil(10 / 3) = 4; FanOut 0 / 1 -> 2; a zero stride -> 1."""
    from rsos_hip.fingerprint import Aggregate, Fingerprint
    from rsos_hip.rbsr import Comparison, FixedFanOut, Split, fan_out
    z = Fingerprint((0, 0, 0, 0))
    c = Comparison(Aggregate(10, Fingerprint((1, 0, 0, 0))), Aggregate(7, z))
    assert FixedFanOut(3).decide(c) == Split(4)
    assert fan_out(0) == fan_out(1) == 2
    assert Split(0).stride == 1


def test_batched_driver_host_logic_matches_oracle(oracle_lib):
    """rsos_hip.rbsr's batched driver, fed by the oracle FTM, reproduces the literal driver's
    rounds on a u32 reconciliation with one-sided keys, changed values and an empty range."""
    from rsos_hip import rbsr as R
    rng = np.random.default_rng(4)
    keys = rng.choice(2**31, 3000, replace=False)
    a_pairs = {int(k): int(k) % 977 for k in keys[:2800]}
    b_pairs = dict(a_pairs)
    for k in keys[2800:2900]:
        a_pairs[int(k)] = 1
    for k in keys[2900:]:
        b_pairs[int(k)] = 2
    for k in keys[:40]:
        b_pairs[int(k)] += 5
    va = OR.FtmView(_ftm(_u32_recs(a_pairs.items())), True)
    vb = OR.FtmView(_ftm(_u32_recs(b_pairs.items())), True)
    for policy, decide in [(R.FixedFanOut(16), OR.fixed_fan_out(16)), (R.SqrtFanOut(), OR.sqrt_fan_out),
                           (R.FixedFanOut(2), OR.fixed_fan_out(2))]:
        want = reconcile(va, vb, lambda v, act, ch, en: OR.protocol_round(v, decide, act, ch, en),
                         OR.initial_ranges)
        pa, pb = BatchedFtm(va), BatchedFtm(vb)

        def prod(v, act, ch, en):
            o = R.protocol_round_with_policy(v, policy, _to_product(act) if act and isinstance(act[0], tuple)
                                             else act, ch, en)
            return (o.skipped, o.enumerated, o.split, o.children, o.dropped_malformed)
        got = reconcile(pa, pb, prod, R.initial_ranges)
        assert len(got[0]) == len(want[0])
        for (gc, ge, go), (wc, we, wo) in zip(got[0], want[0]):
            assert go == wo and ge == we and gc == wc
        # soundness: every one-sided key is enumerated by its holder
        lt = lambda x, y: x < y  # noqa: E731
        for k in keys[2800:2900]:
            assert _covered(int(k), want[1], lt)
        for k in keys[2900:]:
            assert _covered(int(k), want[2], lt)
        for k in keys[:40]:
            assert _covered(int(k), want[1], lt) or _covered(int(k), want[2], lt)


def test_c_reconciliation_matches_literal_driver(oracle_lib):
    """oracle.c's whole-reconciliation loop (the bench's native CPU baseline) takes the same
    rounds, answers the same segments and enumerates the same ranges as the Python driver."""
    rng = np.random.default_rng(8)
    keys = rng.choice(2**31, 5000, replace=False)
    a_pairs = {int(k): 7 for k in keys[:4900]}
    b_pairs = dict(a_pairs)
    for k in keys[4900:4950]:
        a_pairs[int(k)] = 1
    for k in keys[4950:]:
        b_pairs[int(k)] = 2
    for k in keys[:30]:
        b_pairs[int(k)] = 9
    ta, tb = _ftm(_u32_recs(a_pairs.items())), _ftm(_u32_recs(b_pairs.items()))
    va, vb = OR.FtmView(ta, True), OR.FtmView(tb, True)
    for b in (16, 2, 5):
        log, ea, eb = reconcile(va, vb, lambda v, act, ch, en: OR.protocol_round(v, OR.fixed_fan_out(b), act, ch, en),
                                OR.initial_ranges)
        want = (len(log), 1 + sum(len(c) for c, _, _ in log[:-1]), len(ea) + len(eb))
        assert O.reconcile_fixed(ta, tb, b) == want


def test_oracle_drops_inverted_segment(oracle_lib):
    a = OR.FtmView(_ftm(_u32_recs([(i, i) for i in range(100)])), True)
    children, enums = [], []
    out = OR.protocol_round(a, OR.fixed_fan_out(16), [(50, 10, ((1, 0, 0, 0), 3))], children, enums)
    assert out == (0, 0, 0, 0, 1) and children == [] and enums == []


# ---- GPU: the batched driver on the device store against the literal oracle driver --------------

def _dated_sets(seed, n_common, n_a, n_b, n_mod):
    rng = np.random.default_rng(seed)
    tot = n_common + n_a + n_b
    keys = np.unique(rng.integers(0, 256, (tot + 64, 16), dtype=np.uint8), axis=0)[:tot]
    rng.shuffle(keys)
    vals = rng.integers(0, 256, (tot, 64), dtype=np.uint8)
    phys = (1_700_000_000_000 + np.arange(tot)).astype(np.uint64)

    def cols(idx, bump=()):
        idx = np.array(sorted(idx, key=lambda i: keys[i].tobytes()))
        p = phys[idx].copy()
        for j, i in enumerate(idx):
            if i in bump:
                p[j] += 1
        n = len(idx)
        return {"keys": keys[idx].copy(), "values": vals[idx].copy(), "phys": p,
                "logical": np.zeros(n, np.uint32), "node": np.ones(n, np.uint64), "tags": np.zeros(n, np.uint8)}
    common = list(range(n_common))
    a_idx = common + list(range(n_common, n_common + n_a))
    b_idx = common + list(range(n_common + n_a, tot))
    mod = set(range(n_mod))
    return keys, cols(a_idx), cols(b_idx, bump=mod), a_idx[n_common:], b_idx[n_common:], sorted(mod)


def _cat(*cols):
    return {k: np.concatenate([c[k] for c in cols]) for k in cols[0]}


def _rows(cols, sel):
    return {k: v[sel] for k, v in cols.items()}


def _store_via_delta(schema, c, seed):
    """A GPU store holding exactly c's records with its delta run pending: a different base
    (withheld rows, extra rows, stale versions), then two batches -- the withheld rows inserted,
    the extra rows deleted, the stale rows overwritten, and keys inserted by the first batch and
    deleted by the second.  Rounds must read base + run without compacting it."""
    from rsos_hip import GpuFingerprintStore
    rng = np.random.default_rng(seed)
    n = len(c["keys"])
    idx = rng.permutation(n)
    nw, no = max(n // 40, 4), max(n // 60, 4)
    w, o = np.sort(idx[:nw]), np.sort(idx[nw:nw + no])
    have = {k.tobytes() for k in c["keys"]}
    fresh = []
    while len(fresh) < 2 * nw:
        k = rng.integers(0, 256, 16, dtype=np.uint8)
        if k.tobytes() not in have:
            have.add(k.tobytes())
            fresh.append(k)
    fresh = np.array(fresh)

    def fresh_cols(ks):
        m = len(ks)
        return {"keys": ks, "values": rng.integers(0, 256, (m, 64), dtype=np.uint8),
                "phys": np.full(m, 1_600_000_000_000, np.uint64), "logical": np.zeros(m, np.uint32),
                "node": np.ones(m, np.uint64), "tags": np.zeros(m, np.uint8)}
    keep = np.ones(n, bool)
    keep[w] = False
    base = _rows(c, keep)
    stale = {k: v.copy() for k, v in c.items()}
    stale["values"][o] ^= 0x5A
    stale["phys"][o] -= 5
    kept_idx = np.flatnonzero(keep)
    base["values"], base["phys"] = stale["values"][kept_idx], stale["phys"][kept_idx]
    xs, ys = fresh_cols(fresh[:nw]), fresh_cols(fresh[nw:])  # X: in the base; Y: batch 1 only
    base = _cat(base, xs)
    order = sorted(range(len(base["keys"])), key=lambda i: base["keys"][i].tobytes())
    base = _rows(base, np.array(order))
    st = GpuFingerprintStore(schema)
    st.load_bulk(base)
    hw, ho, hx = nw // 2, no // 2, nw // 2
    b1 = _cat(_rows(c, w[:hw]), _rows(c, o[:ho]), _rows(xs, slice(0, hx)), ys)
    ops1 = np.concatenate([np.zeros(hw + ho, np.uint8), np.ones(hx, np.uint8), np.zeros(nw, np.uint8)])
    b2 = _cat(_rows(c, w[hw:]), _rows(c, o[ho:]), _rows(xs, slice(hx, None)), ys)
    ops2 = np.concatenate([np.zeros(nw - hw + no - ho, np.uint8), np.ones(nw - hx, np.uint8),
                           np.ones(nw, np.uint8)])
    st.apply(b1, ops1)
    st.apply(b2, ops2)
    s = st.stats()
    assert s["delta_rows"] > 0 and s["compactions"] == 0 and st.size() == n
    return st


def _gpu_and_oracle(schema, c):
    from rsos_hip import GpuFingerprintStore
    st = GpuFingerprintStore(schema)
    st.load_bulk(c)
    sc = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
    recs = O.Records(sc, c["keys"], c["values"], c["phys"], c["logical"], c["node"], c["tags"])
    return st, OR.FtmView(_ftm(recs), False)


@pytest.mark.gpu
@pytest.mark.parametrize("rowp", ["row_prefix", "block_prefix"])
@pytest.mark.parametrize("native", [True, False])
@pytest.mark.parametrize("policy", ["fixed16", "sqrt", "fixed2"])
def test_gpu_reconciliation_rounds_match_oracle(gpu, oracle_lib, policy, native, rowp, monkeypatch):
    """Base-only stores; row_prefix: the base's row prefix formed in order (RSOS_HIP_ROW_PREFIX=2),
    so every round's sums are its differences (k_round_bounds_pre / k_round_emit_pre, the tiny
    rounds' lane sums); block_prefix: none (the wave-per-range kernels)."""
    monkeypatch.setenv("RSOS_HIP_ROW_PREFIX", "2" if rowp == "row_prefix" else "0")
    from rsos_hip import RecordSchema, rbsr as R
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(7, 20_000, 60, 45, 30)
    ga, oa = _gpu_and_oracle(schema, ca)
    gb, ob = _gpu_and_oracle(schema, cb)
    pol, decide = {"fixed16": (R.FixedFanOut(16), OR.fixed_fan_out(16)), "sqrt": (R.SqrtFanOut(), OR.sqrt_fan_out),
                   "fixed2": (R.FixedFanOut(2), OR.fixed_fan_out(2))}[policy]
    want = reconcile(oa, ob, lambda v, act, ch, en: OR.protocol_round(v, decide, act, ch, en), OR.initial_ranges)

    def prod(st, act, ch, en):
        o = R.protocol_round_with_policy(st, pol, act, ch, en, native=native)
        return (o.skipped, o.enumerated, o.split, o.children, o.dropped_malformed)

    def prod_init(st):
        return R.initial_ranges(st)
    got_log, got_ea, got_eb = reconcile(ga, gb, prod, prod_init)
    assert len(got_log) == len(want[0]) > 2
    for (gc, ge, go), (wc, we, wo) in zip(got_log, want[0]):
        assert go == wo
        assert ge == we
        assert gc == wc
    lt = lambda x, y: x < y  # noqa: E731  (memcmp order of [u8; 16])
    for i in only_a:
        assert _covered(keys[i].tobytes(), got_ea, lt)
    for i in only_b:
        assert _covered(keys[i].tobytes(), got_eb, lt)
    for i in mod:
        assert _covered(keys[i].tobytes(), got_ea, lt) or _covered(keys[i].tobytes(), got_eb, lt)
    ga.close()
    gb.close()


@pytest.mark.gpu
def test_gpu_round_edge_segments(gpu, oracle_lib):
    """Inverted, empty, beyond-the-end and unbounded segments, u64 keys, an empty store, and a
    store with a pending delta run (the one-call round reads base + run as they stand; the
    two-call path compacts first)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    rng = np.random.default_rng(9)
    keys = np.unique(rng.integers(0, 2**40, 5000, dtype=np.uint64))
    vals = rng.integers(0, 2**63, len(keys), dtype=np.uint64)
    n = len(keys)
    schema = RecordSchema.plain("u64", "u64")
    st = GpuFingerprintStore(schema)
    st.load_bulk({"keys": keys[:-100].view(np.uint8).reshape(-1, 8), "values": vals[:-100].view(np.uint8).reshape(-1, 8)})
    # the last 100 records arrive as a batch: they sit in the delta run (the one-call round reads
    # it in place, the two-call path compacts it)
    st.apply({"keys": keys[-100:].view(np.uint8).reshape(-1, 8), "values": vals[-100:].view(np.uint8).reshape(-1, 8)},
             np.zeros(100, np.uint8))
    recs = O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0), keys.view(np.uint8).reshape(n, 8),
                     vals.view(np.uint8).reshape(n, 8))
    ov = OR.FtmView(_ftm(recs), True)
    k = [int(x) for x in keys]
    segs = [(k[3000], k[100], ((0, 0, 0, 0), 5)),           # inverted: dropped
            (k[10], k[10], ((1, 0, 0, 0), 1)),              # empty local range, remote 1
            (k[-1] + 1, None, ((0, 0, 0, 0), 0)),           # beyond the end, remote empty: SKIP
            (None, k[7], ((0, 0, 0, 0), 0)),                # remote empty: IDLIST, no bounce
            (k[20], k[21], ((9, 9, 9, 9), 1)),              # 1 vs 1: IDLIST + bounce
            (None, None, ((5, 0, 0, 0), 9)),                # whole store: SPLIT
            (0, 2**64 - 1, ((5, 0, 0, 0), 2))]
    for pol, decide in [(R.FixedFanOut(16), OR.fixed_fan_out(16)), (R.SqrtFanOut(), OR.sqrt_fan_out)]:
        wc, we = [], []
        wo = OR.protocol_round(ov, decide, segs, wc, we)
        for native in (True, False):
            gc, ge = [], []
            o = R.protocol_round_with_policy(st, pol, _to_product(segs), gc, ge, native=native)
            assert (o.skipped, o.enumerated, o.split, o.children, o.dropped_malformed) == wo
            assert wo[4] == 1
            assert ge == we and _norm(gc) == wc
    empty = GpuFingerprintStore(schema)
    empty.load_bulk({"keys": np.zeros((0, 8), np.uint8), "values": np.zeros((0, 8), np.uint8)})
    gc, ge = [], []
    o = R.protocol_round(empty, _to_product(segs[1:]), gc, ge)  # native (FixedFanOut 16)
    eo = OR.FtmView(_ftm(O.Records(O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0),
                                   np.zeros((0, 8), np.uint8), np.zeros((0, 8), np.uint8))), True)
    wc, we = [], []
    assert (o.skipped, o.enumerated, o.split, o.children, o.dropped_malformed) == \
        OR.protocol_round(eo, OR.fixed_fan_out(16), segs[1:], wc, we)
    assert ge == we and _norm(gc) == wc
    st.close()
    empty.close()


@pytest.mark.gpu
def test_gpu_soa_reconciliation_and_wire(gpu, oracle_lib):
    """A reconciliation that stays in SoA form end to end (protocol_round_segments), each round's
    children shipped through the wire codec (ComparisonItem datagram bytes) and decoded by the
    peer, equals the object-level rounds; the children of a SPLIT sum to their parent."""
    from rsos_hip import RecordSchema, rbsr as R, wire
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(13, 30_000, 80, 70, 50)
    ga, _ = _gpu_and_oracle(schema, ca)
    gb, _ = _gpu_and_oracle(schema, cb)
    want, _, _ = reconcile(ga, gb, lambda v, act, ch, en: _outcome(R.protocol_round(v, act, ch, en)),
                           R.initial_ranges)
    pol = R.FixedFanOut(16)
    active = R.initial_segments(ga)
    sides = [gb, ga]
    k = 0
    while len(active):
        side = sides[k % 2]
        ch, en, o = R.protocol_round_segments(side, pol, active)
        wc, we, wo = want[k]
        assert _outcome(o) == wo
        assert _norm(ch.items(schema)) == wc
        assert [en.bounds(schema, i) for i in range(en.n)] == we
        # over the wire: encode the children as ComparisonItems, decode on the other side
        items = ch.items(schema)
        data = wire.encode(schema, items, msg_tag=wire.COMPARISON_ITEM)
        back, used = wire.decode_stream(schema, data, len(items), msg_tag=wire.COMPARISON_ITEM)
        assert back == items and used == len(data)
        active = R.Segments.from_items(schema, back)
        k += 1
    assert k == len(want)
    # zero-copy ping-pong: each store's output arrays feed the peer store directly
    active, k = R.initial_segments(ga), 0
    while len(active):
        active, en, o = R.protocol_round_segments(sides[k % 2], pol, active, copy=False)
        assert _outcome(o) == want[k][2]
        assert _norm(active.items(schema)) == want[k][0]
        assert [en.bounds(schema, i) for i in range(en.n)] == want[k][1]
        k += 1
    assert k == len(want)
    ga.close()
    gb.close()


def _outcome(o):
    return (o.skipped, o.enumerated, o.split, o.children, o.dropped_malformed)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["u32_u32", "b32_b64", "u64_b64"])
def test_gpu_reconciliation_other_key_types(gpu, oracle_lib, shape):
    """The round on every store key type (u32 numeric order, 32-byte memcmp order, u64): the
    native round equals the literal driver over the FTM, round by round."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    rng = np.random.default_rng(21)
    kk, kl, vname, vl = {"u32_u32": ("u32", 4, "u32", 4), "b32_b64": ("bytes32", 32, "bytes64", 64),
                         "u64_b64": ("u64", 8, "bytes64", 64)}[shape]
    schema = RecordSchema.plain(kk, vname)
    n = 12_000
    if kk == "u32":
        keys = np.unique(rng.integers(0, 2**32, n + 100, dtype=np.uint64).astype(np.uint32))[:n]
        krows = keys.view(np.uint8).reshape(-1, 4)
        key_int = True
    elif kk == "u64":
        keys = np.unique(rng.integers(0, 2**63, n + 100, dtype=np.uint64))[:n]
        krows = keys.view(np.uint8).reshape(-1, 8)
        key_int = True
    else:
        krows = np.unique(rng.integers(0, 256, (n + 100, kl), dtype=np.uint8), axis=0)[:n]
        key_int = False
    n = len(krows)
    vals = rng.integers(0, 256, (n, vl), dtype=np.uint8)
    drop = rng.choice(n, 40, replace=False)
    keep = np.ones(n, bool)
    keep[drop[:20]] = False
    vals_b = vals.copy()
    vals_b[drop[20:]] ^= 0x5A
    stores, views = [], []
    for kr, vv in ((krows, vals), (krows[keep], vals_b[keep])):
        st = GpuFingerprintStore(schema)
        st.load_bulk({"keys": np.ascontiguousarray(kr), "values": np.ascontiguousarray(vv)})
        sc = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
        t = _ftm(O.Records(sc, np.ascontiguousarray(kr), np.ascontiguousarray(vv)))
        stores.append(st)
        views.append(OR.FtmView(t, key_int))
    want = reconcile(views[0], views[1],
                     lambda v, act, ch, en: OR.protocol_round(v, OR.fixed_fan_out(16), act, ch, en), OR.initial_ranges)
    got = reconcile(stores[0], stores[1], lambda v, act, ch, en: _outcome(R.protocol_round(v, act, ch, en)),
                    R.initial_ranges)
    assert len(got[0]) == len(want[0]) > 2
    for (gc, ge, go), (wc, we, wo) in zip(got[0], want[0]):
        assert go == wo and ge == we and gc == wc
    for st in stores:
        st.close()


from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(a=st.dictionaries(st.integers(0, 400), st.integers(0, 3), max_size=120),
       b=st.dictionaries(st.integers(0, 400), st.integers(0, 3), max_size=120),
       fan=st.sampled_from([0, 2, 3, 16, 1000]), sqrt=st.booleans())
def test_batched_driver_property(oracle_lib, a, b, fan, sqrt):
    """Random replica pairs (empty, equal, disjoint, overlapping with changed values) under
    random policies: the batched driver's host logic reproduces the literal driver round by round,
    and every key the replicas disagree on is enumerated by a side that holds it."""
    from rsos_hip import rbsr as R
    va = OR.FtmView(_ftm(_u32_recs(a.items())), True)
    vb = OR.FtmView(_ftm(_u32_recs(b.items())), True)
    pol, decide = (R.SqrtFanOut(), OR.sqrt_fan_out) if sqrt else (R.FixedFanOut(fan), OR.fixed_fan_out(fan))
    want = reconcile(va, vb, lambda v, act, ch, en: OR.protocol_round(v, decide, act, ch, en), OR.initial_ranges)

    def prod(v, act, ch, en):
        o = R.protocol_round_with_policy(v, pol, act, ch, en)
        return (o.skipped, o.enumerated, o.split, o.children, o.dropped_malformed)
    got = reconcile(BatchedFtm(va), BatchedFtm(vb), prod, R.initial_ranges)
    assert len(got[0]) == len(want[0])
    for (gc, ge, go), (wc, we, wo) in zip(got[0], want[0]):
        assert go == wo and ge == we and gc == wc
    lt = lambda x, y: x < y  # noqa: E731
    for k in set(a) | set(b):
        if a.get(k) != b.get(k):
            holders = ([want[1]] if k in a else []) + ([want[2]] if k in b else [])
            assert any(_covered(k, r, lt) for r in holders), k


@pytest.mark.gpu
@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow,
                                                                  HealthCheck.function_scoped_fixture])
@given(a=st.dictionaries(st.integers(0, 2**32 - 1), st.integers(0, 3), max_size=300),
       b=st.dictionaries(st.integers(0, 2**32 - 1), st.integers(0, 3), max_size=300),
       fan=st.sampled_from([0, 2, 16]), sqrt=st.booleans())
def test_gpu_native_round_property(gpu, oracle_lib, a, b, fan, sqrt):
    """Random u32 replica pairs on GPU stores (including empty ones) under random policies: the
    library's one-call round equals the literal driver over the FTM, round by round."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R

    def store(d):
        pairs = sorted(d.items())
        s = GpuFingerprintStore(RecordSchema.plain("u32", "u32"))
        s.load_bulk({"keys": np.array([k for k, _ in pairs], np.uint32).view(np.uint8).reshape(-1, 4),
                     "values": np.array([v for _, v in pairs], np.uint32).view(np.uint8).reshape(-1, 4)})
        return s
    va = OR.FtmView(_ftm(_u32_recs(a.items())), True)
    vb = OR.FtmView(_ftm(_u32_recs(b.items())), True)
    pol, decide = (R.SqrtFanOut(), OR.sqrt_fan_out) if sqrt else (R.FixedFanOut(fan), OR.fixed_fan_out(fan))
    want = reconcile(va, vb, lambda v, act, ch, en: OR.protocol_round(v, decide, act, ch, en), OR.initial_ranges)
    ga, gb = store(a), store(b)
    got = reconcile(ga, gb, lambda v, act, ch, en: _outcome(R.protocol_round_with_policy(v, pol, act, ch, en)),
                    R.initial_ranges)
    assert len(got[0]) == len(want[0])
    for (gc, ge, go), (wc, we, wo) in zip(got[0], want[0]):
        assert go == wo and ge == we and gc == wc
    ga.close()
    gb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["fixed16", "sqrt"])
def test_gpu_native_round_large_batches(gpu, policy):
    """Rounds of tens of thousands of segments -- the per-array input copies, the header-first
    readback and, under SqrtFanOut, more children than the first capacity guess -- answered by the
    one-call device round equal the two-call path (host decisions, tested above against the
    literal driver) round by round."""
    from rsos_hip import RecordSchema, rbsr as R
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(17, 200_000, 1000, 1000, 1000)
    ga, _ = _gpu_and_oracle(schema, ca)
    gb, _ = _gpu_and_oracle(schema, cb)
    pol = {"fixed16": R.FixedFanOut(16), "sqrt": R.SqrtFanOut()}[policy]
    active, sides, k, widest, log = R.initial_segments(ga), [gb, ga], 0, 0, []
    while len(active):
        side = sides[k % 2]
        widest = max(widest, len(active))
        items = active.items(schema)
        ch, en, o = R.protocol_round_segments(side, pol, active)
        want_ch, want_en = [], []
        wo = R.protocol_round_with_policy(side, pol, items, want_ch, want_en, native=False)
        assert _outcome(o) == _outcome(wo)
        assert _norm(ch.items(schema)) == _norm(want_ch)
        assert [en.bounds(schema, i) for i in range(en.n)] == want_en
        log.append((_outcome(o), _norm(want_ch), want_en))
        active, k = ch, k + 1
    assert widest > 4000 and k > 3
    # the same rounds handed over in place (each store's output arrays, in mapped page-locked
    # memory, are the peer's next input: read in by a kernel, not copied)
    active, k = R.initial_segments(ga), 0
    while len(active):
        active, en, o = R.protocol_round_segments(sides[k % 2], pol, active, copy=False)
        assert (_outcome(o), _norm(active.items(schema)), [en.bounds(schema, i) for i in range(en.n)]) == log[k]
        k += 1
    assert k == len(log)
    ga.close()
    gb.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fused", ["fused", "fused_block", "unfused", "unfused_block"])
@pytest.mark.parametrize("policy", ["fixed16", "sqrt", "fixed2"])
def test_gpu_rounds_over_pending_delta_run_match_oracle(gpu, oracle_lib, policy, fused, monkeypatch):
    """Both replicas reach their contents through batches that stay in the delta run (inserts,
    deletes of base keys, overwrites, a key inserted then deleted): the one-call device round reads
    base + run in place (select over both, sums over both) and must equal the literal driver over
    the final contents round by round -- without compacting either store.  fused: tiny rounds in
    one launch (round_tiny.hpp k_round_tiny, the default); unfused: RSOS_HIP_ROUND_FUSED=0, the two
    searches and k_round_small_view, with the run's columns from the eight launches
    (RSOS_HIP_RUNCOL_FUSED=0) rather than k_run_columns_small.  *_block: RSOS_HIP_ROW_PREFIX=0, sums
    from the block prefixes (head and tail rows plus a difference) instead of the row prefixes' one
    difference (formed in order, RSOS_HIP_ROW_PREFIX=2, so that every question reads them)."""
    monkeypatch.setenv("RSOS_HIP_ROUND_FUSED", "1" if fused.startswith("fused") else "0")
    monkeypatch.setenv("RSOS_HIP_QUERY_FUSED", "1" if fused.startswith("fused") else "0")
    monkeypatch.setenv("RSOS_HIP_ROW_PREFIX", "0" if fused.endswith("_block") else "2")
    monkeypatch.setenv("RSOS_HIP_RUNCOL_FUSED", "1" if fused.startswith("fused") else "0")
    from rsos_hip import RecordSchema, rbsr as R
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(11, 20_000, 60, 45, 30)
    ga, gb = _store_via_delta(schema, ca, 1), _store_via_delta(schema, cb, 2)
    _, oa = _gpu_and_oracle(schema, ca)
    _, ob = _gpu_and_oracle(schema, cb)
    pol, decide = {"fixed16": (R.FixedFanOut(16), OR.fixed_fan_out(16)), "sqrt": (R.SqrtFanOut(), OR.sqrt_fan_out),
                   "fixed2": (R.FixedFanOut(2), OR.fixed_fan_out(2))}[policy]
    want = reconcile(oa, ob, lambda v, act, ch, en: OR.protocol_round(v, decide, act, ch, en), OR.initial_ranges)
    got = reconcile(ga, gb, lambda v, act, ch, en: _outcome(R.protocol_round_with_policy(v, pol, act, ch, en)),
                    R.initial_ranges)
    assert len(got[0]) == len(want[0]) > 2
    for (gc, ge, go), (wc, we, wo) in zip(got[0], want[0]):
        assert go == wo and ge == we and gc == wc
    for g in (ga, gb):
        s = g.stats()
        assert s["delta_rows"] > 0 and s["compactions"] == 0
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rowp", ["row_prefix", "block_prefix"])
@pytest.mark.parametrize("policy", ["fixed16", "sqrt"])
def test_gpu_large_rounds_over_pending_delta_run(gpu, policy, rowp, monkeypatch):
    """Rounds of thousands of segments over a replica whose delta run is pending equal the same
    rounds over a freshly loaded replica with the same contents (the base-only path, tested above
    against the literal driver), round by round, and leave the delta run in place.  row_prefix:
    both replicas with their row prefixes formed in order (a thread per segment and per child,
    k_bounds_view_pre / k_round_emit_view_pre); block_prefix: without (a wave each)."""
    monkeypatch.setenv("RSOS_HIP_ROW_PREFIX", "2" if rowp == "row_prefix" else "0")
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(23, 200_000, 1000, 1000, 1000)
    va = _store_via_delta(schema, ca, 3)
    fa = GpuFingerprintStore(schema)
    fa.load_bulk(ca)
    gb = GpuFingerprintStore(schema)
    gb.load_bulk(cb)
    pol = {"fixed16": R.FixedFanOut(16), "sqrt": R.SqrtFanOut()}[policy]
    active, k, widest = R.initial_segments(gb), 0, 0
    while len(active):
        if k % 2 == 0:
            widest = max(widest, len(active))
            ch, en, o = R.protocol_round_segments(va, pol, active)
            wch, wen, wo = R.protocol_round_segments(fa, pol, active)
            assert _outcome(o) == _outcome(wo)
            assert _norm(ch.items(schema)) == _norm(wch.items(schema))
            assert [en.bounds(schema, i) for i in range(en.n)] == [wen.bounds(schema, i) for i in range(wen.n)]
        else:
            ch, en, o = R.protocol_round_segments(gb, pol, active)
        active, k = ch, k + 1
    assert widest > 1024 and k > 3
    s = va.stats()
    assert s["delta_rows"] > 0 and s["compactions"] == 0
    for g in (va, fa, gb):
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fused", ["fused", "fused_block", "unfused"])
def test_tiny_questions_over_pending_delta_run(gpu, oracle_lib, fused, monkeypatch):
    """The small questions a device answers when the host tier is off or stale -- rank, ranks of up
    to 64 keys, select and dumps of up to 64 keys, an aggregate over a key range with every bound
    kind -- in one launch each (round_tiny.hpp k_query_tiny) over a store whose delta run is pending,
    against a freshly loaded store with the same contents and the oracle FTM; with
    RSOS_HIP_QUERY_FUSED=0 the same questions take the multi-launch paths; fused_block: without the
    row prefixes (RSOS_HIP_ROW_PREFIX=0)."""
    monkeypatch.setenv("RSOS_HIP_QUERY_FUSED", "1" if fused.startswith("fused") else "0")
    monkeypatch.setenv("RSOS_HIP_ROW_PREFIX", "0" if fused.endswith("_block") else "2")
    monkeypatch.setenv("RSOS_HIP_RUNCOL_FUSED", "1" if fused.startswith("fused") else "0")
    from rsos_hip import GpuFingerprintStore, RecordSchema, _abi as A
    from rsos_hip.store import KeyRange
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(29, 20_000, 80, 10, 10)
    va = _store_via_delta(schema, ca, 5)
    monkeypatch.setenv("RSOS_HIP_QUERY_FUSED", "0")
    fa = GpuFingerprintStore(schema)  # the base-only, multi-launch reference
    fa.load_bulk(ca)
    _, ov = _gpu_and_oracle(schema, ca)
    ftm = ov.t
    rng = np.random.default_rng(3)
    n = fa.size()
    assert va.size() == n
    present = [bytes(k) for k in ca["keys"][rng.integers(0, n, 120)]]
    absent = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(120)]
    probes = present + absent + [b"\x00" * 16, b"\xff" * 16]
    for z in probes:
        assert va.rank(z) == fa.rank(z) == ftm.rank(z)
    for m in (1, 64, 65):
        pk = np.frombuffer(b"".join(probes[:m]), np.uint8).reshape(m, 16)
        assert (va.ranks(pk) == fa.ranks(pk)).all()
    for r in [0, n - 1] + [int(x) for x in rng.integers(0, n, 60)]:
        assert va.select(r) == fa.select(r)
    for lo, cnt in ((0, 64), (n - 64, 64), (n // 2, 65), (7, 1)):
        k1, k2 = np.zeros(cnt * 16, np.uint8), np.zeros(cnt * 16, np.uint8)
        A.check(A.lib().rh_store_keys(va._h, lo, lo + cnt, k1.ctypes.data), "keys")
        A.check(A.lib().rh_store_keys(fa._h, lo, lo + cnt, k2.ctypes.data), "keys")
        assert (k1 == k2).all()
    kinds = ["unbounded", "included", "excluded"]
    for i in range(120):
        a, b = sorted((probes[int(rng.integers(len(probes)))], probes[int(rng.integers(len(probes)))]))
        if i % 7 == 0:
            a, b = b, a  # inverted: ZERO
        lk, hk = kinds[i % 3], kinds[(i // 3) % 3]
        rg = KeyRange(None if lk == "unbounded" else a, None if hk == "unbounded" else b, lk, hk)
        got = va.aggregate(rg)
        assert got == fa.aggregate(rg), (i, lk, hk)
        if lk == "included" and hk == "excluded" and a <= b:  # the oracle FTM's own range form
            fp, size = ftm.aggregate(a, b)
            assert got.size == size and list(got.fingerprint.limbs) == [int(x) for x in fp]
    s = va.stats()
    assert s["delta_rows"] > 0 and s["compactions"] == 0
    for g in (va, fa):
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("run_rows", [1, 255, 256, 4094, 4095, 4096, 9000])
def test_run_columns_at_the_one_launch_limit(gpu, oracle_lib, run_rows, monkeypatch):
    """A delta run of run_rows entries on a base whose size is no multiple of 256: its columns
    from k_run_columns_small (up to RUNCOL_SMALL = 4,095 entries; the eight-launch path above it)
    against the eight launches (RSOS_HIP_RUNCOL_FUSED=0), each with the row prefixes formed in
    order and without them, and against a store loaded with the final contents: ranks, selects,
    key-range aggregates and a whole reconciliation round by round."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    from rsos_hip.store import KeyRange
    schema = RecordSchema.dated("bytes16", "bytes64")
    rng = np.random.default_rng(run_rows)
    n = 20_011
    keys = np.unique(rng.integers(0, 256, (n + run_rows + 64, 16), dtype=np.uint8), axis=0)[:n + run_rows]
    rng.shuffle(keys)
    tot = len(keys)
    cols = {"keys": keys, "values": rng.integers(0, 256, (tot, 64), dtype=np.uint8),
            "phys": (1_700_000_000_000 + np.arange(tot)).astype(np.uint64), "logical": np.zeros(tot, np.uint32),
            "node": np.ones(tot, np.uint64), "tags": np.zeros(tot, np.uint8)}

    def part(idx):
        idx = np.array(sorted(idx, key=lambda i: keys[i].tobytes()))
        return {k: v[idx].copy() for k, v in cols.items()}
    base, batch, final = part(range(n)), part(range(n, tot)), part(range(tot))
    stores = {}
    for fusedc in ("1", "0"):
        for rowp in ("2", "0"):
            monkeypatch.setenv("RSOS_HIP_RUNCOL_FUSED", fusedc)
            monkeypatch.setenv("RSOS_HIP_ROW_PREFIX", rowp)
            st = GpuFingerprintStore(schema)
            st.load_bulk(base)
            st.apply(batch, np.zeros(len(batch["keys"]), np.uint8))
            assert st.stats()["delta_rows"] == run_rows
            stores[(fusedc, rowp)] = st
    ref = GpuFingerprintStore(schema)
    ref.load_bulk(final)
    probes = [bytes(k) for k in final["keys"][rng.integers(0, tot, 80)]] + \
        [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in range(40)]
    kinds = ["unbounded", "included", "excluded"]
    for st in stores.values():
        assert st.size() == ref.size() == tot
        assert st.aggregate() == ref.aggregate()
        for z in probes[:40]:
            assert st.rank(z) == ref.rank(z)
        for r in [0, tot - 1] + [int(x) for x in rng.integers(0, tot, 30)]:
            assert st.select(r) == ref.select(r)
        for i in range(60):
            a, b = sorted((probes[int(rng.integers(len(probes)))], probes[int(rng.integers(len(probes)))]))
            rg = KeyRange(a, b, kinds[i % 3] if i % 3 else "included", kinds[(i // 3) % 3] if (i // 3) % 3 else "excluded")
            assert st.aggregate(rg) == ref.aggregate(rg), i
    peer = GpuFingerprintStore(schema)
    peer.load_bulk(part([i for i in range(tot) if i % 97]))
    want = reconcile(ref, peer, lambda v, act, ch, en: _outcome(R.protocol_round_with_policy(v, R.FixedFanOut(16), act, ch, en)),
                     R.initial_ranges)
    for st in stores.values():
        got = reconcile(st, peer, lambda v, act, ch, en: _outcome(R.protocol_round_with_policy(v, R.FixedFanOut(16), act, ch, en)),
                        R.initial_ranges)
        assert got[0] == want[0]
        assert st.stats()["compactions"] == 0
        st.close()
    ref.close()
    peer.close()


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["fixed16", "sqrt"])
def test_gpu_large_base_rounds_row_prefix_equal_block_prefix(gpu, policy, monkeypatch):
    """Rounds of thousands of segments over a base-only replica: with the base's row prefix
    (RSOS_HIP_ROW_PREFIX=2: a thread per segment and per child, k_round_bounds_pre /
    k_round_emit_pre) equal the wave-per-range kernels without it (RSOS_HIP_ROW_PREFIX=0), whose
    rounds the tests above hold to the literal driver -- round by round, children with their bounds
    and sums, enumerations and outcomes.  The first plans a large round in three launches
    (k_round_plan_part / _scan_parts / _apply), the second with k_round_plan and library scans
    (RSOS_HIP_ROUND_PLAN3=0)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(31, 200_000, 1500, 1000, 1000)
    st = {}
    for rowp in ("2", "0"):
        monkeypatch.setenv("RSOS_HIP_ROW_PREFIX", rowp)
        monkeypatch.setenv("RSOS_HIP_ROUND_PLAN3", "1" if rowp == "2" else "0")
        s = GpuFingerprintStore(schema)
        s.load_bulk(ca)
        st[rowp] = s
    gb = GpuFingerprintStore(schema)
    gb.load_bulk(cb)
    pol = {"fixed16": R.FixedFanOut(16), "sqrt": R.SqrtFanOut()}[policy]
    active, k, widest = R.initial_segments(gb), 0, 0
    while len(active):
        if k % 2 == 0:
            widest = max(widest, len(active))
            ch, en, o = R.protocol_round_segments(st["2"], pol, active)
            wch, wen, wo = R.protocol_round_segments(st["0"], pol, active)
            assert _outcome(o) == _outcome(wo)
            assert _norm(ch.items(schema)) == _norm(wch.items(schema))
            assert [en.bounds(schema, i) for i in range(en.n)] == [wen.bounds(schema, i) for i in range(wen.n)]
        else:
            ch, en, o = R.protocol_round_segments(gb, pol, active)
        active, k = ch, k + 1
    assert widest > 1024 and k > 3
    for g in (*st.values(), gb):
        g.close()


@pytest.mark.gpu
def test_raw_round_handoff_equals_views(gpu):
    """protocol_round_segments(raw=True) hands a round's output to the peer as the library returned
    it (RawSegments, bench.py's rbsr loop): the same rounds, outcomes and enumeration counts as
    copied Segments."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    schema = RecordSchema.dated("bytes16", "bytes64")
    keys, ca, cb, only_a, only_b, mod = _dated_sets(37, 50_000, 400, 300, 300)
    a, b = GpuFingerprintStore(schema), GpuFingerprintStore(schema)
    a.load_bulk(ca)
    b.load_bulk(cb)
    pol = R.FixedFanOut(16)

    def run(raw):
        active, k, log = R.initial_segments(a), 0, []
        while len(active):
            kw = {"raw": True} if raw else {"copy": True}
            active, en, o = R.protocol_round_segments((b, a)[k % 2], pol, active, **kw)
            log.append((_outcome(o), len(active), len(en)))
            k += 1
        return log
    got, want = run(True), run(False)
    assert got == want and len(got) > 3
    a.close()
    b.close()
