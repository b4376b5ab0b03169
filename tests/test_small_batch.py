"""The store's small-batch path (csrc/small_batch.hpp) against the large-batch path and the oracle.

A batch of up to small_batch_max rows (1,024; 512 for 32-byte keys) is sorted, lifted, searched and
turned into delta records by one workgroup, then merged into the delta run by a second launch --
the path of a replica's network merge (src/replica/dispatch.rs:188-196) and of a staged
Rsos::insert.  Every case runs twice, with the small path on (the default) and off
(RSOS_HIP_SMALL_MAX=0: every batch through the large-batch path), through host batches
(rh_store_apply), device batches (rh_store_apply_device) and staged rows (rh_store_stage, where a key
staged more than once keeps its last operation), across compactions; after every batch the size
and root, and at the end the whole rank order (keys and fingerprints), ranks and selects, equal a
model folded with FingerprintTreeMap's semantics (insert-or-overwrite replaces the element's
fingerprint, remove drops it: rsos/src/fingerprint_tree_map/mutate.rs:23-154) over the oracle's
lifts (oracle/oracle.c)."""
import numpy as np
import pytest

M256 = 1 << 256

SCHEMAS = [("dated", "bytes16", "bytes64", True), ("plain", "u64", "u64", False),
           ("projection", "bytes32", "bytes64", True), ("dated", "u32", "u32", True)]


def _gen(rng, sch, n, tombstones):
    """n random host rows of schema sch (keys distinct)."""
    kl, vl = sch.key_row, sch.value_row
    keys = rng.integers(0, 256, size=(n, kl), dtype=np.uint8)
    cols = {"keys": keys, "values": rng.integers(0, 256, size=(n, vl), dtype=np.uint8)}
    if sch.dated_kind:
        cols["phys"] = rng.integers(0, 1 << 62, size=n, dtype=np.uint64)
        cols["logical"] = rng.integers(0, 1 << 31, size=n, dtype=np.uint32)
        cols["node"] = rng.integers(0, 1 << 62, size=n, dtype=np.uint64)
    if tombstones:
        cols["tags"] = (rng.random(n) < 0.1).astype(np.uint8)
    return cols


def _order(sch, k: bytes):
    return int.from_bytes(k, "little") if sch.key_kind in (1, 2) else k


class Model:
    """FingerprintTreeMap's contents: key -> fingerprint (last write wins, deletes remove)."""

    def __init__(self, O, sch):
        self.O, self.sch, self.d = O, sch, {}
        self.osch = O.Schema(sch.key_kind, sch.key_len, sch.value_kind, sch.value_len, sch.record_kind, 0)

    def lifts(self, cols):
        g = lambda c: cols.get(c)  # noqa: E731
        return self.O.Records(self.osch, g("keys"), g("values"), g("phys"), g("logical"), g("node"), g("tags")).lift()

    def apply(self, cols, ops):
        """rows in order; returns (new, overwritten, deleted) as the store counts them for a batch
        of distinct keys"""
        fps = self.lifts(cols)
        new = over = dele = 0
        for i in range(len(ops)):
            k = cols["keys"][i].tobytes()
            live = k in self.d
            if ops[i]:
                dele += live
                self.d.pop(k, None)
            else:
                new += not live
                over += live
                self.d[k] = fps[i].tobytes()
        return new, over, dele

    def root(self):
        return sum(int.from_bytes(f, "little") for f in self.d.values()) % M256, len(self.d)

    def sorted_keys(self):
        return sorted(self.d, key=lambda k: _order(self.sch, k))


def _batch(rng, sch, model, m, tombstones, repeats=False):
    """m rows: fresh keys, overwrites of live keys, deletes of live and of absent keys; with
    repeats, some keys appear two or three times (staged rows only)."""
    cols = _gen(rng, sch, m, tombstones)
    ops = np.zeros(m, np.uint8)
    live = model.sorted_keys()
    if live:
        for i in range(m):
            u = rng.random()
            if u < 0.2:  # overwrite a live key
                cols["keys"][i] = np.frombuffer(live[rng.integers(len(live))], np.uint8)
            elif u < 0.27:  # delete a live key
                cols["keys"][i] = np.frombuffer(live[rng.integers(len(live))], np.uint8)
                ops[i] = 1
            elif u < 0.3:  # delete an absent key
                ops[i] = 1
    if repeats and m > 2:
        for i in range(1, m, 3):
            cols["keys"][i] = cols["keys"][i - 1]
            ops[i] = rng.integers(0, 2)
    if not repeats:  # distinct keys: keep the first of any accidental repeat
        _, first = np.unique(cols["keys"], axis=0, return_index=True)
        keep = np.sort(first)
        cols = {c: v[keep] for c, v in cols.items()}
        ops = ops[keep]
    return cols, ops


def _run(O, spec, small_on, monkeypatch, seed=3):
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    if small_on:
        monkeypatch.delenv("RSOS_HIP_SMALL_MAX", raising=False)
    else:
        monkeypatch.setenv("RSOS_HIP_SMALL_MAX", "0")
    kind, kname, vname, tomb = spec
    sch = getattr(RecordSchema, kind)(kname, vname)
    rng = np.random.default_rng(seed)
    model = Model(O, sch)
    base = _gen(rng, sch, 6000, tomb)
    _, first = np.unique(base["keys"], axis=0, return_index=True)
    base = {c: v[np.sort(first)] for c, v in base.items()}
    order = sorted(range(len(base["keys"])), key=lambda i: _order(sch, base["keys"][i].tobytes()))
    base = {c: np.ascontiguousarray(v[order]) for c, v in base.items()}
    model.apply(base, np.zeros(len(base["keys"]), np.uint8))
    st = GpuFingerprintStore(sch)
    st.set_compaction(2, 1500)  # compactions every few batches
    st.load_bulk(base)
    sbm = 512 if sch.key_row == 32 else 1024
    sizes = [1, 2, 3, 63, 64, 65, 300, sbm, sbm + 1, 5, 1, 700, 1]
    trace = []
    for bi, m in enumerate(sizes):
        how = ("host", "device", "staged")[bi % 3]
        cols, ops = _batch(rng, sch, model, m, tomb, repeats=how == "staged")
        if how == "host":
            got = st.apply(cols, ops)
        elif how == "device":
            dc = {c: torch.from_numpy(np.ascontiguousarray(v)).cuda() for c, v in cols.items()}
            got = st.apply_device(dc, torch.from_numpy(ops).cuda())
        else:
            st.stage(cols, ops)
            got = None
        want = model.apply(cols, ops)
        if got is not None:
            assert got == want, (how, m)
        root, size = model.root()
        agg = st.aggregate()
        assert agg.size == size == st.size(), (how, m)
        assert agg.fingerprint.to_int() == root, (how, m)
        trace.append((got, agg.size, agg.fingerprint.to_int()))
    # a batch with a repeated key through apply is refused, the store unchanged
    cols, ops = _batch(rng, sch, model, 4, tomb)
    cols = {c: np.concatenate([v, v[:1]]) for c, v in cols.items()}
    ops = np.concatenate([ops, ops[:1]])
    with pytest.raises(Exception):
        st.apply(cols, ops)
    assert st.aggregate().fingerprint.to_int() == model.root()[0]
    # the whole rank order, ranks and selects
    keys = model.sorted_keys()
    fps = st.fingerprints()
    assert np.array_equal(fps, np.stack([np.frombuffer(model.d[k], np.uint8) for k in keys]))
    for r in list(range(0, len(keys), 97)) + [len(keys) - 1]:
        k = st.select(r)
        kb = k.to_bytes(sch.key_row, "little") if isinstance(k, int) else k
        assert kb == keys[r]
        assert st.rank(k) == r
    stats = st.batch_stats()
    comps = st.stats()["compactions"]
    st.close()
    return trace, stats, comps


@pytest.mark.gpu
@pytest.mark.parametrize("spec", SCHEMAS, ids=lambda s: "%s-%s-%s" % s[:3])
def test_small_batch_path_equals_large_path_and_oracle(gpu, oracle_lib, monkeypatch, spec):
    small, s_stats, s_comp = _run(oracle_lib, spec, True, monkeypatch)
    large, l_stats, l_comp = _run(oracle_lib, spec, False, monkeypatch)
    assert small == large
    assert s_stats["small"] >= 10 and l_stats["small"] == 0 and l_stats["large"] >= 12
    assert s_comp > 0 and l_comp > 0


@pytest.mark.gpu
def test_staged_large_batch_keeps_last_operation(gpu, oracle_lib, monkeypatch):
    """A staged batch past the small path (5,000 rows, a third of the keys repeated with mixed
    operations) is sorted on the device and reduced to the last row of each key: the same root and
    rank order as the model folding the rows in order, with no host sort."""
    from rsos_hip import GpuFingerprintStore, RecordSchema
    monkeypatch.delenv("RSOS_HIP_SMALL_MAX", raising=False)
    sch = RecordSchema.dated("bytes16", "bytes64")
    rng = np.random.default_rng(11)
    model = Model(oracle_lib, sch)
    st = GpuFingerprintStore(sch)
    for rnd in range(3):
        cols, ops = _batch(rng, sch, model, 5000, True, repeats=True)
        st.stage(cols, ops)
        model.apply(cols, ops)
        root, size = model.root()
        agg = st.aggregate()
        assert (agg.size, agg.fingerprint.to_int()) == (size, root), rnd
    keys = model.sorted_keys()
    assert np.array_equal(st.fingerprints(), np.stack([np.frombuffer(model.d[k], np.uint8) for k in keys]))
    assert st.batch_stats()["large"] >= 3
    st.close()


@pytest.mark.gpu
def test_failed_small_merge_is_reported_and_sticks_until_a_load(gpu, oracle_lib):
    """A small batch commits on the host once its first kernel's result word lands, with the delta
    merge still queued behind it.  If that merge fails, the next call on the store reports it
    (RH_ERR_HIP, naming the small batch's merge), and so does every call after it -- the host's
    bookkeeping is ahead of the device -- until a load replaces the contents (fail point
    "small_batch.merge" stands in for the device fault)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, _abi as A
    sch = RecordSchema.plain("u64", "u64")
    rng = np.random.default_rng(9)
    st = GpuFingerprintStore(sch)
    cols = _gen(rng, sch, 2000, False)
    order = np.argsort(cols["keys"].copy().view("<u8").ravel())
    cols = {c: v[order] for c, v in cols.items()}
    _, first = np.unique(cols["keys"], axis=0, return_index=True)
    cols = {c: v[np.sort(first)] for c, v in cols.items()}
    st.load_bulk(cols)
    n0 = st.size()
    one = _gen(rng, sch, 1, False)
    A.check(A.lib().rh_debug_fail_point(b"small_batch.merge"), "fail point")
    st.apply(one, np.zeros(1, np.uint8))  # commits: the merge's failure is not known yet
    for _ in range(2):
        with pytest.raises(A.RsosHipError) as e:
            st.size()
        assert e.value.code == A.ERR_HIP and "small batch's delta merge failed" in str(e.value)
    with pytest.raises(A.RsosHipError):
        st.aggregate()
    st.load_bulk(cols)  # a load replaces the contents: the store works again
    assert st.size() == n0
    st.apply(one, np.zeros(1, np.uint8))
    assert st.size() == n0 + 1
    assert st.batch_stats()["small"] >= 2
    st.close()
