"""The Rust binding's insert path through the C ABI (examples/insert_latency.c): one rh_store_stage
per record, then a question that applies the staged rows as one device batch (and folds it into the
host tier).  The root and size it reports must equal the oracle FingerprintTreeMap's after the same
inserts, one at a time (rsos/src/fingerprint_tree_map/mutate.rs:23-88); and the write -> round cycle
of examples/rbsr_latency.c (write rows staged into both replicas, then a whole reconciliation) must
run the same rounds from the host tier as from the device, without copying the map again."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "reconcile-rs_amd", "examples")
M64 = (1 << 64) - 1


def splitmix64(i: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (i.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def oracle_root(O, n, m):
    """The FTM restatement after loading the resident keys, then inserting m keys one by one."""
    res = np.unique(splitmix64(np.arange(n, dtype=np.uint64)))
    ins = splitmix64(np.arange(n, n + m, dtype=np.uint64))
    keys = np.concatenate([res, ins])
    with np.errstate(over="ignore"):
        vals = keys * np.uint64(2654435761)
    sc = O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0)
    r = O.Records(sc, keys.view(np.uint8).reshape(-1, 8), vals.view(np.uint8).reshape(-1, 8))
    t = O.FingerprintTreeMap(r)
    t.fill(0, len(keys))
    fp, size = t.root()
    return len(res), fp, size


def test_generator_restated():
    """The harness's SplitMix64 and the test's agree on known values (no GPU needed)."""
    z = splitmix64(np.array([0, 1, 41], dtype=np.uint64))
    assert [int(x) for x in z] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, int(z[2])]


@pytest.mark.gpu
@pytest.mark.parametrize("tier,batches,m", [(0, 1, 100_000), (1, 1, 100_000), (1, 1, 50_000), (1, 7, 50_000)])
def test_staged_inserts_root_equals_oracle_ftm(gpu, oracle_lib, tier, batches, m):
    n = 100_000
    r = subprocess.run([os.path.join(EX, "insert_latency"), str(n), str(m), str(tier), str(batches)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    nr, fp, size = oracle_root(oracle_lib, n, m)
    assert out["resident"] == nr and out["size"] == size
    want = "".join("%016x" % (int(fp[q]) & M64) for q in (3, 2, 1, 0))
    assert out["root"] == want
    if tier and m <= 65_536:  # within the tier's delta bound (max(base / 8, 2^16)): folded, never copied
        assert out["tier_refreshes"] == 0 and out["tier_folds"] == batches


@pytest.mark.gpu
@pytest.mark.parametrize("d,wrows", [(1, 1), (1, 1000), (7, 300)])
def test_write_round_cycle_host_tier_equals_device(gpu, d, wrows):
    n = 200_000
    out = {}
    for tier in (0, 1):
        r = subprocess.run([os.path.join(EX, "rbsr_latency"), str(n), str(d), "4", str(tier), str(wrows)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        out[tier] = json.loads(r.stdout)
    keys = ("rounds", "ranges", "idlists", "enumerated", "wire_bytes")
    assert {k: out[0][k] for k in keys} == {k: out[1][k] for k in keys}
    # every write batch was folded into the tier; the map was never copied down again
    assert out[1]["tier_refreshes"] == 0 and out[1]["tier_folds"] == 4
