"""The host tier under large write batches (examples/tier_interleave.c): batches the tier's delta
tree cannot take start a background refresh (csrc/rsos_hip_abi.hip start_refresh: the device
compacts, a copy stream brings the new base down), the drives in between are answered by the
device, and writes go on without waiting for the copy; batches the tree takes are folded.  Whatever the path,
every reconciliation between the two replicas (FixedFanOut(16), the reference's
reconciliation_drive, benches/protocol.rs:455-520) sees the same rounds, ranges, IDLIST ranges and
enumerated keys as with the tier off -- the device path, itself checked round by round against
oracle/rbsr.py by tests/test_rbsr_latency.py / tests/test_rbsr.py."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "reconcile-rs_amd", "examples", "tier_interleave")


@pytest.mark.gpu
@pytest.mark.parametrize("shape,n,m,policy", [("u64", 200_000, 80_000, "1"), ("c5", 200_000, 80_000, "1"),
                                              ("u64", 200_000, 80_000, "0"), ("c5", 200_000, 80_000, "0"),
                                              ("u64", 200_000, 2_000, "1"), ("c5", 300_000, 500, "1")])
def test_interleaved_drives_equal_device_path(gpu, shape, n, m, policy):
    """policy: RSOS_HIP_TIER_SYNC -- 1 (the default: writes keep the tier fresh; batches past the
    tree take run copies) or 0 (writes never wait; the device answers while a copy is in flight)."""
    out = {}
    env = dict(os.environ, RSOS_HIP_TIER_SYNC=policy)
    for tier in (0, 1):
        r = subprocess.run([EX, str(n), str(m), "5", str(tier), shape, "1"], capture_output=True, text=True,
                           timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        out[tier] = json.loads(r.stdout)
    keys = ("size", "rounds", "ranges", "idlists", "enumerated", "wire_bytes")
    assert {k: out[0][k] for k in keys} == {k: out[1][k] for k in keys}
    assert out[1]["size"] == n + 6 * m and out[1]["idlists"] >= 1
    if m > 65_536:  # past the tier's delta tree (max(2^16, min(n / 8, 2^18)) at these sizes): refreshed
        assert out[1]["tier_refreshes"] >= 1 and out[1]["tier_folds"] == 0
    else:  # folded, never copied again
        assert out[1]["tier_refreshes"] == 0 and out[1]["tier_folds"] == 5  # store a's folds


@pytest.mark.gpu
@pytest.mark.parametrize("policy", ["1", "0"])
@pytest.mark.parametrize("shape", ["u64", "c5"])
def test_small_writes_after_large_batches(gpu, shape, policy):
    """After each large batch (a run copy under the default policy) three single rows staged into
    both replicas, each followed by a reconciliation: the rows fold into the tier's tree over base +
    run copy (no copy), and every reconciliation sees what the device path sees.  policy "0"
    (writes never wait): the large batch starts a background run copy (or a base refresh after a
    compaction) that the small writes overtake, so the device answers those drives; the answers
    must still be the device path's."""
    # 130 k rows: past the tree (RSOS_HIP_TIER_TREE=50000 here, as the map grows past n / 8) -> a
    # run copy, and past the compaction threshold (n / 6) every second batch -> a base refresh:
    # both paths, then folds
    n, m, small = 1_000_000, 130_000, 3
    out = {}
    env = dict(os.environ, RSOS_HIP_TIER_TREE="50000", RSOS_HIP_TIER_SYNC=policy)
    for tier in (0, 1):
        r = subprocess.run([EX, str(n), str(m), "4", str(tier), shape, "1", str(small)], capture_output=True,
                           text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr
        out[tier] = json.loads(r.stdout)
    keys = ("size", "rounds", "ranges", "idlists", "enumerated", "wire_bytes")
    assert {k: out[0][k] for k in keys} == {k: out[1][k] for k in keys}
    assert out[1]["size"] == n + 5 * m + 4 * small and out[1]["small_cycles"] == 4 * small
    if policy == "1":
        assert out[1]["tier_folds"] == 4 * small  # store a's: every staged row folded, no large batch
        assert out[1]["tier_refreshes"] >= 4  # every large batch: a run copy or a base refresh
