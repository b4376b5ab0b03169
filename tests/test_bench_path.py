"""bench.py's multi-GPU path, end to end.

GPU (one MI355X): the exact path the driver's N-GPU run times -- bench.py starting its own ranks
(torch.distributed.run child), each rank lifting its key-range shard on a high-priority stream,
gather_async of the per-shard (R x 40 B) aggregates after every step, the device
combine_aggregates -- run at world size 2 with gloo (both ranks share the one GPU), checked bit
for bit against the same workload in one process, and against an independent torch reduction of
the whole set's lifts.  Strong scaling: both runs hash the same 100 M-shaped data set (the
synthetic generator is counter-based, so a shard is the same rows at any world size).

CPU: the launcher's argument checks (no GPU needed).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M256 = 1 << 256


def _bench(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_refuses_more_gpus_than_visible():
    """--gpus 2 on a host with fewer GPUs must fail loudly, not report a one-GPU number."""
    import torch
    have = torch.cuda.device_count()
    r = _bench(["--gpus", str(have + 1), "--steps", "1", "--warmup", "0"], timeout=120)
    assert r.returncode != 0
    assert "GPU" in (r.stderr + r.stdout)


def test_bench_refuses_world_size_mismatch():
    r = _bench(["--gpus", "2", "--steps", "1"], env_extra={"WORLD_SIZE": "3", "RANK": "0"}, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in (r.stderr + r.stdout)


def _agg_int(row):
    return sum((int(x) & (2**64 - 1)) << (64 * i) for i, x in enumerate(row[:4]))


@pytest.mark.gpu
def test_bench_world2_gloo_equals_single_process(tmp_path, gpu):
    total = 3_000_001  # not a multiple of the world size: shards of 1,500,000 and 1,500,001
    common = ["--config", "config4", "--records", str(total), "--steps", "3", "--warmup", "1",
              "--cpu-baseline", "0", "--e2e", "0", "--spinup-ms", "0", "--check", "0"]
    one, two = tmp_path / "one.json", tmp_path / "two.json"
    r1 = _bench(common + ["--gpus", "1", "--dump-aggregates", str(one)])
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = _bench(common + ["--gpus", "2", "--dump-aggregates", str(two)], env_extra={"BENCH_BACKEND": "gloo"})
    assert r2.returncode == 0, r2.stderr[-3000:]
    line2 = json.loads(r2.stdout.strip().splitlines()[-1])
    assert line2["n_gpus"] == 2 and line2["dist"] == {"backend": "gloo", "world_size": 2}
    assert line2["scaling"] == "strong"
    assert line2["config"]["records_per_rank"] == [1_500_000, 1_500_001]
    a, b = json.loads(one.read_text()), json.loads(two.read_text())
    assert a["world"] == 1 and b["world"] == 2
    assert a["ranges"] == b["ranges"]  # the 16 combined range aggregates, bit for bit
    # and the whole set's root against an independent torch reduction of its lifts
    import torch
    from rsos_hip import RecordSchema, lift_records
    from rsos_hip.synth import make_records
    s = RecordSchema.dated("bytes16", "bytes64")
    cols = make_records(s, total, seed=42, key_space=total)
    fps, _ = lift_records(s, cols, block_sums=False)
    limbs16 = fps.view(torch.int16).to(torch.int64) & 0xFFFF
    col = limbs16.sum(dim=0).cpu().tolist()
    want = sum(int(c) << (16 * i) for i, c in enumerate(col)) % M256
    assert sum(_agg_int(r) for r in a["ranges"]) % M256 == want
    assert sum(int(r[4]) for r in a["ranges"]) == total
    # equal-count ranges: range j holds rows [total*j/16, total*(j+1)/16)
    assert [int(r[4]) for r in a["ranges"]] == [total * (j + 1) // 16 - total * j // 16 for j in range(16)]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [4, 8])
def test_bench_world_n_gloo_equals_single_process(tmp_path, gpu, world):
    """The driver's N = 4 / 8 sharding rehearsed on one GPU (gloo; every rank shares the card):
    bench.py starts `world` ranks, each lifts its uneven key-range shard of one 3,000,007-record
    set, and the 16 combined range aggregates equal the one-process run's bit for bit."""
    total = 3_000_007
    common = ["--config", "config4", "--records", str(total), "--steps", "2", "--warmup", "1",
              "--cpu-baseline", "0", "--e2e", "0", "--spinup-ms", "0", "--check", "0"]
    one, many = tmp_path / "one.json", tmp_path / "many.json"
    r1 = _bench(common + ["--gpus", "1", "--dump-aggregates", str(one)])
    assert r1.returncode == 0, r1.stderr[-3000:]
    rn = _bench(common + ["--gpus", str(world), "--dump-aggregates", str(many)], env_extra={"BENCH_BACKEND": "gloo"},
                timeout=300)
    assert rn.returncode == 0, rn.stderr[-3000:]
    line = json.loads(rn.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["dist"] == {"backend": "gloo", "world_size": world}
    assert line["config"]["records_per_rank"] == [total * (r + 1) // world - total * r // world for r in range(world)]
    a, b = json.loads(one.read_text()), json.loads(many.read_text())
    assert b["world"] == world and a["ranges"] == b["ranges"]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_config5_routed_batches_equal_one_store(tmp_path, gpu, world):
    """config5 at N ranks (gloo rehearsal on one GPU): every step's global batch of N x --batch
    random records is routed by key range, each rank applies what its shard owns, and the per-shard
    roots are all_gathered and carry-added on the device.  The combined root and 16 key-range
    aggregates must equal, bit for bit, one store that loaded the whole resident set and applied
    every global batch (src/replica/dispatch.rs:188-196)."""
    import torch
    from rsos_hip import GpuFingerprintStore, RecordSchema
    from rsos_hip.store import KeyRange
    from rsos_hip.synth import make_records
    n, m, warm, steps = 200_000, 20_000, 1, 3
    out = tmp_path / "c5.json"
    r = _bench(["--config", "config5", "--records", str(n), "--batch", str(m), "--steps", str(steps), "--warmup",
                str(warm), "--cpu-baseline", "0", "--spinup-ms", "0", "--gpus", str(world), "--dump-aggregates",
                str(out)], env_extra={"BENCH_BACKEND": "gloo"}, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world and line["dist"] == {"backend": "gloo", "world_size": world}
    got = json.loads(out.read_text())
    s = RecordSchema.dated("bytes16", "bytes64")
    total = n * world
    st = GpuFingerprintStore(s)
    st.load_bulk_device(make_records(s, total, seed=42, key_space=total))
    for k in range(warm + steps):
        st.apply_device(make_records(s, m * world, seed=1000 + k, random_keys=True))
    root = st.aggregate()
    assert got["root"] == [x - (1 << 64) if x >> 63 else x for x in root.fingerprint.limbs] + [root.size]
    assert line["root_size"] == root.size
    bk = [bytes(make_records(s, 1, seed=42, first_index=total * j // 16, key_space=total)["keys"].cpu().numpy().tobytes())
          for j in range(1, 16)]
    for j in range(16):
        a = st.aggregate(KeyRange(None if j == 0 else bk[j - 1], None if j == 15 else bk[j]))
        assert got["ranges"][j] == [x - (1 << 64) if x >> 63 else x for x in a.fingerprint.limbs] + [a.size]
    st.close()
    torch.cuda.synchronize()


def test_records_by_index_equal_the_rows_of_the_set():
    """bench.py's overwrites regenerate the picked resident rows from their global indices
    (make_records(indices=...)) instead of gathering them from the 10^8-row columns: the same bytes
    as the rows of the whole set, for byte and integer keys (CPU, no GPU needed)."""
    import torch
    from rsos_hip import RecordSchema
    from rsos_hip.synth import make_records
    for s in (RecordSchema.dated("bytes16", "bytes64"), RecordSchema.plain("u64", "u64")):
        whole = make_records(s, 50_000, seed=42, device="cpu", first_index=200_000, key_space=400_000)
        rows = torch.randperm(50_000, generator=torch.Generator().manual_seed(3))[:4_000]
        picked = make_records(s, 4_000, seed=42, device="cpu", key_space=400_000, indices=rows + 200_000)
        assert set(picked) == set(whole)
        for c in whole:
            assert torch.equal(whole[c][rows], picked[c]), c
