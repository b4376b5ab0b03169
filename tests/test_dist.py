"""Multi-process (gloo, world_size 2, CPU) test of the sharded path's exchange step: key-range
shards, per-shard partial range aggregates, all_gather of the (R x 5) int64 aggregates, and the
carry-add combine -- equal to the same range aggregates over the unsharded set.

No GPU here: each rank's per-shard aggregates are computed by the oracle (test infrastructure)
in place of the kernels; the code under test is rsos_hip.shard (range intersection, gather,
combine) and the synthetic key-range sharding of rsos_hip.synth.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, n, R, out_q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reconcile-rs_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from rsos_hip import RecordSchema
        from rsos_hip.shard import combine_host, equal_count_ranges, gather, local_ranges, shard_rows
        from rsos_hip.synth import make_records, to_host
        s = RecordSchema.dated("bytes16", "bytes64")
        base, _ = shard_rows(rank, world, n)
        cols = make_records(s, n, seed=42, device="cpu", first_index=base, key_space=n * world)
        h = to_host(cols)
        sc = O.Schema(s.key_kind, s.key_len, s.value_kind, s.value_len, s.record_kind, 0)
        fps = O.Records(sc, h["keys"], h["values"], h["phys"], h["logical"], h["node"]).lift(threads=2)
        ranges = equal_count_ranges(n * world, R)
        lo, hi = local_ranges(ranges, base, n)
        # per-range aggregates of this shard (lo[j] .. hi[j])
        aggs = []
        for a, b in zip(lo, hi):
            (limbs, size), = O.range_aggregates(fps, [a, b]) if b > a else [([0, 0, 0, 0], 0)]
            aggs.append(limbs + [size])
        out = torch.tensor(np.array(aggs, dtype=np.uint64).view(np.int64), dtype=torch.int64)
        g = gather(dist, out)  # (world, R, 5)
        parts = []
        for p in range(world):
            rows = g[p].numpy().view(np.uint64)
            parts.append([(sum(int(x) << (64 * i) for i, x in enumerate(r[:4])), int(r[4])) for r in rows])
        combined = combine_host(parts)
        # keys must be globally sorted across the shard boundary
        first_key, last_key = h["keys"][0].tobytes(), h["keys"][-1].tobytes()
        edge = torch.tensor(np.frombuffer(first_key + last_key, np.uint8).astype(np.int64))
        edges = [torch.empty_like(edge) for _ in range(world)]
        dist.all_gather(edges, edge)
        if rank == 0:
            out_q.put(("ok", combined, [e.numpy().astype(np.uint8).tobytes() for e in edges]))
    except Exception as e:  # surface the failure to the parent
        out_q.put(("err", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_sharded_range_aggregates_gloo_world2(oracle_lib):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reconcile-rs_amd"))
    from rsos_hip import RecordSchema
    from rsos_hip.shard import equal_count_ranges
    from rsos_hip.synth import make_records, to_host
    world, n, R = 2, 3000, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, R, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, combined, edges = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert status == "ok", combined
    # shards are consecutive key ranges: last key of shard 0 < first key of shard 1
    assert edges[0][16:] < edges[1][:16]
    # reference: the same ranges over the unsharded set
    O = oracle_lib
    s = RecordSchema.dated("bytes16", "bytes64")
    sc = O.Schema(s.key_kind, s.key_len, s.value_kind, s.value_len, s.record_kind, 0)
    fps = []
    for r in range(world):
        h = to_host(make_records(s, n, seed=42, device="cpu", first_index=r * n, key_space=n * world))
        fps.append(O.Records(sc, h["keys"], h["values"], h["phys"], h["logical"], h["node"]).lift(threads=2))
    allf = np.concatenate(fps)
    for j, (a, b) in enumerate(equal_count_ranges(n * world, R)):
        (limbs, size), = O.range_aggregates(allf, [a, b])
        assert combined[j] == (sum(x << (64 * i) for i, x in enumerate(limbs)), size)
