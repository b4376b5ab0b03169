#!/usr/bin/env python3
"""bench.py -- device-resident fingerprint-hash throughput of the reconcile-rs hot path on MI355X.

One step = one pass of the path over one batch resident in HBM:
  lift every record of this GPU's key-range shard (BLAKE3 over the synthesised canonical
  encoding, fused with the 256-row block sums) -> super-block sums -> the R = 16 range
  aggregates of rbsr's default fan-out (rbsr/src/protocol.rs:40) -> (N > 1) all_gather of the
  per-shard (R x 40 B) aggregates over RCCL + carry-add combine.

Default workload (BASELINE.json configs[3], the north_star's shape): 100 M records in total,
16 B key / 64 B value, dated (FingerprintTreeMap<[u8;16], Entry<Timestamp, Vec<u8>>>, 120
canonical bytes per record), one globally key-sorted set cut into N equal-count key-range
shards.  Strong scaling: at N = 1 one MI355X holds all 100 M records (the north_star target);
at N = 8 each GPU holds 12.5 M.  `--config config2` is BASELINE configs[1] (10 M per GPU, weak).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config config1|config2|config3|config3_full|config4|config5|encoded|snapshot|rbsr|bench_u32]

--gpus N > 1 without a launcher: bench.py starts `python -m torch.distributed.run
--nproc-per-node N` as a child process (no exec) and exits with its status; under a launcher
(RANK / WORLD_SIZE set) WORLD_SIZE must equal N.  Fewer visible GPUs than N is an error.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.environ.get("RSOS_HIP_TREE") or os.path.join(ROOT, "reconcile-rs_amd"))  # override: A/B of builds

import torch  # noqa: E402

CONFIGS = {
    # name: (key, value, record kind, records, description); `records` are per GPU (weak scaling)
    # unless the config is in STRONG (the total, cut into one key-range shard per GPU)
    "config1": ("u64", "bytes64", "plain", 1_000_000,
                "BASELINE configs[0]: the reference's CPU case, FingerprintTreeMap<u64, Vec<u8>> of {per} "
                "u64-key / 64 B-value records per GPU (GPU lift beside the CPU fill)"),
    "config2": ("bytes16", "bytes64", "dated", 10_000_000,
                "BASELINE configs[1]: {per} records per GPU, 16 B key / 64 B value, dated Entry<Timestamp,Vec<u8>>"),
    "config3": ("bytes16", "bytes1024", "dated", 10_000_000,
                "BASELINE configs[2] shape: {per} records per GPU, 16 B key / 1 KiB value, dated"),
    "config3_full": ("bytes16", "bytes1024", "dated", 100_000_000,
                     "BASELINE configs[2]: {total} records in total ({per} per GPU), 16 B key / 1 KiB value, dated"),
    "config4": ("bytes16", "bytes64", "dated", 100_000_000,
                "BASELINE configs[3] (north_star shape): {total} records in total, 16 B key / 64 B value, dated "
                "Entry<Timestamp,Vec<u8>>, key-range sharded over {world} GPU(s) ({per} per GPU)"),
    "bench_u32": ("u32", "u32", "plain", 10_000_000,
                  "benches/bench.rs fill shape: FingerprintTreeMap<u32,u32>, {per} records per GPU"),
    "config5": ("bytes16", "bytes64", "dated", 100_000_000,
                "BASELINE configs[4]: 1M random inserts per batch into a 100M-record resident map"),
    "rbsr": ("bytes16", "bytes64", "dated", 10_000_000,
             "rbsr reconciliation (SURVEY 8a row a13): two GPU-resident replicas of 10M records/GPU "
             "(16 B key / 64 B value, dated) differing in --diffs keys, FixedFanOut(16) rounds until no "
             "segment is left"),
    "encoded": ("bytes16", "bytes64", "dated", 10_000_000,
                "the drop-in encoded map (HipEncodedMap / EncodedFingerprintMap over rh_estore_*): {per} records "
                "per GPU of Entry<Timestamp, Vec<u8>> with [u8; 16] keys and 64 B values as canonical bytes "
                "(120 B each, what rsos::encoding::encode_to_vec gives), hashed by the fixed-length kernel"),
    "snapshot": ("bytes16", "bytes64", "dated", 10_000_000,
                 "snapshot reload (SURVEY 8f row 4): RCNL v1 file of 10M entries (16 B key / 64 B value, "
                 "10% tombstones) resident in HBM -> dated + projection stores"),
}
STRONG = {"config4", "config3_full"}  # total fixed as N grows
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level table (spec)


def _count(x: int) -> str:
    return f"{x / 1e6:g}M" if x % 100_000 == 0 else str(x)


def describe(config: str, total: int, per: int, world: int) -> str:
    return CONFIGS[config][4].format(total=_count(total), per=_count(per), world=world)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="config4", choices=sorted(CONFIGS))
    p.add_argument("--records", type=int, default=0,
                   help="override the record count: the total for config4 / config3_full (strong scaling), "
                        "per GPU for the others")
    p.add_argument("--ranges", type=int, default=16)
    p.add_argument("--dump-aggregates", default="", help="write the step's combined range aggregates (JSON) here")
    p.add_argument("--cpu-baseline", type=int, default=1, help="0 to skip the CPU baseline leg")
    p.add_argument("--cpu-sample", type=int, default=0,
                   help="records in the CPU baseline sample (0: min(shard, 10M), ~3 s of serial fill)")
    p.add_argument("--batch", type=int, default=1_000_000, help="config5: records per update batch")
    p.add_argument("--pipeline", type=int, default=1,
                   help="config5: 1 = the timed batches through one apply_device_many call (batch i + 1 "
                        "key-sorted while batch i's result returns); 0 = one apply_device call per batch")
    p.add_argument("--compact-div", type=int, default=0,
                   help="config5: compaction divisor (the delta run merges into the base past base / divisor rows; "
                        "0 = the library's default)")
    p.add_argument("--overwrite", type=float, default=0.0,
                   help="config5: fraction of each batch that re-stamps existing keys (the new - old delta)")
    p.add_argument("--e2e", type=int, default=-1,
                   help="also time host->device->host end to end (DESIGN.md): 1 on, 0 off; "
                        "default on for config2 at one GPU")
    p.add_argument("--diffs", type=int, default=10_000, help="rbsr: keys in which the two replicas differ")
    p.add_argument("--dual", action="store_true",
                   help="dated configs: both lifts of Replica::map_insert (dated + projection) per record")
    p.add_argument("--check", type=int, default=1, help="oracle spot-check of a sample before timing")
    p.add_argument("--spinup-ms", type=float, default=300.0,
                   help="untimed lift launches for this long before the warmup steps: the GPU raises its "
                        "clocks over the first ~50 ms of load (DESIGN.md section 6)")
    return p.parse_args()


def gpu_spinup(ms: float, dev) -> dict:
    """Untimed, stateless device load (lifts of 4 M synthetic records) until `ms` of wall time
    have passed, so the timed steps run at the clocks the chip sustains rather than during its
    ramp from idle.  Touches no state any workload reads."""
    from rsos_hip import RecordSchema, lift_records
    from rsos_hip.synth import make_records
    if ms <= 0:
        return {"ms": 0, "launches": 0}
    # u64 / u64 plain records: a lift instantiation no workload here uses, so kernel statistics
    # and counter passes keep the workload's launches apart from these
    schema = RecordSchema.plain("u64", "u64")
    cols = make_records(schema, 4_000_000, seed=99, device=dev)
    torch.cuda.synchronize()
    t0, k = time.perf_counter(), 0
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(20):
            lift_records(schema, cols)
        k += 20
        torch.cuda.synchronize()
    del cols
    torch.cuda.synchronize()
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "launches": k}


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 from a plain `python bench.py`: start N ranks (one per GPU) under
    torch.distributed.run as a child process and return its exit status.  Nothing here touches
    the GPU (torch.cuda.device_count() does not initialise it), so the parent never holds a
    device while the ranks run.  None: this process is already a rank (or N = 1)."""
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        return None
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    have = torch.cuda.device_count()
    if have < 1:
        raise SystemExit("bench: no GPU visible")
    # gloo rehearsal (BENCH_BACKEND=gloo) may put several ranks on one GPU; RCCL needs one each
    if args.gpus > have and backend == "nccl":
        raise SystemExit(f"bench: --gpus {args.gpus} but only {have} GPU(s) are visible")
    if args.gpus == 1:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # a torch.distributed launcher (it sets RANK / WORLD_SIZE) gets the process group even at
    # world size 1, so the RCCL path (init, all_gather, barrier, all_reduce) also runs on one GPU
    launched = "RANK" in os.environ and "WORLD_SIZE" in os.environ
    if world > 1 or launched:
        import torch.distributed as dist
        backend = os.environ.get("BENCH_BACKEND", "nccl")  # gloo: functional rehearsal only
        ngpu = torch.cuda.device_count()
        if backend == "nccl" and world > ngpu:
            raise SystemExit(f"bench: {world} ranks but only {ngpu} GPU(s): RCCL needs one GPU per rank")
        torch.cuda.set_device(local % max(ngpu, 1))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import rsos_hip
    from rsos_hip import RecordSchema, lift_records, lift_dual, range_aggregates, reduce_blocks, combine_aggregates
    from rsos_hip.synth import make_records
    from rsos_hip.shard import equal_count_ranges, gather_async, local_ranges

    if args.config == "config5":
        return incremental(args, world, rank, dev, dist)
    if args.config == "snapshot":
        return reload(args, world, rank, dev, dist)
    if args.config == "encoded":
        return encoded(args, world, rank, dev, dist)
    if args.config == "rbsr":
        return reconcile(args, world, rank, dev, dist)
    kname, vname, kind, n_default, _ = CONFIGS[args.config]
    strong = args.config in STRONG
    if strong:  # equal-count key-range shards of one fixed total: rank r holds [r*T/N, (r+1)*T/N)
        total = args.records or n_default
        base = total * rank // world
        n = total * (rank + 1) // world - base
    else:       # every rank holds its own n-record shard of one n*N-record set
        n = args.records or n_default
        total = n * world
        base = rank * n
    desc = describe(args.config, total, n, world)
    schema = getattr(RecordSchema, kind)(kname, vname)
    rec_bytes = schema.record_len()                     # canonical bytes BLAKE3 absorbs
    read_bytes = schema.key_row + schema.value_row + (20 if schema.dated_kind else 0)
    hbm_bytes = read_bytes + 32                          # + fingerprint write
    dual = args.dual and kind == "dated"
    if dual:  # + the projection's canonical bytes and its fingerprint (src/replica/write.rs:44-45)
        rec_bytes += schema.with_kind(2).record_len()
        hbm_bytes += 32

    # this rank's shard of the globally sorted key space: global rows [base, base + n)
    cols = make_records(schema, n, seed=42, device=dev, first_index=base, key_space=total)
    if dist is not None:
        # the steps run on a high-priority stream: HIP maps it to its own hardware queue, so RCCL's
        # per-step all_gather (a normal-priority stream) cannot sit in front of the next lift
        torch.cuda.synchronize()
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))
    R = args.ranges
    lo_l, hi_l = local_ranges(equal_count_ranges(total, R), base, n)
    lo = torch.tensor(lo_l, dtype=torch.int64, device=dev)
    hi = torch.tensor(hi_l, dtype=torch.int64, device=dev)

    nb = (n + 255) // 256
    fps = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    bs = torch.empty((nb, 32), dtype=torch.uint8, device=dev)
    dual_out = (fps, bs, torch.empty((n, 32), dtype=torch.uint8, device=dev),
                torch.empty((nb, 32), dtype=torch.uint8, device=dev)) if dual else None
    # per-step aggregates and their gathers: RCCL runs each step's all_gather on its own stream
    # after that step's range queries; the compute stream never waits for it, so the ranks only
    # meet in the collectives and at the end, where every step's gather is combined
    outs = [torch.empty((R, 5), dtype=torch.int64, device=dev) for _ in range(2)]
    stream = torch.cuda.current_stream()

    # correctness gate before timing: sampled rows vs the oracle (rank 0)
    checked = None
    if args.check and rank == 0:
        checked = spot_check(schema, cols, n)

    lift_ms = []
    state = {"pending": [], "res": None, "k": 0}

    # each step's gather is combined on a side stream that waits for it (work.wait() inside the
    # side stream's context), so neither the compute stream nor the host ever waits for RCCL and
    # the combines overlap the following lifts instead of queueing up behind the last one
    side = torch.cuda.Stream(device=dev) if dist is not None else None

    def finish():  # the last step's combined aggregates, once every combine has been issued
        if side is not None:
            stream.wait_stream(side)
        state["pending"] = []
        return state["res"]

    def step(timed: bool):
        if dist is None:
            out = outs[state["k"] % 2]
        else:  # held by the pending gather until finish()
            out = torch.empty((R, 5), dtype=torch.int64, device=dev)
        if timed:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        if dual:
            lift_dual(schema, cols, out=dual_out)
        else:
            lift_records(schema, cols, fps=fps, bsums=bs)
        if timed:
            e1.record(stream)
            lift_ms.append((e0, e1))
        ss = reduce_blocks(bs)
        range_aggregates(fps, bs, ss, lo, hi, out=out)
        if dist is None:
            state["res"] = out
        else:
            g = torch.empty((world, R, 5), dtype=torch.int64, device=dev)
            work, g = gather_async(dist, out, g)
            side.wait_stream(stream)  # gloo: the gathered copy was made on the compute stream
            with torch.cuda.stream(side):
                work.wait()
                state["res"] = combine_aggregates(g)
            state["pending"].append((work, g, out))  # keeps the step's buffers alive
        state["k"] += 1

    spin = gpu_spinup(args.spinup_ms, dev)
    for _ in range(args.warmup):
        step(False)
    finish()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    res = finish()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    lift_avg_s = sum(a.elapsed_time(b) for a, b in lift_ms) / len(lift_ms) / 1e3

    root = res.cpu().numpy()  # the step's result: R combined range aggregates over all shards
    per_rank = [n]
    if dist is not None:  # every rank's record count, for the line (checked to cover the total)
        cnt = torch.tensor([n], dtype=torch.int64, device=dev)
        parts = [torch.empty_like(cnt) for _ in range(world)]
        dist.all_gather(parts, cnt)
        per_rank = [int(p.item()) for p in parts]
        if sum(per_rank) != total:
            raise SystemExit(f"bench: shards hold {sum(per_rank)} records, expected {total}")
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    if int(root[:, 4].sum()) != total:
        raise SystemExit(f"bench: combined range aggregates count {int(root[:, 4].sum())} records, expected {total}")
    if args.dump_aggregates:
        with open(args.dump_aggregates, "w") as f:
            json.dump({"world": world, "total": total, "ranges": [[int(x) for x in row] for row in root]}, f)

    recs = total * args.steps
    gib_s = recs * rec_bytes / elapsed / 2**30
    achieved = hbm_bytes * n / lift_avg_s / 1e9
    traffic = None if dual else load_traffic(args.config, n)
    line = {
        "metric": "fingerprint-hash GiB/s + M records/s (device-resident) at 1/2/4/8 MI355X",
        "value": round(gib_s, 2),
        "unit": "GiB/s",
        "mrec_per_s": round(recs / elapsed / 1e6, 1),
        "n_gpus": world,
        # the process group actually in use: "nccl" is RCCL on ROCm; "gloo" only in CPU-side rehearsals
        "dist": {"backend": dist.get_backend() if dist is not None else None,
                 "world_size": dist.get_world_size() if dist is not None else 1},
        "steps": args.steps,
        "warmup": args.warmup, "spinup": spin,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded, SURVEY §8d generator), resident in HBM before timing",
        "config": {"workload": desc + ("; both lifts of Replica::map_insert (dated + projection)" if dual else ""),
                   "records_per_gpu": n, "records_per_rank": per_rank, "records_total": total, "ranges": R,
                   "canonical_bytes_per_record": rec_bytes, "hbm_bytes_per_record": hbm_bytes,
                   "parallelism": f"key-range shards x{world}" + (
                       (" + RCCL all_gather per step (off the compute stream; combined at the end)" if dist.get_backend() == "nccl"
                        else " + gloo all_gather (rehearsal)") if dist is not None else "")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "rh::k_lift_dual (dated + projection lifts + block sums)" if dual else
                               "rh::k_lift (lift + block sums)", "kernel_avg_us": round(lift_avg_s * 1e6, 2)},
        "oracle_spot_check": checked,
        "total_aggregate_size": int(root[:, 4].sum()),
    }
    valu = None if dual else load_valu(args.config, n, lift_avg_s)
    if valu:
        line["valu"] = valu
    if args.cpu_baseline:  # rank 0 only, on the host's cores, once per run at every N
        line["cpu_baseline"] = cpu_baseline(schema, cols, args.cpu_sample or min(n, 10_000_000), dual)
    if args.e2e == 1 or (args.e2e < 0 and args.config in ("config2", "config4") and world == 1):
        line["end_to_end"] = end_to_end(schema, cols, n)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _agg_row(a) -> list:
    """An Aggregate as the (fp limbs as int64 bit patterns, size) row the device combine takes."""
    return [x - (1 << 64) if x >> 63 else x for x in a.fingerprint.limbs] + [a.size]


def _route_keys(keys: torch.Tensor, splitters: torch.Tensor) -> torch.Tensor:
    """Owner shard of each 16-byte key: the number of shard splitters (the first key of shards
    1..N-1, memcmp order = the Ord of [u8; 16]) at or below it -- bisect_right over the splitters,
    as ShardedStore.apply routes (rsos_hip/sharded.py), on the device."""
    def words(k):  # big-endian u64 halves, sign-flipped so signed int64 order = unsigned order
        hi = k[:, :8].flip(1).contiguous().view(torch.int64).view(-1)
        lo = k[:, 8:16].flip(1).contiguous().view(torch.int64).view(-1)
        flip = torch.iinfo(torch.int64).min
        return hi ^ flip, lo ^ flip
    kh, kl = words(keys)
    sh, sl = words(splitters)
    owner = torch.zeros(keys.shape[0], dtype=torch.int64, device=keys.device)
    for j in range(splitters.shape[0]):
        owner += ((kh > sh[j]) | ((kh == sh[j]) & (kl >= sl[j]))).to(torch.int64)
    return owner


def incremental(args, world, rank, dev, dist):
    """config5: GPU-resident store of N records per GPU; each step applies one batch of `--batch`
    random records per GPU (insert-or-overwrite; fresh random 128-bit keys are essentially all new)
    through the device sort / search / merge / re-sum path.  Timed: apply_device_many over the
    steps' batches (or apply_device per batch), then the whole map's root.

    N > 1 ("the incremental config"): the resident set is one key-sorted set of N x n
    records cut into N equal-count key-range shards; every step's update batch is one global batch
    of N x --batch uniformly random records, routed by key range (the shard splitters) so that each
    rank applies exactly the updates its range owns -- the multi-GPU form of a replica's network
    merge (src/replica/dispatch.rs:188-196).  The per-shard roots (1 x 40 B each) are all_gathered
    over RCCL and carry-added on the device: the whole map's root (initial_ranges,
    rbsr/src/protocol.rs:100).  The routing is data preparation (untimed): a sender routes by key
    range before the records reach a shard."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, combine_aggregates
    from rsos_hip.synth import make_records
    from rsos_hip.shard import gather
    kname, vname, kind, n_default, desc = CONFIGS["config5"]
    n = args.records or n_default
    schema = getattr(RecordSchema, kind)(kname, vname)
    st = GpuFingerprintStore(schema, device=dev.index)
    if args.compact_div:
        st.set_compaction(args.compact_div, 65536)
    base = make_records(schema, n, seed=42, device=dev, first_index=rank * n, key_space=n * world)
    # shard splitters: the first key of every shard but the first (the generator is counter-based)
    splitters = torch.cat([make_records(schema, 1, seed=42, device=dev, first_index=r * n, key_space=n * world)["keys"]
                           for r in range(1, world)]) if world > 1 else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st.load_bulk_device(base)
    load_s = time.perf_counter() - t0
    m = args.batch
    m_over = int(m * args.overwrite)
    batches = []
    gen = torch.Generator(device=dev)
    gen.manual_seed(7 + rank)
    for k in range(args.warmup + args.steps):
        if world > 1:  # one global batch, routed by key range
            g = make_records(schema, m * world, seed=1000 + k, device=dev, random_keys=True)
            mine = (_route_keys(g["keys"], splitters) == rank).nonzero().view(-1)
            b = {c: t.index_select(0, mine).contiguous() for c, t in g.items()}
            del g
        else:
            b = make_records(schema, m, seed=1000 + k, device=dev, random_keys=True)
        if m_over:  # re-stamp distinct existing keys of this shard: an overwrite, the new - old delta (mutate.rs:31-41)
            rows = torch.randperm(n, generator=gen, device=dev)[:m_over]
            mo = min(m_over, b["keys"].shape[0])
            # the picked resident rows regenerated from their global indices (the generator is
            # counter-based), not gathered from the 10^8-row columns: torch's gathers of 10^8
            # output rows return wrong rows on this image (profiles/r04_torch_large_ops_repro.log)
            old = make_records(schema, mo, seed=42, device=dev, key_space=n * world, indices=rows[:mo] + rank * n)
            b["keys"][:mo] = old["keys"]
            b["phys"][:mo] = old["phys"] + 1_000_000
            del old
        batches.append(b)
    del base
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    # capacity for the map this run grows into (its resident rows plus every batch), reserved
    # before the first batch the way a replica sizes its store: no reallocation in the loop
    mmax = max(b["keys"].shape[0] for b in batches)
    reserved = n + sum(b["keys"].shape[0] for b in batches)
    st.reserve(reserved, mmax)
    spin = gpu_spinup(args.spinup_ms, dev)
    for k in range(args.warmup):
        st.apply_device(batches[k])
    def global_root():
        """The whole map's root: this shard's root, all_gathered with the others' and carry-added
        on the device (one shard: the root itself)."""
        a = st.aggregate()  # the shard's root, O(1) (the store keeps it on the host)
        if dist is None:
            return a
        root_t = torch.tensor([_agg_row(a)], dtype=torch.int64, device=dev)
        return combine_aggregates(gather(dist, root_t))

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    counts = [0, 0, 0]
    comp0 = st.stats()["compactions"]
    from rsos_hip import _abi as A
    A.check(A.lib().rh_debug_batch_timing(1), "rh_debug_batch_timing")  # HIP events around k_lift_search
    t0 = time.perf_counter()
    if args.pipeline:  # the queued batches drained in order by one call, then the root
        for c in st.apply_device_many(batches[args.warmup:args.warmup + args.steps]):
            counts = [a + b for a, b in zip(counts, c)]
        root_g = global_root()
    else:  # one batch at a time, the root exchanged after each
        for k in range(args.steps):
            c = st.apply_device(batches[args.warmup + k])
            counts = [a + b for a, b in zip(counts, c)]
            root_g = global_root()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ls_us, ls_n = C.c_double(), C.c_uint64()
    A.check(A.lib().rh_debug_batch_kernel_us(C.byref(ls_us), C.byref(ls_n)), "rh_debug_batch_kernel_us")
    A.check(A.lib().rh_debug_batch_timing(0), "rh_debug_batch_timing")
    applied = [sum(b["keys"].shape[0] for b in batches[args.warmup:args.warmup + args.steps])]
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor(counts + applied, dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        counts, applied = [int(x) for x in tot[:3].tolist()], [int(tot[3].item())]
    stats = st.stats()
    root_size = root_g.size if dist is None else int(root_g[0, 4].item())
    size_all = torch.tensor([st.size()], dtype=torch.int64, device=dev)
    if dist is not None:
        dist.all_reduce(size_all)
    if root_size != int(size_all.item()):  # the combined root counts every shard's rows
        raise SystemExit(f"bench: combined root counts {root_size} rows, the shards hold {int(size_all.item())}")
    dump = None
    if args.dump_aggregates:
        # the combined root and 16 key-range aggregates (bounds: the keys of equal-count rows of the
        # original resident set), for tests/test_bench_path.py to check against one store
        total = n * world
        bk = [make_records(schema, 1, seed=42, device=dev, first_index=total * j // 16, key_space=total)["keys"]
              for j in range(1, 16)]
        from rsos_hip.store import KeyRange
        parts = []
        for j in range(16):
            lo = None if j == 0 else bytes(bk[j - 1].cpu().numpy().tobytes())
            hi = None if j == 15 else bytes(bk[j].cpu().numpy().tobytes())
            a = st.aggregate(KeyRange(lo, hi))
            parts.append(_agg_row(a))
        loc = torch.tensor(parts, dtype=torch.int64, device=dev)
        comb = combine_aggregates(gather(dist, loc)) if dist is not None else loc
        rt = root_g if dist is not None else torch.tensor([_agg_row(root_g)], dtype=torch.int64)
        dump = {"world": world, "root": [int(x) for x in rt.cpu().view(-1).tolist()],
                "ranges": [[int(x) for x in row] for row in comb.cpu().tolist()]}
    if rank == 0:
        if dump is not None:
            with open(args.dump_aggregates, "w") as f:
                json.dump(dump, f)
        recs = applied[0]
        line = {
            "metric": "incremental update: batched inserts into a GPU-resident map (M records/s)",
            "value": round(recs / elapsed / 1e6, 2), "unit": "M records/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "spinup": spin,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded): sorted resident set + uniformly random update keys",
            "config": {"workload": desc + (f"; {args.overwrite:.0%} of each batch overwrites existing keys"
                                           if m_over else ""),
                       "resident_records_per_gpu": n, "batch": m, "overwrites_per_batch": m_over,
                       "parallelism": f"key-range shards x{world}" + (
                           " (each global batch of N x --batch records routed by key range; per-shard roots "
                           "all_gathered and carry-added on the device)" if world > 1 else "")},
            "dist": {"backend": (dist.get_backend() if dist is not None else None), "world_size": world},
            "batch_counts": {"new": counts[0], "overwritten": counts[1], "deleted": counts[2]},
            "root_size": root_size, "bulk_load_s": round(load_s, 3),
            "step": ("apply_device_many over the K queued batches (each: key sort, lift fused with the "
                     "base/delta searches, delta records + merge, amortised compaction; the next batch key-sorted while this one's result "
                     "returns) + the whole map's root" if args.pipeline else
                     "apply_device per batch (key sort, lift fused with the base/delta searches, delta "
                     "records + merge; amortised "
                     "compaction) + the whole map's root after each"),
            "compactions_in_timed_steps": stats["compactions"] - comp0, "delta_rows_at_end": stats["delta_rows"],
            "reserved_rows": reserved, "compaction_divisor": args.compact_div or 6,
            "roofline": config5_roofline(schema, n, m, args.compact_div or 6, elapsed / args.steps,
                                         ls_us.value / max(ls_n.value, 1), int(ls_n.value)),
        }
        if args.cpu_baseline:
            line["cpu_baseline"] = cpu_baseline_incremental(schema, m, args.cpu_sample or 10_000_000)
        print(json.dumps(line), flush=True)
    st.close()
    if dist is not None:
        dist.destroy_process_group()


def config5_roofline(schema, n, m, div, step_s, ls_us, launches):
    """config5's roofline ("config5: algorithmic bytes"): the dominant kernel,
    k_lift_search (the fused lift + base / delta searches), timed with HIP events on the store's
    stream over the timed batches (rh_debug_batch_timing), against its algorithmic bytes per
    launch; and the whole batch's steady-state byte model against ms_per_step.  traffic: the
    kernel's DRAM bytes per launch from the committed PMC summary (TCC_EA0_RDREQ_DRAM_32B x 32 +
    the write requests; scripts/pmc_c5.sh, pmc_c5_summary.py)."""
    rec = schema.key_row + (20 if schema.dated_kind else 0) + schema.value_row  # the record columns read
    line = 128  # one random key line per search (the tables and sample lines stay in L2)
    per_key = {"records": rec, "fingerprint_write": 32, "search_results": 2 * (4 + 1), "position": 4,
               "base_key_line": line, "delta_key_line": line}
    ls_bytes = m * sum(per_key.values())
    achieved = ls_bytes / (ls_us * 1e-6) / 1e9 if ls_us > 0 else 0.0
    # the batch, steady state: the delta run grows from 0 to T = n / div rows between compactions
    T = max(n // div, 65_536)
    batches_per_cycle = max(T / m, 1.0)
    terms = {
        "sort": m * (schema.key_row * 2 + 4),                       # keys read, sorted keys + positions written
        "lift_search": ls_bytes,
        "delta_records": m * (32 + 40 + 1),                         # fingerprints in, DeltaRecs + drop flags out
        "delta_merge": int((T / 2 + m) * (schema.key_row + 4) * 2),  # the run's (key, slot) rows read + written
        "compaction": int(((n + T / 2) * (schema.key_row + 32) * 2 + T * (schema.key_row + 4 + 40)) / batches_per_cycle),
    }
    batch_bytes = sum(terms.values())
    batch_gbs = batch_bytes / step_s / 1e9
    traffic = None
    p = _profile_any("pmc_config5.json")
    if p:
        try:
            with open(p) as f:
                k = next(v for name, v in json.load(f)["kernels"].items() if name.startswith("k_lift_search"))
            traffic = {"bytes_per_launch": int(k["dram_read_bytes"] + k["dram_write_bytes"]),
                       "source": os.path.relpath(p, ROOT)}
        except (OSError, ValueError, KeyError, StopIteration):
            traffic = None
    return {"bound": "hbm", "kernel": "k_lift_search", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "algorithmic_bytes_per_launch": ls_bytes, "algorithmic_bytes_per_key": per_key,
            "kernel_avg_us": round(ls_us, 2), "launches_timed": launches,
            "batch_model": {"algorithmic_bytes_per_batch": batch_bytes, "terms": terms,
                            "achieved": round(batch_gbs, 1), "frac": round(batch_gbs / HBM_PEAK_GBS, 4),
                            "delta_threshold_rows": T}}


def _profile_any(suffix):
    """The newest committed profiles/rNN_<suffix>, or None."""
    import glob
    ps = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_" + suffix)), reverse=True)
    return ps[0] if ps else None


def _encode_host(h) -> "np.ndarray":
    """(n, 120) canonical bytes of dated 16 B / 64 B present records from host columns (numpy,
    vectorised): u64 16 ‖ key ‖ phys ‖ logical ‖ node ‖ u32 0 ‖ u64 64 ‖ value -- the bytes
    rsos::encoding::encode_to_vec of the key then the Entry gives (rsos/src/encoding.rs:17-35)."""
    import numpy as np
    n = h["keys"].shape[0]
    out = np.empty((n, 120), np.uint8)
    out[:, 0:8] = np.frombuffer((16).to_bytes(8, "little"), np.uint8)
    out[:, 8:24] = h["keys"]
    out[:, 24:32] = h["phys"].view(np.uint8).reshape(n, 8)
    out[:, 32:36] = h["logical"].view(np.uint8).reshape(n, 4)
    out[:, 36:44] = h["node"].view(np.uint8).reshape(n, 8)
    out[:, 44:48] = 0
    out[:, 48:56] = np.frombuffer((64).to_bytes(8, "little"), np.uint8)
    out[:, 56:120] = h["values"]
    return out


def encoded(args, world, rank, dev, dist):
    """--config encoded: the drop-in map for serde K / V (HipEncodedMap, rust/rsos-hip/src/encoded.rs;
    its Python twin rsos_hip.emap.EncodedFingerprintMap) on the north_star record.  Records reach the
    library as canonical bytes (rsos::encoding::encode_to_vec of the key then the value,
    public-api/rsos.txt:61): here [u8; 16] keys and Entry<Timestamp, Vec<u8>> of 64 B, 120 B each.
    A batch whose records share one length is hashed by the compile-time fixed-length kernel
    (k_lift_fixed_ct<120>).  One step = one device-resident lift + block sums of the n encoded
    records (what rh_estore_load runs after its upload).  Also timed, once: the host encode
    (numpy, vectorised, for this fixed shape -- the Rust binding runs encode_to_vec per record), the
    fill (rh_estore_load from host bytes: the bulk path of just_insert_bulk /
    src/replica/write.rs:107-121 through the encoded store) and one 1 M-record batch
    (rh_estore_apply of rank-addressed inserts, the map's staged-batch flush).  The ABI calls are the
    ones HipEncodedMap::load_bulk / flush make; the Python map's own per-key index (a SortedList of
    Python objects) is not what is timed."""
    import ctypes as C
    import numpy as np
    from rsos_hip import RecordSchema, lift_fixed, lift_records, reduce_blocks
    from rsos_hip import _abi as A
    from rsos_hip.synth import make_records, to_host
    kname, vname, kind, n_default, desc = CONFIGS["encoded"]
    n = args.records or n_default
    m = min(args.batch, n)
    schema = getattr(RecordSchema, kind)(kname, vname)
    L = schema.record_len()
    cols = make_records(schema, n, seed=42, device=dev, first_index=rank * n, key_space=n * world)
    h = to_host(cols)
    t0 = time.perf_counter()
    rows = _encode_host(h)
    encode_s = time.perf_counter() - t0
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(L)
    es = C.c_void_p()
    A.check(A.lib().rh_estore_create(dev.index, C.byref(es)), "rh_estore_create")
    t0 = time.perf_counter()
    A.check(A.lib().rh_estore_load(es, rows.ctypes.data, offs.ctypes.data, n), "rh_estore_load")
    fill_s = time.perf_counter() - t0
    root0 = A.Aggregate()
    A.check(A.lib().rh_estore_root(es, C.byref(root0)), "rh_estore_root")
    # one batch of m fresh records, rank-addressed into the key order (the map's flush)
    b = make_records(schema, m, seed=1000 + rank, device=dev, random_keys=True)
    bh = to_host(b)
    order = np.argsort(bh["keys"].copy().view("S16").ravel(), kind="stable")
    bh = {k: np.ascontiguousarray(v[order]) for k, v in bh.items()}
    existing = h["keys"].copy().view("S16").ravel()
    bk = bh["keys"].copy().view("S16").ravel()
    pos = np.searchsorted(existing, bk).astype(np.uint64)
    present = (pos < n) & (existing[np.minimum(pos, n - 1)] == bk)
    kinds = present.astype(np.uint8)  # 0 insert, 1 overwrite
    t1 = time.perf_counter()
    brows = _encode_host(bh)
    bencode_s = time.perf_counter() - t1
    boffs = np.arange(m + 1, dtype=np.uint64) * np.uint64(L)
    t1 = time.perf_counter()
    A.check(A.lib().rh_estore_apply(es, pos.ctypes.data, kinds.ctypes.data, m, brows.ctypes.data, boffs.ctypes.data, m),
            "rh_estore_apply")
    apply_s = time.perf_counter() - t1
    root1 = A.Aggregate()
    A.check(A.lib().rh_estore_root(es, C.byref(root1)), "rh_estore_root")
    # the root moved by exactly the batch's lifts (all fresh keys): the schema kernel's sum of them
    bfps, _ = lift_records(schema, {k: v.clone() for k, v in b.items()})
    lim = bfps.view(torch.int16).to(torch.int64) & 0xFFFF
    bsum = sum(int(c) << (16 * i) for i, c in enumerate(lim.sum(dim=0).cpu().tolist())) % (1 << 256)
    r0 = sum(int(x) << (64 * i) for i, x in enumerate(root0.fingerprint))
    r1 = sum(int(x) << (64 * i) for i, x in enumerate(root1.fingerprint))
    if int(present.sum()) == 0 and ((r1 - r0) % (1 << 256) != bsum or root1.size != n + m):
        raise SystemExit("bench: the encoded store's root after the batch differs from root + Σ batch lifts")
    A.lib().rh_estore_destroy(es)
    # device-resident steps: the encoded records' lift over bytes already in HBM
    flat = torch.from_numpy(rows).to(dev).view(-1)
    ref, _ = lift_records(schema, cols)
    got, _ = lift_fixed(flat, L)
    if not torch.equal(got, ref):
        raise SystemExit("bench: encoded-bytes lift differs from the schema kernel's")
    del got
    spin = gpu_spinup(args.spinup_ms, dev)
    for _ in range(args.warmup):
        lift_fixed(flat, L)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _, bs = lift_fixed(flat, L)
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_s = sum(a.elapsed_time(c) for a, c in ev) / len(ev) / 1e3
    # the schema kernel on the same records, for the ratio (median of 10)
    sev = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lift_records(schema, cols)
        e1.record()
        sev.append((e0, e1))
    torch.cuda.synchronize()
    schema_s = sorted(a.elapsed_time(c) for a, c in sev)[5] / 1e3
    if rank == 0:
        recs = n * args.steps * world
        hbm = (L + 32) * n / kern_s / 1e9
        line = {
            "metric": "fingerprint-hash GiB/s + M records/s (device-resident) at 1/2/4/8 MI355X",
            "value": round(recs * L / elapsed / 2**30, 2), "unit": "GiB/s",
            "mrec_per_s": round(recs / elapsed / 1e6, 1),
            "n_gpus": world, "dist": {"backend": dist.get_backend() if dist is not None else None, "world_size": world},
            "steps": args.steps, "warmup": args.warmup, "spinup": spin,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded, SURVEY §8d generator) encoded to canonical bytes on the host; "
                    "device-resident bytes for the timed steps",
            "config": {"workload": describe("encoded", n * world, n, world), "records_per_gpu": n,
                       "canonical_bytes_per_record": L, "hbm_bytes_per_record": L + 32,
                       "parallelism": f"key-range shards x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(hbm / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "rh::k_lift_fixed_ct<120> (lift + block sums)", "kernel_avg_us": round(kern_s * 1e6, 2)},
            "schema_kernel_us": round(schema_s * 1e6, 2), "encoded_over_schema": round(kern_s / schema_s, 4),
            "map_path": {"host_encode_s": round(encode_s, 4), "host_encode_ns_per_record": round(encode_s / n * 1e9, 1),
                         "encoder": "numpy, vectorised for this fixed shape",
                         "fill_s": round(fill_s, 4), "fill_m_rec_per_s": round(n / fill_s / 1e6, 1),
                         "fill": "rh_estore_load from pageable host bytes (H2D + lift + sums + root)",
                         "batch": m, "batch_encode_s": round(bencode_s, 4), "apply_s": round(apply_s, 4),
                         "apply_m_rec_per_s": round(m / apply_s / 1e6, 1),
                         "apply": "rh_estore_apply: rank-addressed inserts (H2D + lift + segment merge + sums + root)",
                         "root_check": "root after the batch == root before + Σ schema-kernel lifts of the batch"},
        }
        if args.cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(schema, cols, args.cpu_sample or min(n, 10_000_000))
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def reload(args, world, rank, dev, dist):
    """Snapshot reload: one step = rh_store_load_snapshot of a device-resident RCNL file into the
    dated and the projection store (entry walk + transfer-function tree + the fused pass: listing,
    both lifts, keys, samples, block sums + the stores' super sums), i.e.
    ReplicatedMap::with_persistence's replay (src/replicated_map/persistence.rs:108-143)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, lift_records, range_aggregates, reduce_blocks
    from rsos_hip.snapshot import load_snapshot
    from rsos_hip.synth import make_records, make_snapshot
    kname, vname, kind, n_default, desc = CONFIGS["snapshot"]
    n = args.records or n_default
    sd, sp = RecordSchema.dated(kname, vname), RecordSchema.projection(kname, vname)
    cols = make_records(sd, n, seed=42, device=dev, first_index=rank * n, key_space=n * world,
                        tombstone_fraction=0.1)
    blob = make_snapshot(cols, sd)
    file_bytes = blob.numel()
    # the expected dated root: Σ GPU lifts of the source rows (checked after timing)
    fps, bs = lift_records(sd, cols)
    want = range_aggregates(fps, bs, reduce_blocks(bs), torch.tensor([0], device=dev),
                            torch.tensor([n], device=dev)).cpu()
    del fps, bs
    dated, proj = GpuFingerprintStore(sd, device=dev.index), GpuFingerprintStore(sp, device=dev.index)
    spin = gpu_spinup(args.spinup_ms, dev)
    for _ in range(args.warmup):
        load_snapshot(blob, dated, proj)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        info = load_snapshot(blob, dated, proj)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    root = dated.aggregate()
    ok = root.size == n == info.keys and root.fingerprint.limbs == tuple(int(x) & (2**64 - 1) for x in want[0, :4])
    if not ok:
        raise SystemExit("bench: reloaded root aggregate differs from the lifted source rows")
    # roofline of the dominant kernel, the fused pass k_snap_lift (listing + both lifts + keys +
    # samples + block sums), timed with HIP events on the loading store's stream
    # (rh_debug_reload_timing): algorithmic bytes = the file read once + per entry two
    # fingerprints, the key once per store and the two stores' search samples (1 u64 per 8 keys)
    import ctypes as C
    from rsos_hip import _abi as A
    lib = A.lib()
    lib.rh_debug_reload_timing(1)
    stages = []
    for _ in range(3):
        load_snapshot(blob, dated, proj)
        loc, lift = C.c_double(), C.c_double()
        lib.rh_debug_last_reload_us(C.byref(loc), C.byref(lift))
        stages.append((lift.value, loc.value))
    lib.rh_debug_reload_timing(0)
    lift_us, locate_us = min(stages)
    alg_bytes = file_bytes + n * (2 * 32 + 2 * sd.key_row + 2)
    achieved = alg_bytes / (lift_us * 1e-6) / 1e9
    if rank == 0:
        recs = n * args.steps * world
        line = {
            "metric": "snapshot reload into dated + projection GPU stores (M entries/s)",
            "value": round(recs / elapsed / 1e6, 2), "unit": "M entries/s",
            "gib_s_file": round(file_bytes * args.steps * world / elapsed / 2**30, 2),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "spinup": spin,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded): sorted unique keys, 10% tombstones, file bytes resident in HBM",
            "config": {"workload": desc, "entries_per_gpu": n, "file_bytes": file_bytes,
                       "parallelism": f"key-range shards x{world}"},
            "tombstones": info.tombstones,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic("snapshot", n),
                         "kernel": "rh::k_snap_lift (fused listing + dated and projection lifts + keys + "
                                   "samples + block sums)",
                         "kernel_avg_us": round(lift_us, 1), "algorithmic_bytes": alg_bytes,
                         "locate_us": round(locate_us, 1)},
            "root_check": "dated root == Σ lift(source rows)",
        }
        valu = load_valu("snapshot", n, lift_us * 1e-6)  # the fused pass is VALU-bound, like the lift
        if valu:
            line["valu"] = valu
        if args.e2e == 1:  # the file's bytes in (pinned) host memory: H2D inside the reload
            host = blob.cpu().pin_memory()
            best = None
            for _ in range(3):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                load_snapshot(host.numpy(), dated, proj)
                dt = time.perf_counter() - t1
                best = dt if best is None else min(best, dt)
            line["end_to_end"] = {"entries": n, "seconds": round(best, 5), "m_entries_per_s": round(n / best / 1e6, 1),
                                  "from": "pinned host bytes (H2D of the whole file inside the call)"}
        if args.cpu_baseline:  # rank 0 at every N: the same per-GPU workload's sample on this host
            line["cpu_baseline"] = cpu_baseline_reload(sd, sp, cols, args.cpu_sample or 1_000_000)
        print(json.dumps(line), flush=True)
    dated.close()
    proj.close()
    if dist is not None:
        dist.destroy_process_group()


def reconcile(args, world, rank, dev, dist):
    """rbsr: one step = one whole reconciliation between two GPU stores (replica A, and replica B
    = A minus d/2 keys, with d/2 records re-stamped): FixedFanOut(16) rounds, each answered by
    rh_store_protocol_round on the responding store, the children handed to the peer store, until
    no segment is left (rbsr/src/protocol.rs:97-317 driven as src/replica/dispatch.rs does)."""
    from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
    from rsos_hip.synth import make_records
    kname, vname, kind, n_default, desc = CONFIGS["rbsr"]
    n = args.records or n_default
    d = max(2, args.diffs)
    schema = getattr(RecordSchema, kind)(kname, vname)
    cols = make_records(schema, n, seed=42, device=dev, first_index=rank * n, key_space=n * world)
    a, b = GpuFingerprintStore(schema, device=dev.index), GpuFingerprintStore(schema, device=dev.index)
    a.load_bulk_device(cols)
    b.load_bulk_device(cols)
    g = torch.Generator(device=dev)
    g.manual_seed(11 + rank)
    rows = torch.randperm(n, generator=g, device=dev)[:d]
    batch = {k: v[rows].clone() for k, v in cols.items()}
    batch["phys"] += 1_000_000
    ops = torch.zeros(d, dtype=torch.uint8, device=dev)
    ops[: d // 2] = 1  # B lacks these keys; the other half differ in their stamp
    b.apply_device(batch, ops)
    b.compact()
    cpu_line = None
    if args.cpu_baseline and world == 1:  # the same replicas and differences, reconciled on the CPU
        cpu_line = cpu_baseline_reconcile(schema, cols, rows.cpu().numpy(), args.cpu_sample or n)
    del cols, batch
    pol = R.FixedFanOut(16)

    kl = schema.key_row
    pcie = {"in": 0, "out": 0}

    def run():
        active, k, segs, enum = R.initial_segments(a), 0, 0, 0
        pcie["in"] = pcie["out"] = 0
        while len(active):
            segs += len(active)
            r = len(active)
            active, en, _ = R.protocol_round_segments((b, a)[k % 2], pol, active, raw=True)
            enum += len(en)
            pcie["in"] += round_in_bytes(r, kl)
            pcie["out"] += round_out_bytes(len(active), len(en), kl)
            k += 1
        return k, segs, enum

    spin = gpu_spinup(args.spinup_ms, dev)
    for _ in range(max(args.warmup, 1)):
        rounds, segs, enum = run()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rounds, segs, enum = run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        line = {
            "metric": "rbsr reconciliation on GPU stores (segments answered per second)",
            "value": round(segs * args.steps * world / elapsed / 1e6, 3), "unit": "M segments/s",
            "reconciliations_per_s": round(args.steps * world / elapsed, 2),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "spinup": spin,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (seeded): sorted resident set; replica B lacks d/2 keys and re-stamps d/2",
            "config": {"workload": desc, "records_per_replica": n, "diffs": d, "policy": "FixedFanOut(16)",
                       "parallelism": f"key-range shards x{world} (each rank reconciles its own shard pair)"},
            "rounds": rounds, "segments_per_reconciliation": segs, "enumerations": enum,
            "step": "initial_ranges + protocol rounds (rh_store_protocol_round, one device round trip each) "
                    "until no segment is left",
        }
        line["roofline"] = rbsr_roofline(pcie["in"], pcie["out"], elapsed / args.steps, rounds)
        if cpu_line:
            line["cpu_baseline"] = cpu_line
        print(json.dumps(line), flush=True)
    a.close()
    b.close()
    if dist is not None:
        dist.destroy_process_group()


def _pad16(x):
    return (x + 15) // 16 * 16


def round_in_bytes(r, kl):
    """A round's segments as the device reads them (rsos_hip_abi.hip protocol_round): start / end
    kinds, start then end keys, the peer's aggregates -- one copy up, or read in place when tiny."""
    return _pad16(_pad16(r) + _pad16(r) + 2 * r * kl) + 40 * r


def round_out_bytes(nc, ne, kl):
    """A round's output in round_layout() (internal.hpp): the 64-byte header, the children's kinds,
    keys and aggregates, the enumerations' kinds and keys -- written by the emit kernel into mapped
    page-locked memory (or copied down when small)."""
    return 64 + 2 * _pad16(nc) + 2 * _pad16(nc * kl) + _pad16(40 * nc) + 2 * _pad16(ne) + 2 * _pad16(ne * kl)


def rbsr_roofline(in_bytes, out_bytes, step_s, rounds):
    """The rbsr line's bound: a reconciliation moves its rounds' inputs up and
    outputs down over PCIe, one device round trip per round.  achieved = those bytes per
    reconciliation / its time, against the link's measured ceiling -- a kernel's 16-byte stores
    into mapped page-locked memory, the fastest form measured (microbench/pcie_copy.hip,
    profiles/r04_pcie_copy.jsonl); model_ms = the inputs at the measured copy rate plus the
    outputs at the mapped-store rate, the time the bytes alone would take."""
    w_gbs, h2d_gbs, src = 54.6, 21.7, None
    p = os.path.join(ROOT, "profiles", "r04_pcie_copy.jsonl")
    try:
        rows = [json.loads(x) for x in open(p) if x.strip()]
        big = max(r["bytes"] for r in rows)
        w_gbs = max(r["kernel_write_GBs"] for r in rows if r["bytes"] == big)
        h2d_gbs = max(r["h2d_GBs"] for r in rows if r["bytes"] == big)
        src = os.path.relpath(p, ROOT)
    except (OSError, ValueError, KeyError):
        pass
    total = in_bytes + out_bytes
    achieved = total / step_s / 1e9 if step_s > 0 else 0.0
    model_s = in_bytes / (h2d_gbs * 1e9) + out_bytes / (w_gbs * 1e9)
    return {"bound": "pcie", "achieved": round(achieved, 2), "peak": w_gbs, "unit": "GB/s",
            "frac": round(achieved / w_gbs, 4), "traffic": None,
            "bytes_per_reconciliation": {"in": in_bytes, "out": out_bytes},
            "peak_h2d_copy_GBs": h2d_gbs, "model_ms": round(model_s * 1e3, 3),
            "model_frac_of_step": round(model_s / step_s, 4) if step_s > 0 else None,
            "round_trips": rounds, "source": src}


def cpu_baseline_reconcile(schema, cols, rows, m):
    """The same reconciliation on the CPU: oracle.c's restatement of protocol_round_with_policy
    (one aggregate / rank / select question at a time, FixedFanOut(16)) over two oracle
    FingerprintTreeMaps holding the first m records of each replica."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    from rsos_hip.synth import to_host
    h = to_host(cols, 0, m)
    h.setdefault("tags", np.zeros(m, np.uint8))
    rows = rows[rows < m]
    d = len(rows)
    keep = np.ones(m, bool)
    keep[rows[: d // 2]] = False
    phys = h["phys"].copy()
    phys[rows[d // 2:]] += 1_000_000
    sc = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
    ra = O.Records(sc, h["keys"], h["values"], h["phys"], h["logical"], h["node"], h["tags"])
    rb = O.Records(sc, h["keys"][keep], h["values"][keep], phys[keep], h["logical"][keep], h["node"][keep],
                   h["tags"][keep])
    ta, tb = O.FingerprintTreeMap(ra), O.FingerprintTreeMap(rb)
    ta.fill(0, ra.n)
    tb.fill(0, rb.n)
    t0 = time.perf_counter()
    rounds, segs, _ = O.reconcile_fixed(ta, tb, 16)  # no hashing in a round: the SIMD level does not apply
    dt = time.perf_counter() - t0
    return {"value": round(segs / dt / 1e6, 4), "unit": "M segments/s", "cores": 1, "kind": "port",
            "reconciliation_ms": round(dt * 1e3, 3),
            "sample": f"one reconciliation of two oracle FTMs (oracle.c) of {m} records differing in {d} keys "
                      f"({segs} segments, {rounds} rounds)"}


def cpu_baseline_reload(sd, sp, cols, m):
    """The reference's replay restated (oracle/oracle.c FingerprintTreeMap): just_insert_bulk
    inserts every entry into the dated map and into the projection, serially under the write
    lock (src/replica/write.rs:26-46,107-121).  The bincode decode is not timed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from rsos_hip.synth import to_host
    h = to_host(cols, 0, m)
    dt = 0.0
    level = O.set_simd(2)  # the blake3 crate's SIMD row form (oracle/blake3_simd.c)
    for s in (sd, sp):
        sc = O.Schema(s.key_kind, s.key_len, s.value_kind, s.value_len, s.record_kind, 0)
        dated = s.record_kind == O.REC_DATED
        recs = O.Records(sc, h["keys"], h["values"], h["phys"] if dated else None, h["logical"] if dated else None,
                         h["node"] if dated else None, h["tags"])
        t = O.FingerprintTreeMap(recs)
        t0 = time.perf_counter()
        t.fill(0, m)
        dt += time.perf_counter() - t0
    O.set_simd(0)
    return {"value": round(m / dt / 1e6, 3), "unit": "M entries/s", "cores": 1, "kind": "port",
            "simd": ["portable", "sse4.1", "avx512vl"][level],
            "sample": f"replay of the first {m} entries into two FingerprintTreeMaps (dated + projection; "
                      f"oracle/oracle.c restatement, serial, decode not timed), {dt:.2f} s"}


def cpu_baseline_incremental(schema, m, resident):
    """The reference's update path restated (oracle/oracle.c FingerprintTreeMap): a resident map
    of `resident` records filled untimed, then `m` random-key inserts timed, serially (one writer
    under the map's write lock, src/replica/dispatch.rs:188-196)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from rsos_hip.synth import make_records, to_host
    base = to_host(make_records(schema, resident, seed=7, device="cuda"))
    batch = to_host(make_records(schema, m, seed=8, device="cuda", random_keys=True))
    cols = {k: np.concatenate([base[k], batch[k]]) for k in base}
    sc = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
    recs = O.Records(sc, cols["keys"], cols.get("values"), cols.get("phys"), cols.get("logical"), cols.get("node"),
                     cols.get("tags"))
    t = O.FingerprintTreeMap(recs)
    t.fill(0, resident)
    level = O.set_simd(2)  # the blake3 crate's SIMD row form (oracle/blake3_simd.c)
    t0 = time.perf_counter()
    t.fill(resident, resident + m)
    dt = time.perf_counter() - t0
    O.set_simd(0)
    return {"value": round(m / dt / 1e6, 3), "unit": "M records/s", "cores": 1, "kind": "port",
            "simd": ["portable", "sse4.1", "avx512vl"][level],
            "sample": f"{m} random-key inserts into a {resident}-record FingerprintTreeMap "
                      f"(oracle/oracle.c restatement, serial), {dt:.2f} s"}


def spot_check(schema, cols, n):
    """Lift a few thousand rows and compare with the C oracle (test infrastructure)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle as O
        O.lib()
    except Exception as e:  # the checker is optional; the product path never needs it
        return f"skipped: {e}"
    from rsos_hip import lift_records
    from rsos_hip.synth import to_host
    m = min(n, 4096)
    sub = {k: v[:m] for k, v in cols.items()}
    fps, _ = lift_records(schema, sub, block_sums=False)
    torch.cuda.synchronize()
    h = to_host(cols, 0, m)
    sc = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
    want = O.Records(sc, h["keys"], h.get("values"), h.get("phys"), h.get("logical"), h.get("node"),
                     h.get("tags")).lift(threads=8)
    ok = bool(np.array_equal(fps.cpu().numpy(), want))
    if not ok:
        raise SystemExit("bench: GPU fingerprints differ from the oracle -- refusing to report a number")
    return f"bit-exact on {m} rows"


def usable_cores() -> dict:
    """Host cores this process may run on: the affinity mask, capped by a cgroup CPU quota (the GPU
    box shows every core of the machine in os.cpu_count() but gives a job a share of them)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return {"used": min(aff, quota) if quota else aff, "affinity": aff, "cgroup_quota": quota,
            "os_cpu_count": os.cpu_count()}


def cpu_calibration(O) -> dict:
    """The oracle's FingerprintTreeMap against the reference's own published CPU numbers, on the
    reference's own shapes (same host, same SIMD level as the baseline):
    - benches/contention.rs (README.md:848-875): u64/u64, 100 k sequential keys pre-filled, then
      20 k tail inserts, one writer -> ns per insert (reference: 346 ns = 1 / 2,888,103 ops/s);
    - benches/protocol.rs reconciliation_drive (README.md:584-585): FixedFanOut(16), n = 10^6
      u64/u64, d = 1 scattered -> us per whole reconciliation (reference: 45.0 us, which also
      encodes every round for the wire)."""
    import numpy as np
    m = 120_000
    k = np.arange(m, dtype=np.uint64)
    sc = O.Schema(O.KEY_U64, 8, O.VAL_U64, 8, O.REC_PLAIN, 0)
    r = O.Records(sc, k.view(np.uint8).reshape(m, 8), k.copy().view(np.uint8).reshape(m, 8))
    best = None
    for _ in range(5):
        t = O.FingerprintTreeMap(r)
        t.fill(0, 100_000)
        t0 = time.perf_counter()
        t.fill(100_000, m)
        dt = (time.perf_counter() - t0) / 20_000
        best = dt if best is None else min(best, dt)
    n = 1_000_000
    k = np.arange(n, dtype=np.uint64)
    v = k * np.uint64(2654435761)
    keep = k != (n // 2)

    def ftm(kk, vv):
        rr = O.Records(sc, np.ascontiguousarray(kk).view(np.uint8).reshape(-1, 8),
                       np.ascontiguousarray(vv).view(np.uint8).reshape(-1, 8))
        tt = O.FingerprintTreeMap(rr)
        tt.fill(0, rr.n)
        return tt, rr
    (ta, ra), (tb, rb) = ftm(k, v), ftm(k[keep], v[keep])
    ts = []
    for _ in range(100):
        t0 = time.perf_counter()
        O.reconcile_fixed(ta, tb, 16)
        ts.append(time.perf_counter() - t0)
    rec = sorted(ts)[len(ts) // 2]
    return {"insert_ns": round(best * 1e9, 1), "insert_ns_reference": 346.0,
            "insert_ratio_to_reference": round(best * 1e9 / 346.0, 3),
            "reconcile_d1_n1e6_us": round(rec * 1e6, 1), "reconcile_us_reference": 45.0,
            "reconcile_ratio_to_reference": round(rec * 1e6 / 45.0, 3)}


def cpu_baseline(schema, cols, sample, dual=False):
    """The reference's CPU path restated (oracle/oracle.c): FingerprintTreeMap fill -- one lift per
    insert into an order-6 B-tree with per-node Aggregate caches, serial (one writer holds the map's
    write lock, src/replica/write.rs:117-120), over a bounded sample of the same records.  BLAKE3 runs
    the blake3 crate's own SIMD form (its row-vector compress_in_place, AVX-512VL where the host has
    it, else SSE4.1: oracle/blake3_simd.c), not portable C.  dual: Replica::map_insert's two inserts
    per record, into the dated map and its projection (src/replica/write.rs:44-45).
    Beside it: the batch lift on every usable core (record-parallel, same SIMD form), the best batch
    lift this CPU can do (16 records per AVX-512 vector, not the reference's path), and the
    calibration of the restated FTM against the reference's published CPU numbers."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from rsos_hip.synth import to_host
    level = O.set_simd(2)
    simd = {0: "portable", 1: "sse4.1 (blake3 crate row form)", 2: "avx512vl (blake3 crate row form)"}[level]
    try:
        m = next(iter(cols.values())).shape[0]
        m = min(sample, m) if sample else m
        h = to_host(cols, 0, m)
        sc = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
        recs = O.Records(sc, h["keys"], h.get("values"), h.get("phys"), h.get("logical"), h.get("node"),
                         h.get("tags"))
        rec_bytes = schema.record_len()
        t = O.FingerprintTreeMap(recs)
        t0 = time.perf_counter()
        t.fill(0, m)
        dt = time.perf_counter() - t0
        recs_p = None
        if dual:
            sp = schema.with_kind(2)
            recs_p = O.Records(O.Schema(sp.key_kind, sp.key_len, sp.value_kind, sp.value_len, sp.record_kind, 0),
                               h["keys"], h.get("values"), None, None, None, h.get("tags"))
            tp = O.FingerprintTreeMap(recs_p)
            t0 = time.perf_counter()
            tp.fill(0, m)
            dt += time.perf_counter() - t0
            rec_bytes += sp.record_len()
        del t
        cores = usable_cores()
        threads = cores["used"]
        fill = {"value": round(m * rec_bytes / dt / 2**30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                "simd": simd, "mrec_per_s": round(m / dt / 1e6, 3),
                "sample": f"FingerprintTreeMap fill{'s of the dated map and its projection' if dual else ''} "
                          f"(oracle/oracle.c restatement, serial inserts, BLAKE3 in the crate's {simd} form) of the "
                          f"first {m} records of the benchmark shard, {dt:.2f} s"}
        t0 = time.perf_counter()
        recs.lift(threads=threads)
        if recs_p is not None:
            recs_p.lift(threads=threads)
        dt2 = time.perf_counter() - t0
        fill["batch_lift_all_cores"] = {"value": round(m * rec_bytes / dt2 / 2**30, 4), "unit": "GiB/s",
                                        "cores": threads, "simd": simd, "mrec_per_s": round(m / dt2 / 1e6, 3)}
        if O.has_avx512() and not dual:
            t0 = time.perf_counter()
            recs.lift_x16(threads=threads)
            dt3 = time.perf_counter() - t0
            fill["best_cpu_batch_lift"] = {
                "value": round(m * rec_bytes / dt3 / 2**30, 4), "unit": "GiB/s", "cores": threads,
                "simd": "avx512f, 16 records per vector (not the reference's code path)",
                "mrec_per_s": round(m / dt3 / 1e6, 3)}
        fill["host_cores"] = cores
        fill["calibration"] = cpu_calibration(O)
        return fill
    finally:
        O.set_simd(0)


def end_to_end(schema, cols, n):
    """Host records -> H2D -> lift -> D2H of the fingerprints, from pinned host buffers:
    rh_lift_host (the C ABI's host path: chunked, copy-in / lift / copy-out on three streams),
    and for comparison the same steps issued back to back on one stream."""
    import ctypes as C
    from rsos_hip import _abi as A, lift_records
    host = {k: v.cpu().pin_memory() for k, v in cols.items()}
    fps_h = torch.empty((n, 32), dtype=torch.uint8).pin_memory()
    hc = A.Columns(*[host[k].data_ptr() if k in host else None
                     for k in ("keys", "phys", "logical", "node", "tags", "values")])
    sc = schema.c()
    dev = torch.cuda.current_device()

    def pipelined():
        A.check(A.lib().rh_lift_host(dev, C.byref(sc), C.byref(hc), n, fps_h.data_ptr()), "rh_lift_host")

    def serial():
        dcols = {k: v.to("cuda", non_blocking=True) for k, v in host.items()}
        fps, _ = lift_records(schema, dcols, block_sums=False)
        fps_h.copy_(fps, non_blocking=True)
        torch.cuda.synchronize()

    pcie_bytes = sum(v.numel() * v.element_size() for v in host.values()) + n * 32  # in + out
    out = {"records": n, "pcie_bytes": pcie_bytes}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        best = None
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        out[name] = {"seconds": round(best, 5), "mrec_per_s": round(n / best / 1e6, 1),
                     "gib_s_hashed": round(n * schema.record_len() / best / 2**30, 2),
                     "pcie_gb_s": round(pcie_bytes / best / 1e9, 1)}
    ref, _ = lift_records(schema, cols, block_sums=False)
    out["pipelined_bit_exact"] = bool(torch.equal(ref.cpu(), fps_h))
    return out


def load_valu(config, n, lift_s):
    """The lift's VALU-issue roofline from the committed PMC pass (profiles/rNN_valu_<config>.json:
    SQ_INSTS_VALU / SQ_WAVES / GRBM_GUI_ACTIVE, scripts/pmc_valu.py): VALU wave-instructions per
    launch over this run's measured lift time, against
    - peak_sustained: the rate gfx950 sustains for BLAKE3's instruction mix -- one wave64
      instruction per 4 cycles per SIMD (every rotate form and v_add3 issue at 4 cycles, and so
      does a G function in any encoding: profiles/r02_micro_valu_g.log) -- at the
      chip's maximum engine clock, 2.4 GHz;
    - peak_nominal: the full-rate 2-operand rate, one per 2 cycles per SIMD at 2.4 GHz."""
    p = _profile(f"valu_{config}.json", n)
    if p is None:
        return None
    try:
        with open(p) as f:
            v = json.load(f)
        instr = float(v["valu_wave_instructions_per_launch"])
        sustained = 256 * 4 * 2.4e9 / 4
        nominal = 256 * 4 * 2.4e9 / 2
        achieved = instr / lift_s
        return {"bound": "valu", "achieved": round(achieved / 1e9, 1), "peak_sustained": round(sustained / 1e9, 1),
                "peak_nominal": round(nominal / 1e9, 1), "unit": "G wave-instr/s",
                "frac": round(achieved / sustained, 4), "frac_nominal": round(achieved / nominal, 4),
                "valu_per_wave": round(float(v["valu_per_wave"]), 1),
                "pmc_pass_clock_ghz": round(float(v["effective_clock_ghz"]), 3),
                "source": os.path.relpath(p, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


def load_traffic(config, n):
    """HBM bytes per lift launch from the committed rocprofv3 PMC summary, if one exists for this
    config and size (profiles/traffic_<config>.json; FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction)."""
    p = _profile(f"traffic_{config}.json", n)
    if p is None:
        return None
    with open(p) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def _profile(suffix, n):
    """The newest committed profile summary (profiles/rNN_<suffix>, newest round first) that was
    collected at this record count, or None."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_" + suffix)), reverse=True):
        try:
            with open(p) as f:
                if int(json.load(f).get("records", -1)) == n:
                    return p
        except (OSError, ValueError):
            continue
    return None


if __name__ == "__main__":
    main()
