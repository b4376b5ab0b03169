"""Key-range sharding across GPUs and the one exchange step of the path.

Records are sorted by key and cut into equal-count shards, one per GPU (rank r holds global
rows [r*n, (r+1)*n)).  lift is per record and the Aggregate group is commutative and
associative (rsos/src/fingerprint.rs:44-45, rsos/src/aggregate.rs:79-89), so every GPU
computes, for each requested global range, the aggregate of that range intersected with its
shard; one all_gather of the R x 40 B partial aggregates (RCCL over xGMI with the nccl
backend) and a carry-add combine give the global range aggregates.  There is no other
data-path collective.  The reference has no distribution of this kind.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

M256 = 1 << 256


def shard_rows(rank: int, world: int, n_per: int) -> Tuple[int, int]:
    return rank * n_per, (rank + 1) * n_per


def equal_count_ranges(total: int, r: int) -> List[Tuple[int, int]]:
    """rbsr's fan-out cut of [0, total) into r equal-count rank ranges (protocol.rs:40, b = 16)."""
    return [(total * j // r, total * (j + 1) // r) for j in range(r)]


def local_ranges(ranges: Sequence[Tuple[int, int]], base: int, n: int) -> Tuple[List[int], List[int]]:
    """Each global rank range intersected with the shard [base, base + n), in shard coordinates
    (empty intersections become [x, x))."""
    lo = [min(max(a - base, 0), n) for a, _ in ranges]
    hi = [min(max(b - base, 0), n) for _, b in ranges]
    return lo, hi


def combine_host(parts: Sequence[Sequence[Tuple[int, int]]]) -> List[Tuple[int, int]]:
    """Σ over shards of (fingerprint as int, size) per range -- Aggregate's Add, host form."""
    r = len(parts[0])
    out = []
    for j in range(r):
        fp = sum(p[j][0] for p in parts) % M256
        size = sum(p[j][1] for p in parts)
        out.append((fp, size))
    return out


def gather(dist, out, gathered=None):
    """All-gather one rank's (R, 5) int64 aggregates into (world, R, 5).  nccl (RCCL): one
    all_gather_into_tensor; gloo (CPU rehearsal / tests): list all_gather."""
    import torch
    world = dist.get_world_size()
    if dist.get_backend() == "nccl":
        if gathered is None:
            gathered = torch.empty((world,) + tuple(out.shape), dtype=out.dtype, device=out.device)
        dist.all_gather_into_tensor(gathered, out)
        return gathered
    parts = [torch.empty_like(out) for _ in range(world)]
    dist.all_gather(parts, out)
    return torch.stack(parts)


class _Done:
    def wait(self):
        return None


def gather_async(dist, out, gathered):
    """Start the all-gather of `out` into `gathered` (world, R, 5) without blocking the compute
    stream: (work, gathered).  nccl: RCCL runs it on its own stream and work.wait() only makes
    the current stream wait, so the next step's lift overlaps the collective.  gloo: done
    synchronously (CPU rehearsal)."""
    import torch
    if dist.get_backend() == "nccl":
        return dist.all_gather_into_tensor(gathered, out, async_op=True), gathered
    parts = [torch.empty_like(out) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, out)
    gathered.copy_(torch.stack(parts))
    return _Done(), gathered

