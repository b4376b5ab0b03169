"""Encoded-lift A/B on one box (round 3): 10 M north_star records (16 B key / 64 B value, dated,
120 canonical bytes) hashed by the schema kernel from columns, and from their canonical bytes by
the compile-time fixed-length kernel (k_lift_fixed_ct<120>), the runtime-length fixed kernel
(the same bytes at a 4-byte offset, which the compile-time path refuses), and the offsets kernel.
All four are checked bit-exact against each other first.  Median of 30 launches each, interleaved
over 3 rounds, after a 400 ms clock spin-up."""
import os, sys, time
sys.path.insert(0, os.environ.get("RSOS_HIP_TREE") or
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reconcile-rs_amd"))
import torch
from rsos_hip import RecordSchema, lift_records, lift_encoded, lift_fixed
from rsos_hip.synth import make_records, encode_rows

def timeit(fn, reps=30):
    fn(); torch.cuda.synchronize()
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); ev.append((a, b))
    torch.cuda.synchronize()
    return sorted(x.elapsed_time(y) for x, y in ev)[reps // 2] / 1e3

n = int(os.environ.get("N", 10_000_000))
s = RecordSchema.dated("bytes16", "bytes64")
cols = make_records(s, n, seed=42)
rows = encode_rows(s, cols)
L = rows.shape[1]
flat = rows.view(-1)
mis = torch.zeros(flat.numel() + 16, dtype=torch.uint8, device="cuda")
mis[4:4 + flat.numel()] = flat
mis_view = mis[4:4 + flat.numel()]
offs = torch.arange(0, n + 1, dtype=torch.int64, device="cuda") * L
ref, _ = lift_records(s, cols)
for name, got in [("ct", lift_fixed(flat, L)[0]), ("runtime", lift_fixed(mis_view, L)[0]),
                  ("offsets", lift_encoded(flat, offs)[0])]:
    assert torch.equal(got, ref), name
print(f"bit-exact: {n} records of {L} B, schema / fixed-ct / fixed-runtime / offsets")
t_end = time.perf_counter() + 0.4
while time.perf_counter() < t_end:
    lift_records(s, cols); torch.cuda.synchronize()
res = {k: [] for k in ("schema", "ct", "runtime", "offsets")}
for _ in range(3):
    res["schema"].append(timeit(lambda: lift_records(s, cols)))
    res["ct"].append(timeit(lambda: lift_fixed(flat, L)))
    res["runtime"].append(timeit(lambda: lift_fixed(mis_view, L)))
    res["offsets"].append(timeit(lambda: lift_encoded(flat, offs)))
for k, v in res.items():
    t = sorted(v)[1]
    print(f"{k:8s} {t*1e6:7.1f} us  {n/t/1e9:6.2f} G rec/s  ({' '.join(f'{x*1e6:.0f}' for x in v)})  "
          f"x{t / sorted(res['schema'])[1]:.3f} of schema")
