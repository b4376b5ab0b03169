"""Time the generic encoded-bytes lift (k_lift_encoded) against the schema kernel: 10 M records
of 120 B (the config2 record, pre-encoded) and 10 M variable-length records (u64 key + Vec<u8>
of 0..128 bytes, i.e. 16..144 B)."""
import os, sys, time
sys.path.insert(0, os.environ.get("RSOS_HIP_TREE") or
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reconcile-rs_amd"))
import torch
from rsos_hip import lift_encoded, lift_fixed

def timeit(fn, reps=30):
    fn(); torch.cuda.synchronize()
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); ev.append((a, b))
    torch.cuda.synchronize()
    return sorted(x.elapsed_time(y) for x, y in ev)[reps // 2] / 1e3

n = 10_000_000
g = torch.Generator(device="cuda"); g.manual_seed(1)
data = torch.randint(0, 256, (n * 120,), dtype=torch.uint8, device="cuda", generator=g)
offs = torch.arange(0, n + 1, dtype=torch.int64, device="cuda") * 120
t_end = time.perf_counter() + 0.4  # clock spin-up: the chip raises its clock over the first ~50 ms of load
while time.perf_counter() < t_end:
    lift_encoded(data, offs)
    torch.cuda.synchronize()
t = timeit(lambda: lift_encoded(data, offs))
print(f"fixed 120 B: {t*1e6:.0f} us  {n/t/1e9:.2f} G rec/s  {n*120/t/1e9:.0f} GB/s")
t = timeit(lambda: lift_fixed(data, 120))
print(f"fixed 120 B via rh_lift_fixed_async (no offsets): {t*1e6:.0f} us  {n/t/1e9:.2f} G rec/s  {n*120/t/1e9:.0f} GB/s")
lens = 16 + torch.randint(0, 129, (n,), dtype=torch.int64, device="cuda", generator=g)
offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda"); offs[1:] = torch.cumsum(lens, 0)
tot = int(offs[-1])
data = torch.randint(0, 256, (tot,), dtype=torch.uint8, device="cuda", generator=g)
t = timeit(lambda: lift_encoded(data, offs))
print(f"variable 16..144 B (avg {tot/n:.0f}): {t*1e6:.0f} us  {n/t/1e9:.2f} G rec/s  {tot/t/1e9:.0f} GB/s")
