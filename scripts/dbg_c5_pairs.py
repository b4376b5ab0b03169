"""Debug the 100 M pair check: the store's dumped (key, fp) rows against the expected live set,
sorted on the host with numpy (the keys' leading u64 words are unique here)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reconcile-rs_amd"))
import numpy as np
import torch
from rsos_hip import GpuFingerprintStore, RecordSchema, lift_records, _abi as A
from rsos_hip.synth import make_records
s = RecordSchema.dated("bytes16", "bytes64")
n = int(sys.argv[1]); m, K, touch = 1_000_000, 15, 50_000
base = make_records(s, n, seed=5)
def lift64(cols):
    rows = cols["keys"].shape[0]
    out = torch.empty((rows, 4), dtype=torch.int64, device="cuda")
    for i in range(0, rows, 16_000_000):
        out[i:i + 16_000_000] = lift_records(s, {c: t[i:i + 16_000_000] for c, t in cols.items()}, block_sums=False)[0].view(torch.int64)
    return out
bf = lift64(base)
st = GpuFingerprintStore(s); st.load_bulk_device(base); st.reserve(n + K * m, m)
perm = torch.randperm(n, generator=torch.Generator(device="cuda").manual_seed(9), device="cuda")
batches, ops = [], []
for k in range(K):
    ins = make_records(s, m - 2 * touch, seed=700 + k, random_keys=True)
    rows = perm[k * 2 * touch:(k + 1) * 2 * touch]
    ex = {c: t[rows].clone() for c, t in base.items()}
    ex["values"][:touch] ^= 0x3C; ex["phys"][:touch] += 7
    b = {c: torch.cat([ins[c], ex[c]]).contiguous() for c in ins}
    o = torch.zeros(m, dtype=torch.uint8, device="cuda"); o[m - touch:] = 1
    batches.append(b); ops.append(o)
st.apply_device_many(batches, ops)
keep = torch.ones(n, dtype=torch.bool, device="cuda"); keep[perm[:K * 2 * touch]] = False
kept = keep.nonzero().view(-1)
print("kept", kept.numel(), flush=True)
k64 = [base["keys"].view(torch.int64)[kept]]; f64 = [bf[kept]]
for b in batches:
    part = {c: t[:m - touch] for c, t in b.items()}
    k64.append(part["keys"].view(torch.int64)); f64.append(lift64(part))
k64 = torch.cat(k64).cpu().numpy(); f64 = torch.cat(f64).cpu().numpy()
N = st.size(); print("N", N, k64.shape, flush=True)
dk = np.zeros(N * 16, np.uint8)
A.check(A.lib().rh_store_keys(st._h, 0, N, dk.ctypes.data), "keys")
dk = dk.view(np.uint64).reshape(N, 2)
df = st.fingerprints().view(np.uint64).reshape(N, 4)
t0 = time.time()
hi = k64[:, 0].view(np.uint64).byteswap()  # big-endian leading word
order = np.argsort(hi, kind="stable")
print("sorted in", round(time.time() - t0, 1), "s; unique hi:", np.unique(hi).size == N, flush=True)
ek, ef = k64[order].view(np.uint64), f64[order].view(np.uint64)
kd = np.nonzero((ek != dk).any(axis=1))[0]
fd = np.nonzero((ef != df).any(axis=1))[0]
print("key rows differing", kd.size, kd[:5], "fp rows differing", fd.size, fd[:5], flush=True)
for i in fd[:3]:
    print(i, "key", dk[i], "exp key", ek[i], "fp", df[i], "exp fp", ef[i])
    j = order[i]
    print("   source row", j, "kept" if j < kept.numel() else "batch", flush=True)
