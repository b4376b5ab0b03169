"""Bisect the 100 M store root against an independent torch reduction, batches with overwrites
and deletes of resident keys: per batch (apply_device) or all at once (apply_device_many)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reconcile-rs_amd"))
import torch
from rsos_hip import GpuFingerprintStore, RecordSchema, lift_records
from rsos_hip.synth import make_records
M256 = 1 << 256
def troot(fps, chunk=8_000_000):
    t = 0
    for i in range(0, fps.shape[0], chunk):
        l = fps[i:i + chunk].view(torch.int16).to(torch.int64) & 0xFFFF
        col = l.sum(dim=0).cpu().tolist()
        t += sum(int(c) << (16 * k) for k, c in enumerate(col))
    return t % M256
def lift(s, cols):
    n = cols["keys"].shape[0]
    out = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
    for i in range(0, n, 16_000_000):
        out[i:i + 16_000_000] = lift_records(s, {c: t[i:i + 16_000_000] for c, t in cols.items()}, block_sums=False)[0]
    return out
s = RecordSchema.dated("bytes16", "bytes64")
n = int(sys.argv[1])
many = sys.argv[2] == "1"
K, m, touch = 15, 1_000_000, 50_000
base = make_records(s, n, seed=5)
bf = lift(s, base)
want = troot(bf)
st = GpuFingerprintStore(s)
st.load_bulk_device(base)
st.reserve(n + K * m, m)
perm = torch.randperm(n, generator=torch.Generator(device="cuda").manual_seed(9), device="cuda")
batches, ops, wants = [], [], []
for k in range(K):
    ins = make_records(s, m - 2 * touch, seed=700 + k, random_keys=True)
    rows = perm[k * 2 * touch:(k + 1) * 2 * touch]
    ex = {c: t[rows].clone() for c, t in base.items()}
    ex["values"][:touch] ^= 0x3C
    ex["phys"][:touch] += 7
    b = {c: torch.cat([ins[c], ex[c]]).contiguous() for c in ins}
    o = torch.zeros(m, dtype=torch.uint8, device="cuda")
    o[m - touch:] = 1
    batches.append(b); ops.append(o)
    want = (want + troot(lift(s, {c: t[:m - touch] for c, t in b.items()})) - troot(bf[rows])) % M256
    wants.append(want)
if many:
    print("many", st.apply_device_many(batches, ops)[:2], flush=True)
    r = st.aggregate()
    print("after many", r.size, r.fingerprint.to_int() == wants[-1], st.stats(), flush=True)
else:
    for k in range(K):
        c = st.apply_device(batches[k], ops[k])
        r = st.aggregate()
        print("batch", k, c, r.size, r.fingerprint.to_int() == wants[k], st.stats(), flush=True)
st.compact()
r = st.aggregate()
print("compact", r.size, r.fingerprint.to_int() == wants[-1], st.stats(), flush=True)
# keys: the store's full dump (after the compaction) against the expected live set, sorted
import numpy as np
N = st.size()
dump = np.zeros(N * 16, np.uint8)
import ctypes as C
from rsos_hip import _abi as A
A.check(A.lib().rh_store_keys(st._h, 0, N, dump.ctypes.data), "keys")
dk = torch.from_numpy(dump).cuda().view(N, 16)
keep = torch.ones(n, dtype=torch.bool, device="cuda")
keep[perm[:K * 2 * touch]] = False
kept = keep.nonzero().view(-1)
ek = [base["keys"].view(torch.int64)[kept]] + [b["keys"][:m - touch].contiguous().view(torch.int64) for b in batches]
ek = torch.cat(ek)
flip = torch.iinfo(torch.int64).min
def words(k8):
    return (k8[:, :8].flip(1).contiguous().view(torch.int64).view(-1) ^ flip,
            k8[:, 8:].flip(1).contiguous().view(torch.int64).view(-1) ^ flip)
h, l = words(ek.view(torch.uint8))
p = torch.argsort(l, stable=True)
p = p[torch.argsort(h[p], stable=True)]
es = ek[p].view(torch.uint8)
dh, dl = words(dk)
print("dump sorted:", bool(((dh[1:] > dh[:-1]) | ((dh[1:] == dh[:-1]) & (dl[1:] > dl[:-1]))).all()), flush=True)
eq = (es == dk).all(dim=1)
bad = (~eq).nonzero().view(-1)
print("rows differing:", bad.numel(), "first:", bad[:5].tolist(), flush=True)
if bad.numel():
    i = int(bad[0])
    print("expected", es[i].cpu().numpy().tobytes().hex(), "store", dk[i].cpu().numpy().tobytes().hex(), flush=True)
    print("expected sorted:", bool(((h[p][1:] > h[p][:-1]) | ((h[p][1:] == h[p][:-1]) & (l[p][1:] > l[p][:-1]))).all()))
