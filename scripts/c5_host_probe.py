"""Host-side time of the config5 batch loop: wall time of each apply_device (enqueue + device
work + result wait) and of the root aggregate between batches.  python scripts/c5_host_probe.py [n]"""
import sys
import time

import os
sys.path.insert(0, os.environ.get("RSOS_HIP_TREE", "reconcile-rs_amd"))
import torch  # noqa: E402

from rsos_hip import GpuFingerprintStore, RecordSchema  # noqa: E402
from rsos_hip.synth import make_records  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
div = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # compaction divisor (0: the store's default)
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 24
m = 1_000_000
s = RecordSchema.dated("bytes16", "bytes64")
st = GpuFingerprintStore(s)
if div:
    st.set_compaction(div, 65536)
st.load_bulk_device(make_records(s, n, seed=42))
batches = [make_records(s, m, seed=1000 + k, random_keys=True) for k in range(steps)]
torch.cuda.synchronize()
st.reserve(n + m * steps, m)
rows = []
for k in range(steps):
    t0 = time.perf_counter_ns()
    st.apply_device(batches[k])
    t1 = time.perf_counter_ns()
    st.aggregate()
    t2 = time.perf_counter_ns()
    rows.append((k, (t1 - t0) / 1e3, (t2 - t1) / 1e3, st.stats()["delta_rows"]))
for r in rows:
    print("batch %2d apply %8.1f us aggregate %6.1f us delta_rows %d" % r)
w = rows[len(rows) // 4:]  # past the first cycle's start
print("mean apply over batches %d..%d: %.1f us" % (w[0][0], w[-1][0], sum(r[1] for r in w) / len(w)))
