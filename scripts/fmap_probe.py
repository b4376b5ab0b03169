"""Time 10^6 single-record inserts through FingerprintMap's staged path (rh_store_stage) and the one
device batch the first question applies; prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reconcile-rs_amd"))
from rsos_hip import Entry, FingerprintMap, RecordSchema  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
s = RecordSchema.dated("bytes16", "bytes64")
rng = np.random.default_rng(3)
keys = [rng.bytes(16) for _ in range(n)]
vals = [rng.bytes(64) for _ in range(n)]
fm = FingerprintMap(s)
t0 = time.perf_counter()
for i in range(n):
    fm.insert(keys[i], Entry(vals[i], 1_700_000_000_000 + i, 0, 1))
t1 = time.perf_counter()
root = fm.aggregate()
t2 = time.perf_counter()
q = [fm.aggregate() for _ in range(1000)]
t3 = time.perf_counter()
print(json.dumps({"inserts": n, "host_inserts_s": round(t1 - t0, 3), "first_aggregate_s": round(t2 - t1, 4),
                  "aggregate_after_us": round((t3 - t2) / 1000 * 1e6, 2), "size": root.size}))
