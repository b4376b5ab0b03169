"""Host tier refresh cost: the first key-range aggregate after a load builds the tier, and the
first one after each batch refreshes it (compaction, device prefix sums, one copy of keys and
prefix sums); later ones are host-only.  python scripts/tier_refresh_probe.py [n] [batch]"""
import sys
import time

sys.path.insert(0, "reconcile-rs_amd")
import numpy as np  # noqa: E402

from rsos_hip import GpuFingerprintStore, RecordSchema  # noqa: E402
from rsos_hip.store import KeyRange  # noqa: E402
from rsos_hip.synth import make_records  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
m = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
s = RecordSchema.dated("bytes16", "bytes64")
st = GpuFingerprintStore(s, host_tier=True)
st.load_bulk_device(make_records(s, n, seed=42))
rng = np.random.default_rng(1)
rg = KeyRange(rng.bytes(16), rng.bytes(16))


def timed(f):
    t0 = time.perf_counter()
    f()
    return (time.perf_counter() - t0) * 1e6


print("first aggregate after load: %.0f us" % timed(lambda: st.aggregate(rg)))
print("next aggregate: %.2f us" % timed(lambda: st.aggregate(rg)))
for k in range(5):
    b = make_records(s, m, seed=100 + k, random_keys=True)
    t_apply = timed(lambda: st.apply_device(b))
    t_first = timed(lambda: st.aggregate(rg))
    t_next = timed(lambda: st.aggregate(rg))
    print("batch %d: apply %.0f us, first aggregate (refresh) %.0f us, next %.2f us" % (k, t_apply, t_first, t_next))
