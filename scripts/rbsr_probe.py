"""Time whole two-replica reconciliations (rbsr FixedFanOut(16) ping-pong, rsos_hip.rbsr over two
GPU stores on one device) for n records per replica and d differences: d/2 keys the responder
lacks, d/2 keys whose record differs (re-stamped).  Reports rounds, segments answered, wall time,
and the time inside the two store calls.  CPU side for comparison: the literal oracle driver over
two FTM restatements of a smaller replica (--cpu-n), same d.

usage: python scripts/rbsr_probe.py [--n 10000000] [--d 1,100,10000] [--cpu-n 1000000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "reconcile-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import torch

from rsos_hip import GpuFingerprintStore, RecordSchema, rbsr as R
from rsos_hip.synth import make_records, to_host


class Timed:
    """Wraps a store: counts and times the two batched calls."""

    def __init__(self, st):
        self.st, self.t, self.calls, self.segs = st, 0.0, 0, 0

    def size(self):
        return self.st.size()

    def aggregate(self, *a):
        return self.st.aggregate(*a)

    def resolve_segments(self, segs):
        t0 = time.perf_counter()
        out = self.st.resolve_segments(segs)
        self.t += time.perf_counter() - t0
        self.calls += 1
        self.segs += len(segs)
        return out

    def split_segments(self, sel, lo, hi):
        t0 = time.perf_counter()
        out = self.st.split_segments(sel, lo, hi)
        self.t += time.perf_counter() - t0
        self.calls += 1
        return out


def diff_batch(schema, cols, n, d, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    rows = torch.randperm(n, generator=g, device="cuda")[:d]
    b = {k: v[rows].clone() for k, v in cols.items()}
    b["phys"] += 1_000_000
    ops = torch.zeros(d, dtype=torch.uint8, device="cuda")
    ops[: d // 2] = 1  # delete: the responder lacks these keys; the rest are re-stamped
    return b, ops


def reconcile(a, b, max_rounds=100):
    """Object-level rounds through the two-call path (protocol_round_with_policy, native=False)."""
    active = R.initial_ranges(a)
    side = [b, a]
    rounds = 0
    t0 = time.perf_counter()
    while active and rounds < max_rounds:
        ch, en = [], []
        R.protocol_round_with_policy(side[rounds % 2], R.DEFAULT_POLICY, active, ch, en, native=False)
        active = ch
        rounds += 1
    return rounds, time.perf_counter() - t0


def reconcile_soa(a, b, max_rounds=100):
    """The same ping-pong entirely in SoA form: one rh_store_protocol_round call per round."""
    pol = R.FixedFanOut(16)
    active = R.initial_segments(a)
    side = [b, a]
    rounds = segs = 0
    t0 = time.perf_counter()
    while len(active) and rounds < max_rounds:
        segs += len(active)
        active, _, _ = R.protocol_round_segments(side[rounds % 2], pol, active, copy=False)
        rounds += 1
    return rounds, time.perf_counter() - t0, segs


def cpu_reconcile(schema, cols_h, n, d, seed):
    import oracle as O
    import rbsr as OR
    rng = np.random.default_rng(seed)
    rows = rng.choice(n, d, replace=False)
    sc = O.Schema(schema.key_kind, schema.key_len, schema.value_kind, schema.value_len, schema.record_kind, 0)
    cols_h = dict(cols_h)
    cols_h.setdefault("tags", np.zeros(n, np.uint8))
    ra = O.Records(sc, cols_h["keys"], cols_h["values"], cols_h["phys"], cols_h["logical"], cols_h["node"],
                   cols_h["tags"])
    keep = np.ones(n, bool)
    keep[rows[: d // 2]] = False
    phys = cols_h["phys"].copy()
    phys[rows[d // 2:]] += 1_000_000
    rb = O.Records(sc, cols_h["keys"][keep], cols_h["values"][keep], phys[keep], cols_h["logical"][keep],
                   cols_h["node"][keep], cols_h["tags"][keep])
    ta, tb = O.FingerprintTreeMap(ra), O.FingerprintTreeMap(rb)
    ta.fill(0, ra.n)
    tb.fill(0, rb.n)
    va, vb = OR.FtmView(ta, False), OR.FtmView(tb, False)
    decide = OR.fixed_fan_out(16)
    active = OR.initial_ranges(va)
    side = [vb, va]
    rounds = 0
    t0 = time.perf_counter()
    while active:
        ch, en = [], []
        OR.protocol_round(side[rounds % 2], decide, active, ch, en)
        active = ch
        rounds += 1
    return rounds, time.perf_counter() - t0


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--d", default="1,100,10000,100000")
    p.add_argument("--cpu-n", type=int, default=1_000_000)
    args = p.parse_args()
    schema = RecordSchema.dated("bytes16", "bytes64")
    cols = make_records(schema, args.n, seed=42, device="cuda")
    for d in [int(x) for x in args.d.split(",")]:
        a, b = GpuFingerprintStore(schema), GpuFingerprintStore(schema)
        a.load_bulk_device(cols)
        b.load_bulk_device(cols)
        batch, ops = diff_batch(schema, cols, args.n, d, seed=d)
        b.apply_device(batch, ops)
        b.compact()
        reconcile_soa(a, b)  # warm up: the stores' pinned round buffers reach their size
        rounds, wall, segs = reconcile_soa(a, b)
        line = {"n": args.n, "d": d, "rounds": rounds, "segments": segs,
                "soa_native_ms": round(wall * 1e3, 3)}
        if d <= 1000:  # the two-call path with RangeAggregate objects (Python loop per segment)
            ta, tb = Timed(a), Timed(b)
            r2, wall2 = reconcile(ta, tb)
            line["object_two_call"] = {"rounds": r2, "wall_ms": round(wall2 * 1e3, 3),
                                       "store_call_ms": round((ta.t + tb.t) * 1e3, 3),
                                       "store_calls": ta.calls + tb.calls}
        if args.cpu_n and d <= 10000:
            h = to_host({k: v[: args.cpu_n] for k, v in cols.items()})
            cr, cw = cpu_reconcile(schema, h, args.cpu_n, d, seed=d)
            line["cpu_oracle"] = {"n": args.cpu_n, "rounds": cr, "wall_ms": round(cw * 1e3, 3),
                                  "driver": "oracle/rbsr.py over the C FTM restatement (1 core, Python loop)"}
        print(json.dumps(line), flush=True)
        a.close()
        b.close()


if __name__ == "__main__":
    main()
