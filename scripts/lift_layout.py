"""Why does the lift run faster in some harnesses than in others?  Lifts 10 M records (16 B /
64 B dated) under several conditions, HIP events around each launch, median of 10:
  fresh-out   fresh 10 M-row inputs and outputs, lifts back to back
  view-out    the same inputs, outputs are the first rows of a 100 M-row buffer
  view-in     inputs are the first 10 M rows of 100 M-row columns
  +queries    fresh, with the bench step's super-block sums and 16 range aggregates between lifts
  100M        one launch over all 100 M rows, per 10 M

usage: python scripts/lift_layout.py
"""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "reconcile-rs_amd"))
from rsos_hip import RecordSchema, lift_records, range_aggregates, reduce_blocks  # noqa: E402
from rsos_hip.synth import make_records  # noqa: E402


def timed(schema, cols, fps, bs, reps=10, queries=None):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lift_records(schema, cols, fps=fps, bsums=bs)
        e1.record()
        ts.append((e0, e1))
        if queries is not None:
            lo, hi = queries
            range_aggregates(fps, bs, reduce_blocks(bs), lo, hi)
    torch.cuda.synchronize()
    v = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
    return v[len(v) // 2]


def main():
    schema = RecordSchema.dated("bytes16", "bytes64")
    n = 10_000_000
    nb = (n + 255) // 256
    small = make_records(schema, n, seed=1)
    big = make_records(schema, 10 * n, seed=1)
    view = {k: v[:n] for k, v in big.items()}
    fps_big = torch.empty((10 * n, 32), dtype=torch.uint8, device="cuda")
    bs_big = torch.empty(((10 * n + 255) // 256, 32), dtype=torch.uint8, device="cuda")
    fps, bs = torch.empty((n, 32), dtype=torch.uint8, device="cuda"), torch.empty((nb, 32), dtype=torch.uint8, device="cuda")
    lo = torch.tensor([i * n // 16 for i in range(16)], dtype=torch.int64, device="cuda")
    hi = torch.tensor([(i + 1) * n // 16 for i in range(16)], dtype=torch.int64, device="cuda")
    for _ in range(3):
        timed(schema, small, fps, bs, 3)
    for rnd in range(3):
        r = {
            "fresh-out": timed(schema, small, fps, bs),
            "view-out": timed(schema, small, fps_big[:n], bs_big[:nb]),
            "view-in": timed(schema, view, fps, bs),
            "+queries": timed(schema, small, fps, bs, queries=(lo, hi)),
            "100M": timed(schema, big, fps_big, bs_big, 3) / 10,
        }
        print(f"round {rnd}: " + ", ".join(f"{k} {v:.1f} us" for k, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
