"""CPU restatement of rbsr's protocol round (TEST INFRASTRUCTURE ONLY).

Only tests/ import this, as the checker of rsos_hip.rbsr's batched driver.  It follows
rbsr/src/protocol.rs:212-317 literally: one segment at a time, asking the view
`aggregate(start..end)` (:230), `rank` of both bounds (BoundedRange::parse,
rbsr/src/protocol/rank.rs:85-125), then per SPLIT child `select(cut)` (:305) and
`aggregate(child)` (:297-307), each as a separate call, against any view with
size() / aggregate(start, end) / rank(key) / select(r).  FtmView binds it to the C oracle's
FingerprintTreeMap restatement (oracle.c: the order-6 B-tree of rsos/src/fingerprint_tree_map).

Policies (rbsr/src/policy): shared_cutoffs (cutoffs.rs), FixedFanOut (fixed_fan_out.rs,
stride = ceil(span / b), FanOut::new raises b < 2 to 2), SqrtFanOut (sqrt_fan_out.rs,
stride = (span as f32).sqrt() as usize), SplitStride::per_child raising 0 to 1 (params.rs).

Representation: a segment is (start, end, agg) with start None = Unbounded else Included,
end None = Unbounded else Excluded, agg = (fp limbs tuple, size); enumeration ranges are
(start, end) pairs.
"""
from __future__ import annotations

from typing import List

import numpy as np

ZERO = ((0, 0, 0, 0), 0)


def _split(stride: int):
    return ("split", stride if stride > 0 else 1)


def _cutoffs(local, remote):
    ls, rs = local[1], remote[1]
    if local == remote:
        return ("skip",)
    if rs == 0:
        return ("enumerate",)
    if ls == 0:
        return _split(1)
    if ls == 1 and rs == 1:
        return ("enumerate",)
    if ls == 1:
        return _split(1)
    return None


def fixed_fan_out(b: int = 16):
    b = 2 if b < 2 else b

    def decide(local, remote, children):
        d = _cutoffs(local, remote)
        return d if d is not None else _split((local[1] + b - 1) // b)
    return decide


def sqrt_fan_out(local, remote, children):
    d = _cutoffs(local, remote)
    return d if d is not None else _split(int(np.sqrt(np.float32(local[1]))))


class FtmView:
    """RsosView over the oracle's FingerprintTreeMap (keys: the record columns' key rows)."""

    def __init__(self, ftm, key_kind_int: bool):
        self.t = ftm
        sc = ftm.recs.schema
        self.kl = {1: 4, 2: 8}.get(sc.key_kind, sc.key_len)  # OR_KEY_U32 / OR_KEY_U64 / bytes
        self.key_int = key_kind_int

    def _kb(self, k) -> bytes:
        return int(k).to_bytes(self.kl, "little") if self.key_int else bytes(k)

    def size(self) -> int:
        return len(self.t)

    def aggregate(self, start, end):
        fp, size = self.t.aggregate(None if start is None else self._kb(start),
                                    None if end is None else self._kb(end))
        return tuple(int(x) for x in fp), int(size)

    def rank(self, k) -> int:
        return self.t.rank(self._kb(k))

    def select(self, r: int):
        row = self.t.select(r)
        kb = self.t.recs.keys.reshape(-1)[row * self.kl:(row + 1) * self.kl].tobytes()
        return int.from_bytes(kb, "little") if self.key_int else kb


def initial_ranges(view):
    return [(None, None, view.aggregate(None, None))]


def protocol_round(view, decide, active, child_ranges: List, enumeration_ranges: List):
    """Returns the RoundOutcome as (skipped, enumerated, split, children, dropped_malformed)."""
    skipped = enumerated = split = children = dropped = 0
    for start, end, remote in active:
        local = view.aggregate(start, end)
        size = view.size()
        raw_start = 0 if start is None else view.rank(start)
        raw_end = size if end is None else view.rank(end)
        if raw_end < raw_start:
            dropped += 1
            continue
        start_index, end_index = min(raw_start, size), min(raw_end, size)
        span = local[1]
        d = decide(local, remote, children)
        if d[0] == "split" and span > 1 and d[1] >= span:
            d = ("enumerate",)
        if d[0] == "skip":
            skipped += 1
        elif d[0] == "enumerate":
            enumerated += 1
            if remote[1] != 0:
                child_ranges.append((start, end, ZERO))
                children += 1
            enumeration_ranges.append((start, end))
        else:
            split += 1
            stride = d[1]
            cur_bound, cur_index = start, start_index
            while True:
                nxt = cur_index + stride
                if not nxt < end_index:
                    agg = local if cur_index == start_index else view.aggregate(cur_bound, end)
                    child_ranges.append((cur_bound, end, agg))
                    children += 1
                    break
                key = view.select(nxt)
                child_ranges.append((cur_bound, key, view.aggregate(cur_bound, key)))
                children += 1
                cur_bound, cur_index = key, nxt
    return skipped, enumerated, split, children, dropped
