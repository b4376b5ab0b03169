"""rbsr's protocol driver over a GpuFingerprintStore: one round in two device round trips.

Host-side mirror of rbsr/src/protocol.rs (names, argument meaning, outputs):

  initial_ranges(local)                                   protocol.rs:97-102
  protocol_round(local, active, children, enumerations)   protocol.rs:161-178 (FixedFanOut 16)
  protocol_round_with_policy(local, policy, ...)          protocol.rs:212-317
  RoundOutcome                                            protocol.rs:135-142, protocol/outcome.rs
  Comparison, FixedFanOut, SqrtFanOut, FanOut,
  SplitStride rules                                       rbsr/src/policy/{comparison,cutoffs,
                                                          fixed_fan_out,sqrt_fan_out,params}.rs

The reference walks the active segments one by one and asks its RsosView four questions per
segment and two per SPLIT child, each an O(log n) tree walk.  Against an HBM-resident store each
question would be a device round trip, so the round is answered in two batched calls instead:

  1. rh_store_resolve_segments: for every segment, the raw ranks of both bounds and the local
     aggregate over its key range (BoundedRange::parse and `local.aggregate(..)`, :225-255);
  2. the policy decides every segment on the host, in segment order (Comparison carries the
     children emitted so far, which the cut arithmetic gives without any key);
     rh_store_split_segments then returns the keys at every SPLIT cut (`select`, :305) and the
     aggregate of every child that is not the parent itself (:297-307).

For FixedFanOut and SqrtFanOut, which decide on the span alone, the whole round runs inside
the library instead (rh_store_protocol_round: the same two device steps with the decision loop
in C++ between them), on segments in the wire codec's SoA form (`Segments`); a reconciliation
that never leaves that form (protocol_round_segments) touches no per-segment Python object.

Both calls see one state of the store (rsos_view.rs:36).  The outputs are appended in the
reference's order: child_ranges (SPLIT children, bounced IDLIST parents) and enumeration_ranges
(IDLIST), segment by segment.  A segment is a RangeAggregate (start None = Unbounded, else
Included(start); end None = Unbounded, else Excluded(end)); an enumeration range is a
(start, end) pair in the same convention.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

import ctypes as C

from . import _abi as A
from .fingerprint import Aggregate, Fingerprint
from .wire import RangeAggregate, _key_bytes, _key_out

Key = Union[bytes, int]
EnumerationRange = Tuple[Optional[Key], Optional[Key]]

SKIP = "skip"
ENUMERATE = "enumerate"


@dataclass(frozen=True)
class Split:
    """Decision::Split(SplitStride): elements per child range, never zero (params.rs:52-60)."""
    stride: int

    def __post_init__(self):
        if self.stride <= 0:
            object.__setattr__(self, "stride", 1)


@dataclass(frozen=True)
class Comparison:
    """policy/comparison.rs: the local and remote aggregates of one segment."""
    local: Aggregate
    remote: Aggregate
    children_emitted: int = 0

    def span(self) -> int:
        return self.local.size

    def remote_size(self) -> int:
        return self.remote.size

    def agrees(self) -> bool:
        return self.local == self.remote


def shared_cutoffs(c: Comparison):
    """policy/cutoffs.rs: the outcomes every shipped policy shares."""
    local, remote = c.span(), c.remote_size()
    if c.agrees():
        return SKIP
    if remote == 0:
        return ENUMERATE
    if local == 0:
        return Split(1)
    if local == 1 and remote == 1:
        return ENUMERATE
    if local == 1:
        return Split(1)
    return None


def fan_out(b: int) -> int:
    """FanOut::new: 0 and 1 are raised to 2 (params.rs:82-84)."""
    return 2 if b < 2 else b


class FixedFanOut:
    """At most `fan_out` children per SPLIT, stride ceil(span / b) (fixed_fan_out.rs)."""

    def __init__(self, b: int = 16):  # FanOut::NEGENTROPY
        self.fan_out = fan_out(b)

    def decide(self, c: Comparison):
        d = shared_cutoffs(c)
        if d is not None:
            return d
        return Split(-(-c.span() // self.fan_out))


class SqrtFanOut:
    """Stride floor(sqrt(span)) in f32 arithmetic, as `(span as f32).sqrt() as usize`
    (sqrt_fan_out.rs)."""

    def decide(self, c: Comparison):
        d = shared_cutoffs(c)
        if d is not None:
            return d
        return Split(int(np.sqrt(np.float32(c.span()))))


DEFAULT_POLICY = FixedFanOut(16)


@dataclass
class RoundOutcome:
    """What one round did (protocol.rs:135-142); `+=` accumulates a whole reconciliation."""
    skipped: int = 0
    enumerated: int = 0
    split: int = 0
    children: int = 0
    dropped_malformed: int = 0

    def __iadd__(self, o: "RoundOutcome") -> "RoundOutcome":
        self.skipped += o.skipped
        self.enumerated += o.enumerated
        self.split += o.split
        self.children += o.children
        self.dropped_malformed += o.dropped_malformed
        return self


AGG_DTYPE = np.dtype([("fingerprint", "<u8", (4,)), ("size", "<u8")])  # rh_aggregate


class Segments:
    """A round's segments in SoA form (rh_segments; the arrays rh_wire_* encodes): bound kinds
    (start 0 = Unbounded / 1 = Included, end 0 = Unbounded / 1 = Excluded), key rows and
    aggregates, n items of `cap`."""

    def __init__(self, key_len: int, cap: int):
        cap = max(int(cap), 1)
        self.start_kinds = np.zeros(cap, np.uint8)
        self.start_keys = np.zeros((cap, key_len), np.uint8)
        self.end_kinds = np.zeros(cap, np.uint8)
        self.end_keys = np.zeros((cap, key_len), np.uint8)
        self.aggregates = np.zeros(cap, AGG_DTYPE)
        self.n = 0

    def __len__(self) -> int:
        return self.n

    @property
    def cap(self) -> int:
        return len(self.start_kinds)

    def c(self) -> A.Segments:
        ptrs = self.__dict__.get("_ptrs")
        if ptrs is None or ptrs[0] is not self.start_kinds:  # the arrays' addresses, looked up once
            ptrs = (self.start_kinds, tuple(a.ctypes.data for a in (self.start_kinds, self.start_keys, self.end_kinds,
                                                                    self.end_keys, self.aggregates)))
            self._ptrs = ptrs
        sk, skeys, ek, ekeys, aggs = ptrs[1]
        return A.Segments(sk, skeys, ek, ekeys, aggs, self.n, self.cap)

    @staticmethod
    def from_items(schema, items: Sequence) -> "Segments":
        """From RangeAggregates (or (start, end) pairs, aggregates left ZERO)."""
        seg = Segments(schema.key_row, len(items))
        for i, it in enumerate(items):
            start, end = (it.start, it.end) if hasattr(it, "start") else it
            if start is not None:
                seg.start_kinds[i] = 1
                seg.start_keys[i] = np.frombuffer(_key_bytes(schema, start), np.uint8)
            if end is not None:
                seg.end_kinds[i] = 1
                seg.end_keys[i] = np.frombuffer(_key_bytes(schema, end), np.uint8)
            if hasattr(it, "aggregate"):
                seg.aggregates["fingerprint"][i] = it.aggregate.fingerprint.limbs
                seg.aggregates["size"][i] = it.aggregate.size
        seg.n = len(items)
        return seg

    def bounds(self, schema, i: int) -> EnumerationRange:
        s = _key_out(schema, self.start_keys[i].tobytes()) if self.start_kinds[i] else None
        e = _key_out(schema, self.end_keys[i].tobytes()) if self.end_kinds[i] else None
        return s, e

    def items(self, schema) -> List[RangeAggregate]:
        out = []
        for i in range(self.n):
            s, e = self.bounds(schema, i)
            a = self.aggregates[i]
            out.append(RangeAggregate(s, e, Aggregate(int(a["size"]),
                                                      Fingerprint(tuple(int(x) for x in a["fingerprint"])))))
        return out


class _Raw:
    """A pointer as an __array_interface__: numpy wraps it in ~2 us (a ctypes array's PEP 3118
    format goes through numpy's Python-level parser, ~10 us per array)."""
    __slots__ = ("__array_interface__",)


def _view(ptr, n: int, shape) -> np.ndarray:
    """uint8 array of `shape` at ptr (zeros when n == 0)."""
    if n == 0 or not ptr:
        return np.zeros(shape, np.uint8)
    o = _Raw()
    o.__array_interface__ = {"data": (ptr, False), "shape": shape, "typestr": "|u1", "version": 3}
    return np.asarray(o)


def _wrap(cs: A.Segments, key_len: int, copy: bool, with_aggs: bool) -> "Segments":
    n = int(cs.n)
    seg = Segments.__new__(Segments)
    seg.n = n
    m = max(n, 1)
    seg.start_kinds = _view(cs.start_kinds, n, (m,))
    seg.end_kinds = _view(cs.end_kinds, n, (m,))
    seg.start_keys = _view(cs.start_keys, n, (m, key_len))
    seg.end_keys = _view(cs.end_keys, n, (m, key_len))
    if with_aggs and n:
        seg.aggregates = _view(cs.aggregates, n, (m * AGG_DTYPE.itemsize,)).view(AGG_DTYPE)
    else:
        seg.aggregates = np.zeros(m, AGG_DTYPE)
    if copy and n:
        for k in ("start_kinds", "end_kinds", "start_keys", "end_keys", "aggregates"):
            setattr(seg, k, getattr(seg, k).copy())
    return seg


class RawSegments:
    """A round's output as the library returned it (its rh_segments, pointing into the answering
    store's own buffers, valid until that store's next call): handed to the peer store's round as
    it is, as a C or Rust caller hands the children over -- no numpy views either way."""
    __slots__ = ("cs",)

    def __init__(self, cs: A.Segments):
        self.cs = cs

    def __len__(self) -> int:
        return int(self.cs.n)

    def c(self) -> A.Segments:
        return self.cs


def protocol_round_segments(store, policy, active,
                            copy: bool = True, raw: bool = False) -> Tuple[Segments, Segments, RoundOutcome]:
    """One round of FixedFanOut / SqrtFanOut inside the library: (children, enumerations, outcome).
    copy=False returns views of the store's own output arrays, valid until the store's next call
    (enough to hand the children to the peer store's round); raw=True returns them as RawSegments
    (no views at all).  `active`: Segments or RawSegments."""
    if isinstance(policy, FixedFanOut):
        kind, b = A.POLICY_FIXED_FAN_OUT, policy.fan_out
    elif isinstance(policy, SqrtFanOut):
        kind, b = A.POLICY_SQRT_FAN_OUT, 0
    else:
        raise TypeError("protocol_round_segments runs FixedFanOut / SqrtFanOut; use protocol_round_with_policy")
    kl = store.schema.key_row
    a, cc, ec, oc = active.c(), A.Segments(), A.Segments(), A.RoundOutcome()
    A.check(store._f("protocol_round")(store._h, kind, b, C.byref(a), C.byref(cc), C.byref(ec), C.byref(oc)),
            store._P + "protocol_round")
    if raw:
        return (RawSegments(cc), RawSegments(ec),
                RoundOutcome(int(oc.skipped), int(oc.enumerated), int(oc.split), int(oc.children),
                             int(oc.dropped_malformed)))
    return (_wrap(cc, kl, copy, True), _wrap(ec, kl, copy, False),
            RoundOutcome(int(oc.skipped), int(oc.enumerated), int(oc.split), int(oc.children),
                         int(oc.dropped_malformed)))


def initial_segments(store) -> Segments:
    seg = Segments(store.schema.key_row, 1)
    agg = store.aggregate()
    seg.aggregates["fingerprint"][0] = agg.fingerprint.limbs
    seg.aggregates["size"][0] = agg.size
    seg.n = 1
    return seg


def initial_ranges(local) -> List[RangeAggregate]:
    """{(-inf, +inf), A(whole store)}: the cached root, O(1) (protocol.rs:97-102)."""
    return [RangeAggregate(None, None, local.aggregate())]


def protocol_round(local, active: Sequence[RangeAggregate], child_ranges: List[RangeAggregate],
                   enumeration_ranges: List[EnumerationRange]) -> RoundOutcome:
    return protocol_round_with_policy(local, DEFAULT_POLICY, active, child_ranges, enumeration_ranges)


def protocol_round_with_policy(local, policy, active: Sequence[RangeAggregate],
                               child_ranges: List[RangeAggregate],
                               enumeration_ranges: List[EnumerationRange], native: Optional[bool] = None) -> RoundOutcome:
    """native: None = the library's one-call round when the policy allows it (FixedFanOut,
    SqrtFanOut) and `local` is a GpuFingerprintStore; False = the two-call path for any policy."""
    if native is None:
        native = isinstance(policy, (FixedFanOut, SqrtFanOut)) and hasattr(local, "_h")
    if native:
        ch, en, outcome = protocol_round_segments(local, policy, Segments.from_items(local.schema, active))
        child_ranges.extend(ch.items(local.schema))
        enumeration_ranges.extend(en.bounds(local.schema, i) for i in range(en.n))
        return outcome
    outcome = RoundOutcome()
    if not active:
        return outcome
    raw_lo, raw_hi, locals_ = local.resolve_segments(active)       # round trip 1
    size = local.size()
    # decide every segment in order; SPLIT children are planned as rank ranges
    plan = []        # (kind, segment, payload) in segment order
    sel: List[int] = []          # select() ranks of every cut
    agg_lo: List[int] = []       # child rank ranges whose aggregate is needed
    agg_hi: List[int] = []
    for seg, rl, rh, la in zip(active, raw_lo.tolist(), raw_hi.tolist(), locals_):
        if rh < rl:  # inverted: covers no keys (protocol.rs:232-245)
            outcome.dropped_malformed += 1
            continue
        start_index, end_index = min(rl, size), min(rh, size)   # StoreSize::admit
        comparison = Comparison(la, seg.aggregate, outcome.children)
        span = comparison.span()
        decision = policy.decide(comparison)
        if isinstance(decision, Split) and span > 1 and decision.stride >= span:
            decision = ENUMERATE  # a non-progressing SPLIT becomes an IDLIST (:263-272)
        if decision == SKIP:
            outcome.skipped += 1
        elif decision == ENUMERATE:
            outcome.enumerated += 1
            bounce = seg.aggregate.size != 0
            if bounce:
                outcome.children += 1
            plan.append((ENUMERATE, seg, bounce))
        else:
            outcome.split += 1
            stride = decision.stride
            cuts = list(range(start_index + stride, end_index, stride)) if stride else []
            first_sel = len(sel)
            sel.extend(cuts)
            bounds = [start_index] + cuts + [end_index]
            first_agg = len(agg_lo)
            if cuts:  # an uncut child is the parent: its aggregate is already in hand (:292-296)
                agg_lo.extend(bounds[:-1])
                agg_hi.extend(bounds[1:])
            outcome.children += len(cuts) + 1
            plan.append(("split", seg, (first_sel, len(cuts), first_agg, la)))
    keys, aggs = local.split_segments(sel, agg_lo, agg_hi) if (sel or agg_lo) else ([], [])  # round trip 2
    for kind, seg, p in plan:
        if kind == ENUMERATE:
            if p:
                child_ranges.append(RangeAggregate(seg.start, seg.end, Aggregate.ZERO))
            enumeration_ranges.append((seg.start, seg.end))
            continue
        first_sel, ncuts, first_agg, la = p
        if ncuts == 0:
            child_ranges.append(RangeAggregate(seg.start, seg.end, la))
            continue
        cur = seg.start
        for k in range(ncuts):
            nxt = keys[first_sel + k]
            child_ranges.append(RangeAggregate(cur, nxt, aggs[first_agg + k]))
            cur = nxt
        child_ranges.append(RangeAggregate(cur, seg.end, aggs[first_agg + ncuts]))
    return outcome
