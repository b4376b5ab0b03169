"""Device-resident batch API: torch CUDA(HIP) tensors in, kernels enqueued on torch's
current stream (no synchronisation, no host copies).

Every shape is checked on the host before a launch: the kernels index rows by `n`, so a
column shorter than n rows would read out of bounds.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple

import torch

from . import _abi as A
from .schema import RecordSchema

COLS = ("keys", "phys", "logical", "node", "tags", "values")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def block_sums_for(n: int) -> int:
    return (n + A.BLOCK - 1) // A.BLOCK


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


_NEED: Dict[tuple, tuple] = {}  # per schema: (column, row width) of every required column


def _need(schema: RecordSchema) -> tuple:
    key = (schema.key_row, schema.value_row, bool(schema.dated_kind))
    got = _NEED.get(key)
    if got is None:
        need = [("keys", schema.key_row), ("values", schema.value_row)]
        if schema.dated_kind:
            need += [("phys", 8), ("logical", 4), ("node", 8)]
        got = _NEED[key] = tuple((c, w) for c, w in need if w)
    return got


def _check_cols(schema: RecordSchema, cols: Dict[str, torch.Tensor]) -> int:
    """The row count, after checking every column the schema needs: present, a contiguous device
    tensor, and exactly n rows of its width (the kernels index rows by n)."""
    for k in cols:
        if k not in COLS:
            raise ValueError(f"unknown column {k!r}")
    if schema.key_row:
        n = cols["keys"].nbytes // schema.key_row
    else:
        n = cols["values"].nbytes // max(schema.value_row, 1)
    for name, width in _need(schema):
        t = cols.get(name)
        if t is None:
            raise ValueError(f"column {name!r} is required by {schema}")
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"column {name!r} must be a contiguous device tensor")
        if t.nbytes != n * width:
            raise ValueError(f"column {name!r} has {t.nbytes} bytes, expected {n} x {width}")
    t = cols.get("tags")
    if t is not None and (t.nbytes != n or not t.is_cuda):
        raise ValueError("tags must be n device bytes")
    return n


def _columns(cols: Dict[str, torch.Tensor]) -> A.Columns:
    return A.Columns(*[_ptr(cols.get(k)) for k in COLS])


def lift_records(schema: RecordSchema, cols: Dict[str, torch.Tensor], block_sums: bool = True,
                 fps: Optional[torch.Tensor] = None, bsums: Optional[torch.Tensor] = None
                 ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """fps[i] = lift(key_i, record_i) as 32 LE bytes; bsums[g] = Σ fps over rows 256g..256g+255."""
    n = _check_cols(schema, cols)
    dev = next(iter(cols.values())).device
    if fps is None:
        fps = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    if block_sums and bsums is None:
        bsums = torch.empty((block_sums_for(n), 32), dtype=torch.uint8, device=dev)
    if fps.shape != (n, 32) or (bsums is not None and bsums.shape != (block_sums_for(n), 32)):
        raise ValueError("output shape mismatch")
    s, c = schema.c(), _columns(cols)
    A.check(A.lib().rh_lift_records_async(C.byref(s), C.byref(c), n, _ptr(fps),
                                          _ptr(bsums) if block_sums else None, _stream()),
            "rh_lift_records_async")
    return fps, (bsums if block_sums else None)


def lift_dual(schema: RecordSchema, cols: Dict[str, torch.Tensor], out=None):
    """Both lifts of Replica::map_insert (src/replica/write.rs:44-45) from one read of the
    records: (dated fps, dated block sums, projection fps, projection block sums).  `out`: the
    same four tensors, preallocated (reused across calls)."""
    if schema.record_kind != A.REC_DATED:
        raise ValueError("dual lift needs a DATED schema")
    n = _check_cols(schema, cols)
    dev = next(iter(cols.values())).device
    if out is not None:
        fd, bd, fp, bp = out
        if fd.shape != (n, 32) or fp.shape != (n, 32) or bd.shape[0] < block_sums_for(n) or \
                bp.shape[0] < block_sums_for(n):
            raise ValueError("out tensors have the wrong shape")
    else:
        fd = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        fp = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        bd = torch.empty((block_sums_for(n), 32), dtype=torch.uint8, device=dev)
        bp = torch.empty((block_sums_for(n), 32), dtype=torch.uint8, device=dev)
    s, c = schema.c(), _columns(cols)
    A.check(A.lib().rh_lift_dual_async(C.byref(s), C.byref(c), n, _ptr(fd), _ptr(bd), _ptr(fp), _ptr(bp),
                                       _stream()), "rh_lift_dual_async")
    return fd, bd, fp, bp


def lift_encoded(data: torch.Tensor, offsets: torch.Tensor, block_sums: bool = True):
    """BLAKE3 of pre-encoded canonical records: record i = data[offsets[i]:offsets[i+1]]."""
    if offsets.dtype != torch.int64 or not offsets.is_cuda or offsets.dim() != 1:
        raise ValueError("offsets must be a 1-D int64 device tensor of n+1 entries")
    n = offsets.numel() - 1
    dev = offsets.device
    fps = torch.empty((max(n, 0), 32), dtype=torch.uint8, device=dev)
    bs = torch.empty((block_sums_for(n), 32), dtype=torch.uint8, device=dev) if block_sums else None
    # the kernel may read the last dword containing data[offsets[n]-1]: pad to 4
    if data.numel() % 4:
        data = torch.cat([data, torch.zeros(4 - data.numel() % 4, dtype=torch.uint8, device=dev)])
    A.check(A.lib().rh_lift_encoded_async(_ptr(data), data.numel(), _ptr(offsets), n, _ptr(fps), _ptr(bs),
                                          _stream()),
            "rh_lift_encoded_async")
    return fps, bs


def lift_fixed(data: torch.Tensor, record_len: int, n: Optional[int] = None, block_sums: bool = True):
    """BLAKE3 of fixed-length canonical records: record i = data[i*record_len:(i+1)*record_len]
    (n defaults to data.numel() // record_len; trailing bytes are padding)."""
    if data.dtype != torch.uint8 or not data.is_cuda or data.dim() != 1:
        raise ValueError("data must be a 1-D uint8 device tensor")
    if record_len < 0:
        raise ValueError("record_len must be >= 0")
    if n is None:
        if record_len == 0:
            raise ValueError("n is required when record_len is 0")
        n = data.numel() // record_len
    dev = data.device
    fps = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    bs = torch.empty((block_sums_for(n), 32), dtype=torch.uint8, device=dev) if block_sums else None
    if data.numel() % 4:
        data = torch.cat([data, torch.zeros(4 - data.numel() % 4, dtype=torch.uint8, device=dev)])
    A.check(A.lib().rh_lift_fixed_async(_ptr(data), data.numel(), record_len, n, _ptr(fps), _ptr(bs), _stream()),
            "rh_lift_fixed_async")
    return fps, bs


def reduce_blocks(x: torch.Tensor) -> torch.Tensor:
    """out[g] = Σ x[256g .. 256g+255] (mod 2^256)."""
    n = x.shape[0]
    out = torch.empty((block_sums_for(n), 32), dtype=torch.uint8, device=x.device)
    A.check(A.lib().rh_reduce_blocks_async(_ptr(x), n, _ptr(out), _stream()), "rh_reduce_blocks_async")
    return out


def range_aggregates(fps: torch.Tensor, bsums: Optional[torch.Tensor], ssums: Optional[torch.Tensor],
                     lo: torch.Tensor, hi: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(r, 5) int64 device tensor: per rank range [lo, hi), fingerprint limbs 0..3 then size."""
    n = fps.shape[0]
    r = lo.numel()
    if hi.numel() != r or lo.dtype != torch.int64 or hi.dtype != torch.int64:
        raise ValueError("lo / hi must be int64 of equal length")
    if bsums is not None and bsums.shape[0] != block_sums_for(n):
        raise ValueError("block sums do not match fps")
    if ssums is not None and (bsums is None or ssums.shape[0] != block_sums_for(bsums.shape[0])):
        raise ValueError("super-block sums do not match block sums")
    if out is None:
        out = torch.empty((r, 5), dtype=torch.int64, device=fps.device)
    A.check(A.lib().rh_range_aggregates_async(_ptr(fps), _ptr(bsums), _ptr(ssums), n, _ptr(lo), _ptr(hi), r,
                                              _ptr(out), _stream()), "rh_range_aggregates_async")
    return out


def combine_aggregates(parts: torch.Tensor) -> torch.Tensor:
    """parts: (P, r, 5) int64 gathered aggregates -> (r, 5) Σ over P (Aggregate's Add)."""
    p, r, five = parts.shape
    assert five == 5
    out = torch.empty((r, 5), dtype=torch.int64, device=parts.device)
    A.check(A.lib().rh_combine_aggregates_async(_ptr(parts.contiguous()), p, r, _ptr(out), _stream()),
            "rh_combine_aggregates_async")
    return out
