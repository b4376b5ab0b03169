"""Snapshot reload onto the GPU.

The load side of FileSnapshot (src/snapshot.rs:30-98) and the replay that follows it in
ReplicatedMap::with_persistence (src/replicated_map/persistence.rs:108-143): every entry of
PersistedState.entries (lww-register/src/persistence.rs:32,62-70) is inserted into the dated
map and its value-only projection (just_insert_bulk, src/replica/write.rs:107-121).

On the GPU the entries are located and decoded by librsos_hip.so (rh_store_load_snapshot:
a parallel walk over the bincode entry Vec, then a column scatter), both stores are lifted and
summed from the decoded columns, and a key that appears twice keeps its last entry -- what the
sequential replay leaves.  PersistedState.members and .tombstone_acks, which follow the entries
in the file, are host state; `decode_tail` reads them on the host.

Errors are the reference's: a short file, a wrong magic or format version, or entries that do
not parse raise RsosHipError with code ERR_DATA (io::ErrorKind::InvalidData) -- never a
silent fresh start (persistence.rs:111-114).
"""
from __future__ import annotations

import ctypes as C
import ipaddress
import struct
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _abi as A
from .schema import RecordSchema

_FORMS = {"array": A.FORM_ARRAY, "vec": A.FORM_VEC}


@dataclass(frozen=True)
class SnapshotInfo:
    entries: int       # PersistedState.entries.len()
    tombstones: int    # entries holding State::Tombstone
    entries_end: int   # file offset of PersistedState.members
    keys: int          # distinct keys loaded

    @staticmethod
    def from_c(i: A.SnapshotInfo) -> "SnapshotInfo":
        return SnapshotInfo(int(i.entries), int(i.tombstones), int(i.entries_end), int(i.keys))


def _host_buffer(data) -> Tuple[int, int, object]:
    a = np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data, np.uint8)
    return (a.ctypes.data if a.size else None), a.size, a


def read_header(data, length: Optional[int] = None) -> int:
    """Validate the RCNL header of the file's first bytes; returns the entry count.  `length`:
    the whole file's length when `data` holds only its start."""
    head = bytes(np.asarray(data[:16], np.uint8).tobytes() if not isinstance(data, (bytes, bytearray, memoryview))
                 else bytes(data[:16]))
    buf = C.create_string_buffer(head, max(len(head), 1))
    out = C.c_uint64()
    A.check(A.lib().rh_snapshot_header(buf, len(data) if length is None else length, C.byref(out)),
            "rh_snapshot_header")
    return int(out.value)


def load_snapshot(data, dated=None, projection=None, key_form: str = "array") -> SnapshotInfo:
    """Replace the contents of the dated and / or projection GpuFingerprintStore with the
    snapshot's entries.  `data`: the file's bytes on the host (bytes / bytearray / memoryview /
    numpy), or a contiguous uint8 torch tensor already in HBM."""
    if dated is None and projection is None:
        raise ValueError("no store given")
    info = A.SnapshotInfo()
    is_dev = hasattr(data, "is_cuda") and data.is_cuda
    if is_dev:
        if not data.is_contiguous():
            raise ValueError("device snapshot must be contiguous")
        ptr, size, keep = data.data_ptr(), data.numel() * data.element_size(), data
    else:
        ptr, size, keep = _host_buffer(data)
    stream = None
    if is_dev:
        import torch
        stream = torch.cuda.current_stream(data.device).cuda_stream
    A.check(A.lib().rh_store_load_snapshot(dated._h if dated is not None else None,
                                           projection._h if projection is not None else None,
                                           _FORMS[key_form], ptr, size, 1 if is_dev else 0, C.byref(info), stream),
            "rh_store_load_snapshot")
    del keep
    return SnapshotInfo.from_c(info)


def decode_entries_device(schema: RecordSchema, data, key_form: str = "array"):
    """Decode a device-resident snapshot's entries into device columns (keys, phys, logical,
    node, tags, values); returns (columns, SnapshotInfo)."""
    import torch
    if not (data.is_cuda and data.is_contiguous() and data.dtype == torch.uint8):
        raise ValueError("data must be a contiguous uint8 device tensor")
    n = read_header(data[:16].cpu().numpy(), data.numel())
    dev = data.device
    cols = {
        "keys": torch.empty((n, schema.key_row), dtype=torch.uint8, device=dev),
        "phys": torch.empty(n, dtype=torch.int64, device=dev),
        "logical": torch.empty(n, dtype=torch.int32, device=dev),
        "node": torch.empty(n, dtype=torch.int64, device=dev),
        "tags": torch.empty(n, dtype=torch.uint8, device=dev),
        "values": torch.empty((n, schema.value_row), dtype=torch.uint8, device=dev),
    }
    c = A.Columns(*[cols[k].data_ptr() if cols[k].numel() else None
                    for k in ("keys", "phys", "logical", "node", "tags", "values")])
    s, info = schema.with_kind(A.REC_DATED).c(), A.SnapshotInfo()
    stream = torch.cuda.current_stream(dev).cuda_stream
    A.check(A.lib().rh_snapshot_decode_device(C.byref(s), _FORMS[key_form], data.data_ptr(), data.numel(),
                                              C.byref(c), n, C.byref(info), stream), "rh_snapshot_decode_device")
    return cols, SnapshotInfo.from_c(info)


# ---- the host part of the file: members and tombstone acks --------------------------------------
class _Rd:
    def __init__(self, d: bytes, p: int):
        self.d, self.p = d, p

    def take(self, k: int) -> bytes:
        if self.p + k > len(self.d):
            raise A.RsosHipError(A.ERR_DATA, "decode_tail", "io error: unexpected end of file")
        b = self.d[self.p:self.p + k]
        self.p += k
        return b

    def u64(self) -> int:
        return struct.unpack("<Q", self.take(8))[0]

    def ip(self):
        tag = struct.unpack("<I", self.take(4))[0]  # IpAddr: V4 = 0, V6 = 1, then the octets
        if tag > 1:
            raise A.RsosHipError(A.ERR_DATA, "decode_tail",
                                 f"invalid value: integer `{tag}`, expected variant index 0 <= i < 2")
        return ipaddress.ip_address(self.take(4 if tag == 0 else 16))


def decode_tail(data, entries_end: int, schema: RecordSchema, key_form: str = "array"
                ) -> Tuple[List, Dict[bytes, Dict[object, int]]]:
    """PersistedState.members (HashSet<IpAddr>) and .tombstone_acks (HashMap<K, HashMap<IpAddr,
    u64>>), bincode fixint, starting at entries_end.  Keys are returned as their column bytes."""
    r = _Rd(bytes(data), entries_end)
    members = [r.ip() for _ in range(r.u64())]
    acks: Dict[bytes, Dict[object, int]] = {}
    for _ in range(r.u64()):
        if key_form == "vec" and r.u64() != schema.key_row:
            raise A.RsosHipError(A.ERR_DATA, "decode_tail", "ack key length differs from the schema's")
        k = r.take(schema.key_row)
        peers = {}
        for _ in range(r.u64()):
            ip = r.ip()
            peers[ip] = r.u64()
        acks[k] = peers
    return members, acks
