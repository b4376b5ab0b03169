"""Canonical encoding of typed keys and values (rsos::encoding, rsos/src/encoding.rs:17-35) on the host.

The GPU hashes records it is handed as bytes (the encoded store, rh_estore_*); this module produces
those bytes for key / value types without a fixed-width column form -- what the Rust binding gets
from `rsos::encoding::encode_to_vec` (public-api/rsos.txt:61).  A type is described by a small
spec, mirroring the serde data model the reference's Serializer sees:

  "bool" | "u8" "u16" "u32" "u64" "u128" | "i8" "i16" "i32" "i64" "i128"   fixed-width LE
  "str" / "bytes"      u64 LE length, then the bytes         (String, &str, serde_bytes)
  ("vec", T)           u64 LE count, then the elements       (Vec<T>; Vec<u8> = "bytes" bytes)
  ("array", T, N)      u64 LE count N, then the elements     ([T; N] is a serde tuple)
  ("option", T)        0, or 1 then the value
  ("tuple", T1, ...)   u64 LE count, then the elements
  ("struct", T1, ...)  the fields in declaration order, nothing else
  "unit"               nothing
  ("entry", V)         Entry<Timestamp, V> (lww-register/src/entry.rs:88-94): value is an
                       Entry(value, phys, logical, node, tombstone) -> Timestamp as u64 / u32 /
                       u64 (clock.rs:143-181), then State: u32 0 + V, or u32 1
  ("state", V)         State<V> (entry.rs:24-29), the projection: u32 0 + V, or u32 1
"""
from __future__ import annotations

import struct
from typing import Any

_INT = {"u8": "<B", "u16": "<H", "u32": "<I", "u64": "<Q", "i8": "<b", "i16": "<h", "i32": "<i", "i64": "<q"}


def encode(spec: Any, value: Any) -> bytes:
    out = bytearray()
    _put(out, spec, value)
    return bytes(out)


def _put(out: bytearray, spec: Any, v: Any) -> None:
    if isinstance(spec, str):
        if spec in _INT:
            out += struct.pack(_INT[spec], v)
        elif spec in ("u128", "i128"):
            out += int(v).to_bytes(16, "little", signed=spec == "i128")
        elif spec == "bool":
            out.append(1 if v else 0)
        elif spec in ("str", "bytes"):
            b = v.encode("utf-8") if isinstance(v, str) else bytes(v)
            out += struct.pack("<Q", len(b))
            out += b
        elif spec == "unit":
            pass
        else:
            raise ValueError(f"unknown type {spec!r}")
        return
    kind = spec[0]
    if kind == "vec":
        items = list(v)
        if spec[1] == "u8" and isinstance(v, (bytes, bytearray)):
            out += struct.pack("<Q", len(v)) + bytes(v)
            return
        out += struct.pack("<Q", len(items))
        for x in items:
            _put(out, spec[1], x)
    elif kind == "array":
        items = list(v)
        if len(items) != spec[2]:
            raise ValueError(f"array of {spec[2]} elements expected, got {len(items)}")
        out += struct.pack("<Q", spec[2])
        for x in items:
            _put(out, spec[1], x)
    elif kind == "option":
        if v is None:
            out.append(0)
        else:
            out.append(1)
            _put(out, spec[1], v)
    elif kind == "tuple":
        if len(v) != len(spec) - 1:
            raise ValueError("tuple arity mismatch")
        out += struct.pack("<Q", len(v))
        for t, x in zip(spec[1:], v):
            _put(out, t, x)
    elif kind == "struct":
        if len(v) != len(spec) - 1:
            raise ValueError("struct field count mismatch")
        for t, x in zip(spec[1:], v):
            _put(out, t, x)
    elif kind in ("entry", "state"):
        if kind == "entry":
            out += struct.pack("<QIQ", v.phys, v.logical, v.node)
        if v.tombstone:
            out += struct.pack("<I", 1)
        else:
            out += struct.pack("<I", 0)
            _put(out, spec[1], v.value)
    else:
        raise ValueError(f"unknown type {spec!r}")
