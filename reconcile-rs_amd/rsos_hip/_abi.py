"""ctypes declarations of librsos_hip.so (include/rsos_hip.h).

The library is the product: there is no CPU fallback.  If the .so is missing, `lib()`
raises -- build it with `make -C reconcile-rs_amd` (or `__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_lib", "librsos_hip.so")

# rh_status
OK, ERR_ARG, ERR_HIP, ERR_OOM, ERR_UNSUPPORTED, ERR_STATE, ERR_DATA = 0, -1, -2, -3, -4, -5, -6
# schema enums (rsos_hip.h)
KEY_UNIT, KEY_U32, KEY_U64, KEY_BYTES = 0, 1, 2, 3
VAL_UNIT, VAL_U32, VAL_U64, VAL_BYTES = 0, 1, 2, 3
REC_PLAIN, REC_DATED, REC_PROJECTION = 0, 1, 2
BLOCK, SUPER = 256, 65536
FORM_ARRAY, FORM_VEC = 0, 1  # rh_key_form: [u8; L] | Vec<u8> / String


class Schema(C.Structure):
    _fields_ = [("key_kind", C.c_int32), ("key_len", C.c_uint32), ("value_kind", C.c_int32),
                ("value_len", C.c_uint32), ("record_kind", C.c_int32), ("reserved", C.c_uint32)]


class Columns(C.Structure):
    _fields_ = [("keys", C.c_void_p), ("phys", C.c_void_p), ("logical", C.c_void_p),
                ("node", C.c_void_p), ("tags", C.c_void_p), ("values", C.c_void_p)]


class Aggregate(C.Structure):
    _fields_ = [("fingerprint", C.c_uint64 * 4), ("size", C.c_uint64)]


class Segments(C.Structure):  # rh_segments
    _fields_ = [("start_kinds", C.c_void_p), ("start_keys", C.c_void_p), ("end_kinds", C.c_void_p),
                ("end_keys", C.c_void_p), ("aggregates", C.c_void_p), ("n", C.c_size_t), ("cap", C.c_size_t)]


class RoundOutcome(C.Structure):  # rh_round_outcome
    _fields_ = [("skipped", C.c_uint64), ("enumerated", C.c_uint64), ("split", C.c_uint64),
                ("children", C.c_uint64), ("dropped_malformed", C.c_uint64)]


POLICY_FIXED_FAN_OUT, POLICY_SQRT_FAN_OUT = 0, 1


class SnapshotInfo(C.Structure):
    _fields_ = [("entries", C.c_uint64), ("tombstones", C.c_uint64), ("entries_end", C.c_uint64),
                ("keys", C.c_uint64)]


# (name, restype, argtypes) -- every entry point include/rsos_hip.h declares
P, U8P, U64P, SZ, VP = C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p
SIGNATURES = [
    ("rh_abi_version", C.c_int, []),
    ("rh_last_error", C.c_char_p, []),
    ("rh_schema_supported", C.c_int, [C.POINTER(Schema)]),
    ("rh_schema_record_len", C.c_int64, [C.POINTER(Schema), C.c_int]),
    ("rh_num_blocks", C.c_size_t, [SZ]),
    ("rh_num_superblocks", C.c_size_t, [SZ]),
    ("rh_lift_records_async", C.c_int, [C.POINTER(Schema), C.POINTER(Columns), SZ, U8P, U8P, VP]),
    ("rh_lift_dual_async", C.c_int, [C.POINTER(Schema), C.POINTER(Columns), SZ, U8P, U8P, U8P, U8P, VP]),
    ("rh_lift_encoded_async", C.c_int, [U8P, SZ, U64P, SZ, U8P, U8P, VP]),
    ("rh_lift_fixed_async", C.c_int, [U8P, SZ, SZ, SZ, U8P, U8P, VP]),
    ("rh_reduce_blocks_async", C.c_int, [U8P, SZ, U8P, VP]),
    ("rh_range_aggregates_async", C.c_int, [U8P, U8P, U8P, SZ, U64P, U64P, SZ, P, VP]),
    ("rh_combine_aggregates_async", C.c_int, [P, SZ, SZ, P, VP]),
    ("rh_lift_host", C.c_int, [C.c_int, C.POINTER(Schema), C.POINTER(Columns), SZ, U8P]),
    ("rh_host_alloc", C.c_int, [SZ, C.POINTER(C.c_void_p)]),
    ("rh_host_free", C.c_int, [C.c_void_p]),
    ("rh_fp_add", None, [U64P, U64P, U64P]),
    ("rh_fp_sub", None, [U64P, U64P, U64P]),
    ("rh_store_create", C.c_int, [C.c_int, C.POINTER(Schema), C.POINTER(C.c_void_p)]),
    ("rh_store_destroy", C.c_int, [P]),
    ("rh_store_load", C.c_int, [P, C.POINTER(Columns), SZ]),
    ("rh_store_load_device", C.c_int, [P, C.POINTER(Columns), SZ, VP]),
    ("rh_store_len", C.c_int, [P, C.POINTER(C.c_uint64)]),
    ("rh_store_aggregate", C.c_int, [P, C.c_uint64, C.c_uint64, C.POINTER(Aggregate)]),
    ("rh_store_aggregates", C.c_int, [P, U64P, U64P, SZ, P]),
    ("rh_store_aggregate_keys", C.c_int, [P, C.c_int, VP, C.c_int, VP, C.POINTER(Aggregate)]),
    ("rh_store_rank", C.c_int, [P, VP, C.POINTER(C.c_uint64)]),
    ("rh_store_ranks", C.c_int, [P, VP, SZ, U64P]),
    ("rh_store_keys", C.c_int, [P, C.c_uint64, C.c_uint64, VP]),
    ("rh_store_select", C.c_int, [P, C.c_uint64, VP]),
    ("rh_store_fingerprints", C.c_int, [P, C.c_uint64, C.c_uint64, U8P]),
    ("rh_store_resolve_segments", C.c_int, [P, SZ, U8P, VP, U8P, VP, U64P, U64P, P]),
    ("rh_store_split_segments", C.c_int, [P, SZ, U64P, VP, SZ, U64P, U64P, P]),
    ("rh_store_protocol_round", C.c_int, [P, C.c_int, C.c_uint64, C.POINTER(Segments), C.POINTER(Segments),
                                          C.POINTER(Segments), C.POINTER(RoundOutcome)]),
    ("rh_store_apply", C.c_int, [P, C.POINTER(Columns), U8P, SZ, C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("rh_store_apply_device", C.c_int, [P, C.POINTER(Columns), U8P, SZ, C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), VP]),
    ("rh_store_apply_device_many", C.c_int, [P, C.POINTER(Columns), C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                             SZ, C.POINTER(C.c_uint64), VP]),
    ("rh_store_compact", C.c_int, [P]),
    ("rh_store_set_compaction", C.c_int, [P, C.c_uint64, C.c_uint64]),
    ("rh_store_set_host_tier", C.c_int, [P, C.c_int, C.c_uint64]),
    ("rh_store_stage", C.c_int, [P, C.POINTER(Columns), U8P, SZ]),
    ("rh_store_reserve", C.c_int, [P, C.c_uint64, C.c_uint64]),
    ("rh_store_stats", C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("rh_store_batch_stats", C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("rh_store_tier_stats", C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64)]),
    ("rh_store_tier_sync", C.c_int, [P]),
    ("rh_store_set_tier_policy", C.c_int, [P, C.c_int]),
    ("rh_snapshot_header", C.c_int, [VP, SZ, C.POINTER(C.c_uint64)]),
    ("rh_snapshot_decode_device", C.c_int, [C.POINTER(Schema), C.c_int, VP, SZ, C.POINTER(Columns), SZ,
                                            C.POINTER(SnapshotInfo), VP]),
    ("rh_store_load_snapshot", C.c_int, [P, P, C.c_int, VP, SZ, C.c_int, C.POINTER(SnapshotInfo), VP]),
    ("rh_wire_encode_range_aggregates", C.c_int, [C.POINTER(Schema), C.c_int, C.c_int, U8P, VP, U8P, VP, P, SZ,
                                                  U8P, SZ, C.POINTER(C.c_size_t)]),
    ("rh_wire_decode_range_aggregates", C.c_int, [C.POINTER(Schema), C.c_int, C.c_int, U8P, SZ, SZ, U8P, VP, U8P,
                                                  VP, P, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    ("rh_estore_create", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("rh_estore_destroy", C.c_int, [P]),
    ("rh_estore_load", C.c_int, [P, VP, U64P, SZ]),
    ("rh_estore_apply", C.c_int, [P, U64P, U8P, SZ, VP, U64P, SZ]),
    ("rh_estore_len", C.c_int, [P, C.POINTER(C.c_uint64)]),
    ("rh_estore_root", C.c_int, [P, C.POINTER(Aggregate)]),
    ("rh_estore_aggregates", C.c_int, [P, U64P, U64P, SZ, P]),
    ("rh_estore_fingerprints", C.c_int, [P, C.c_uint64, C.c_uint64, U8P]),
    ("rh_estore_set_host_tier", C.c_int, [P, C.c_int]),
    ("rh_sstore_create", C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(Schema), C.POINTER(C.c_void_p)]),
    ("rh_sstore_destroy", C.c_int, [P]),
    ("rh_sstore_shard_count", C.c_int, [P]),
    ("rh_sstore_shard", C.c_int, [P, C.c_int, C.POINTER(C.c_void_p)]),
    ("rh_sstore_splitters", C.c_int, [P, VP]),
    ("rh_sstore_set_splitters", C.c_int, [P, VP]),
    ("rh_sstore_load", C.c_int, [P, C.POINTER(Columns), SZ]),
    ("rh_sstore_stage", C.c_int, [P, C.POINTER(Columns), U8P, SZ]),
    ("rh_sstore_apply", C.c_int, [P, C.POINTER(Columns), U8P, SZ, C.POINTER(C.c_uint64),
                                  C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("rh_sstore_len", C.c_int, [P, C.POINTER(C.c_uint64)]),
    ("rh_sstore_aggregates", C.c_int, [P, U64P, U64P, SZ, P]),
    ("rh_sstore_aggregate_keys", C.c_int, [P, C.c_int, VP, C.c_int, VP, C.POINTER(Aggregate)]),
    ("rh_sstore_rank", C.c_int, [P, VP, C.POINTER(C.c_uint64)]),
    ("rh_sstore_ranks", C.c_int, [P, VP, SZ, U64P]),
    ("rh_sstore_select", C.c_int, [P, C.c_uint64, VP]),
    ("rh_sstore_keys", C.c_int, [P, C.c_uint64, C.c_uint64, VP]),
    ("rh_sstore_fingerprints", C.c_int, [P, C.c_uint64, C.c_uint64, U8P]),
    ("rh_sstore_resolve_segments", C.c_int, [P, SZ, U8P, VP, U8P, VP, U64P, U64P, P]),
    ("rh_sstore_split_segments", C.c_int, [P, SZ, U64P, VP, SZ, U64P, U64P, P]),
    ("rh_sstore_protocol_round", C.c_int, [P, C.c_int, C.c_uint64, C.POINTER(Segments), C.POINTER(Segments),
                                           C.POINTER(Segments), C.POINTER(RoundOutcome)]),
    ("rh_sstore_set_host_tier", C.c_int, [P, C.c_int, C.c_uint64]),
    ("rh_sstore_set_tier_policy", C.c_int, [P, C.c_int]),
    ("rh_sstore_reserve", C.c_int, [P, C.c_uint64, C.c_uint64]),
    ("rh_sstore_compact", C.c_int, [P]),
    ("rh_debug_fail_point", C.c_int, [C.c_char_p]),
    ("rh_debug_reload_timing", C.c_int, [C.c_int]),
    ("rh_debug_last_reload_us", C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("rh_debug_batch_timing", C.c_int, [C.c_int]),
    ("rh_debug_batch_kernel_us", C.c_int, [C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
]

_lib = None


class RsosHipError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where} failed ({code}): {msg}")
        self.code = code


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"librsos_hip.so not found at {LIB_PATH}: the HIP path is the only path; "
                "build it with `make -C reconcile-rs_amd` or __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.rh_abi_version() != 1:
            raise RuntimeError("librsos_hip.so ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, where: str) -> int:
    if rc < 0:
        raise RsosHipError(rc, where, (lib().rh_last_error() or b"").decode())
    return rc
