//! Raw declarations of include/rsos_hip.h (the C ABI of librsos_hip.so).  Every item here is
//! one-to-one with the header; the safe layer is in lib.rs.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub const RH_ABI_VERSION: c_int = 1;
pub const RH_BLOCK: usize = 256;
pub const RH_SUPER: usize = 65536;
/// One `rh_store` holds fewer than this many rows (`include/rsos_hip.h`, "Row cap").
pub const RH_STORE_MAX_ROWS: u64 = 2147483648;
pub const RH_OK: c_int = 0;
pub const RH_KEY_UNIT: i32 = 0;
pub const RH_KEY_U32: i32 = 1;
pub const RH_KEY_U64: i32 = 2;
pub const RH_KEY_BYTES: i32 = 3;
pub const RH_VAL_UNIT: i32 = 0;
pub const RH_VAL_U32: i32 = 1;
pub const RH_VAL_U64: i32 = 2;
pub const RH_VAL_BYTES: i32 = 3;
pub const RH_REC_PLAIN: i32 = 0;
pub const RH_REC_DATED: i32 = 1;
pub const RH_REC_PROJECTION: i32 = 2;

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rh_schema {
    pub key_kind: i32,
    pub key_len: u32,
    pub value_kind: i32,
    pub value_len: u32,
    pub record_kind: i32,
    pub reserved: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rh_columns {
    pub keys: *const c_void,
    pub phys: *const u64,
    pub logical: *const u32,
    pub node: *const u64,
    pub tags: *const u8,
    pub values: *const c_void,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct rh_aggregate {
    pub fingerprint: [u64; 4],
    pub size: u64,
}

#[repr(C)]
pub struct rh_store {
    _private: [u8; 0],
}

#[repr(C)]
pub struct rh_estore {
    _private: [u8; 0],
}

#[repr(C)]
pub struct rh_sstore {
    _private: [u8; 0],
}

#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct rh_snapshot_info {
    pub entries: u64,
    pub tombstones: u64,
    pub entries_end: u64,
    pub keys: u64,
}

pub const RH_POLICY_FIXED_FAN_OUT: c_int = 0;
pub const RH_POLICY_SQRT_FAN_OUT: c_int = 1;

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rh_segments {
    pub start_kinds: *mut u8,
    pub start_keys: *mut c_void,
    pub end_kinds: *mut u8,
    pub end_keys: *mut c_void,
    pub aggregates: *mut rh_aggregate,
    pub n: usize,
    pub cap: usize,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct rh_round_outcome {
    pub skipped: u64,
    pub enumerated: u64,
    pub split: u64,
    pub children: u64,
    pub dropped_malformed: u64,
}

pub const RH_ERR_ARG: c_int = -1;
pub const RH_ERR_HIP: c_int = -2;
pub const RH_ERR_OOM: c_int = -3;
pub const RH_ERR_UNSUPPORTED: c_int = -4;
pub const RH_ERR_STATE: c_int = -5;
pub const RH_ERR_DATA: c_int = -6;
pub const RH_FORM_ARRAY: c_int = 0;
pub const RH_FORM_VEC: c_int = 1;

// Every entry point of include/rsos_hip.h, in header order.
extern "C" {
    pub fn rh_abi_version() -> c_int;
    pub fn rh_last_error() -> *const c_char;
    pub fn rh_schema_supported(schema: *const rh_schema) -> c_int;
    pub fn rh_schema_record_len(schema: *const rh_schema, tombstone: c_int) -> i64;
    pub fn rh_num_blocks(n: usize) -> usize;
    pub fn rh_num_superblocks(n: usize) -> usize;
    pub fn rh_lift_records_async(schema: *const rh_schema, dev_cols: *const rh_columns, n: usize, dev_fps: *mut u8,
                                 dev_block_sums: *mut u8, stream: *mut c_void) -> c_int;
    pub fn rh_lift_dual_async(schema: *const rh_schema, dev_cols: *const rh_columns, n: usize, fps_dated: *mut u8,
                              bsums_dated: *mut u8, fps_proj: *mut u8, bsums_proj: *mut u8,
                              stream: *mut c_void) -> c_int;
    pub fn rh_lift_encoded_async(dev_bytes: *const u8, bytes_len: usize, dev_offsets: *const u64, n: usize,
                                 dev_fps: *mut u8, dev_block_sums: *mut u8, stream: *mut c_void) -> c_int;
    pub fn rh_lift_fixed_async(dev_bytes: *const u8, bytes_len: usize, record_len: usize, n: usize,
                               dev_fps: *mut u8, dev_block_sums: *mut u8, stream: *mut c_void) -> c_int;
    pub fn rh_reduce_blocks_async(dev_in: *const u8, n_in: usize, dev_out: *mut u8, stream: *mut c_void) -> c_int;
    pub fn rh_range_aggregates_async(dev_fps: *const u8, dev_block_sums: *const u8, dev_super_sums: *const u8,
                                     n: usize, dev_lo: *const u64, dev_hi: *const u64, r: usize,
                                     dev_out: *mut rh_aggregate, stream: *mut c_void) -> c_int;
    pub fn rh_combine_aggregates_async(dev_in: *const rh_aggregate, parts: usize, r: usize, dev_out: *mut rh_aggregate,
                                       stream: *mut c_void) -> c_int;
    pub fn rh_lift_host(device: c_int, schema: *const rh_schema, cols: *const rh_columns, n: usize, fps: *mut u8) -> c_int;
    pub fn rh_host_alloc(bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn rh_host_free(p: *mut c_void) -> c_int;
    pub fn rh_fp_add(a: *const u64, b: *const u64, out: *mut u64);
    pub fn rh_fp_sub(a: *const u64, b: *const u64, out: *mut u64);
    pub fn rh_store_create(device: c_int, schema: *const rh_schema, out: *mut *mut rh_store) -> c_int;
    pub fn rh_store_destroy(store: *mut rh_store) -> c_int;
    pub fn rh_store_load(store: *mut rh_store, cols: *const rh_columns, n: usize) -> c_int;
    pub fn rh_store_load_device(store: *mut rh_store, dev_cols: *const rh_columns, n: usize,
                                after_stream: *mut c_void) -> c_int;
    pub fn rh_store_len(store: *mut rh_store, out: *mut u64) -> c_int;
    pub fn rh_store_aggregate(store: *mut rh_store, lo: u64, hi: u64, out: *mut rh_aggregate) -> c_int;
    pub fn rh_store_aggregates(store: *mut rh_store, lo: *const u64, hi: *const u64, r: usize, out: *mut rh_aggregate) -> c_int;
    pub fn rh_store_aggregate_keys(store: *mut rh_store, lo_kind: c_int, lo_key: *const c_void, hi_kind: c_int,
                                   hi_key: *const c_void, out: *mut rh_aggregate) -> c_int;
    pub fn rh_store_rank(store: *mut rh_store, key: *const c_void, out: *mut u64) -> c_int;
    pub fn rh_store_ranks(store: *mut rh_store, keys: *const c_void, m: usize, out: *mut u64) -> c_int;
    pub fn rh_store_select(store: *mut rh_store, r: u64, key_out: *mut c_void) -> c_int;
    pub fn rh_store_keys(store: *mut rh_store, lo: u64, hi: u64, host_out: *mut c_void) -> c_int;
    pub fn rh_store_fingerprints(store: *mut rh_store, lo: u64, hi: u64, host_out: *mut u8) -> c_int;
    pub fn rh_store_resolve_segments(store: *mut rh_store, r: usize, start_kinds: *const u8,
                                     start_keys: *const c_void, end_kinds: *const u8, end_keys: *const c_void,
                                     raw_start: *mut u64, raw_end: *mut u64, local: *mut rh_aggregate) -> c_int;
    pub fn rh_store_split_segments(store: *mut rh_store, m: usize, select_ranks: *const u64, keys_out: *mut c_void,
                                   q: usize, lo: *const u64, hi: *const u64, out: *mut rh_aggregate) -> c_int;
    pub fn rh_store_protocol_round(store: *mut rh_store, policy: c_int, fan_out: u64, active: *const rh_segments,
                                   children: *mut rh_segments, enumerations: *mut rh_segments,
                                   outcome: *mut rh_round_outcome) -> c_int;
    pub fn rh_store_apply(store: *mut rh_store, cols: *const rh_columns, ops: *const u8, n: usize,
                          n_new: *mut u64, n_over: *mut u64, n_del: *mut u64) -> c_int;
    pub fn rh_store_apply_device(store: *mut rh_store, dev_cols: *const rh_columns, dev_ops: *const u8, n: usize,
                                 n_new: *mut u64, n_over: *mut u64, n_del: *mut u64,
                                 after_stream: *mut c_void) -> c_int;
    pub fn rh_store_apply_device_many(store: *mut rh_store, dev_cols: *const rh_columns, dev_ops: *const *const u8,
                                      n: *const usize, k: usize, counts: *mut u64, after_stream: *mut c_void)
                                      -> c_int;
    pub fn rh_store_compact(store: *mut rh_store) -> c_int;
    pub fn rh_store_stage(store: *mut rh_store, cols: *const rh_columns, ops: *const u8, n: usize) -> c_int;
    pub fn rh_store_set_host_tier(store: *mut rh_store, enable: c_int, round_max: u64) -> c_int;
    pub fn rh_store_tier_stats(store: *mut rh_store, base_rows: *mut u64, delta_entries: *mut u64,
                               refreshes: *mut u64, folds: *mut u64) -> c_int;
    pub fn rh_store_tier_sync(store: *mut rh_store) -> c_int;
    pub fn rh_store_set_tier_policy(store: *mut rh_store, keep_fresh: c_int) -> c_int;
    pub fn rh_store_set_compaction(store: *mut rh_store, divisor: u64, min_rows: u64) -> c_int;
    pub fn rh_store_reserve(store: *mut rh_store, rows: u64, batch_rows: u64) -> c_int;
    pub fn rh_store_stats(store: *mut rh_store, base_rows: *mut u64, delta_rows: *mut u64,
                          compactions: *mut u64) -> c_int;
    pub fn rh_store_batch_stats(store: *mut rh_store, small_batches: *mut u64, large_batches: *mut u64) -> c_int;
    pub fn rh_snapshot_header(bytes: *const c_void, len: usize, entries: *mut u64) -> c_int;
    pub fn rh_snapshot_decode_device(schema: *const rh_schema, key_form: c_int, dev_bytes: *const c_void, len: usize,
                                     dev_out: *const rh_columns, cap: usize, info: *mut rh_snapshot_info,
                                     stream: *mut c_void) -> c_int;
    pub fn rh_store_load_snapshot(dated: *mut rh_store, projection: *mut rh_store, key_form: c_int,
                                  bytes: *const c_void, len: usize, bytes_on_device: c_int,
                                  info: *mut rh_snapshot_info, after_stream: *mut c_void) -> c_int;
    pub fn rh_wire_encode_range_aggregates(schema: *const rh_schema, key_form: c_int, msg_tag: c_int,
                                           start_kinds: *const u8, start_keys: *const c_void, end_kinds: *const u8,
                                           end_keys: *const c_void, aggregates: *const rh_aggregate, r: usize,
                                           out: *mut u8, cap: usize, out_len: *mut usize) -> c_int;
    pub fn rh_wire_decode_range_aggregates(schema: *const rh_schema, key_form: c_int, msg_tag: c_int, input: *const u8,
                                           len: usize, r_cap: usize, start_kinds: *mut u8, start_keys: *mut c_void,
                                           end_kinds: *mut u8, end_keys: *mut c_void, aggregates: *mut rh_aggregate,
                                           r_out: *mut usize, consumed: *mut usize) -> c_int;
    pub fn rh_estore_create(device: c_int, out: *mut *mut rh_estore) -> c_int;
    pub fn rh_estore_destroy(store: *mut rh_estore) -> c_int;
    pub fn rh_estore_load(store: *mut rh_estore, bytes: *const u8, offsets: *const u64, n: usize) -> c_int;
    pub fn rh_estore_apply(store: *mut rh_estore, pos: *const u64, kinds: *const u8, m: usize, bytes: *const u8,
                           offsets: *const u64, nrec: usize) -> c_int;
    pub fn rh_estore_len(store: *mut rh_estore, out: *mut u64) -> c_int;
    pub fn rh_estore_root(store: *mut rh_estore, out: *mut rh_aggregate) -> c_int;
    pub fn rh_estore_aggregates(store: *mut rh_estore, lo: *const u64, hi: *const u64, r: usize,
                                out: *mut rh_aggregate) -> c_int;
    pub fn rh_estore_fingerprints(store: *mut rh_estore, lo: u64, hi: u64, host_out: *mut u8) -> c_int;
    pub fn rh_estore_set_host_tier(store: *mut rh_estore, enable: c_int) -> c_int;
    pub fn rh_sstore_create(devices: *const c_int, n: c_int, schema: *const rh_schema, out: *mut *mut rh_sstore) -> c_int;
    pub fn rh_sstore_destroy(store: *mut rh_sstore) -> c_int;
    pub fn rh_sstore_shard_count(store: *mut rh_sstore) -> c_int;
    pub fn rh_sstore_shard(store: *mut rh_sstore, i: c_int, out: *mut *mut rh_store) -> c_int;
    pub fn rh_sstore_splitters(store: *mut rh_sstore, out: *mut c_void) -> c_int;
    pub fn rh_sstore_set_splitters(store: *mut rh_sstore, keys: *const c_void) -> c_int;
    pub fn rh_sstore_load(store: *mut rh_sstore, cols: *const rh_columns, n: usize) -> c_int;
    pub fn rh_sstore_stage(store: *mut rh_sstore, cols: *const rh_columns, ops: *const u8, m: usize) -> c_int;
    pub fn rh_sstore_apply(store: *mut rh_sstore, cols: *const rh_columns, ops: *const u8, n: usize,
                           n_new: *mut u64, n_over: *mut u64, n_del: *mut u64) -> c_int;
    pub fn rh_sstore_len(store: *mut rh_sstore, out: *mut u64) -> c_int;
    pub fn rh_sstore_aggregates(store: *mut rh_sstore, lo: *const u64, hi: *const u64, r: usize,
                                out: *mut rh_aggregate) -> c_int;
    pub fn rh_sstore_aggregate_keys(store: *mut rh_sstore, lo_kind: c_int, lo_key: *const c_void, hi_kind: c_int,
                                    hi_key: *const c_void, out: *mut rh_aggregate) -> c_int;
    pub fn rh_sstore_rank(store: *mut rh_sstore, key: *const c_void, out: *mut u64) -> c_int;
    pub fn rh_sstore_ranks(store: *mut rh_sstore, keys: *const c_void, m: usize, out: *mut u64) -> c_int;
    pub fn rh_sstore_select(store: *mut rh_sstore, r: u64, key_out: *mut c_void) -> c_int;
    pub fn rh_sstore_keys(store: *mut rh_sstore, lo: u64, hi: u64, host_out: *mut c_void) -> c_int;
    pub fn rh_sstore_fingerprints(store: *mut rh_sstore, lo: u64, hi: u64, host_out: *mut u8) -> c_int;
    pub fn rh_sstore_resolve_segments(store: *mut rh_sstore, r: usize, start_kinds: *const u8,
                                      start_keys: *const c_void, end_kinds: *const u8, end_keys: *const c_void,
                                      raw_start: *mut u64, raw_end: *mut u64, local: *mut rh_aggregate) -> c_int;
    pub fn rh_sstore_split_segments(store: *mut rh_sstore, m: usize, select_ranks: *const u64, keys_out: *mut c_void,
                                    q: usize, lo: *const u64, hi: *const u64, out: *mut rh_aggregate) -> c_int;
    pub fn rh_sstore_protocol_round(store: *mut rh_sstore, policy: c_int, fan_out: u64, active: *const rh_segments,
                                    children: *mut rh_segments, enumerations: *mut rh_segments,
                                    outcome: *mut rh_round_outcome) -> c_int;
    pub fn rh_sstore_set_host_tier(store: *mut rh_sstore, enable: c_int, round_max: u64) -> c_int;
    pub fn rh_sstore_set_tier_policy(store: *mut rh_sstore, keep_fresh: c_int) -> c_int;
    pub fn rh_sstore_reserve(store: *mut rh_sstore, rows: u64, batch_rows: u64) -> c_int;
    pub fn rh_sstore_compact(store: *mut rh_sstore) -> c_int;
    pub fn rh_debug_fail_point(name: *const c_char) -> c_int;
    pub fn rh_debug_reload_timing(on: c_int) -> c_int;
    pub fn rh_debug_last_reload_us(locate_us: *mut f64, lift_us: *mut f64) -> c_int;
    pub fn rh_debug_batch_timing(on: c_int) -> c_int;
    pub fn rh_debug_batch_kernel_us(lift_search_us: *mut f64, launches: *mut u64) -> c_int;
}
