//! Raw declarations of include/rsos_hip.h (the C ABI of librsos_hip.so).  Every item here is
//! one-to-one with the header; the safe layer is in lib.rs.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

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

extern "C" {
    pub fn rh_abi_version() -> c_int;
    pub fn rh_last_error() -> *const c_char;
    pub fn rh_schema_supported(schema: *const rh_schema) -> c_int;
    pub fn rh_schema_record_len(schema: *const rh_schema, tombstone: c_int) -> i64;
    pub fn rh_lift_host(device: c_int, schema: *const rh_schema, cols: *const rh_columns, n: usize, fps: *mut u8) -> c_int;
    pub fn rh_fp_add(a: *const u64, b: *const u64, out: *mut u64);
    pub fn rh_fp_sub(a: *const u64, b: *const u64, out: *mut u64);
    pub fn rh_store_create(device: c_int, schema: *const rh_schema, out: *mut *mut rh_store) -> c_int;
    pub fn rh_store_destroy(store: *mut rh_store) -> c_int;
    pub fn rh_store_load(store: *mut rh_store, cols: *const rh_columns, n: usize) -> c_int;
    pub fn rh_store_len(store: *const rh_store, out: *mut u64) -> c_int;
    pub fn rh_store_aggregate(store: *mut rh_store, lo: u64, hi: u64, out: *mut rh_aggregate) -> c_int;
    pub fn rh_store_aggregates(store: *mut rh_store, lo: *const u64, hi: *const u64, r: usize, out: *mut rh_aggregate) -> c_int;
    pub fn rh_store_aggregate_keys(store: *mut rh_store, lo_kind: c_int, lo_key: *const c_void, hi_kind: c_int,
                                   hi_key: *const c_void, out: *mut rh_aggregate) -> c_int;
    pub fn rh_store_rank(store: *mut rh_store, key: *const c_void, out: *mut u64) -> c_int;
    pub fn rh_store_apply(store: *mut rh_store, cols: *const rh_columns, ops: *const u8, n: usize,
                          n_new: *mut u64, n_over: *mut u64, n_del: *mut u64) -> c_int;
}
