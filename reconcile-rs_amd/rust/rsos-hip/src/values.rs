//! The reference's record types as device columns: `GpuRecord` for `Entry<Timestamp, V>` and
//! `State<V>` (lww-register/src/entry.rs:24-29,88-94) over a `FixedValue` trait, implemented here
//! -- in the crate that owns `GpuRecord` -- because the orphan rule forbids a facade crate from
//! implementing a foreign trait for a foreign type.
//!
//! The column synthesis must reproduce `rsos::encoding` byte for byte (rsos/src/encoding.rs:17-35):
//! * `Timestamp { hlc: Hlc { physical, logical }, node_id }`: 20 bytes, no framing
//!   (lww-register/src/clock.rs:143-181) -> the phys / logical / node columns;
//! * `State::Present(v)` = u32 variant 0 then `v`; `State::Tombstone` = u32 variant 1 -> the tag
//!   column (the variant word is synthesised on the device);
//! * `v`: a `u32` / `u64` is its LE bytes (value kinds U32 / U64, no prefix); a byte string
//!   (`Vec<u8>`, `String`, `[u8; N]`, `FixedBytes<N>`) is a u64 length prefix then the bytes
//!   (encoding/serializer.rs:105-113, :162-179) -> value kind BYTES, the prefix synthesised.
//! A value whose byte length differs from the map's value column is a panic, never a padded row:
//! a padded row would hash some other record and reconcile silently wrongly (rsos_trait.rs:54-56).

use lww_register::{Entry, State, Timestamp};
use serde::{Deserialize, Deserializer, Serialize, Serializer};

use crate::{ffi, GpuRecord, RecordRow};

/// A value type the device hashes from one fixed-width column.
pub trait FixedValue: Serialize {
    /// `RH_VAL_U32`, `RH_VAL_U64` or `RH_VAL_BYTES`
    const KIND: i32;
    /// Bytes of the value column (for BYTES: the byte string's length, without its prefix).
    const LEN: u32;
    /// Append the column bytes: LE integers, or the byte string without its length prefix.
    fn column(&self, out: &mut Vec<u8>);
}

impl FixedValue for u32 {
    const KIND: i32 = ffi::RH_VAL_U32;
    const LEN: u32 = 4;
    fn column(&self, out: &mut Vec<u8>) {
        out.extend_from_slice(&self.to_le_bytes());
    }
}

impl FixedValue for u64 {
    const KIND: i32 = ffi::RH_VAL_U64;
    const LEN: u32 = 8;
    fn column(&self, out: &mut Vec<u8>) {
        out.extend_from_slice(&self.to_le_bytes());
    }
}

// `ReplicatedSet<K>` is `ReplicatedMap<K, ()>` (src/replicated_set.rs): `State::Present(())` is
// the variant word alone (serializer.rs:133-141) -- the UNIT value kind, no value column
impl FixedValue for () {
    const KIND: i32 = ffi::RH_VAL_UNIT;
    const LEN: u32 = 0;
    fn column(&self, _out: &mut Vec<u8>) {}
}

// serde serialises [u8; N] (N <= 32) as a tuple: rsos's canonical Serializer writes the tuple's
// length as a u64 prefix then the elements (encoding/serializer.rs:176-179), i.e. the same bytes as
// a 16-byte Vec<u8> -- the BYTES value kind.
macro_rules! fixed_array {
    ($($n:literal)*) => {$(
        impl FixedValue for [u8; $n] {
            const KIND: i32 = ffi::RH_VAL_BYTES;
            const LEN: u32 = $n;
            fn column(&self, out: &mut Vec<u8>) {
                out.extend_from_slice(self);
            }
        }
    )*};
}
fixed_array!(4 8 16 32);

/// A byte string of exactly `N` bytes (`N` > 32: serde has no array impl there).  It serialises --
/// for rsos's canonical encoder, bincode on the wire and any other serde format -- exactly as a
/// `Vec<u8>` of the same bytes, so a map of `FixedBytes<64>` values has the fingerprints, wire
/// bytes and snapshots of a reference map of 64-byte `Vec<u8>` values.  Construction checks the
/// length; deserialising another length is an error.
#[derive(Clone, Debug, PartialEq, Eq, Hash, PartialOrd, Ord)]
pub struct FixedBytes<const N: usize>(Vec<u8>);

impl<const N: usize> FixedBytes<N> {
    /// `None` unless `bytes.len() == N`.
    pub fn new(bytes: Vec<u8>) -> Option<Self> {
        (bytes.len() == N).then_some(FixedBytes(bytes))
    }
    pub fn as_slice(&self) -> &[u8] {
        &self.0
    }
    pub fn into_vec(self) -> Vec<u8> {
        self.0
    }
}

impl<const N: usize> Default for FixedBytes<N> {
    fn default() -> Self {
        FixedBytes(vec![0; N])
    }
}

impl<const N: usize> Serialize for FixedBytes<N> {
    fn serialize<S: Serializer>(&self, s: S) -> Result<S::Ok, S::Error> {
        self.0.serialize(s) // Vec<u8>'s own impl: a sequence of N u8
    }
}

impl<'de, const N: usize> Deserialize<'de> for FixedBytes<N> {
    fn deserialize<D: Deserializer<'de>>(d: D) -> Result<Self, D::Error> {
        let v = Vec::<u8>::deserialize(d)?;
        let len = v.len();
        FixedBytes::new(v).ok_or_else(|| serde::de::Error::invalid_length(len, &"exactly N bytes"))
    }
}

impl<const N: usize> FixedValue for FixedBytes<N> {
    const KIND: i32 = ffi::RH_VAL_BYTES;
    const LEN: u32 = N as u32;
    fn column(&self, out: &mut Vec<u8>) {
        out.extend_from_slice(&self.0);
    }
}

fn stamp_columns(t: &Timestamp, row: &mut RecordRow) {
    row.phys = t.physical().millis();
    row.logical = t.logical().get();
    row.node = t.node_id().get();
}

fn state_columns<V: FixedValue>(s: &State<V>, row: &mut RecordRow) {
    match s {
        State::Present(v) => {
            row.tombstone = false;
            v.column(&mut row.value);
        }
        State::Tombstone => row.tombstone = true,
    }
}

/// `Replica.map`'s records (src/replica.rs:69): `lift(k, Entry<Timestamp, V>)`, the DATED kind.
impl<V: FixedValue> GpuRecord for Entry<Timestamp, V> {
    const VALUE_KIND: i32 = V::KIND;
    const VALUE_LEN: u32 = V::LEN;
    const RECORD_KIND: i32 = ffi::RH_REC_DATED;
    fn write(&self, row: &mut RecordRow) {
        stamp_columns(&self.stamp, row);
        state_columns(&self.state, row);
    }
}

/// `Replica.projection`'s records (src/replica.rs:74): `lift(k, State<V>)`, the PROJECTION kind.
impl<V: FixedValue> GpuRecord for State<V> {
    const VALUE_KIND: i32 = V::KIND;
    const VALUE_LEN: u32 = V::LEN;
    const RECORD_KIND: i32 = ffi::RH_REC_PROJECTION;
    fn write(&self, row: &mut RecordRow) {
        state_columns(self, row);
    }
}

// A plain `FingerprintTreeMap<K, V>` (benches/bench.rs:47-92 fills `u32 -> u32`): `lift(k, v)`.
macro_rules! plain_record {
    ($($t:ty)*) => {$(
        impl GpuRecord for $t {
            const VALUE_KIND: i32 = <$t as FixedValue>::KIND;
            const VALUE_LEN: u32 = <$t as FixedValue>::LEN;
            const RECORD_KIND: i32 = ffi::RH_REC_PLAIN;
            fn write(&self, row: &mut RecordRow) {
                self.column(&mut row.value);
            }
        }
    )*};
}
plain_record!(u32 u64);

impl<const N: usize> GpuRecord for FixedBytes<N> {
    const VALUE_KIND: i32 = ffi::RH_VAL_BYTES;
    const VALUE_LEN: u32 = N as u32;
    const RECORD_KIND: i32 = ffi::RH_REC_PLAIN;
    fn write(&self, row: &mut RecordRow) {
        self.column(&mut row.value);
    }
}
