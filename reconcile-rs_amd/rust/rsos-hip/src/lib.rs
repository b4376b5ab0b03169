//! `rsos-hip`: an `rsos::Rsos<K>` realisation whose fingerprints and range aggregates are
//! computed on an AMD Instinct MI355X by librsos_hip.so (include/rsos_hip.h).
//!
//! `HipFingerprintMap<K, V>` is a drop-in for `FingerprintTreeMap<K, V>` behind the `Rsos<K>`
//! trait (rsos/src/rsos_trait.rs:39-90); `rbsr` consumes it through its blanket
//! `impl<K, T: Rsos<K>> RsosView<K> for T` (rbsr/src/rsos_view.rs:75-91), so
//! `public-api/rbsr.txt` is unchanged.
//!
//! Ownership follows the reference: the map owns `K` and `V` in host memory (select /
//! enumerate return borrows into it); the device holds the keys, the per-element
//! fingerprints and the block / super-block sums.  Laws:
//! * **summary-folds-lift** -- every fingerprint is computed by the GPU lift, which is
//!   bit-exact with `rsos::lift` (pinned by the reference's golden vectors in the
//!   MI355X repository's tests);
//! * **one-snapshot-per-round** -- every FFI call is synchronous (the device stream is
//!   drained before it returns), so a reader holding the map's read lock never sees a
//!   half-applied batch.
//! Errors: a non-zero status from the library is a bug or a device failure; the reference
//! fails loudly on those (`lift` panics on an encoder failure, fingerprint.rs:240-246), so
//! this crate panics with the library's message.

mod ffi;

use std::cmp::Ordering;
use std::ffi::CStr;
use std::ops::{Bound, RangeBounds};
use std::os::raw::c_void;

use rsos::{Aggregate, Fingerprint, Rsos};
use serde::Serialize;

fn check(rc: i32, what: &str) {
    if rc != ffi::RH_OK {
        // SAFETY: rh_last_error returns a NUL-terminated thread-local string.
        let msg = unsafe { CStr::from_ptr(ffi::rh_last_error()) }.to_string_lossy();
        panic!("rsos-hip: {what} failed ({rc}): {msg}");
    }
}

/// A key type with a fixed-width canonical form the device can order and hash.
pub trait GpuKey: Ord + Clone + Serialize {
    const KIND: i32;
    const LEN: u32;
    /// The key column bytes: LE integer for u32 / u64, the raw bytes for `[u8; N]`.
    fn column_bytes(&self) -> Vec<u8>;
}

impl GpuKey for u32 {
    const KIND: i32 = ffi::RH_KEY_U32;
    const LEN: u32 = 4;
    fn column_bytes(&self) -> Vec<u8> { self.to_le_bytes().to_vec() }
}
impl GpuKey for u64 {
    const KIND: i32 = ffi::RH_KEY_U64;
    const LEN: u32 = 8;
    fn column_bytes(&self) -> Vec<u8> { self.to_le_bytes().to_vec() }
}
impl GpuKey for [u8; 16] {
    const KIND: i32 = ffi::RH_KEY_BYTES;
    const LEN: u32 = 16;
    fn column_bytes(&self) -> Vec<u8> { self.to_vec() }
}
impl GpuKey for [u8; 32] {
    const KIND: i32 = ffi::RH_KEY_BYTES;
    const LEN: u32 = 32;
    fn column_bytes(&self) -> Vec<u8> { self.to_vec() }
}

/// One record's device columns (what the kernels read to synthesise the canonical encoding).
#[derive(Clone, Debug, Default)]
pub struct RecordRow {
    pub value: Vec<u8>,
    pub phys: u64,
    pub logical: u32,
    pub node: u64,
    pub tombstone: bool,
}

/// A value type whose canonical encoding the device synthesises from fixed-width columns.
/// Implement it for `lww_register::Entry<Timestamp, V>` (RECORD_KIND = DATED),
/// `State<V>` (PROJECTION) or a plain `V` (PLAIN).  `write` must produce exactly the
/// fields `rsos::encoding` would serialise; the library's tests pin that equivalence.
pub trait GpuRecord: Serialize {
    const VALUE_KIND: i32;
    const VALUE_LEN: u32;
    const RECORD_KIND: i32;
    fn write(&self, row: &mut RecordRow);
}

/// `Rsos<K>` on an MI355X.
pub struct HipFingerprintMap<K: GpuKey, V: GpuRecord> {
    store: *mut ffi::rh_store,
    /// rank-ordered host mirror (owns K and V; select / enumerate borrow from it)
    entries: Vec<(K, V)>,
}

// SAFETY: the C store serialises all calls with an internal mutex; the host mirror follows
// Rust's aliasing rules through &self / &mut self.
unsafe impl<K: GpuKey + Send, V: GpuRecord + Send> Send for HipFingerprintMap<K, V> {}
unsafe impl<K: GpuKey + Sync, V: GpuRecord + Sync> Sync for HipFingerprintMap<K, V> {}

fn schema<K: GpuKey, V: GpuRecord>() -> ffi::rh_schema {
    ffi::rh_schema {
        key_kind: K::KIND,
        key_len: K::LEN,
        value_kind: V::VALUE_KIND,
        value_len: V::VALUE_LEN,
        record_kind: V::RECORD_KIND,
        reserved: 0,
    }
}

/// Column buffers of a batch of records, kept alive for the duration of one FFI call.
struct Batch {
    keys: Vec<u8>,
    values: Vec<u8>,
    phys: Vec<u64>,
    logical: Vec<u32>,
    node: Vec<u64>,
    tags: Vec<u8>,
}

impl Batch {
    fn new<'a, K: GpuKey + 'a, V: GpuRecord + 'a>(items: impl Iterator<Item = (&'a K, Option<&'a V>)>) -> Batch {
        let mut b = Batch { keys: vec![], values: vec![], phys: vec![], logical: vec![], node: vec![], tags: vec![] };
        for (k, v) in items {
            b.keys.extend(k.column_bytes());
            let mut row = RecordRow::default();
            if let Some(v) = v {
                v.write(&mut row);
            }
            row.value.resize(V::VALUE_LEN as usize, 0);
            b.values.extend(&row.value);
            b.phys.push(row.phys);
            b.logical.push(row.logical);
            b.node.push(row.node);
            b.tags.push(row.tombstone as u8);
        }
        b
    }
    fn columns(&self) -> ffi::rh_columns {
        ffi::rh_columns {
            keys: self.keys.as_ptr() as *const c_void,
            phys: self.phys.as_ptr(),
            logical: self.logical.as_ptr(),
            node: self.node.as_ptr(),
            tags: self.tags.as_ptr(),
            values: self.values.as_ptr() as *const c_void,
        }
    }
}

impl<K: GpuKey, V: GpuRecord> HipFingerprintMap<K, V> {
    /// An empty map on HIP device `device`.
    pub fn new(device: i32) -> Self {
        let s = schema::<K, V>();
        let mut store = std::ptr::null_mut();
        // SAFETY: valid schema pointer and out-pointer.
        check(unsafe { ffi::rh_store_create(device, &s, &mut store) }, "rh_store_create");
        HipFingerprintMap { store, entries: Vec::new() }
    }

    /// Bulk fill (FromIterator / ReplicatedMap::load_bulk): sort, de-duplicate keeping the
    /// last value per key, one device lift of the whole batch.
    pub fn load_bulk(&mut self, mut items: Vec<(K, V)>) {
        items.reverse();
        items.sort_by(|a, b| a.0.cmp(&b.0)); // stable: the last occurrence now comes first
        items.dedup_by(|a, b| a.0 == b.0);
        let batch = Batch::new(items.iter().map(|(k, v)| (k, Some(v))));
        let cols = batch.columns();
        // SAFETY: the column buffers outlive the synchronous call.
        check(unsafe { ffi::rh_store_load(self.store, &cols, items.len()) }, "rh_store_load");
        self.entries = items;
    }

    fn bound_rank(&self, b: Bound<&K>, lower: bool) -> usize {
        match b {
            Bound::Unbounded => if lower { 0 } else { self.entries.len() },
            Bound::Included(k) => {
                if lower { self.entries.partition_point(|(e, _)| e < k) }
                else { self.entries.partition_point(|(e, _)| e <= k) }
            }
            Bound::Excluded(k) => {
                if lower { self.entries.partition_point(|(e, _)| e <= k) }
                else { self.entries.partition_point(|(e, _)| e < k) }
            }
        }
    }

    /// `r` range aggregates by rank in one device launch (one rbsr SPLIT's children).
    pub fn aggregates_by_rank(&self, ranges: &[(usize, usize)]) -> Vec<Aggregate> {
        let lo: Vec<u64> = ranges.iter().map(|r| r.0 as u64).collect();
        let hi: Vec<u64> = ranges.iter().map(|r| r.1 as u64).collect();
        let mut out = vec![ffi::rh_aggregate::default(); ranges.len()];
        // SAFETY: buffers sized r.
        check(unsafe { ffi::rh_store_aggregates(self.store, lo.as_ptr(), hi.as_ptr(), ranges.len(), out.as_mut_ptr()) },
              "rh_store_aggregates");
        out.into_iter().map(|a| Aggregate::new(a.size as usize, Fingerprint(a.fingerprint))).collect()
    }

    fn apply(&mut self, key: &K, value: Option<&V>) -> (u64, u64, u64) {
        let batch = Batch::new(std::iter::once((key, value)));
        let cols = batch.columns();
        let op = [if value.is_some() { 0u8 } else { 1u8 }];
        let (mut a, mut b, mut d) = (0u64, 0u64, 0u64);
        // SAFETY: buffers outlive the synchronous call.
        check(unsafe { ffi::rh_store_apply(self.store, &cols, op.as_ptr(), 1, &mut a, &mut b, &mut d) },
              "rh_store_apply");
        (a, b, d)
    }
}

impl<K: GpuKey, V: GpuRecord> Drop for HipFingerprintMap<K, V> {
    fn drop(&mut self) {
        // SAFETY: store came from rh_store_create and is destroyed once.
        unsafe { ffi::rh_store_destroy(self.store) };
    }
}

impl<K: GpuKey, V: GpuRecord> Rsos<K> for HipFingerprintMap<K, V> {
    type Value = V;

    fn size(&self) -> usize {
        self.entries.len()
    }

    fn aggregate<R: RangeBounds<K>>(&self, range: R) -> Aggregate {
        let lo = self.bound_rank(range.start_bound(), true);
        let hi = self.bound_rank(range.end_bound(), false).max(lo); // inverted -> ZERO
        self.aggregates_by_rank(&[(lo, hi)])[0]
    }

    fn rank(&self, z: &K) -> usize {
        self.entries.partition_point(|(e, _)| e.cmp(z) == Ordering::Less)
    }

    fn select(&self, r: usize) -> &K {
        &self.entries[r].0 // panics if r >= size(), as the reference does
    }

    fn enumerate<'a, R: RangeBounds<K> + 'a>(&'a self, range: R) -> impl Iterator<Item = (&'a K, &'a V)> + 'a
    where
        K: Ord + 'a,
        V: 'a,
    {
        let lo = self.bound_rank(range.start_bound(), true);
        let hi = self.bound_rank(range.end_bound(), false).max(lo);
        self.entries[lo..hi].iter().map(|(k, v)| (k, v))
    }

    fn insert(&mut self, key: K, value: V) -> Option<V> {
        self.apply(&key, Some(&value));
        match self.entries.binary_search_by(|(e, _)| e.cmp(&key)) {
            Ok(i) => Some(std::mem::replace(&mut self.entries[i].1, value)),
            Err(i) => {
                self.entries.insert(i, (key, value));
                None
            }
        }
    }

    fn delete(&mut self, key: &K) -> Option<V> {
        match self.entries.binary_search_by(|(e, _)| e.cmp(key)) {
            Ok(i) => {
                self.apply(key, None);
                Some(self.entries.remove(i).1)
            }
            Err(_) => None,
        }
    }
}
