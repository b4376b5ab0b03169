//! `rsos-hip`: an `rsos::Rsos<K>` realisation whose fingerprints and range aggregates are
//! computed on an AMD Instinct MI355X by librsos_hip.so (include/rsos_hip.h).
//!
//! `HipFingerprintMap<K, V>` is a drop-in for `FingerprintTreeMap<K, V>` behind the `Rsos<K>`
//! trait (rsos/src/rsos_trait.rs:39-90); `rbsr` consumes it through its blanket
//! `impl<K, T: Rsos<K>> RsosView<K> for T` (rbsr/src/rsos_view.rs:75-91), so
//! `public-api/rbsr.txt` is unchanged.
//!
//! Ownership follows the reference: the map owns `K` and `V` in host memory (select /
//! enumerate return borrows into it) in a sorted-blocks index (`sorted.rs`: O(log n) rank /
//! select, O(log n + B) insert); the device holds the keys, the per-element fingerprints and the
//! block / super-block sums, and the library's host tier (rh_store_set_host_tier) answers
//! `aggregate` without a device round trip.  `insert` / `delete` stage one row in the library
//! (rh_store_stage); everything staged reaches the device as ONE batch before the next
//! `aggregate`, so a bulk seed through single inserts (just_insert_bulk,
//! src/replica/write.rs:107-121) costs host work per record and one device batch.  Laws:
//! * **summary-folds-lift** -- every fingerprint is computed by the GPU lift, which is
//!   bit-exact with `rsos::lift` (pinned by the reference's golden vectors in the
//!   MI355X repository's tests);
//! * **one-snapshot-per-round** -- every FFI call is synchronous (the device stream is
//!   drained before it returns), so a reader holding the map's read lock never sees a
//!   half-applied batch.
//! Errors: a non-zero status from the library is a bug or a device failure; the reference
//! fails loudly on those (`lift` panics on an encoder failure, fingerprint.rs:240-246), so
//! this crate panics with the library's message.

mod encoded;
mod ffi;
mod round;
mod sharded;
mod sorted;
mod values;

pub use encoded::HipEncodedMap;
pub use round::RoundPolicy;
pub use sharded::HipShardedMap;
pub use values::{FixedBytes, FixedValue};

use std::ffi::CStr;
use std::ops::{Bound, RangeBounds};
use std::os::raw::{c_int, c_void};

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
    /// The key of `LEN` column bytes (the inverse of `column_bytes`: keys the library returns).
    fn from_column_bytes(b: &[u8]) -> Self;
}

impl GpuKey for u32 {
    const KIND: i32 = ffi::RH_KEY_U32;
    const LEN: u32 = 4;
    fn column_bytes(&self) -> Vec<u8> { self.to_le_bytes().to_vec() }
    fn from_column_bytes(b: &[u8]) -> Self { u32::from_le_bytes(b.try_into().expect("4 key bytes")) }
}
impl GpuKey for u64 {
    const KIND: i32 = ffi::RH_KEY_U64;
    const LEN: u32 = 8;
    fn column_bytes(&self) -> Vec<u8> { self.to_le_bytes().to_vec() }
    fn from_column_bytes(b: &[u8]) -> Self { u64::from_le_bytes(b.try_into().expect("8 key bytes")) }
}
impl GpuKey for [u8; 16] {
    const KIND: i32 = ffi::RH_KEY_BYTES;
    const LEN: u32 = 16;
    fn column_bytes(&self) -> Vec<u8> { self.to_vec() }
    fn from_column_bytes(b: &[u8]) -> Self { b.try_into().expect("16 key bytes") }
}
impl GpuKey for [u8; 32] {
    const KIND: i32 = ffi::RH_KEY_BYTES;
    const LEN: u32 = 32;
    fn column_bytes(&self) -> Vec<u8> { self.to_vec() }
    fn from_column_bytes(b: &[u8]) -> Self { b.try_into().expect("32 key bytes") }
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
/// Implemented in this crate (values.rs) for `lww_register::Entry<Timestamp, V>` (RECORD_KIND =
/// DATED) and `State<V>` (PROJECTION) over any `V: FixedValue`, and for plain `u32` / `u64` /
/// `FixedBytes<N>` values (PLAIN).  `write` must produce exactly the fields `rsos::encoding` would
/// serialise; the library's tests pin that equivalence.
pub trait GpuRecord: Serialize {
    const VALUE_KIND: i32;
    const VALUE_LEN: u32;
    const RECORD_KIND: i32;
    fn write(&self, row: &mut RecordRow);
}

/// The library's store, owned: the one place its pointer lives and its one `Drop`, so the map
/// types carry no bounds on their definitions (a generic `Drop` impl must repeat them, E0367) --
/// `FingerprintTreeMap<K, V>` has none either (rsos/src/fingerprint_tree_map.rs:94), and
/// `Replica`'s fields name the map with unbounded `K`, `V` (src/replica.rs:68-74).
pub(crate) struct StoreHandle(pub(crate) *mut ffi::rh_store);

impl StoreHandle {
    fn create(device: i32, s: &ffi::rh_schema) -> StoreHandle {
        let mut store = std::ptr::null_mut();
        // SAFETY: valid schema pointer and out-pointer.
        check(unsafe { ffi::rh_store_create(device, s, &mut store) }, "rh_store_create");
        StoreHandle(store)
    }
}

impl Drop for StoreHandle {
    fn drop(&mut self) {
        // SAFETY: the pointer came from rh_store_create and is destroyed once, here.
        unsafe { ffi::rh_store_destroy(self.0) };
    }
}

// SAFETY: the C store serialises every call with its internal mutex; a handle has no other state.
unsafe impl Send for StoreHandle {}
unsafe impl Sync for StoreHandle {}

/// The HIP device a map created by `new()` / `default()` lives on: `RSOS_HIP_DEVICE`, else 0
/// (`FingerprintTreeMap::new()` takes no arguments, src/replica/construct.rs:205-206).
pub fn default_device() -> i32 {
    std::env::var("RSOS_HIP_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0)
}

/// `Rsos<K>` on an MI355X.  No bounds on the type: the methods carry them.
///
/// Row cap: one map holds fewer than [`ffi::RH_STORE_MAX_ROWS`] (2^31) rows, the limit of one
/// `rh_store` (`include/rsos_hip.h`, "Row cap").  A load, batch or insert that would pass it
/// panics with the library's message (`store size limit (2^31 rows) exceeded`) and leaves the
/// map unchanged.  `Rsos::size()` is a `usize` (`rsos/src/rsos_trait.rs:44`): a map of 2^31 rows
/// or more is a [`HipShardedMap`], every shard under the cap (one MI355X holds ~2.1 x 10^9 rows
/// of 16 B keys, so one device can hold several shards).
pub struct HipFingerprintMap<K, V> {
    store: StoreHandle,
    /// rank-ordered host index (owns K and V; select / enumerate borrow from it)
    entries: sorted::SortedBlocks<K, V>,
    /// held while a round's outputs (the library's buffers) are read
    round_mu: std::sync::Mutex<()>,
}

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
            match v {
                Some(v) => {
                    v.write(&mut row);
                    // a present value must fill the value column exactly: padding or truncating it
                    // would hash some other record and reconcile silently wrongly (rsos_trait.rs:54-56)
                    if !row.tombstone {
                        assert_eq!(row.value.len(), V::VALUE_LEN as usize,
                                   "rsos-hip: GpuRecord::write produced a {}-byte value for a {}-byte value column",
                                   row.value.len(), V::VALUE_LEN);
                    } else {
                        assert!(row.value.is_empty(), "rsos-hip: a tombstone row carries no value bytes");
                        row.value = vec![0; V::VALUE_LEN as usize]; // never hashed (State::Tombstone)
                    }
                }
                None => row.value = vec![0; V::VALUE_LEN as usize], // a delete: the value columns are ignored
            }
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
    /// An empty map on the default device (`FingerprintTreeMap::new()`).
    pub fn new() -> Self {
        Self::on_device(default_device())
    }

    /// An empty map on HIP device `device`.
    pub fn on_device(device: i32) -> Self {
        let store = StoreHandle::create(device, &schema::<K, V>());
        // SAFETY: store was just created.
        check(unsafe { ffi::rh_store_set_host_tier(store.0, 1, 0) }, "rh_store_set_host_tier");
        HipFingerprintMap { store, entries: sorted::SortedBlocks::new(), round_mu: std::sync::Mutex::new(()) }
    }

    /// Whether a write that outgrows the host tier's delta tree waits for the tier's copy
    /// (`true`, the default: every later read is answered from host memory) or returns at once
    /// (`false`: reads go to the device until the copy lands) -- `rh_store_set_tier_policy`.
    pub fn set_tier_policy(&self, keep_fresh: bool) {
        // SAFETY: the handle is live for &self.
        check(unsafe { ffi::rh_store_set_tier_policy(self.store.0, keep_fresh as c_int) },
              "rh_store_set_tier_policy");
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
        check(unsafe { ffi::rh_store_load(self.store.0, &cols, items.len()) }, "rh_store_load");
        self.entries = sorted::SortedBlocks::from_sorted(items);
    }

    fn bound_rank(&self, b: Bound<&K>, lower: bool) -> usize {
        match b {
            Bound::Unbounded => if lower { 0 } else { self.entries.len() },
            Bound::Included(k) => if lower { self.entries.rank(k) } else { self.entries.rank_incl(k) },
            Bound::Excluded(k) => if lower { self.entries.rank_incl(k) } else { self.entries.rank(k) },
        }
    }

    /// `r` range aggregates by rank in one device launch (one rbsr SPLIT's children).
    pub fn aggregates_by_rank(&self, ranges: &[(usize, usize)]) -> Vec<Aggregate> {
        let lo: Vec<u64> = ranges.iter().map(|r| r.0 as u64).collect();
        let hi: Vec<u64> = ranges.iter().map(|r| r.1 as u64).collect();
        let mut out = vec![ffi::rh_aggregate::default(); ranges.len()];
        // SAFETY: buffers sized r.
        check(unsafe { ffi::rh_store_aggregates(self.store.0, lo.as_ptr(), hi.as_ptr(), ranges.len(), out.as_mut_ptr()) },
              "rh_store_aggregates");
        out.into_iter().map(|a| Aggregate::new(a.size as usize, Fingerprint(a.fingerprint))).collect()
    }

    /// Stage one insert-or-overwrite (`value` Some) or delete in the library's pending batch; the
    /// library applies everything staged as one device batch before the next question.
    fn stage(&mut self, key: &K, value: Option<&V>) {
        let batch = Batch::new(std::iter::once((key, value)));
        let cols = batch.columns();
        let op = [if value.is_some() { 0u8 } else { 1u8 }];
        // SAFETY: the library copies the row before returning.
        check(unsafe { ffi::rh_store_stage(self.store.0, &cols, op.as_ptr(), 1) }, "rh_store_stage");
    }

    fn key_bound(b: Bound<&K>, lower: bool) -> (i32, Vec<u8>) {
        // rh_store_aggregate_keys bound kinds: 0 = unbounded, 1 = included, 2 = excluded
        let _ = lower;
        match b {
            Bound::Unbounded => (0, Vec::new()),
            Bound::Included(k) => (1, k.column_bytes()),
            Bound::Excluded(k) => (2, k.column_bytes()),
        }
    }
}

/// What one batched round did (the fields of `rbsr::RoundOutcome`, which has no public
/// constructor).
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct RoundCounts {
    pub skipped: usize,
    pub enumerated: usize,
    pub split: usize,
    pub children: usize,
    pub dropped_malformed: usize,
}

impl<K: GpuKey, V: GpuRecord> HipFingerprintMap<K, V> {
    /// One `rbsr` protocol round (`protocol_round_with_policy`, rbsr/src/protocol.rs:212-317) answered
    /// by the library in one call (`rh_store_protocol_round`): from the host tier for rounds of up
    /// to 128 segments, else in one device round trip.  Outputs are appended in the reference's
    /// order; any other `RefinementPolicy` goes through `rbsr::protocol_round_with_policy` on the
    /// `Rsos<K>` surface.
    pub fn protocol_round(
        &self,
        policy: RoundPolicy,
        active: Vec<rbsr::RangeAggregate<K>>,
        child_ranges: &mut Vec<rbsr::RangeAggregate<K>>,
        enumeration_ranges: &mut Vec<rbsr::EnumerationRange<K>>,
    ) -> RoundCounts {
        let _g = self.round_mu.lock().unwrap_or_else(|e| e.into_inner());
        let store = self.store.0;
        // SAFETY: the handle is live for &self; run_round passes valid segment buffers.
        round::run_round(
            |p, b, a, c, e, o| unsafe { ffi::rh_store_protocol_round(store, p, b, a, c, e, o) },
            policy,
            active,
            child_ranges,
            enumeration_ranges,
        )
    }

    /// `protocol_round` under `FixedFanOut(fan_out)` (16 = `protocol_round`'s default).
    pub fn protocol_round_fixed(
        &self,
        fan_out: usize,
        active: Vec<rbsr::RangeAggregate<K>>,
        child_ranges: &mut Vec<rbsr::RangeAggregate<K>>,
        enumeration_ranges: &mut Vec<rbsr::EnumerationRange<K>>,
    ) -> RoundCounts {
        self.protocol_round(RoundPolicy::FixedFanOut(fan_out), active, child_ranges, enumeration_ranges)
    }
}

impl<K: GpuKey, V: GpuRecord> Rsos<K> for HipFingerprintMap<K, V> {
    type Value = V;

    fn size(&self) -> usize {
        self.entries.len()
    }

    /// One ABI call: the library applies any staged rows, then its host tier answers from the
    /// fingerprint prefix sums (an inverted range gives ZERO, rbsr/src/protocol.rs:230-232).
    fn aggregate<R: RangeBounds<K>>(&self, range: R) -> Aggregate {
        let (lk, lb) = Self::key_bound(range.start_bound(), true);
        let (hk, hb) = Self::key_bound(range.end_bound(), false);
        let mut out = ffi::rh_aggregate::default();
        let ptr = |b: &Vec<u8>| if b.is_empty() { std::ptr::null() } else { b.as_ptr() as *const c_void };
        // SAFETY: bound keys are key_len bytes (or NULL when unbounded); out is one aggregate.
        check(unsafe { ffi::rh_store_aggregate_keys(self.store.0, lk, ptr(&lb), hk, ptr(&hb), &mut out) },
              "rh_store_aggregate_keys");
        Aggregate::new(out.size as usize, Fingerprint(out.fingerprint))
    }

    fn rank(&self, z: &K) -> usize {
        self.entries.rank(z)
    }

    fn select(&self, r: usize) -> &K {
        &self.entries.at(r).0 // panics if r >= size(), as the reference does
    }

    fn enumerate<'a, R: RangeBounds<K> + 'a>(&'a self, range: R) -> impl Iterator<Item = (&'a K, &'a V)> + 'a
    where
        K: Ord + 'a,
        V: 'a,
    {
        let lo = self.bound_rank(range.start_bound(), true);
        let hi = self.bound_rank(range.end_bound(), false).max(lo);
        self.entries.range(lo, hi).map(|(k, v)| (k, v))
    }

    fn insert(&mut self, key: K, value: V) -> Option<V> {
        self.stage(&key, Some(&value)); // panics on a value of the wrong length (Batch::new)
        self.entries.insert(key, value)
    }

    fn delete(&mut self, key: &K) -> Option<V> {
        let old = self.entries.remove(key)?;
        self.stage(key, None);
        Some(old)
    }
}

// ---- the inherent FingerprintTreeMap surface the facade calls (public-api/rsos.txt:129-194) ----
// The same surface HipEncodedMap has, on the fixed-width column store, so the drop-in at
// src/replica.rs:69,74 gets the schema kernels (the canonical encoding synthesised in registers,
// no host-side encode_to_vec per record): `FingerprintTreeMap<[u8; 16], Entry<Timestamp, V>>` ->
// `HipFingerprintMap<[u8; 16], Entry<Timestamp, V>>` when V has a GpuRecord form.  Every mutation
// is one staged row (rh_store_stage); every fingerprint is still the GPU lift.

impl<K: GpuKey, V: GpuRecord> Default for HipFingerprintMap<K, V> {
    fn default() -> Self {
        HipFingerprintMap::new()
    }
}

impl<K: GpuKey, V: GpuRecord> HipFingerprintMap<K, V> {
    pub fn len(&self) -> usize {
        self.entries.len()
    }

    pub fn is_empty(&self) -> bool {
        self.entries.len() == 0
    }

    pub fn clear(&mut self) {
        let keys: Vec<K> = self.entries.iter().map(|(k, _)| k.clone()).collect();
        for k in &keys {
            self.stage(k, None);
        }
        self.entries.clear();
    }

    pub fn get<Q: Ord + ?Sized>(&self, key: &Q) -> Option<&V>
    where
        K: std::borrow::Borrow<Q>,
    {
        self.entries.get(key)
    }

    pub fn contains_key<Q: Ord + ?Sized>(&self, key: &Q) -> bool
    where
        K: std::borrow::Borrow<Q>,
    {
        self.entries.get(key).is_some()
    }

    pub fn position<Q: Ord + ?Sized>(&self, key: &Q) -> Option<usize>
    where
        K: std::borrow::Borrow<Q>,
    {
        self.entries.position(key)
    }

    pub fn insert(&mut self, key: K, value: V) -> Option<V> {
        <Self as Rsos<K>>::insert(self, key, value)
    }

    pub fn remove<Q: Ord + ?Sized>(&mut self, key: &Q) -> Option<V>
    where
        K: std::borrow::Borrow<Q>,
    {
        let k = self.entries.at(self.entries.position(key)?).0.clone();
        <Self as Rsos<K>>::delete(self, &k)
    }

    /// Keep the entries `f` accepts (FingerprintTreeMap::retain): the others are deleted, each a
    /// staged row of one batch.
    pub fn retain<F: FnMut(&K, &V) -> bool>(&mut self, mut f: F) {
        let gone: Vec<K> = self.entries.iter().filter(|(k, v)| !f(k, v)).map(|(k, _)| k.clone()).collect();
        for k in gone {
            <Self as Rsos<K>>::delete(self, &k);
        }
    }

    /// In-place edit (FingerprintTreeMap::with_mut + Relift, rsos/src/fingerprint_tree_map/access.rs:46-76):
    /// `f` sees the value (or None); the edited value is staged again, so its fingerprint replaces
    /// the old one -- the `new - old` delta -- in the next batch.
    pub fn with_mut<R, F: FnOnce(Option<&mut V>) -> R>(&mut self, key: &K, f: F) -> R {
        let r = f(self.entries.get_mut(key));
        if let Some(v) = self.entries.get(key) {
            let batch = Batch::new(std::iter::once((key, Some(v))));
            let cols = batch.columns();
            let op = [0u8];
            // SAFETY: the library copies the row before returning.
            check(unsafe { ffi::rh_store_stage(self.store.0, &cols, op.as_ptr(), 1) }, "rh_store_stage");
        }
        r
    }

    pub fn entry(&mut self, key: K) -> HipEntry<'_, K, V> {
        HipEntry { map: self, key }
    }

    pub fn range<R: RangeBounds<K>>(&self, range: R) -> impl Iterator<Item = (&K, &V)> + '_ {
        let lo = self.bound_rank(range.start_bound(), true);
        let hi = self.bound_rank(range.end_bound(), false).max(lo);
        self.entries.range(lo, hi).map(|(k, v)| (k, v))
    }

    pub fn iter(&self) -> impl Iterator<Item = (&K, &V)> + '_ {
        self.entries.iter().map(|(k, v)| (k, v))
    }

    pub fn keys(&self) -> impl Iterator<Item = &K> + '_ {
        self.entries.iter().map(|(k, _)| k)
    }

    pub fn values(&self) -> impl Iterator<Item = &V> + '_ {
        self.entries.iter().map(|(_, v)| v)
    }

    pub fn first_key_value(&self) -> Option<(&K, &V)> {
        self.entries.first().map(|(k, v)| (k, v))
    }

    pub fn last_key_value(&self) -> Option<(&K, &V)> {
        self.entries.last().map(|(k, v)| (k, v))
    }

    pub fn aggregate<R: RangeBounds<K>>(&self, range: R) -> Aggregate {
        <Self as Rsos<K>>::aggregate(self, range)
    }

    pub fn rank<Q: Ord + ?Sized>(&self, key: &Q) -> usize
    where
        K: std::borrow::Borrow<Q>,
    {
        self.entries.rank(key)
    }

    pub fn select(&self, r: usize) -> &K {
        &self.entries.at(r).0
    }

    /// The device holds exactly the host index (sizes agree after the staged rows apply).
    pub fn check_invariants(&self) {
        let mut n = 0u64;
        // SAFETY: out-pointer.
        check(unsafe { ffi::rh_store_len(self.store.0, &mut n) }, "rh_store_len");
        assert_eq!(n as usize, self.entries.len(), "rsos-hip: device and host sizes differ");
    }
}

/// The reference's `rsos::Entry` (public-api/rsos.txt:118-121) for the column store.
pub struct HipEntry<'a, K, V> {
    map: &'a mut HipFingerprintMap<K, V>,
    key: K,
}

impl<'a, K: GpuKey, V: GpuRecord> HipEntry<'a, K, V> {
    pub fn and_modify(self, f: impl FnOnce(&mut V)) -> Self {
        let key = self.key.clone();
        self.map.with_mut(&key, |v| {
            if let Some(v) = v {
                f(v)
            }
        });
        self
    }

    pub fn or_insert_with(self, f: impl FnOnce() -> V) -> &'a V {
        let HipEntry { map, key } = self;
        if map.entries.get(&key).is_none() {
            <HipFingerprintMap<K, V> as Rsos<K>>::insert(map, key.clone(), f());
        }
        let map: &'a HipFingerprintMap<K, V> = map;
        map.entries.get(&key).expect("just inserted")
    }

    pub fn or_insert(self, value: V) -> &'a V {
        self.or_insert_with(|| value)
    }

    pub fn or_default(self) -> &'a V
    where
        V: Default,
    {
        self.or_insert_with(V::default)
    }
}

impl<K: GpuKey, V: GpuRecord> FromIterator<(K, V)> for HipFingerprintMap<K, V> {
    fn from_iter<T: IntoIterator<Item = (K, V)>>(iter: T) -> Self {
        let mut m = HipFingerprintMap::new();
        m.load_bulk(iter.into_iter().collect());
        m
    }
}
