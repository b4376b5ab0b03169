//! `HipShardedMap<K, V>`: one map over several GPUs -- the north_star's key-range shards inside
//! one replica (`Inner<K, V>` is one process's map, src/replica.rs:68-74) -- behind the same
//! `Rsos<K>` and inherent `FingerprintTreeMap` surface as `HipFingerprintMap`, on the library's
//! sharded store (`rh_sstore_*`, include/rsos_hip.h).
//!
//! The library keeps one column store per device, shard s holding the keys in
//! `[split[s - 1], split[s])` (before the first bulk load the key space is cut evenly, so single
//! inserts spread over the shards; `load_bulk` cuts at equal counts), drives the shards from one
//! host thread each, and decomposes every question with no device-to-device traffic: sizes and
//! ranks add up, an aggregate is the Add of the shards' parts (rsos/src/aggregate.rs:79-89), a
//! protocol round's segments inside one shard are that shard's own round and the few that
//! straddle a boundary are resolved from their two boundary shards.  The host keeps `K` and `V`
//! in its own rank-ordered index, as `HipFingerprintMap` does; every fingerprint is the GPU lift.

use std::ops::{Bound, RangeBounds};
use std::os::raw::{c_int, c_void};

use rsos::{Aggregate, Fingerprint, Rsos};

use crate::round::{run_round, RoundPolicy};
use crate::{check, ffi, schema, sorted, Batch, GpuKey, GpuRecord, RoundCounts};

/// The library's sharded store, owned (its one `Drop`; see `StoreHandle`).
pub(crate) struct ShardedHandle(pub(crate) *mut ffi::rh_sstore);

impl Drop for ShardedHandle {
    fn drop(&mut self) {
        // SAFETY: the pointer came from rh_sstore_create and is destroyed once, here.
        unsafe { ffi::rh_sstore_destroy(self.0) };
    }
}

// SAFETY: the C sharded store serialises every call with its internal mutex.
unsafe impl Send for ShardedHandle {}
unsafe impl Sync for ShardedHandle {}

/// `Rsos<K>` over key-range shards on several MI355X.  No bounds on the type: the methods carry them.
pub struct HipShardedMap<K, V> {
    store: ShardedHandle,
    entries: sorted::SortedBlocks<K, V>,
    round_mu: std::sync::Mutex<()>,
}

/// The devices a map created by `new()` / `default()` spans: `RSOS_HIP_DEVICES` (comma-separated
/// ids, a device may repeat), else every visible device (`RSOS_HIP_DEVICE_COUNT`, else 1).
pub fn default_devices() -> Vec<i32> {
    if let Ok(v) = std::env::var("RSOS_HIP_DEVICES") {
        let ids: Vec<i32> = v.split(',').filter_map(|x| x.trim().parse().ok()).collect();
        if !ids.is_empty() {
            return ids;
        }
    }
    let n: i32 = std::env::var("RSOS_HIP_DEVICE_COUNT").ok().and_then(|v| v.parse().ok()).unwrap_or(1);
    (0..n.max(1)).collect()
}

impl<K: GpuKey, V: GpuRecord> HipShardedMap<K, V> {
    /// An empty map over the default devices (`FingerprintTreeMap::new()` takes no arguments).
    pub fn new() -> Self {
        Self::on_devices(&default_devices())
    }

    /// An empty map with shard s on HIP device `devices[s]`; the host tier of every shard on.
    pub fn on_devices(devices: &[i32]) -> Self {
        assert!(!devices.is_empty(), "rsos-hip: a sharded map needs at least one device");
        let mut p = std::ptr::null_mut();
        let s = schema::<K, V>();
        // SAFETY: valid device array, schema and out-pointer.
        check(unsafe { ffi::rh_sstore_create(devices.as_ptr(), devices.len() as c_int, &s, &mut p) },
              "rh_sstore_create");
        let store = ShardedHandle(p);
        // SAFETY: store was just created.
        check(unsafe { ffi::rh_sstore_set_host_tier(store.0, 1, 0) }, "rh_sstore_set_host_tier");
        HipShardedMap { store, entries: sorted::SortedBlocks::new(), round_mu: std::sync::Mutex::new(()) }
    }

    pub fn shard_count(&self) -> usize {
        // SAFETY: the handle is live for &self.
        unsafe { ffi::rh_sstore_shard_count(self.store.0) as usize }
    }

    /// Rows per shard (each shard's `len`).
    pub fn shard_sizes(&self) -> Vec<usize> {
        (0..self.shard_count())
            .map(|i| {
                let (mut st, mut n) = (std::ptr::null_mut(), 0u64);
                // SAFETY: i < shard_count; the shard is borrowed from the live sharded store.
                check(unsafe { ffi::rh_sstore_shard(self.store.0, i as c_int, &mut st) }, "rh_sstore_shard");
                check(unsafe { ffi::rh_store_len(st, &mut n) }, "rh_store_len");
                n as usize
            })
            .collect()
    }

    /// Whether writes wait for the shards' host-tier copies (`rh_sstore_set_tier_policy`).
    pub fn set_tier_policy(&self, keep_fresh: bool) {
        // SAFETY: the handle is live for &self.
        check(unsafe { ffi::rh_sstore_set_tier_policy(self.store.0, keep_fresh as c_int) },
              "rh_sstore_set_tier_policy");
    }

    /// Capacity for `rows` resident rows in all and batches of up to `batch_rows` (`rh_sstore_reserve`).
    pub fn reserve(&self, rows: usize, batch_rows: usize) {
        // SAFETY: the handle is live for &self.
        check(unsafe { ffi::rh_sstore_reserve(self.store.0, rows as u64, batch_rows as u64) }, "rh_sstore_reserve");
    }

    /// Bulk fill (FromIterator / ReplicatedMap::load_bulk): sort, keep the last value per key, cut
    /// at equal counts over the shards, one device lift per shard.
    pub fn load_bulk(&mut self, mut items: Vec<(K, V)>) {
        items.reverse();
        items.sort_by(|a, b| a.0.cmp(&b.0)); // stable: the last occurrence now comes first
        items.dedup_by(|a, b| a.0 == b.0);
        let batch = Batch::new(items.iter().map(|(k, v)| (k, Some(v))));
        let cols = batch.columns();
        // SAFETY: the column buffers outlive the synchronous call.
        check(unsafe { ffi::rh_sstore_load(self.store.0, &cols, items.len()) }, "rh_sstore_load");
        self.entries = sorted::SortedBlocks::from_sorted(items);
    }

    fn stage(&mut self, key: &K, value: Option<&V>) {
        let batch = Batch::new(std::iter::once((key, value)));
        let cols = batch.columns();
        let op = [if value.is_some() { 0u8 } else { 1u8 }];
        // SAFETY: the library copies the row (into its shard's pending batch) before returning.
        check(unsafe { ffi::rh_sstore_stage(self.store.0, &cols, op.as_ptr(), 1) }, "rh_sstore_stage");
    }

    fn bound_rank(&self, b: Bound<&K>, lower: bool) -> usize {
        match b {
            Bound::Unbounded => if lower { 0 } else { self.entries.len() },
            Bound::Included(k) => if lower { self.entries.rank(k) } else { self.entries.rank_incl(k) },
            Bound::Excluded(k) => if lower { self.entries.rank_incl(k) } else { self.entries.rank(k) },
        }
    }

    /// `r` range aggregates by rank, each cut over the shards holding it.
    pub fn aggregates_by_rank(&self, ranges: &[(usize, usize)]) -> Vec<Aggregate> {
        let lo: Vec<u64> = ranges.iter().map(|r| r.0 as u64).collect();
        let hi: Vec<u64> = ranges.iter().map(|r| r.1 as u64).collect();
        let mut out = vec![ffi::rh_aggregate::default(); ranges.len()];
        // SAFETY: buffers sized r.
        check(unsafe { ffi::rh_sstore_aggregates(self.store.0, lo.as_ptr(), hi.as_ptr(), ranges.len(), out.as_mut_ptr()) },
              "rh_sstore_aggregates");
        out.into_iter().map(|a| Aggregate::new(a.size as usize, Fingerprint(a.fingerprint))).collect()
    }

    /// One `rbsr` protocol round answered by the library (`rh_sstore_protocol_round`): the runs of
    /// segments inside one shard by that shard (its host tier, or one device round trip), the
    /// shards concurrently.
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
        run_round(
            |p, b, a, c, e, o| unsafe { ffi::rh_sstore_protocol_round(store, p, b, a, c, e, o) },
            policy,
            active,
            child_ranges,
            enumeration_ranges,
        )
    }

    /// The device holds exactly the host index.
    pub fn check_invariants(&self) {
        let mut n = 0u64;
        // SAFETY: out-pointer.
        check(unsafe { ffi::rh_sstore_len(self.store.0, &mut n) }, "rh_sstore_len");
        assert_eq!(n as usize, self.entries.len(), "rsos-hip: device and host sizes differ");
    }
}

impl<K: GpuKey, V: GpuRecord> Rsos<K> for HipShardedMap<K, V> {
    type Value = V;

    fn size(&self) -> usize {
        self.entries.len()
    }

    /// One ABI call: the shards wholly inside the range give their cached roots, at most two
    /// boundary shards answer from their host tiers (an inverted range gives ZERO).
    fn aggregate<R: RangeBounds<K>>(&self, range: R) -> Aggregate {
        let bound = |b: Bound<&K>| match b {
            Bound::Unbounded => (0, Vec::new()),
            Bound::Included(k) => (1, k.column_bytes()),
            Bound::Excluded(k) => (2, k.column_bytes()),
        };
        let (lk, lb) = bound(range.start_bound());
        let (hk, hb) = bound(range.end_bound());
        let ptr = |b: &Vec<u8>| if b.is_empty() { std::ptr::null() } else { b.as_ptr() as *const c_void };
        let mut out = ffi::rh_aggregate::default();
        // SAFETY: bound keys are key_len bytes (or NULL when unbounded); out is one aggregate.
        check(unsafe { ffi::rh_sstore_aggregate_keys(self.store.0, lk, ptr(&lb), hk, ptr(&hb), &mut out) },
              "rh_sstore_aggregate_keys");
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
        self.stage(&key, Some(&value));
        self.entries.insert(key, value)
    }

    fn delete(&mut self, key: &K) -> Option<V> {
        let old = self.entries.remove(key)?;
        self.stage(key, None);
        Some(old)
    }
}

// ---- the inherent FingerprintTreeMap surface the facade calls (public-api/rsos.txt:129-194) ----

impl<K: GpuKey, V: GpuRecord> Default for HipShardedMap<K, V> {
    fn default() -> Self {
        HipShardedMap::new()
    }
}

impl<K: GpuKey, V: GpuRecord> HipShardedMap<K, V> {
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

    pub fn retain<F: FnMut(&K, &V) -> bool>(&mut self, mut f: F) {
        let gone: Vec<K> = self.entries.iter().filter(|(k, v)| !f(k, v)).map(|(k, _)| k.clone()).collect();
        for k in gone {
            <Self as Rsos<K>>::delete(self, &k);
        }
    }

    /// In-place edit (FingerprintTreeMap::with_mut, rsos/src/fingerprint_tree_map/access.rs:46-76):
    /// the edited value is staged again on its key's shard.
    pub fn with_mut<R, F: FnOnce(Option<&mut V>) -> R>(&mut self, key: &K, f: F) -> R {
        let r = f(self.entries.get_mut(key));
        if let Some(v) = self.entries.get(key) {
            let batch = Batch::new(std::iter::once((key, Some(v))));
            let cols = batch.columns();
            let op = [0u8];
            // SAFETY: the library copies the row before returning.
            check(unsafe { ffi::rh_sstore_stage(self.store.0, &cols, op.as_ptr(), 1) }, "rh_sstore_stage");
        }
        r
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
}

impl<K: GpuKey, V: GpuRecord> FromIterator<(K, V)> for HipShardedMap<K, V> {
    fn from_iter<T: IntoIterator<Item = (K, V)>>(iter: T) -> Self {
        let mut m = HipShardedMap::new();
        m.load_bulk(iter.into_iter().collect());
        m
    }
}
