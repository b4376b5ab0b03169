//! `HipEncodedMap<K, V>`: `rsos::Rsos<K>` for any serde `K` / `V` -- `ReplicatedMap<String,
//! String>` (examples/k8s/main.rs:53), `Vec<u8>`, structs -- over the library's encoded store
//! (`rh_estore_*`, include/rsos_hip.h).
//!
//! A record reaches the device as its canonical bytes, `rsos::encoding::encode_to_vec(&k)` followed
//! by `encode_to_vec(&v)` (public-api/rsos.txt:61); `lift(k, v)` is BLAKE3 of exactly that
//! concatenation (rsos/src/fingerprint.rs:270-275), computed by the GPU.  The keys and their order
//! (`K: Ord` -- for `String` not the order of the length-prefixed encodings) stay on the host: the
//! device is addressed by rank.  `insert` / `delete` update the host index at once (returning the
//! displaced value) and queue the device operation; the next `aggregate` applies every queued
//! operation as one rank-addressed batch (`rh_estore_apply`).  The Python twin is
//! `rsos_hip.emap.EncodedFingerprintMap`, whose tests pin this logic.

use std::collections::BTreeMap;
use std::ops::{Bound, RangeBounds};
use std::sync::Mutex;

use rsos::{Aggregate, Fingerprint, Rsos};
use serde::Serialize;

use crate::{check, ffi, sorted::SortedBlocks};

/// What the device holds (its keys in rank order) and the operations not yet applied to it.
struct DevState<K> {
    keys: SortedBlocks<K, ()>,
    pending: BTreeMap<K, Option<Vec<u8>>>, // Some(record bytes) = insert / overwrite, None = delete
}

/// The library's encoded store, owned (its one `Drop`: see `StoreHandle` in lib.rs).
struct EStoreHandle(*mut ffi::rh_estore);

impl Drop for EStoreHandle {
    fn drop(&mut self) {
        // SAFETY: the pointer came from rh_estore_create and is destroyed once, here.
        unsafe { ffi::rh_estore_destroy(self.0) };
    }
}

// SAFETY: the C store serialises every call with its own mutex; a handle has no other state.
unsafe impl Send for EStoreHandle {}
unsafe impl Sync for EStoreHandle {}

/// `Rsos<K>` for any serde `K` / `V` on an MI355X.  No bounds on the type (as
/// `FingerprintTreeMap<K, V>`, rsos/src/fingerprint_tree_map.rs:94): `Replica`'s field
/// `Arc<RwLock<HipEncodedMap<K, Entry<Timestamp, V>>>>` (src/replica.rs:69) is well-formed for
/// its unbounded `K`, `V`; the methods need `K: Ord + Clone + Serialize, V: Serialize`, which
/// `lww_register::Key` / `Value` imply (lww-register/src/bounds.rs:21,31).
pub struct HipEncodedMap<K, V> {
    store: EStoreHandle,
    entries: SortedBlocks<K, V>,
    dev: Mutex<DevState<K>>,
}

fn record<K: Serialize, V: Serialize>(k: &K, v: &V) -> Vec<u8> {
    // encode_to_vec fails only for a hand-written Serialize that errors; lift panics then too
    // (rsos/src/fingerprint.rs:240-246)
    let mut r = rsos::encoding::encode_to_vec(k).expect("rsos-hip: key does not encode");
    r.extend(rsos::encoding::encode_to_vec(v).expect("rsos-hip: value does not encode"));
    r
}

fn pack(records: &[Vec<u8>]) -> (Vec<u8>, Vec<u64>) {
    let mut offs = Vec::with_capacity(records.len() + 1);
    offs.push(0u64);
    let mut bytes = Vec::new();
    for r in records {
        bytes.extend_from_slice(r);
        offs.push(bytes.len() as u64);
    }
    if bytes.is_empty() {
        bytes.push(0);
    }
    (bytes, offs)
}

impl<K: Ord + Clone + Serialize, V: Serialize> HipEncodedMap<K, V> {
    /// An empty map on the default device (`FingerprintTreeMap::new()`, src/replica/construct.rs:205-206).
    pub fn new() -> Self {
        Self::on_device(crate::default_device())
    }

    /// An empty map on HIP device `device`.
    pub fn on_device(device: i32) -> Self {
        let mut store = std::ptr::null_mut();
        // SAFETY: valid out-pointer.
        check(unsafe { ffi::rh_estore_create(device, &mut store) }, "rh_estore_create");
        let store = EStoreHandle(store);
        // SAFETY: store was just created.
        check(unsafe { ffi::rh_estore_set_host_tier(store.0, 1) }, "rh_estore_set_host_tier");
        HipEncodedMap {
            store,
            entries: SortedBlocks::new(),
            dev: Mutex::new(DevState { keys: SortedBlocks::new(), pending: BTreeMap::new() }),
        }
    }

    /// Bulk fill: the last value of a repeated key wins; one device lift of the whole set.
    pub fn load_bulk(&mut self, mut items: Vec<(K, V)>) {
        items.reverse();
        items.sort_by(|a, b| a.0.cmp(&b.0)); // stable: the last occurrence now comes first
        items.dedup_by(|a, b| a.0 == b.0);
        let recs: Vec<Vec<u8>> = items.iter().map(|(k, v)| record(k, v)).collect();
        let (bytes, offs) = pack(&recs);
        // SAFETY: buffers outlive the synchronous call.
        check(unsafe { ffi::rh_estore_load(self.store.0, bytes.as_ptr(), offs.as_ptr(), items.len()) },
              "rh_estore_load");
        let keys = items.iter().map(|(k, _)| (k.clone(), ())).collect();
        *self.dev.get_mut().expect("rsos-hip: poisoned") =
            DevState { keys: SortedBlocks::from_sorted(keys), pending: BTreeMap::new() };
        self.entries = SortedBlocks::from_sorted(items);
    }

    /// Apply every queued operation as one rank-addressed device batch.
    fn flush(&self) {
        let mut st = self.dev.lock().expect("rsos-hip: poisoned");
        if st.pending.is_empty() {
            return;
        }
        let pending = std::mem::take(&mut st.pending);
        let (mut pos, mut kinds, mut recs) = (Vec::new(), Vec::new(), Vec::new());
        let (mut adds, mut dels) = (Vec::new(), Vec::new());
        for (k, op) in pending {
            let p = st.keys.rank(&k);
            let present = p < st.keys.len() && st.keys.at(p).0 == k;
            match op {
                None if present => {
                    pos.push(p as u64);
                    kinds.push(2u8);
                    dels.push(k);
                }
                None => {}
                Some(r) => {
                    pos.push(p as u64);
                    kinds.push(if present { 1u8 } else { 0u8 });
                    recs.push(r);
                    if !present {
                        adds.push(k);
                    }
                }
            }
        }
        if pos.is_empty() {
            return;
        }
        let (bytes, offs) = pack(&recs);
        // SAFETY: buffers outlive the synchronous call; positions are sorted (BTreeMap order).
        check(unsafe {
            ffi::rh_estore_apply(self.store.0, pos.as_ptr(), kinds.as_ptr(), pos.len(), bytes.as_ptr(), offs.as_ptr(),
                                 recs.len())
        }, "rh_estore_apply");
        for k in dels {
            st.keys.remove(&k);
        }
        for k in adds {
            st.keys.insert(k, ());
        }
    }

    fn bound_rank(&self, b: Bound<&K>, lower: bool) -> usize {
        match b {
            Bound::Unbounded => if lower { 0 } else { self.entries.len() },
            Bound::Included(k) => if lower { self.entries.rank(k) } else { self.entries.rank_incl(k) },
            Bound::Excluded(k) => if lower { self.entries.rank_incl(k) } else { self.entries.rank(k) },
        }
    }
}


impl<K: Ord + Clone + Serialize, V: Serialize> Rsos<K> for HipEncodedMap<K, V> {
    type Value = V;

    fn size(&self) -> usize {
        self.entries.len()
    }

    fn aggregate<R: RangeBounds<K>>(&self, range: R) -> Aggregate {
        self.flush(); // the device then holds exactly `entries`, in the same rank order
        let lo = self.bound_rank(range.start_bound(), true) as u64;
        let hi = (self.bound_rank(range.end_bound(), false) as u64).max(lo); // inverted -> ZERO
        let mut out = ffi::rh_aggregate::default();
        // SAFETY: one range in, one aggregate out.
        check(unsafe { ffi::rh_estore_aggregates(self.store.0, &lo, &hi, 1, &mut out) }, "rh_estore_aggregates");
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
        let rec = record(&key, &value);
        self.dev.get_mut().expect("rsos-hip: poisoned").pending.insert(key.clone(), Some(rec));
        self.entries.insert(key, value)
    }

    fn delete(&mut self, key: &K) -> Option<V> {
        let old = self.entries.remove(key)?;
        self.dev.get_mut().expect("rsos-hip: poisoned").pending.insert(key.clone(), None);
        Some(old)
    }
}

// ---- the inherent FingerprintTreeMap surface the facade calls (public-api/rsos.txt:129-194) ----
// With these, `Replica`'s maps (src/replica.rs:69,74) and `ReadReplicaMap`'s
// (src/read_replica_map.rs:61) change type in one line: FingerprintTreeMap<K, V> ->
// HipEncodedMap<K, V>.  Every mutation goes through the staged device batch; every fingerprint
// is still the GPU lift of the record's canonical bytes.

impl<K: Ord + Clone + Serialize, V: Serialize> Default for HipEncodedMap<K, V> {
    fn default() -> Self {
        HipEncodedMap::new()
    }
}

impl<K: Ord + Clone + Serialize, V: Serialize> HipEncodedMap<K, V> {
    fn stage(&mut self, key: &K) {
        // re-encode the key's current value (or a delete) into the pending batch
        let rec = self.entries.get(key).map(|v| record(key, v));
        self.dev.get_mut().expect("rsos-hip: poisoned").pending.insert(key.clone(), rec);
    }

    pub fn len(&self) -> usize {
        self.entries.len()
    }

    pub fn is_empty(&self) -> bool {
        self.entries.len() == 0
    }

    pub fn clear(&mut self) {
        let keys: Vec<K> = self.entries.iter().map(|(k, _)| k.clone()).collect();
        self.entries.clear();
        let st = self.dev.get_mut().expect("rsos-hip: poisoned");
        for k in keys {
            st.pending.insert(k, None);
        }
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

    /// Keep the entries `f` accepts (FingerprintTreeMap::retain): the others are deleted, one
    /// staged batch.
    pub fn retain<F: FnMut(&K, &V) -> bool>(&mut self, mut f: F) {
        let gone: Vec<K> = self.entries.iter().filter(|(k, v)| !f(k, v)).map(|(k, _)| k.clone()).collect();
        for k in gone {
            <Self as Rsos<K>>::delete(self, &k);
        }
    }

    /// In-place edit (FingerprintTreeMap::with_mut + Relift, rsos/src/fingerprint_tree_map/access.rs:46-76):
    /// `f` sees the value (or None), and the edited value's fingerprint replaces the old one --
    /// the `new - old` delta -- through the staged batch.
    pub fn with_mut<R, F: FnOnce(Option<&mut V>) -> R>(&mut self, key: &K, f: F) -> R {
        let r = f(self.entries.get_mut(key));
        if self.entries.get(key).is_some() {
            self.stage(key);
        }
        r
    }

    pub fn entry(&mut self, key: K) -> Entry<'_, K, V> {
        Entry { map: self, key }
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

    /// The device holds exactly the host index: same size, and the root equals the root of
    /// the fingerprints it lifted (checked through the library).  Panics otherwise.
    pub fn check_invariants(&self) {
        self.flush();
        let mut n = 0u64;
        // SAFETY: out-pointer.
        check(unsafe { ffi::rh_estore_len(self.store.0, &mut n) }, "rh_estore_len");
        assert_eq!(n as usize, self.entries.len(), "rsos-hip: device and host sizes differ");
    }
}

/// The reference's `rsos::Entry` (public-api/rsos.txt:118-121).
pub struct Entry<'a, K, V> {
    map: &'a mut HipEncodedMap<K, V>,
    key: K,
}

impl<'a, K: Ord + Clone + Serialize, V: Serialize> Entry<'a, K, V> {
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
        let Entry { map, key } = self;
        if map.entries.get(&key).is_none() {
            <HipEncodedMap<K, V> as Rsos<K>>::insert(map, key.clone(), f());
        }
        let map: &'a HipEncodedMap<K, V> = map;
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

impl<K: Ord + Clone + Serialize, V: Serialize> FromIterator<(K, V)> for HipEncodedMap<K, V> {
    fn from_iter<T: IntoIterator<Item = (K, V)>>(iter: T) -> Self {
        let mut m = HipEncodedMap::new();
        m.load_bulk(iter.into_iter().collect());
        m
    }
}
