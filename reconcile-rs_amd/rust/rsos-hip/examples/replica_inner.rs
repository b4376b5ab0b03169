//! The reference's `Replica` state with its two maps swapped for the MI355X ones -- the field
//! declarations of src/replica.rs:68-74, the construction of src/replica/construct.rs:205-206 and
//! the dual insert of `Replica::map_insert` (src/replica/write.rs:26-46) -- written against the
//! reference's own bounds.  It is what INTEGRATION.md's diff does to `Inner<K, V>`; building this
//! example (`cargo build --example replica_inner`) is the compile check of that diff.
//!
//! (`std::sync::RwLock` stands in for `parking_lot::RwLock`: the lock type does not take part in
//! the bounds.)
use std::hash::Hash;
use std::sync::{Arc, RwLock};

use lww_register::{Entry, Key, State, Timestamp, Value};
use rsos_hip::{FixedValue, GpuKey, HipEncodedMap, HipFingerprintMap};

/// src/replica.rs:68-74 with `FingerprintTreeMap` -> `HipEncodedMap`: no bound on `K`, `V` (any
/// serde key and value; the canonical bytes are encoded on the host, hashed on the device).
pub struct Inner<K, V> {
    pub map: Arc<RwLock<HipEncodedMap<K, Entry<Timestamp, V>>>>,
    pub projection: Arc<RwLock<HipEncodedMap<K, State<V>>>>,
}

/// The same with `HipFingerprintMap` (fixed-width keys and values, the canonical encoding
/// synthesised in registers): the field declarations still take unbounded `K`, `V`.
pub struct InnerFixed<K, V> {
    pub map: Arc<RwLock<HipFingerprintMap<K, Entry<Timestamp, V>>>>,
    pub projection: Arc<RwLock<HipFingerprintMap<K, State<V>>>>,
}

/// Replica's own bounds (src/replica/construct.rs:74: `impl<K: Key + Hash, V: Value>`) suffice
/// for the encoded map: `Key` / `Value` imply `Ord + Clone + Serialize` / `Serialize`
/// (lww-register/src/bounds.rs:21,31), and `Entry<Timestamp, V>` / `State<V>` derive `Serialize`.
impl<K: Key + Hash, V: Value> Inner<K, V> {
    pub fn build() -> Self {
        let map = HipEncodedMap::<K, Entry<Timestamp, V>>::new();
        let projection = HipEncodedMap::<K, State<V>>::new();
        Inner { map: Arc::new(RwLock::new(map)), projection: Arc::new(RwLock::new(projection)) }
    }

    /// Replica::map_insert's two inserts under the two write locks (write.rs:44-45)
    pub fn map_insert(&self, key: K, value: Entry<Timestamp, V>) -> Option<Entry<Timestamp, V>> {
        self.projection.write().unwrap().insert(key.clone(), value.state.clone());
        self.map.write().unwrap().insert(key, value)
    }

    pub fn fingerprint(&self) -> rsos::Aggregate {
        self.map.read().unwrap().aggregate(..)
    }
}

/// The fixed-width map needs the two extra bounds INTEGRATION.md adds to the impl blocks:
/// `K: GpuKey` and `V: FixedValue` (then `Entry<Timestamp, V>: GpuRecord` and
/// `State<V>: GpuRecord` come from rsos-hip's own impls).
impl<K: Key + Hash + GpuKey, V: Value + FixedValue> InnerFixed<K, V> {
    pub fn build() -> Self {
        let map = HipFingerprintMap::<K, Entry<Timestamp, V>>::new();
        let projection = HipFingerprintMap::<K, State<V>>::new();
        InnerFixed { map: Arc::new(RwLock::new(map)), projection: Arc::new(RwLock::new(projection)) }
    }

    pub fn map_insert(&self, key: K, value: Entry<Timestamp, V>) -> Option<Entry<Timestamp, V>> {
        self.projection.write().unwrap().insert(key.clone(), value.state.clone());
        self.map.write().unwrap().insert(key, value)
    }

    pub fn fingerprint(&self) -> rsos::Aggregate {
        self.map.read().unwrap().aggregate(..)
    }
}

fn main() {
    use lww_register::clock::{Hlc, LogicalCounter, NodeId, PhysicalTime};
    let stamp = Timestamp::new(Hlc::new(PhysicalTime::from_millis(1_700_000_000_000), LogicalCounter::new(0)),
                               NodeId::new(1));
    let fixed: InnerFixed<[u8; 16], rsos_hip::FixedBytes<64>> = InnerFixed::build();
    fixed.map_insert([7; 16], Entry::present(stamp, rsos_hip::FixedBytes::new(vec![1; 64]).unwrap()));
    let encoded: Inner<String, String> = Inner::build();
    encoded.map_insert("k".into(), Entry::present(stamp, "v".into()));
    println!("{:?} {:?}", fixed.fingerprint(), encoded.fingerprint());
}
