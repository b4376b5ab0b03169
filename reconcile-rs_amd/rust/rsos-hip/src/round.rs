//! One `rbsr` protocol round answered inside the library (`rh_store_protocol_round` /
//! `rh_sstore_protocol_round`, include/rsos_hip.h): `protocol_round_with_policy`
//! (rbsr/src/protocol.rs:212-317) for the policies that decide on the span alone.
//!
//! The round's logic -- the shared cutoffs (policy/cutoffs.rs:21-38), the policy's stride
//! (fixed_fan_out.rs:74-80, sqrt_fan_out.rs), the cut rule (protocol/rank.rs:75-78), the
//! non-progressing SPLIT turned IDLIST (protocol.rs:263-272) -- exists once, in the library,
//! where it is checked round by round against a literal restatement of the reference's round
//! (MI355X repository: tests/test_rbsr.py, tests/test_sharded.py).  This file only converts the
//! segments to the wire codec's SoA form and the outputs back, in the reference's order.

use std::ops::Bound;
use std::os::raw::{c_int, c_void};

use rsos::{Aggregate, Fingerprint};

use crate::{check, ffi, GpuKey, RoundCounts};

/// The shipped policies the library decides on the device or its host tier: `FixedFanOut(b)`
/// (`b < 2` is raised to 2, `FanOut::new`; 16 = `FanOut::NEGENTROPY`, `protocol_round`'s default)
/// and `SqrtFanOut`.
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum RoundPolicy {
    FixedFanOut(usize),
    SqrtFanOut,
}

/// `call(policy, fan_out, active, children, enumerations, outcome)` is one of the two entry
/// points on the caller's store; the outputs it fills point into the store's own buffers, read
/// here before anything else can call the store (the caller holds its round lock).
pub(crate) fn run_round<K: GpuKey>(
    call: impl FnOnce(c_int, u64, *const ffi::rh_segments, *mut ffi::rh_segments, *mut ffi::rh_segments,
                      *mut ffi::rh_round_outcome) -> c_int,
    policy: RoundPolicy,
    active: Vec<rbsr::RangeAggregate<K>>,
    child_ranges: &mut Vec<rbsr::RangeAggregate<K>>,
    enumeration_ranges: &mut Vec<rbsr::EnumerationRange<K>>,
) -> RoundCounts {
    let kl = K::LEN as usize;
    let n = active.len();
    let mut sk = vec![0u8; n.max(1)];
    let mut ek = vec![0u8; n.max(1)];
    let mut skeys = vec![0u8; n * kl + 1];
    let mut ekeys = vec![0u8; n * kl + 1];
    let mut aggs = vec![ffi::rh_aggregate::default(); n.max(1)];
    for (j, seg) in active.iter().enumerate() {
        // a RangeAggregate's start is Included or Unbounded, its end Excluded or Unbounded
        // (KeyRange, rbsr/src/protocol.rs:63-88)
        match seg.start_bound() {
            Bound::Included(k) | Bound::Excluded(k) => {
                sk[j] = 1;
                skeys[j * kl..(j + 1) * kl].copy_from_slice(&k.column_bytes());
            }
            Bound::Unbounded => {}
        }
        match seg.end_bound() {
            Bound::Included(k) | Bound::Excluded(k) => {
                ek[j] = 1;
                ekeys[j * kl..(j + 1) * kl].copy_from_slice(&k.column_bytes());
            }
            Bound::Unbounded => {}
        }
        let a = seg.aggregate();
        aggs[j] = ffi::rh_aggregate { fingerprint: a.fingerprint().0, size: a.size() as u64 };
    }
    let input = ffi::rh_segments {
        start_kinds: sk.as_mut_ptr(),
        start_keys: skeys.as_mut_ptr() as *mut c_void,
        end_kinds: ek.as_mut_ptr(),
        end_keys: ekeys.as_mut_ptr() as *mut c_void,
        aggregates: aggs.as_mut_ptr(),
        n,
        cap: n,
    };
    let (kind, b) = match policy {
        RoundPolicy::FixedFanOut(b) => (ffi::RH_POLICY_FIXED_FAN_OUT, b as u64),
        RoundPolicy::SqrtFanOut => (ffi::RH_POLICY_SQRT_FAN_OUT, 0),
    };
    let empty = ffi::rh_segments {
        start_kinds: std::ptr::null_mut(),
        start_keys: std::ptr::null_mut(),
        end_kinds: std::ptr::null_mut(),
        end_keys: std::ptr::null_mut(),
        aggregates: std::ptr::null_mut(),
        n: 0,
        cap: 0,
    };
    let (mut ch, mut en, mut oc) = (empty, empty, ffi::rh_round_outcome::default());
    check(call(kind, b, &input, &mut ch, &mut en, &mut oc), "protocol_round");
    // SAFETY: the library filled ch / en with arrays of ch.n / en.n items (keys kl bytes each),
    // valid until the store's next call, which the caller's round lock excludes.
    unsafe {
        let key = |p: *mut c_void, i: usize| K::from_column_bytes(std::slice::from_raw_parts((p as *const u8).add(i * kl), kl));
        for i in 0..ch.n {
            let s = (*ch.start_kinds.add(i) != 0).then(|| key(ch.start_keys, i));
            let e = (*ch.end_kinds.add(i) != 0).then(|| key(ch.end_keys, i));
            let a = *ch.aggregates.add(i);
            child_ranges.push(rbsr::RangeAggregate::new(s, e, Aggregate::new(a.size as usize, Fingerprint(a.fingerprint))));
        }
        for i in 0..en.n {
            let s = if *en.start_kinds.add(i) != 0 { Bound::Included(key(en.start_keys, i)) } else { Bound::Unbounded };
            let e = if *en.end_kinds.add(i) != 0 { Bound::Excluded(key(en.end_keys, i)) } else { Bound::Unbounded };
            enumeration_ranges.push((s, e));
        }
    }
    RoundCounts {
        skipped: oc.skipped as usize,
        enumerated: oc.enumerated as usize,
        split: oc.split as usize,
        children: oc.children as usize,
        dropped_malformed: oc.dropped_malformed as usize,
    }
}
