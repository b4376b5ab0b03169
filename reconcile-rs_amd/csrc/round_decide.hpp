// round_decide.hpp -- one segment's decision in an rbsr protocol round, on the host: the host
// tier's rounds (host_tier.hpp HostTier::round) and the sharded store's segments that straddle a
// shard boundary (sharded_store.cpp) take it from here; the device path restates it in
// aggregate_kernels.hip (round_decide).
//
// protocol_round_with_policy (rbsr/src/protocol.rs:212-317) for the policies that decide on the
// span alone: SKIP on equal aggregates (:236-241), the shared cutoffs (policy/cutoffs.rs:21-38:
// an empty remote side or a 1-vs-1 span is enumerated, a span of 0 or 1 against a larger remote
// side is split with stride 1), the policy's stride -- FixedFanOut ceil(span / b)
// (fixed_fan_out.rs:74-80), SqrtFanOut (span as f32).sqrt() (sqrt_fan_out.rs) -- a SPLIT that
// would not progress turned IDLIST (:263-272), an IDLIST with a non-empty remote side bounced
// back as one child with the ZERO aggregate, a SPLIT's children cut at every stride-th rank
// (:288-313).  Plain C++: no HIP, no allocation.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/rsos_hip.h"

namespace rh {

struct SegDecision {
    int kind;          // 0 skip, 1 IDLIST, 2 SPLIT, 3 dropped (malformed: the end ranks below the start)
    uint64_t stride;   // SPLIT: ranks per child
    uint64_t children; // children emitted (SPLIT: the cut pieces; IDLIST: 1 if bounced back)
    uint64_t enums;    // enumerations emitted (IDLIST: 1)
};

// lo / hi: the segment's raw ranks (BoundedRange::parse, rbsr/src/protocol/rank.rs); loc: the
// local aggregate over them (ZERO when hi < lo); rem: the peer's aggregate; b: the fan-out (>= 2)
inline SegDecision decide_segment(uint64_t lo, uint64_t hi, const rh_aggregate &loc, const rh_aggregate &rem,
                                  int sqrt_policy, uint64_t b) {
    SegDecision d{3, 0, 0, 0};
    if (hi < lo) return d;
    const uint64_t span = loc.size, r = rem.size;
    uint64_t st = 0;
    int k;
    if (span == r && !memcmp(loc.fingerprint, rem.fingerprint, 32)) k = 0;
    else if (r == 0) k = 1;
    else if (span == 0) k = 2, st = 1;
    else if (span == 1 && r == 1) k = 1;
    else if (span == 1) k = 2, st = 1;
    else {
        k = 2;
        st = sqrt_policy ? (uint64_t)std::sqrt((float)span) : (span + b - 1) / b;
        if (st == 0) st = 1;  // SplitStride::per_child
    }
    if (k == 2 && span > 1 && st >= span) k = 1;
    d.kind = k;
    d.stride = st;
    if (k == 1) {
        d.enums = 1;
        d.children = r != 0;
    } else if (k == 2) {
        d.children = (hi > lo ? (hi - lo - 1) / st : 0) + 1;
    }
    return d;
}

}  // namespace rh
