// host_tier.hpp -- the store's host tier: the small questions of a reconciliation answered in
// host memory, with no device round trip.
//
// rbsr's diff path is latency-bound: a d = 1 reconciliation of a 10^6-entry
// map asks ~155 aggregate, ~152 rank and ~70 select questions (benches/README.md:579-585), each
// O(log n) on the reference's FingerprintTreeMap (query.rs:25-167), ~45 us in all.  One device
// round trip per round costs more than that.  The host tier keeps, next to the HBM-resident store,
//   - the keys in rank order (what select() returns, rbsr/src/rsos_view.rs:70),
//   - the exclusive prefix sums of the per-row fingerprints, P[i] = Σ lift(row j), j < i, mod 2^256,
//     computed on the device (launch_prefix) from the fingerprints the GPU lift produced, so
//     summary-folds-lift holds by construction (rsos_trait.rs:46-60): aggregate over rank range
//     [lo, hi) = (P[hi] - P[lo], hi - lo) -- the Fingerprint group's inverse (fingerprint.rs:159-173),
//   - the leading 8 key bytes (order-preserving) of every 64th key, so a rank is a search of a
//     cache-resident sample array and then of one 64-key window.
// It is refreshed from the device on the first question after the store changes.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/rsos_hip.h"
#include "internal.hpp"

namespace rh {

struct HostTier {
    uint32_t kl = 0;
    int kk = RH_KEY_BYTES;
    uint64_t n = 0;
    const uint8_t *keys = nullptr;     // n * kl bytes, rank order
    const uint64_t *prefix = nullptr;  // (n + 1) * 4 LE limbs
    std::vector<uint64_t> samp;        // digit(keys[64 j])
    static constexpr unsigned SHIFT = 6;

    // an order-preserving u64 of a key's leading bytes: the integer for u32 / u64 keys, the first 8
    // bytes big-endian for byte keys (memcmp order, the Ord of [u8; L])
    uint64_t digit(const uint8_t *k) const {
        if (kk == RH_KEY_U32) {
            uint32_t v;
            memcpy(&v, k, 4);
            return v;
        }
        uint64_t v;
        memcpy(&v, k, 8);
        return kk == RH_KEY_U64 ? v : __builtin_bswap64(v);
    }
    int cmp(const uint8_t *a, const uint8_t *b) const {
        const uint64_t x = digit(a), y = digit(b);
        if (x != y) return x < y ? -1 : 1;
        return kk == RH_KEY_BYTES && kl > 8 ? memcmp(a + 8, b + 8, kl - 8) : 0;
    }
    void build(uint32_t key_len, int key_kind, uint64_t rows, const uint8_t *k, const uint64_t *p) {
        kl = key_len;
        kk = key_kind;
        n = rows;
        keys = k;
        prefix = p;
        samp.clear();
        if (!keys) return;  // the encoded store keeps its keys on the host side of the ABI
        samp.resize((n + 63) >> SHIFT);
        for (uint64_t j = 0; j < samp.size(); j++) samp[j] = digit(keys + (j << SHIFT) * kl);
    }
    // rank(z) = number of keys strictly below z (query.rs:93-121)
    uint64_t rank(const uint8_t *key) const {
        if (n == 0) return 0;
        const uint64_t d = digit(key);
        const uint64_t jl = std::lower_bound(samp.begin(), samp.end(), d) - samp.begin();
        const uint64_t jh = std::upper_bound(samp.begin() + jl, samp.end(), d) - samp.begin();
        uint64_t lo = jl ? ((jl - 1) << SHIFT) + 1 : 0;  // keys[64 (jl - 1)] < key
        uint64_t hi = std::min<uint64_t>(n, jh << SHIFT);  // keys[64 jh] > key
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (cmp(keys + mid * kl, key) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // Aggregate over rank range [lo, hi), clamped as the device query clamps (hi <= n, lo <= hi)
    void agg(uint64_t lo, uint64_t hi, rh_aggregate *o) const {
        if (hi > n) hi = n;
        if (lo > hi) lo = hi;
        const uint64_t *a = prefix + 4 * hi, *b = prefix + 4 * lo;
        unsigned char borrow = 0;
        for (int q = 0; q < 4; q++) {
            const uint64_t x = a[q], y = b[q];
            const uint64_t d = x - y - borrow;
            borrow = (x < y) || (x == y && borrow);
            o->fingerprint[q] = d;
        }
        o->size = hi - lo;
    }
    // rank of a bound: kind 0 = unbounded (lower: 0, upper: n), 1 = included, 2 = excluded
    uint64_t bound_rank(int kind, const uint8_t *key, bool lower) const {
        if (kind == 0) return lower ? 0 : n;
        const uint64_t r = rank(key);  // keys < key
        const bool present = r < n && cmp(keys + r * kl, key) == 0;
        if (lower) return kind == 1 ? r : r + present;   // Included(k): k.., Excluded(k): k is out
        return kind == 2 ? r : r + present;              // Excluded(k): ..k, Included(k): ..=k
    }

    // ---- one protocol round (protocol_round_with_policy, rbsr/src/protocol.rs:212-317) ------------
    // The same decisions as the device path (round_decide, aggregate_kernels.hip) and the same output
    // layout (round_layout): SKIP on equal aggregates, the shared cutoffs (policy/cutoffs.rs), the
    // policy's stride (FixedFanOut ceil(span / b), SqrtFanOut (span as f32).sqrt()), a non-progressing
    // SPLIT turned IDLIST (:263-272), an IDLIST with a non-empty remote side bounced back as one child
    // with the ZERO aggregate, a SPLIT's children cut at every stride-th rank (:288-313).
    struct Seg {
        int kind;  // 0 skip, 1 IDLIST, 2 SPLIT, 3 dropped
        uint64_t stride, si, ei, children, enums;
        rh_aggregate loc;
    };
    std::vector<Seg> segs;
    void round(int sqrt_policy, uint64_t b, const rh_segments &in, std::vector<uint8_t> &out, uint64_t hdr[5]) {
        const size_t r = in.n;
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        segs.resize(r);
        uint64_t nc = 0, ne = 0, cnt[5] = {0, 0, 0, 0, 0};
        for (size_t j = 0; j < r; j++) {
            Seg &g = segs[j];
            const uint64_t l = sk[j] ? rank(skeys + j * kl) : 0, h = ek[j] ? rank(ekeys + j * kl) : n;
            agg(l, h, &g.loc);
            const rh_aggregate &R = in.aggregates[j];
            g = Seg{3, 0, 0, 0, 0, 0, g.loc};
            if (h >= l) {
                g.si = std::min(l, n);
                g.ei = std::min(h, n);
                const uint64_t span = g.loc.size, rem = R.size;
                uint64_t st = 0;
                int k;
                if (span == rem && !memcmp(g.loc.fingerprint, R.fingerprint, 32)) k = 0;
                else if (rem == 0) k = 1;
                else if (span == 0) k = 2, st = 1;
                else if (span == 1 && rem == 1) k = 1;
                else if (span == 1) k = 2, st = 1;
                else {
                    k = 2;
                    st = sqrt_policy ? (uint64_t)std::sqrt((float)span) : (span + b - 1) / b;
                    if (st == 0) st = 1;  // SplitStride::per_child
                }
                if (k == 2 && span > 1 && st >= span) k = 1;
                g.kind = k;
                g.stride = st;
                if (k == 1) {
                    g.enums = 1;
                    g.children = rem != 0;
                } else if (k == 2) {
                    g.children = (g.ei > g.si ? (g.ei - g.si - 1) / st : 0) + 1;
                }
            }
            cnt[g.kind == 3 ? 4 : g.kind]++;
            nc += g.children;
            ne += g.enums;
        }
        hdr[0] = cnt[0], hdr[1] = ne, hdr[2] = cnt[2], hdr[3] = nc, hdr[4] = cnt[4];
        const RoundLayout L = round_layout(nc, ne, kl);
        out.resize(L.end);
        uint8_t *o = out.data();
        memcpy(o, hdr, 40);
        uint64_t c = 0, e = 0;
        auto put_key = [&](uint64_t off, const uint8_t *k) {
            if (k) memcpy(o + off, k, kl);
            else memset(o + off, 0, kl);
        };
        auto child = [&](uint8_t skd, const uint8_t *skey, uint8_t ekd, const uint8_t *ekey, const rh_aggregate &a) {
            o[L.csk + c] = skd;
            o[L.cek + c] = ekd;
            put_key(L.cskeys + c * kl, skd ? skey : nullptr);
            put_key(L.cekeys + c * kl, ekd ? ekey : nullptr);
            memcpy(o + L.caggs + 40 * c, &a, 40);
            c++;
        };
        const rh_aggregate zero{{0, 0, 0, 0}, 0};
        for (size_t j = 0; j < r; j++) {
            const Seg &g = segs[j];
            const uint8_t *s0 = sk[j] ? skeys + j * kl : nullptr, *e0 = ek[j] ? ekeys + j * kl : nullptr;
            if (g.kind == 1) {
                o[L.esk + e] = sk[j];
                o[L.eek + e] = ek[j];
                put_key(L.eskeys + e * kl, s0);
                put_key(L.eekeys + e * kl, e0);
                e++;
                if (g.children) child(sk[j], s0, ek[j], e0, zero);
            } else if (g.kind == 2) {
                const uint64_t ncuts = g.children - 1;
                if (ncuts == 0) {
                    child(sk[j], s0, ek[j], e0, g.loc);
                    continue;
                }
                for (uint64_t k = 0; k <= ncuts; k++) {
                    const uint64_t lo = g.si + k * g.stride, hi = k == ncuts ? g.ei : g.si + (k + 1) * g.stride;
                    rh_aggregate a;
                    agg(lo, hi, &a);
                    child(k ? 1 : sk[j], k ? keys + lo * kl : s0, k != ncuts ? 1 : ek[j], k != ncuts ? keys + hi * kl : e0,
                          a);
                }
            }
        }
    }
};

}  // namespace rh
