// round_device.hpp -- device pieces of the store's rank-range sums and rbsr protocol rounds,
// shared by the round kernels (aggregate_kernels.hip) and the fused tiny round that also runs the
// bound keys' searches (round_tiny.hpp, instantiated per key type in store_kernels.hip).
#pragma once
#include "blake3_device.hpp"
#include "internal.hpp"
#include "search_device.hpp"

namespace rh {

// fingerprint i of an array whose entries are `stride` bytes apart (32 for plain fingerprint
// arrays; the store's delta records carry their 32-byte contribution first, stride 40: 8-byte
// aligned, so those are read as 8-byte words)
__device__ __forceinline__ void load_fp(const uint8_t *src, uint64_t i, uint32_t f[8], uint32_t stride = 32) {
    if ((stride & 15) == 0) {
        const uint4 *p = reinterpret_cast<const uint4 *>(src + (uint64_t)stride * i);
        uint4 a = p[0], b = p[1];
        f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
        f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
    } else {
        const uint2 *p = reinterpret_cast<const uint2 *>(src + (uint64_t)stride * i);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint2 v = p[k];
            f[2 * k] = v.x;
            f[2 * k + 1] = v.y;
        }
    }
}

// One wave per query (4 per workgroup), for batches of many queries over a run with block and
// super-block sums (a protocol round's segments and children): the same head rows + blocks +
// super-blocks decomposition, lanes striding by 64, a wave butterfly instead of the workgroup
// reduction.  The one-workgroup form above wastes 3 of 4 waves on the short ranges a round has.
__device__ __forceinline__ void acc_span_lane(Acc &a, const uint8_t *src, uint64_t lo, uint64_t hi, uint32_t lane,
                                              uint32_t stride = 32) {
    for (uint64_t i = lo + lane; i < hi; i += 64) {
        uint32_t f[8];
        load_fp(src, i, f, stride);
        acc_add_fp(a, f);
    }
}

// Σ over rank range [lo, hi) (already clamped) by one wave, as four 64-bit limbs (lane 0's are the sum)
__device__ __forceinline__ void wave_range_fp(const uint8_t *fps, uint32_t stride, const uint8_t *bsums,
                                              const uint8_t *ssums, uint64_t lo, uint64_t hi, uint32_t lane,
                                              uint64_t fp[4]) {
    Acc a;
    acc_zero(a);
    const uint64_t B = 256;
    const uint64_t b1 = (lo + B - 1) / B, b2 = hi / B;
    if (b1 >= b2) {
        acc_span_lane(a, fps, lo, hi, lane, stride);
    } else {
        acc_span_lane(a, fps, lo, b1 * B, lane, stride);
        acc_span_lane(a, fps, b2 * B, hi, lane, stride);
        const uint64_t s1 = (b1 + B - 1) / B, s2 = b2 / B;
        if (s1 >= s2) {
            acc_span_lane(a, bsums, b1, b2, lane);
        } else {
            acc_span_lane(a, bsums, b1, s1 * B, lane);
            acc_span_lane(a, bsums, s2 * B, b2, lane);
            acc_span_lane(a, ssums, s1, s2, lane);
        }
    }
    acc_wave_reduce(a);
    uint32_t f[8];
    acc_normalise(a, f);
    fp[0] = (uint64_t)f[0] | ((uint64_t)f[1] << 32);
    fp[1] = (uint64_t)f[2] | ((uint64_t)f[3] << 32);
    fp[2] = (uint64_t)f[4] | ((uint64_t)f[5] << 32);
    fp[3] = (uint64_t)f[6] | ((uint64_t)f[7] << 32);
}

// the same; lane 0 writes the rh_aggregate {u64 fp[4]; u64 size} at o
__device__ __forceinline__ void wave_range_agg(const uint8_t *fps, uint32_t stride, const uint8_t *bsums,
                                               const uint8_t *ssums, uint64_t lo, uint64_t hi, uint32_t lane,
                                               uint64_t *o) {
    uint64_t fp[4];
    wave_range_fp(fps, stride, bsums, ssums, lo, hi, lane, fp);
    if (lane == 0) {
        o[0] = fp[0];
        o[1] = fp[1];
        o[2] = fp[2];
        o[3] = fp[3];
        o[4] = hi - lo;
    }
}

// ---- one rbsr protocol round on the device (protocol_round_with_policy, rbsr/src/protocol.rs:212-317) ----
// round_decide takes a segment's decision from its resolved rank range and local / remote
// aggregates: SKIP on equal aggregates, the shared cutoffs (rbsr/src/policy/cutoffs.rs), then
// the policy's stride -- FixedFanOut ceil(span / b) (policy/fixed_fan_out.rs), SqrtFanOut
// (span as f32).sqrt() (policy/sqrt_fan_out.rs) -- and a non-progressing SPLIT turned IDLIST
// (protocol.rs:263-272).  An IDLIST with a non-empty remote side bounces its range back as one
// child with the ZERO aggregate; a SPLIT's children are cut at every stride-th rank
// (protocol.rs:288-313).  kind: 0 skip, 1 IDLIST, 2 SPLIT, 3 dropped (inverted, :232-245).
struct RoundSeg {
    int kind;
    uint64_t stride, si, ei, children, enums;
};

__device__ __forceinline__ RoundSeg round_decide(uint64_t l, uint64_t h, const uint64_t *L, const uint64_t *R,
                                                 uint64_t n, int sqrt_policy, uint64_t b) {
    RoundSeg g{3, 0, 0, 0, 0, 0};
    if (h < l) return g;
    g.si = l < n ? l : n;
    g.ei = h < n ? h : n;
    const uint64_t span = L[4], rem = R[4];
    uint64_t st = 0;
    int k;
    if (span == rem && L[0] == R[0] && L[1] == R[1] && L[2] == R[2] && L[3] == R[3]) k = 0;
    else if (rem == 0) k = 1;
    else if (span == 0) k = 2, st = 1;
    else if (span == 1 && rem == 1) k = 1;
    else if (span == 1) k = 2, st = 1;
    else {
        k = 2;
        st = sqrt_policy ? (uint64_t)__fsqrt_rn((float)span) : (span + b - 1) / b;
        if (st == 0) st = 1;  // SplitStride::per_child
    }
    if (k == 2 && span > 1 && st >= span) k = 1;
    g.kind = k;
    g.stride = st;
    if (k == 1) {
        g.enums = 1;
        g.children = rem != 0;
    } else if (k == 2) {
        g.children = (g.ei > g.si ? (g.ei - g.si - 1) / st : 0) + 1;  // cuts at si + i * st < ei, i >= 1
    }
    return g;
}

// Child c (k-th of segment j), by one wave: its bounds (the parent's own, or the keys at the cut
// ranks) and its aggregate -- the parent's local one for an uncut SPLIT, ZERO for a bounced
// IDLIST, else the rank range summed like k_range_query_wave.
__device__ __forceinline__ void round_emit_child(uint64_t c, uint64_t j, uint64_t k, const RoundLayout &L,
                                                 uint32_t kl, uint32_t lane, const RoundIn &in, const RoundSegs &g,
                                                 uint8_t *out) {
    uint8_t skd = in.sk[j], ekd = in.ek[j];
    const uint8_t *skey = skd ? in.skeys + j * kl : nullptr, *ekey = ekd ? in.ekeys + j * kl : nullptr;
    uint64_t *agg = reinterpret_cast<uint64_t *>(out + L.caggs) + 5 * c;
    const uint64_t ncuts = g.nch[j] - 1;
    if (g.kind[j] == 1 || ncuts == 0) {
        if (lane < 5) agg[lane] = g.kind[j] == 1 ? 0ull : g.loc[5 * j + lane];
    } else {
        const uint64_t st = g.stride[j], s0 = g.si[j];
        const uint64_t lo = s0 + k * st, hi = k == ncuts ? g.ei[j] : s0 + (k + 1) * st;
        if (k) skd = 1, skey = in.bkeys + lo * kl;
        if (k != ncuts) ekd = 1, ekey = in.bkeys + hi * kl;
        wave_range_agg(in.fps, 32, in.bsums, in.ssums, lo, hi, lane, agg);
    }
    if (lane == 0) {
        out[L.csk + c] = skd;
        out[L.cek + c] = ekd;
    }
    if (lane < kl / 4) {
        reinterpret_cast<uint32_t *>(out + L.cskeys + c * kl)[lane] =
            skey ? reinterpret_cast<const uint32_t *>(skey)[lane] : 0u;
        reinterpret_cast<uint32_t *>(out + L.cekeys + c * kl)[lane] =
            ekey ? reinterpret_cast<const uint32_t *>(ekey)[lane] : 0u;
    }
}

// Segment j's IDLIST range as enumeration e (unbounded sides' keys written as zeros)
__device__ __forceinline__ void round_emit_enum(uint64_t j, uint64_t e, const RoundLayout &L, uint32_t kl,
                                                const RoundIn &in, const RoundSegs &, uint8_t *out) {
    const uint8_t skd = in.sk[j], ekd = in.ek[j];
    out[L.esk + e] = skd;
    out[L.eek + e] = ekd;
    uint32_t *os = reinterpret_cast<uint32_t *>(out + L.eskeys + e * kl);
    uint32_t *oe = reinterpret_cast<uint32_t *>(out + L.eekeys + e * kl);
    const uint32_t *is = reinterpret_cast<const uint32_t *>(in.skeys + j * kl);
    const uint32_t *ie = reinterpret_cast<const uint32_t *>(in.ekeys + j * kl);
    for (uint32_t w = 0; w < kl / 4; w++) {
        os[w] = skd ? is[w] : 0u;
        oe[w] = ekd ? ie[w] : 0u;
    }
}

// j = the last segment with choff[j] <= c (it owns child c)
__device__ __forceinline__ uint64_t round_owner(const uint64_t *choff, uint64_t r, uint64_t c) {
    uint64_t a = 0, z = r;
    while (a < z) {
        const uint64_t mid = (a + z) >> 1;
        if (choff[mid] <= c) a = mid + 1;
        else z = mid;
    }
    return a - 1;
}

// ---- rounds over base + delta run (RoundRun, internal.hpp) ----
__device__ __forceinline__ void fp_add256(uint64_t a[4], const uint64_t *b) {
    uint64_t c = 0;
    for (int i = 0; i < 4; i++) {
        const uint64_t s = a[i] + b[i], t = s + c;
        c = (uint64_t)(s < a[i]) | (uint64_t)(t < s);
        a[i] = t;
    }
}

__device__ __forceinline__ bool run_live(const RoundRun &R, uint64_t j) { return R.flags[j] & 2; }

__device__ __forceinline__ bool run_in_base(const RoundRun &R, uint64_t j) { return R.flags[j] & 1; }

// live view keys <= run entry j (non-decreasing in j)
__device__ __forceinline__ int64_t run_g(const RoundRun &R, uint64_t j) {
    return (int64_t)R.brank[j] + R.cntp[j] + (run_live(R, j) ? 1 : 0);
}

struct ViewPlace {
    uint64_t b, j;
    const uint8_t *key;
};

// select: the view key of rank v < nv and its place (host_tier.hpp HostTier::view_at): the first
// entry with G(j) > v is that key itself, or the key is an untouched base row between entries
// j - 1 and j.  Every lane computes the same (uniform loads).
__device__ __forceinline__ ViewPlace view_at(const RoundRun &R, const uint8_t *bkeys, uint32_t kl, uint64_t v) {
    const uint64_t ns = (R.n + 63) >> 6;
    uint64_t a = 0, z = ns;
    while (a < z) {  // the first sampled entry with G > v bounds a window of 64 entries
        const uint64_t mid = (a + z) >> 1;
        if ((uint64_t)R.gsamp[mid] > v) z = mid;
        else a = mid + 1;
    }
    uint64_t lo = a ? ((a - 1) << 6) + 1 : 0, hi = a << 6 < R.n ? a << 6 : R.n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((uint64_t)run_g(R, mid) > v) hi = mid;
        else lo = mid + 1;
    }
    const uint64_t j = lo;
    if (j < R.n && run_live(R, j) && (uint64_t)((int64_t)R.brank[j] + R.cntp[j]) == v)
        return ViewPlace{R.brank[j], j, R.keys + j * kl};
    const uint64_t gprev = j ? (uint64_t)run_g(R, j - 1) : 0;
    const uint64_t b0 = j ? R.brank[j - 1] + (run_in_base(R, j - 1) ? 1 : 0) : 0;
    const uint64_t b = b0 + (v - gprev);
    return ViewPlace{b, j, bkeys + b * kl};
}

// view_at by a group of W lanes (W = 16 or 64): the same answer, the first sampled entry with
// G > v and then the entry inside its 64-entry window found by W-way probes (G(j) needs the entry's
// base rank, count prefix and flags: three loads per probe, issued together) -- a few dependent
// loads where view_at walks ~log2(n / 64) + 6.  gl: the lane's index in its group.
template <int W>
__device__ __forceinline__ ViewPlace view_at_group(const RoundRun &R, const uint8_t *bkeys, uint32_t kl, uint64_t v,
                                                   uint32_t gl) {
    const uint64_t ns = (R.n + 63) >> 6;
    // a = the number of sampled entries with G <= v (G is non-decreasing)
    uint64_t lo = 0, hi = ns;
    while (hi > lo) {
        const uint64_t step = (hi - lo + W - 1) / W;
        const uint64_t p = lo + gl * step;
        const bool le = p < hi && (uint64_t)R.gsamp[p] <= v;
        const uint32_t c = __popcll(group_ballot<W>(le));
        if (c == 0) {
            hi = lo;
            break;
        }
        const uint64_t pc = lo + (c - 1) * step;
        lo = pc + 1;
        hi = pc + step < hi ? pc + step : hi;
        if (step == 1) break;
    }
    const uint64_t a = lo;
    // j = the first entry in ((a - 1) * 64, min(a * 64, n)] with G(j) > v
    uint64_t elo = a ? ((a - 1) << 6) + 1 : 0, ehi = a << 6 < R.n ? a << 6 : R.n;
    while (ehi > elo) {
        const uint64_t step = (ehi - elo + W - 1) / W;
        const uint64_t p = elo + gl * step;
        const bool le = p < ehi && (uint64_t)run_g(R, p) <= v;
        const uint32_t c = __popcll(group_ballot<W>(le));
        if (c == 0) {
            ehi = elo;
            break;
        }
        const uint64_t pc = elo + (c - 1) * step;
        elo = pc + 1;
        ehi = pc + step < ehi ? pc + step : ehi;
        if (step == 1) break;
    }
    const uint64_t j = elo;
    if (j < R.n && run_live(R, j) && (uint64_t)((int64_t)R.brank[j] + R.cntp[j]) == v)
        return ViewPlace{R.brank[j], j, R.keys + j * kl};
    const uint64_t gprev = j ? (uint64_t)run_g(R, j - 1) : 0;
    const uint64_t b0 = j ? R.brank[j - 1] + (run_in_base(R, j - 1) ? 1 : 0) : 0;
    const uint64_t b = b0 + (v - gprev);
    return ViewPlace{b, j, bkeys + b * kl};
}
// two's complement mod 2^256 (a fingerprint subtracted by adding it)
__device__ __forceinline__ void neg256(uint32_t f[8]) {
    uint32_t c = 1;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t x = ~f[k], s = x + c;
        c = s < x ? 1u : 0u;
        f[k] = s;
    }
}
// One part's (base or run) range [lo, hi) of n rows as at most two signed pieces, each <= 128
// rows and at most one bpre entry: a short range is its rows; a longer one is P(hi) - P(lo), P(x) =
// Σ rows [0, x) taken from the nearer block edge -- bpre[x/256] + rows [256(x/256), x) or
// bpre[x/256 + 1] - rows [x, 256(x/256 + 1)) (bpre's last entry is the total, so the last partial
// block's edge is n).  k < 0: no bpre entry.
struct PrePiece {
    uint64_t a, b;
    int64_t k;
    bool neg_rows, neg_pre;
};
__device__ __forceinline__ PrePiece pre_end(uint64_t x, uint64_t n, bool neg) {
    const uint64_t k = x >> 8, off = x & 255;
    if (off <= 128) return PrePiece{x - off, x, (int64_t)k, neg, neg};
    const uint64_t e = ((k + 1) << 8) < n ? (k + 1) << 8 : n;
    return PrePiece{x, e, (int64_t)k + 1, !neg, neg};
}
__device__ __forceinline__ void pre_pieces(uint64_t lo, uint64_t hi, uint64_t n, PrePiece &p, PrePiece &q) {
    const PrePiece none{0, 0, -1, false, false};
    if (hi <= lo) p = q = none;
    else if (hi - lo <= 128) p = PrePiece{lo, hi, -1, false, false}, q = none;
    else p = pre_end(hi, n, false), q = pre_end(lo, n, true);
}
__device__ __forceinline__ void piece_load(const uint8_t *fps, const PrePiece &p, uint32_t lane, uint32_t f0[8],
                                           uint32_t f1[8], bool &v0, bool &v1) {
    const uint64_t i0 = p.a + lane, i1 = i0 + 64;
    v0 = i0 < p.b;
    v1 = i1 < p.b;
    if (v0) load_fp(fps, i0, f0);
    if (v1) load_fp(fps, i1, f1);
}
__device__ __forceinline__ void acc_signed(Acc &a, uint32_t f[8], bool v, bool neg) {
    if (!v) return;
    if (neg) neg256(f);
    acc_add_fp(a, f);
}

// (a - b) mod 2^256, as 8 x u32
__device__ __forceinline__ void sub256(uint32_t a[8], const uint32_t b[8]) {
    uint32_t br = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t x = a[k], d = x - b[k], e = d - br;
        br = (x < b[k] || d < br) ? 1u : 0u;
        a[k] = e;
    }
}
// the row prefixes' difference between two places by one lane: Σ base [b0, b1) + Σ run [j0, j1)
// = pre_b[b1] - pre_b[b0] + pre_r[j1] - pre_r[j0] (four independent 32-B loads, one round of
// latency; the lanes of a wave that ask the same places share the loads)
__device__ __forceinline__ bool has_row_prefix(const RoundIn &in, const RoundRun &R) {
    return in.pre && (R.n == 0 || R.pre);
}
__device__ __forceinline__ void pre_range_fp(const RoundIn &in, const RoundRun &R, uint64_t b0, uint64_t j0,
                                             uint64_t b1, uint64_t j1, uint64_t fp[4]) {
    uint32_t x[8], y[8], u[8], v[8];
    const bool br = b1 > b0, rr = j1 > j0;
    if (br) load_fp(in.pre, b1, x), load_fp(in.pre, b0, y);
    if (rr) load_fp(R.pre, j1, u), load_fp(R.pre, j0, v);
    uint32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (br) {
        sub256(x, y);
#pragma unroll
        for (int k = 0; k < 8; k++) s[k] = x[k];
    }
    if (rr) {
        sub256(u, v);
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint64_t t = (uint64_t)s[k] + u[k] + c;
            s[k] = (uint32_t)t;
            c = (uint32_t)(t >> 32);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) fp[q] = (uint64_t)s[2 * q] | ((uint64_t)s[2 * q + 1] << 32);
}

// two pieces of one part into a: four row loads per lane and two prefix entries (lanes 0, 1)
// issued before any is added
__device__ __forceinline__ void acc_pieces2(Acc &a, const uint8_t *fps, const uint8_t *bpre, const PrePiece &p0,
                                            const PrePiece &p1, uint32_t lane) {
    uint32_t f[4][8], pf[8];
    bool v[4];
    piece_load(fps, p0, lane, f[0], f[1], v[0], v[1]);
    piece_load(fps, p1, lane, f[2], f[3], v[2], v[3]);
    const PrePiece &pq = lane == 0 ? p0 : p1;
    const bool pv = lane < 2 && pq.k >= 0;
    if (pv) load_fp(bpre, (uint64_t)pq.k, pf);
    acc_signed(a, f[0], v[0], p0.neg_rows);
    acc_signed(a, f[1], v[1], p0.neg_rows);
    acc_signed(a, f[2], v[2], p1.neg_rows);
    acc_signed(a, f[3], v[3], p1.neg_rows);
    acc_signed(a, pf, pv, pq.neg_pre);
}

// Σ of the live view keys between two places (lane 0's limbs): base rows [b0, b1) plus run
// contributions [j0, j1).  With both block prefixes present every load of the four pieces (eight
// per lane, and four prefix entries on lanes 0-3) is issued before any is added: one round of
// memory latency whatever the ranges' lengths.  With the row prefixes, their difference
// (pre_range_fp).  Wide = false (a 1,024-lane workgroup, 128 VGPRs a
// lane): the base's pieces, then the run's -- two rounds, no scratch.
template <bool Wide = true>
__device__ __forceinline__ void view_range_fp(const RoundIn &in, const RoundRun &R, uint64_t b0, uint64_t j0,
                                              uint64_t b1, uint64_t j1, uint32_t lane, uint64_t fp[4]) {
    if (has_row_prefix(in, R)) {  // every lane the same sum (the loads are shared)
        pre_range_fp(in, R, b0, j0, b1, j1, fp);
        return;
    }
    if (in.bpre && (R.n == 0 || R.bpre)) {
        PrePiece p0, p1, p2, p3;
        pre_pieces(b0, b1, R.nb, p0, p1);
        pre_pieces(j0, j1, R.n, p2, p3);
        if (!Wide) {
            Acc a;
            acc_zero(a);
            acc_pieces2(a, in.fps, in.bpre, p0, p1, lane);
            if (j1 > j0) acc_pieces2(a, R.contrib, R.bpre, p2, p3, lane);  // uniform
            acc_wave_reduce(a);
            uint32_t g[8];
            acc_normalise(a, g);
#pragma unroll
            for (int q = 0; q < 4; q++) fp[q] = (uint64_t)g[2 * q] | ((uint64_t)g[2 * q + 1] << 32);
            return;
        }
        uint32_t f[8][8], pf[8];
        bool v[8];
        piece_load(in.fps, p0, lane, f[0], f[1], v[0], v[1]);
        piece_load(in.fps, p1, lane, f[2], f[3], v[2], v[3]);
        piece_load(R.contrib, p2, lane, f[4], f[5], v[4], v[5]);
        piece_load(R.contrib, p3, lane, f[6], f[7], v[6], v[7]);
        // lane q < 4: piece q's prefix entry
        const PrePiece &pq = lane == 0 ? p0 : lane == 1 ? p1 : lane == 2 ? p2 : p3;
        const bool pv = lane < 4 && pq.k >= 0;
        if (pv) load_fp(lane < 2 ? in.bpre : R.bpre, (uint64_t)pq.k, pf);
        Acc a;
        acc_zero(a);
        acc_signed(a, f[0], v[0], p0.neg_rows);
        acc_signed(a, f[1], v[1], p0.neg_rows);
        acc_signed(a, f[2], v[2], p1.neg_rows);
        acc_signed(a, f[3], v[3], p1.neg_rows);
        acc_signed(a, f[4], v[4], p2.neg_rows);
        acc_signed(a, f[5], v[5], p2.neg_rows);
        acc_signed(a, f[6], v[6], p3.neg_rows);
        acc_signed(a, f[7], v[7], p3.neg_rows);
        acc_signed(a, pf, pv, pq.neg_pre);
        acc_wave_reduce(a);
        uint32_t g[8];
        acc_normalise(a, g);
#pragma unroll
        for (int q = 0; q < 4; q++) fp[q] = (uint64_t)g[2 * q] | ((uint64_t)g[2 * q + 1] << 32);
        return;
    }
    uint64_t d[4];
    wave_range_fp(in.fps, 32, in.bsums, in.ssums, b0, b1, lane, fp);
    wave_range_fp(R.contrib, 32, R.bsums, R.ssums, j0, j1, lane, d);
    fp_add256(fp, d);
}

// Segment j's view rank range [l, h), its places and its aggregate (ZERO when inverted), by one
// wave.  The bound keys' ranks are rank_x[ia * j] / rank_x[ib * j + off] (a round: starts then
// ends; the two-call path: interleaved)
template <bool Wide = true>
__device__ __forceinline__ void bounds_view_one(uint64_t j, uint32_t lane, const uint32_t *rank_b,
                                                const uint32_t *rank_j, const uint8_t *sk, const uint8_t *ek,
                                                const RoundIn &in, const RoundRun &R, uint32_t ia, uint32_t ib,
                                                uint64_t off, uint64_t *lo_out, uint64_t *hi_out, uint64_t *agg_out,
                                                uint64_t *place) {
    const uint64_t qs = ia * j, qe = ib * j + off;
    const uint64_t bs = sk[j] ? rank_b[qs] : 0, js = sk[j] ? rank_j[qs] : 0;
    const uint64_t be = ek[j] ? rank_b[qe] : R.nb, je = ek[j] ? rank_j[qe] : R.n;
    const uint64_t l = (uint64_t)((int64_t)bs + R.cntp[js]), h = (uint64_t)((int64_t)be + R.cntp[je]);
    uint64_t fp[4] = {0, 0, 0, 0};
    if (h > l) view_range_fp<Wide>(in, R, bs, js, be, je, lane, fp);  // uniform; an inverted range is ZERO
    if (lane == 0) {
        lo_out[j] = l;
        hi_out[j] = h;
        if (place) {
            place[4 * j] = bs;
            place[4 * j + 1] = js;
            place[4 * j + 2] = be;
            place[4 * j + 3] = je;
        }
        uint64_t *o = agg_out + 5 * j;
        o[0] = fp[0];
        o[1] = fp[1];
        o[2] = fp[2];
        o[3] = fp[3];
        o[4] = h > l ? h - l : 0;
    }
}

// child c (k-th of segment j) over the view: round_emit_child with the cut keys selected from
// base + run and the sums taken between places
template <bool Wide = true>
__device__ __forceinline__ void round_emit_child_view(uint64_t c, uint64_t j, uint64_t k, const RoundLayout &L,
                                                      uint32_t kl, uint32_t lane, const RoundIn &in,
                                                      const RoundRun &R, const RoundSegs &g, const uint64_t *place,
                                                      uint8_t *out) {
    uint8_t skd = in.sk[j], ekd = in.ek[j];
    const uint8_t *skey = skd ? in.skeys + j * kl : nullptr, *ekey = ekd ? in.ekeys + j * kl : nullptr;
    uint64_t *agg = reinterpret_cast<uint64_t *>(out + L.caggs) + 5 * c;
    const uint64_t ncuts = g.nch[j] - 1;
    if (g.kind[j] == 1 || ncuts == 0) {
        if (lane < 5) agg[lane] = g.kind[j] == 1 ? 0ull : g.loc[5 * j + lane];
    } else {
        const uint64_t st = g.stride[j], s0 = g.si[j];
        const uint64_t lo = s0 + k * st, hi = k == ncuts ? g.ei[j] : s0 + (k + 1) * st;
        ViewPlace a{place[4 * j], place[4 * j + 1], nullptr}, z{place[4 * j + 2], place[4 * j + 3], nullptr};
        if (k) {
            a = view_at_group<64>(R, in.bkeys, kl, lo, lane);
            skd = 1, skey = a.key;
        }
        if (k != ncuts) {
            z = view_at_group<64>(R, in.bkeys, kl, hi, lane);
            ekd = 1, ekey = z.key;
        }
        uint64_t fp[4];
        view_range_fp<Wide>(in, R, a.b, a.j, z.b, z.j, lane, fp);
        if (lane == 0) {
            agg[0] = fp[0];
            agg[1] = fp[1];
            agg[2] = fp[2];
            agg[3] = fp[3];
            agg[4] = hi - lo;
        }
    }
    if (lane == 0) {
        out[L.csk + c] = skd;
        out[L.cek + c] = ekd;
    }
    if (lane < kl / 4) {
        reinterpret_cast<uint32_t *>(out + L.cskeys + c * kl)[lane] =
            skey ? reinterpret_cast<const uint32_t *>(skey)[lane] : 0u;
        reinterpret_cast<uint32_t *>(out + L.cekeys + c * kl)[lane] =
            ekey ? reinterpret_cast<const uint32_t *>(ekey)[lane] : 0u;
    }
}

// Medium rounds (r <= ROUND_SMALL): decisions, the children / enumeration offsets (block scan)
// and the header in one workgroup, between k_round_bounds and k_round_emit -- three launches
// where the large path takes six.  Tiny rounds (r <= ROUND_TINY: one segment per wave, at most
// 16 * fan-out children) run whole in k_round_small, one launch.  Both write the per-segment
// arrays, so a round whose children outnumber cap can be emitted again by k_round_emit.
constexpr uint32_t ROUND_SMALL = 1024, ROUND_TINY = 16;

__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *wsum, uint64_t *total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    uint64_t x = v;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (uint32_t i = 0; i < nwv; i++) {
            const uint64_t t = wsum[i];
            wsum[i] = acc;
            acc += t;
        }
        *total = acc;
    }
    __syncthreads();
    return wsum[w] + x - v;
}

}  // namespace rh
