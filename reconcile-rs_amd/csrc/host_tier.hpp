// host_tier.hpp -- the store's host tier: the small questions of a reconciliation answered in
// host memory, with no device round trip.
//
// rbsr's diff path is latency-bound: a d = 1 reconciliation of a 10^6-entry
// map asks ~155 aggregate, ~152 rank and ~70 select questions (benches/README.md:579-585), each
// O(log n) on the reference's FingerprintTreeMap (query.rs:25-167), ~45 us in all.  One device
// round trip per round costs more than that.  The host tier keeps, next to the HBM-resident store,
//   - the base run: its keys in rank order and the exclusive prefix sums of its per-row
//     fingerprints, P[i] = Σ lift(row j), j < i, mod 2^256, computed on the device (launch_prefix)
//     from the fingerprints the GPU lift produced, so summary-folds-lift holds by construction
//     (rsos_trait.rs:46-60), plus the leading 8 key bytes (order-preserving) of every 64th key, so
//     a base rank is a search of a cache-resident sample array and then of one 64-key window;
//   - the delta run: every batch since the base was copied, as the signed deltas the device
//     computed for it (host_delta.hpp), folded in per batch -- O(batch), not O(n).
// A question composes the two as the device does and as FingerprintTreeMap composes its cached
// aggregates (mutate.rs:31-41, :93-154): rank(z) = rank_B(z) + Σ count deltas below z, the prefix
// of the fingerprints at z = P[rank_B(z)] + Σ contribs below z, and an aggregate is the
// difference of two prefixes -- the Fingerprint group's inverse (fingerprint.rs:159-173).  The
// base part is copied down again only when the device base changes (a compaction), not per batch.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/rsos_hip.h"
#include "host_delta.hpp"
#include "internal.hpp"
#include "round_decide.hpp"

namespace rh {

struct HostTier {
    KeyOrder ko;
    uint32_t kl = 0;
    uint64_t nb = 0;                   // base rows
    uint64_t n = 0;                    // live keys: nb + Σ count deltas
    const uint8_t *keys = nullptr;     // nb * kl bytes, rank order
    const uint64_t *prefix = nullptr;  // (nb + 1) * 4 LE limbs
    const uint64_t *samp = nullptr;    // digit(keys[64 j]), j < ns
    uint64_t ns = 0;
    std::vector<uint64_t> samp_own;    // ... when build() forms them itself
    // the index over the samples: samp2[j] = samp[64 j] = digit(keys[4096 j]), j < ns2 -- 8 bytes
    // per 4,096 keys (195 KB at 10^8), cache-resident, so a search of the samples touches a few
    // lines instead of ~10 cold ones (the sample array is 12.5 MB at 10^8)
    const uint64_t *samp2 = nullptr;
    uint64_t ns2 = 0;
    std::vector<uint64_t> samp2_own;
    DeltaTree dt;
    static constexpr unsigned SHIFT = 6;
    // A copy of the device's delta run (the run copy), taken after a batch too large for the
    // tree: its entries in key order, each the DeltaRec the device keeps for the key (the
    // contribution cur - base and the count delta live - in_base relative to the base, its flags
    // and its base rank), with exclusive prefix sums of both, all formed on the device
    // (rsos_hip_abi.hip tier_run_snapshot).  Base + run copy (the *view*) is the whole map, as the
    // device's base + delta run is; later small batches fold into the tree as deltas against the
    // view (entry_vs_base), and the next run copy absorbs them.
    struct Run {
        uint64_t n = 0;
        const uint8_t *keys = nullptr;      // n * kl, key order
        const uint64_t *prefix = nullptr;   // (n + 1) * 4 limbs: Σ contribs of entries [0, i)
        const int32_t *cntp = nullptr;      // n + 1: Σ count deltas of entries [0, i)
        const uint8_t *flags = nullptr;     // n: DeltaRec flags (1 in the base, 2 live)
        const uint32_t *brank = nullptr;    // n: base rows below the key
        const uint64_t *samp = nullptr, *samp2 = nullptr;  // digits of every 64th / 4096th key
        // G(64 k) = live keys <= entry 64 k (brank + cntp + live), k < ns: select's index (nullable)
        const uint64_t *gsamp = nullptr;
        uint64_t ns = 0, ns2 = 0;
    };
    Run run;
    // select's index over the run copy's G samples: every 64th of them (8 B per 4,096 entries,
    // cache-resident), so a select reads a few lines of gsamp instead of binary-searching all of it
    // (at 1.6 x 10^7 run entries gsamp is 2 MB: ~18 dependent misses a select)
    std::vector<uint64_t> gsamp2_own;
    bool has_run() const { return run.n != 0; }
    // hold a run copy (replacing the tree: the run holds every change since the base copy)
    void set_run(const Run &r) {
        run = r;
        run.ns = (r.n + 63) >> SHIFT;
        run.ns2 = (run.ns + 63) >> SHIFT;
        gsamp2_own.clear();
        if (r.gsamp && run.ns > 64) {
            gsamp2_own.resize(run.ns2);
            for (uint64_t k = 0; k < run.ns2; k++) gsamp2_own[k] = r.gsamp[k << SHIFT];
        }
        dt.clear();
        nv = n = (uint64_t)((int64_t)nb + (r.n ? r.cntp[r.n] : 0));
    }
    uint64_t nv = 0;  // live keys of the view (base + run copy)

    uint64_t digit(const uint8_t *k) const { return ko.digit(k); }
    int cmp(const uint8_t *a, const uint8_t *b) const { return ko.cmp(a, b); }
    // smp (optional): the samples, formed on the device with the copy (k_sample, stride 64), and
    // smp2 (optional) their index (stride 4096)
    void build(uint32_t key_len, int key_kind, uint64_t rows, const uint8_t *k, const uint64_t *p,
               const uint64_t *smp = nullptr, const uint64_t *smp2 = nullptr) {
        ko = KeyOrder{key_len, key_kind};
        kl = key_len;
        nb = n = nv = rows;
        keys = k;
        prefix = p;
        dt.set_order(ko);
        samp_own.clear();
        samp2_own.clear();
        run = Run{};
        gsamp2_own.clear();
        samp = samp2 = nullptr;
        ns = ns2 = 0;
        if (!keys) return;  // the encoded store keeps its keys on the host side of the ABI
        ns = (nb + 63) >> SHIFT;
        ns2 = (ns + 63) >> SHIFT;
        if (smp) {
            samp = smp;
        } else {
            samp_own.resize(ns);
            for (uint64_t j = 0; j < ns; j++) samp_own[j] = digit(keys + (j << SHIFT) * kl);
            samp = samp_own.data();
        }
        if (smp2) {
            samp2 = smp2;
        } else {
            samp2_own.resize(ns2);
            for (uint64_t j = 0; j < ns2; j++) samp2_own[j] = samp[j << SHIFT];
            samp2 = samp2_own.data();
        }
    }
    // a window's cache lines requested at once (at 10^8 rows the windows are cold: the binary search
    // in them would otherwise wait for each line in turn)
    static void prefetch_span(const void *p, size_t bytes) {
        const char *c = static_cast<const char *>(p);
        for (size_t o = 0; o < bytes; o += 64) __builtin_prefetch(c + o);
    }
    // the first sample >= d (> d with upper), through the index: samp[64 (i - 1)] < d (<= d) and
    // samp[64 i] >= d (> d) bound a window of 63 samples
    static uint64_t samp_bound(const uint64_t *samp, uint64_t ns, const uint64_t *samp2, uint64_t ns2, uint64_t d,
                               bool upper, uint64_t from = 0) {
        const uint64_t i = upper ? std::upper_bound(samp2, samp2 + ns2, d) - samp2
                                 : std::lower_bound(samp2, samp2 + ns2, d) - samp2;
        const uint64_t lo = std::max<uint64_t>(from, i ? ((i - 1) << SHIFT) + 1 : 0);
        const uint64_t hi = std::min<uint64_t>(ns, i << SHIFT);
        if (lo >= hi) return lo;  // the window is empty: the bound is its start
        prefetch_span(samp + lo, (hi - lo) * 8);
        return upper ? std::upper_bound(samp + lo, samp + hi, d) - samp : std::lower_bound(samp + lo, samp + hi, d) - samp;
    }
    // keys below `key` among n sorted keys with those samples: the samples narrow it to one window
    // of 64 keys (or the run of keys sharing its digit), then a binary search
    uint64_t sampled_lb(const uint8_t *ks, uint64_t nk, const uint64_t *sp, uint64_t nsp, const uint64_t *sp2,
                        uint64_t nsp2, const uint8_t *key) const {
        if (nk == 0) return 0;
        const uint64_t d = digit(key);
        const uint64_t jl = samp_bound(sp, nsp, sp2, nsp2, d, false);
        const uint64_t jh = samp_bound(sp, nsp, sp2, nsp2, d, true, jl);
        uint64_t lo = jl ? ((jl - 1) << SHIFT) + 1 : 0;     // keys[64 (jl - 1)] < key
        uint64_t hi = std::min<uint64_t>(nk, jh << SHIFT);  // keys[64 jh] > key
        if (hi - lo <= 64) prefetch_span(ks + lo * kl, (hi - lo) * kl);
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (cmp(ks + mid * kl, key) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // ---- the same searches for many keys at once: each phase's cache lines are requested for every
    // key before any is read, so the keys' dependent misses overlap (a round's 2r bounds at 10^8 rows
    // were ~4 dependent DRAM misses each, one key after another) -----------------------------------
    struct SampWin {
        uint64_t d, ll, lh, ul, uh;  // the digit, the lower and upper bounds' sample windows
    };
    static SampWin samp_windows(const uint64_t *samp, uint64_t ns, const uint64_t *samp2, uint64_t ns2, uint64_t d) {
        const uint64_t i = std::lower_bound(samp2, samp2 + ns2, d) - samp2;
        const uint64_t iu = std::upper_bound(samp2, samp2 + ns2, d) - samp2;
        SampWin w{d, i ? ((i - 1) << SHIFT) + 1 : 0, std::min<uint64_t>(ns, i << SHIFT),
                  iu ? ((iu - 1) << SHIFT) + 1 : 0, std::min<uint64_t>(ns, iu << SHIFT)};
        if (w.lh > w.ll) prefetch_span(samp + w.ll, (w.lh - w.ll) * 8);
        if (w.uh > w.ul && w.ul != w.ll) prefetch_span(samp + w.ul, (w.uh - w.ul) * 8);
        return w;
    }
    // sampled_lb's key window [lo, hi) from the windows (its lines requested)
    void key_window(const uint8_t *ks, uint64_t nk, const uint64_t *samp, const SampWin &w, uint64_t *lo,
                    uint64_t *hi) const {
        const uint64_t jl = w.ll >= w.lh ? w.ll : std::lower_bound(samp + w.ll, samp + w.lh, w.d) - samp;
        const uint64_t ul = std::max<uint64_t>(jl, w.ul);
        const uint64_t jh = ul >= w.uh ? ul : std::upper_bound(samp + ul, samp + w.uh, w.d) - samp;
        *lo = jl ? ((jl - 1) << SHIFT) + 1 : 0;
        *hi = std::min<uint64_t>(nk, jh << SHIFT);
        if (*hi - *lo <= 64) prefetch_span(ks + *lo * kl, (*hi - *lo) * kl);
    }
    uint64_t key_search(const uint8_t *ks, uint64_t lo, uint64_t hi, const uint8_t *key) const {
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (cmp(ks + mid * kl, key) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // view_lt(z[k], false) for m keys: b[k], j[k] (no tree)
    std::vector<SampWin> bw_, rw_;
    std::vector<uint64_t> blo_, bhi_, rlo_, rhi_;
    void view_lt_batch(const uint8_t *const *z, size_t m, uint64_t *b, uint64_t *j) {
        bw_.resize(m), rw_.resize(m), blo_.resize(m), bhi_.resize(m), rlo_.resize(m), rhi_.resize(m);
        const bool run_on = has_run();
        for (size_t k = 0; k < m; k++) {
            const uint64_t d = digit(z[k]);
            if (nb) bw_[k] = samp_windows(samp, ns, samp2, ns2, d);
            if (run_on) rw_[k] = samp_windows(run.samp, run.ns, run.samp2, run.ns2, d);
        }
        for (size_t k = 0; k < m; k++) {
            if (nb) key_window(keys, nb, samp, bw_[k], &blo_[k], &bhi_[k]);
            if (run_on) key_window(run.keys, run.n, run.samp, rw_[k], &rlo_[k], &rhi_[k]);
        }
        for (size_t k = 0; k < m; k++) {
            b[k] = nb ? key_search(keys, blo_[k], bhi_[k], z[k]) : 0;
            j[k] = run_on ? key_search(run.keys, rlo_[k], rhi_[k], z[k]) : 0;
        }
    }
    // view_at for m ranks (each < nv): their places and keys
    std::vector<uint64_t> alo_, ahi_;
    void view_at_batch(const uint64_t *v, size_t m, uint64_t *b, uint64_t *j, const uint8_t **key) {
        if (!has_run() || !run.gsamp) {
            for (size_t k = 0; k < m; k++) key[k] = view_at(v[k], b[k], j[k]);
            return;
        }
        alo_.resize(m), ahi_.resize(m);
        for (size_t k = 0; k < m; k++) {  // the first sampled entry with G > v: its window's entries requested
            uint64_t q;
            if (!gsamp2_own.empty()) {
                const uint64_t *g2 = gsamp2_own.data();
                const uint64_t i = std::upper_bound(g2, g2 + gsamp2_own.size(), v[k]) - g2;
                const uint64_t l2 = i ? ((i - 1) << SHIFT) + 1 : 0, h2 = std::min<uint64_t>(run.ns, i << SHIFT);
                q = l2 >= h2 ? h2 : std::upper_bound(run.gsamp + l2, run.gsamp + h2, v[k]) - run.gsamp;
            } else {
                q = std::upper_bound(run.gsamp, run.gsamp + run.ns, v[k]) - run.gsamp;
            }
            alo_[k] = q ? ((q - 1) << SHIFT) + 1 : 0;
            ahi_[k] = std::min<uint64_t>(run.n, q << SHIFT);
            const uint64_t lo = alo_[k] ? alo_[k] - 1 : 0, cnt = ahi_[k] - lo + 1;
            prefetch_span(run.brank + lo, cnt * 4);
            prefetch_span(run.cntp + lo, cnt * 4);
            prefetch_span(run.flags + lo, cnt);
        }
        for (size_t k = 0; k < m; k++) {
            uint64_t lo = alo_[k], hi = ahi_[k];
            while (lo < hi) {
                const uint64_t mid = (lo + hi) >> 1;
                if (run_below(mid) + (run_live(mid) ? 1 : 0) > v[k]) hi = mid;
                else lo = mid + 1;
            }
            j[k] = lo;
            if (lo < run.n && run_below(lo) == v[k] && run_live(lo)) {
                b[k] = run.brank[lo];
                key[k] = run.keys + lo * kl;
            } else {
                const uint64_t gprev = lo ? run_below(lo - 1) + (run_live(lo - 1) ? 1 : 0) : 0;
                const uint64_t b0 = lo ? run.brank[lo - 1] + (run_in_base(lo - 1) ? 1 : 0) : 0;
                b[k] = b0 + (v[k] - gprev);
                key[k] = keys + b[k] * kl;
            }
            __builtin_prefetch(key[k]);
        }
    }
    // the prefix sums' lines of places (b, j), requested
    void prefetch_pre(uint64_t b, uint64_t j) const {
        __builtin_prefetch(prefix + 4 * b);
        if (has_run()) __builtin_prefetch(run.prefix + 4 * j);
    }

    // forget everything (tier off)
    void reset() {
        build(0, RH_KEY_BYTES, 0, nullptr, nullptr);
        gsamp2_own = std::vector<uint64_t>();
        samp_own = std::vector<uint64_t>();
        samp2_own = std::vector<uint64_t>();
        segs = std::vector<Seg>();
    }
    bool plain() const { return dt.size() == 0; }
    // Whether the view holds key, and its fingerprint (the run's entry if it has one, else the base)
    bool view_find(const uint8_t *key, uint64_t fp[4]) const {
        if (has_run()) {
            const uint64_t j = rank_run(key);
            if (j < run.n && cmp(run.keys + j * kl, key) == 0) {
                if (!run_live(j)) return false;
                memcpy(fp, run.prefix + 4 * (j + 1), 32);  // contrib = cur - base
                fp4_sub(fp, run.prefix + 4 * j);
                if (run_in_base(j)) {
                    fp4_add(fp, prefix + 4 * (run.brank[j] + 1));
                    fp4_sub(fp, prefix + 4 * run.brank[j]);
                }
                return true;
            }
        }
        const uint64_t b = rank_b(key);
        if (b < nb && cmp(keys + b * kl, key) == 0) {
            memcpy(fp, prefix + 4 * (b + 1), 32);
            fp4_sub(fp, prefix + 4 * b);
            return true;
        }
        return false;
    }
    // One batch row's entry formed against this tier's own view (its base, and its run copy when
    // held): the rule of k_delta_build (store_kernels.hip) -- an upsert is (cur - view, 1 - in_view,
    // live), a delete of a view key (-view, -1, dead), a delete of any other key drops the key's
    // entry (returns true).  cur == nullptr: a delete.
    bool entry_vs_base(const uint8_t *key, const uint64_t *cur, DeltaTree::Rec *r) const {
        uint64_t v[4] = {0, 0, 0, 0};
        const bool in_v = view_find(key, v);
        r->key = key;
        if (cur) memcpy(r->fp, cur, 32);
        else memset(r->fp, 0, 32);
        if (in_v) fp4_sub(r->fp, v);
        r->cnt = (int8_t)((cur ? 1 : 0) - (in_v ? 1 : 0));
        r->live = cur != nullptr;
        return !cur && !in_v;
    }
    // m sorted, distinct rows into the delta tree; drop[j]: remove row j's key.  A batch large
    // against the tree is one merge pass over the whole tree instead of m walks.
    void fold(const DeltaTree::Rec *rows, const uint8_t *drop, size_t m) {
        if (m > 256 && m * 16 > dt.size()) {
            dt.merge_rebuild(rows, drop, m);
        } else {
            for (size_t j = 0; j < m; j++) {
                if (drop[j]) dt.erase(rows[j].key);
                else dt.upsert(rows[j]);
            }
        }
        n = (uint64_t)((int64_t)nv + dt.cnt_total());
    }

    // base rows with key < z
    uint64_t rank_b(const uint8_t *key) const { return sampled_lb(keys, nb, samp, ns, samp2, ns2, key); }
    // run entries with key < z
    uint64_t rank_run(const uint8_t *key) const {
        return sampled_lb(run.keys, run.n, run.samp, run.ns, run.samp2, run.ns2, key);
    }

    // ---- the view: the base copy, merged with the run copy when one is held ----------------------
    // A place in it: b base rows and j run entries below; the live view keys below are then
    // b + Σ count deltas of those run entries.
    bool run_live(uint64_t j) const { return run.flags[j] & 2; }
    bool run_in_base(uint64_t j) const { return run.flags[j] & 1; }
    uint64_t run_below(uint64_t j) const { return (uint64_t)((int64_t)run.brank[j] + run.cntp[j]); }
    uint64_t view_rank(uint64_t b, uint64_t j) const {
        return has_run() ? (uint64_t)((int64_t)b + run.cntp[j]) : b;
    }
    // view keys < z (le: <= z)
    void view_lt(const uint8_t *z, bool le, uint64_t &b, uint64_t &j) const {
        b = rank_b(z);
        if (le && b < nb && cmp(keys + b * kl, z) == 0) b++;
        j = 0;
        if (has_run()) {
            j = rank_run(z);
            if (le && j < run.n && cmp(run.keys + j * kl, z) == 0) j++;
        }
    }
    // the view key of rank v < nv, with its place.  G(j) = live view keys <= run entry j = brank +
    // cntp + live, non-decreasing; the first entry with G(j) > v is that key itself, or the key is
    // an untouched base row between entries j - 1 and j (those rows are consecutive)
    const uint8_t *view_at(uint64_t v, uint64_t &b, uint64_t &j) const {
        if (!has_run()) {
            b = v, j = 0;
            return keys + v * kl;
        }
        uint64_t lo = 0, hi = run.n;
        if (run.gsamp) {  // the first sampled entry with G > v bounds a window of 64 entries
            uint64_t k;
            if (!gsamp2_own.empty()) {  // through the index: gsamp[64 (i - 1)] <= v < gsamp[64 i]
                const uint64_t *g2 = gsamp2_own.data();
                const uint64_t i = std::upper_bound(g2, g2 + gsamp2_own.size(), v) - g2;
                const uint64_t l2 = i ? ((i - 1) << SHIFT) + 1 : 0, h2 = std::min<uint64_t>(run.ns, i << SHIFT);
                if (h2 > l2) prefetch_span(run.gsamp + l2, (h2 - l2) * 8);
                k = l2 >= h2 ? h2 : std::upper_bound(run.gsamp + l2, run.gsamp + h2, v) - run.gsamp;
            } else {
                k = std::upper_bound(run.gsamp, run.gsamp + run.ns, v) - run.gsamp;
            }
            lo = k ? ((k - 1) << SHIFT) + 1 : 0;         // G(64 (k - 1)) <= v
            hi = std::min<uint64_t>(run.n, k << SHIFT);  // G(64 k) > v (or the end)
        }
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (run_below(mid) + (run_live(mid) ? 1 : 0) > v) hi = mid;
            else lo = mid + 1;
        }
        j = lo;
        if (j < run.n && run_below(j) == v && run_live(j)) {
            b = run.brank[j];
            return run.keys + j * kl;
        }
        const uint64_t gprev = j ? run_below(j - 1) + (run_live(j - 1) ? 1 : 0) : 0;
        const uint64_t b0 = j ? run.brank[j - 1] + (run_in_base(j - 1) ? 1 : 0) : 0;
        b = b0 + (v - gprev);
        return keys + b * kl;
    }
    // in-order walk of the view from a place: the next live key (nullptr at the end) and a step
    // past it.  A run entry comes before base row b when b >= its base rank; one in the base
    // replaces that row, a dead one is skipped.
    const uint8_t *view_peek(uint64_t &b, uint64_t &j) const {
        while (j < run.n && b >= run.brank[j] && !run_live(j)) {
            if (run_in_base(j)) b++;
            j++;
        }
        if (j < run.n && b >= run.brank[j]) return run.keys + j * kl;
        return b < nb ? keys + b * kl : nullptr;
    }
    void view_step(uint64_t &b, uint64_t &j) const {
        if (j < run.n && b >= run.brank[j]) {
            if (run_in_base(j)) b++;
            j++;
        } else {
            b++;
        }
    }

    // A place in the merged key order (the view + the tree): r live keys below it; b, j its place
    // in the view; d tree entries below it; k = the live key at rank r (set by at(), r < n).
    struct Cur {
        uint64_t r = 0, b = 0, d = 0;
        const uint8_t *k = nullptr;
        uint64_t j = 0;
    };
    Cur begin() const { return Cur{0, 0, 0, nullptr, 0}; }
    Cur end() const { return Cur{n, nb, dt.size(), nullptr, run.n}; }
    // keys < z (le: keys <= z)
    Cur place(const uint8_t *z, bool le) const {
        Cur c;
        view_lt(z, le, c.b, c.j);
        c.r = view_rank(c.b, c.j);
        if (plain()) return c;
        const DeltaTree::Pos p = dt.lt(z);
        c.d = p.idx + (le && p.found ? 1 : 0);
        c.r = (uint64_t)((int64_t)c.r + p.cnt + (le && p.found ? p.fcnt : 0));
        return c;
    }
    Cur lt(const uint8_t *z) const { return place(z, false); }
    Cur le(const uint8_t *z) const { return place(z, true); }
    // select: the place of the r-th live key (r <= n; r == n is end())
    Cur at(uint64_t r) const {
        if (r >= n) return end();
        Cur c;
        if (plain()) {
            c.k = view_at(r, c.b, c.j);
            c.r = r;
            return c;
        }
        // F(v) = live keys <= view key v, non-decreasing in v; find the smallest v with F(v) > r.
        // |F(v) - v| <= tree entries + 1 brackets the search.
        const uint64_t nt = dt.size();
        uint64_t lo = r > nt ? r - nt : 0, hi = std::min<uint64_t>(nv, r + nt + 1);
        auto F = [&](uint64_t v, DeltaTree::Pos *pp, Cur *vc) {
            uint64_t b, j;
            const uint8_t *k = view_at(v, b, j);
            const DeltaTree::Pos p = dt.lt(k);
            if (pp) *pp = p;
            if (vc) vc->b = b, vc->j = j, vc->k = k;
            return (uint64_t)((int64_t)v + 1 + p.cnt + (p.found ? p.fcnt : 0));
        };
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (F(mid, nullptr, nullptr) > r) hi = mid;
            else lo = mid + 1;
        }
        const uint64_t v = lo;
        if (v < nv) {
            DeltaTree::Pos p;
            const uint64_t f = F(v, &p, &c);
            const bool live = !p.found || p.flive;
            if (live && f - 1 == r) {
                c.r = r;
                c.d = p.idx;
                return c;
            }
        }
        // the r-th live key is an inserted tree key between view keys v - 1 and v: every tree
        // entry in that gap is one (a key not in the view is in the tree only while live)
        uint64_t fprev = 0, d0 = 0;
        if (v > 0) {
            DeltaTree::Pos q;
            fprev = F(v - 1, &q, nullptr);
            d0 = q.idx + (q.found ? 1 : 0);
        }
        const uint64_t d = d0 + (r - fprev);
        const uint8_t *k = dt.key_at(d);
        view_lt(k, false, c.b, c.j);
        c.r = r, c.d = d, c.k = k;
        return c;
    }
    // Σ fingerprints of the live keys below c
    void pre(const Cur &c, uint64_t out[4]) const {
        memcpy(out, prefix + 4 * c.b, 32);
        if (has_run()) fp4_add(out, run.prefix + 4 * c.j);
        if (!plain() && c.d) {
            uint64_t t[4];
            dt.fp_prefix(c.d, t);
            fp4_add(out, t);
        }
    }
    // aggregate between two places (ZERO when hi is below lo: the inverted range)
    void agg(const Cur &lo, const Cur &hi, rh_aggregate *o) const {
        if (hi.r <= lo.r) {
            memset(o, 0, sizeof *o);
            return;
        }
        uint64_t a[4], b[4];
        pre(hi, a);
        pre(lo, b);
        fp4_sub(a, b);
        memcpy(o->fingerprint, a, 32);
        o->size = hi.r - lo.r;
    }
    // rank(z) = number of keys strictly below z (query.rs:93-121)
    uint64_t rank(const uint8_t *key) const { return lt(key).r; }
    // Aggregate over rank range [lo, hi), clamped as the device query clamps (hi <= n, lo <= hi)
    void agg(uint64_t lo, uint64_t hi, rh_aggregate *o) const {
        if (hi > n) hi = n;
        if (lo > hi) lo = hi;
        if (plain() && !has_run()) {
            uint64_t a[4];
            memcpy(a, prefix + 4 * hi, 32);
            fp4_sub(a, prefix + 4 * lo);
            memcpy(o->fingerprint, a, 32);
            o->size = hi - lo;
            return;
        }
        agg(at(lo), at(hi), o);
    }
    // place of a bound: kind 0 = unbounded (lower: begin, upper: end), 1 = included, 2 = excluded
    Cur bound(int kind, const uint8_t *key, bool lower) const {
        if (kind == 0) return lower ? begin() : end();
        if (lower) return kind == 1 ? lt(key) : le(key);  // Included(k): k.., Excluded(k): k is out
        return kind == 2 ? lt(key) : le(key);             // Excluded(k): ..k, Included(k): ..=k
    }
    // the keys of ranks [lo, hi) (hi <= n), in order
    void copy_keys(uint64_t lo, uint64_t hi, uint8_t *out) const {
        if (hi <= lo) return;
        if (plain() && !has_run()) {
            memcpy(out, keys + lo * kl, (hi - lo) * kl);
            return;
        }
        const Cur c = at(lo);
        uint64_t b = c.b, j = c.j;
        DeltaTree::Iter it = dt.iter(c.d);
        for (uint64_t r = lo; r < hi;) {
            const uint8_t *vk = view_peek(b, j);
            const int s = !it.l ? -1 : !vk ? 1 : cmp(vk, it.key());
            if (s < 0) {  // a view key the tree does not touch
                memcpy(out, vk, kl);
                out += kl, r++;
                view_step(b, j);
            } else {
                if (it.live()) {  // inserted (s > 0) or overwritten (s == 0)
                    memcpy(out, it.key(), kl);
                    out += kl, r++;
                }
                if (s == 0) view_step(b, j);
                it.advance();
            }
        }
    }

    // ---- one protocol round (protocol_round_with_policy, rbsr/src/protocol.rs:212-317) ------------
    // The same decisions as the device path (round_decide, aggregate_kernels.hip; on the host
    // decide_segment, round_decide.hpp) and the same output layout (round_layout).
    struct Seg {
        int kind;  // 0 skip, 1 IDLIST, 2 SPLIT, 3 dropped
        uint64_t stride, children, enums;
        Cur cs, ce;
        rh_aggregate loc;
    };
    std::vector<Seg> segs;
    bool batch = true;  // rounds over base + run copy with the batched searches (false: key by key)
    std::vector<const uint8_t *> bq_;
    std::vector<uint64_t> bb_, bj_, cut_r_, cut_b_, cut_j_;
    std::vector<const uint8_t *> cut_k_;
    std::vector<Cur> cuts_;
    void round(int sqrt_policy, uint64_t b, const rh_segments &in, std::vector<uint8_t> &out, uint64_t hdr[5]) {
        if (batch && keys && in.n > 1) return round_batched(sqrt_policy, b, in, out, hdr);
        const size_t r = in.n;
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        segs.resize(r);
        uint64_t nc = 0, ne = 0, cnt[5] = {0, 0, 0, 0, 0};
        for (size_t j = 0; j < r; j++) {
            Seg &g = segs[j];
            g = Seg{3, 0, 0, 0, sk[j] ? lt(skeys + j * kl) : begin(), ek[j] ? lt(ekeys + j * kl) : end(), {}};
            agg(g.cs, g.ce, &g.loc);
            const SegDecision d = decide_segment(g.cs.r, g.ce.r, g.loc, in.aggregates[j], sqrt_policy, b);
            g.kind = d.kind, g.stride = d.stride, g.children = d.children, g.enums = d.enums;
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
                Cur lo = g.cs;
                for (uint64_t k = 0; k <= ncuts; k++) {
                    const Cur hi = k == ncuts ? g.ce : at(g.cs.r + (k + 1) * g.stride);
                    rh_aggregate a;
                    agg(lo, hi, &a);
                    child(k ? 1 : sk[j], k ? lo.k : s0, k != ncuts ? 1 : ek[j], k != ncuts ? hi.k : e0, a);
                    lo = hi;
                }
            }
        }
    }
    // round() with the segments' bounds, their sums and (with no tree) the SPLIT cuts each as one
    // batch of searches (view_lt_batch, view_at_batch), the prefix lines requested before they are
    // read; a tree adds its own (cached) search per bound and keeps select key by key.  The same
    // answers as the key-by-key path (tests/host_tier_check.cpp compares the two).
    void round_batched(int sqrt_policy, uint64_t b, const rh_segments &in, std::vector<uint8_t> &out, uint64_t hdr[5]) {
        const size_t r = in.n;
        const uint8_t *sk = in.start_kinds, *ek = in.end_kinds;
        const uint8_t *skeys = static_cast<const uint8_t *>(in.start_keys);
        const uint8_t *ekeys = static_cast<const uint8_t *>(in.end_keys);
        segs.resize(r);
        bq_.clear();
        for (size_t j = 0; j < r; j++) {
            if (sk[j]) bq_.push_back(skeys + j * kl);
            if (ek[j]) bq_.push_back(ekeys + j * kl);
        }
        const size_t q = bq_.size();
        bb_.resize(q), bj_.resize(q);
        view_lt_batch(bq_.data(), q, bb_.data(), bj_.data());
        for (size_t k = 0; k < q; k++) prefetch_pre(bb_[k], bj_[k]);
        uint64_t nc = 0, ne = 0, cnt[5] = {0, 0, 0, 0, 0};
        size_t qi = 0;
        cut_r_.clear();
        const bool tree = !plain();
        auto bound_place = [&](Cur &c) {  // lt(key) from its view place (+ the tree's entries below it)
            c.r = view_rank(c.b, c.j), c.d = 0, c.k = nullptr;
            if (tree) {
                const DeltaTree::Pos p = dt.lt(bq_[qi]);
                c.d = p.idx;
                c.r = (uint64_t)((int64_t)c.r + p.cnt);
            }
        };
        for (size_t j = 0; j < r; j++) {
            Seg &g = segs[j];
            Cur cs = begin(), ce = end();
            if (sk[j]) cs.b = bb_[qi], cs.j = bj_[qi], bound_place(cs), qi++;
            if (ek[j]) ce.b = bb_[qi], ce.j = bj_[qi], bound_place(ce), qi++;
            g = Seg{3, 0, 0, 0, cs, ce, {}};
            agg(g.cs, g.ce, &g.loc);
            const SegDecision d = decide_segment(g.cs.r, g.ce.r, g.loc, in.aggregates[j], sqrt_policy, b);
            g.kind = d.kind, g.stride = d.stride, g.children = d.children, g.enums = d.enums;
            cnt[g.kind == 3 ? 4 : g.kind]++;
            nc += g.children;
            ne += g.enums;
            if (g.kind == 2 && g.children > 1)
                for (uint64_t k = 0; k + 1 < g.children; k++) cut_r_.push_back(g.cs.r + (k + 1) * g.stride);
        }
        const size_t nq = cut_r_.size();
        cuts_.resize(nq);
        if (!tree) {
            cut_b_.resize(nq), cut_j_.resize(nq), cut_k_.resize(nq);
            view_at_batch(cut_r_.data(), nq, cut_b_.data(), cut_j_.data(), cut_k_.data());
            for (size_t k = 0; k < nq; k++) {
                cuts_[k] = Cur{cut_r_[k], cut_b_[k], 0, cut_k_[k], cut_j_[k]};
                prefetch_pre(cut_b_[k], cut_j_[k]);
            }
        } else {
            for (size_t k = 0; k < nq; k++) cuts_[k] = at(cut_r_[k]);
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
        size_t ci = 0;
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
                Cur lo = g.cs;
                for (uint64_t k = 0; k <= ncuts; k++) {
                    const Cur hi = k == ncuts ? g.ce : cuts_[ci++];
                    rh_aggregate a;
                    agg(lo, hi, &a);
                    child(k ? 1 : sk[j], k ? lo.k : s0, k != ncuts ? 1 : ek[j], k != ncuts ? hi.k : e0, a);
                    lo = hi;
                }
            }
        }
    }
};

}  // namespace rh
