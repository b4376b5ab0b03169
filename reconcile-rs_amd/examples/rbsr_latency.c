/*
 * rbsr_latency.c -- the reference's `reconciliation_drive` (benches/protocol.rs:455-520, :917-940)
 * through the C ABI: one whole FixedFanOut(16) reconciliation between two stores, timed on the
 * host clock, plus the per-question costs of Rsos::aggregate / rank through the same ABI.
 *
 *   rbsr_latency <n> <d> <reps> <host_tier 0|1> [write_rows]
 *
 * write_rows > 0: every repetition first writes write_rows fresh records into both replicas
 * (rh_store_stage, the Rsos::insert path of the Rust binding), then reconciles: the write -> round
 * cycle of a replica that merges updates and then answers rounds (src/replica/dispatch.rs:188-196).
 * The write half (staging + the batch each store applies on its next question) and the round half
 * are timed separately; the host tier folds each batch instead of copying the map again.
 *
 * Stores as the reference bench builds them (benches/protocol.rs:198-232): FingerprintTreeMap<u64,
 * u64> with keys 0..n and values key * 2654435761 (wrapping); the second store lacks d keys
 * scattered at (n / (d + 1)) * i, i = 1..d.  One reconciliation = initial_ranges(a), then rounds
 * alternating responder b, a, b, ... until no segment is left; each round encodes the active
 * segments with the gossip wire codec (bincode varint, as `reconcile` does before every round),
 * answers them (rh_store_protocol_round), and enumerates every IDLIST range's keys (the
 * responder's Enumerate).  Prints one JSON object.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/rsos_hip.h"

#define CHECK(call)                                                                      \
    do {                                                                                 \
        int rc_ = (call);                                                                \
        if (rc_ != RH_OK) {                                                              \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, rh_last_error());        \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int cmp_d(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

/* a round's segments, owned by the driver (copied out of the store's buffers) */
typedef struct {
    uint8_t *sk, *ek;
    uint64_t *skey, *ekey;
    rh_aggregate *agg;
    size_t n, cap;
} segs_t;

static void segs_reserve(segs_t *s, size_t n) {
    if (n <= s->cap) return;
    s->cap = n * 2;
    s->sk = realloc(s->sk, s->cap);
    s->ek = realloc(s->ek, s->cap);
    s->skey = realloc(s->skey, s->cap * 8);
    s->ekey = realloc(s->ekey, s->cap * 8);
    s->agg = realloc(s->agg, s->cap * sizeof(rh_aggregate));
    if (!s->sk || !s->ek || !s->skey || !s->ekey || !s->agg) {
        fprintf(stderr, "out of memory\n");
        exit(2);
    }
}

static void segs_copy(segs_t *dst, const rh_segments *src) {
    segs_reserve(dst, src->n + 1);
    dst->n = src->n;
    memcpy(dst->sk, src->start_kinds, src->n);
    memcpy(dst->ek, src->end_kinds, src->n);
    memcpy(dst->skey, src->start_keys, src->n * 8);
    memcpy(dst->ekey, src->end_keys, src->n * 8);
    memcpy(dst->agg, src->aggregates, src->n * sizeof(rh_aggregate));
}

typedef struct {
    uint64_t rounds, ranges, idlists, enumerated, wire_bytes;
} cost_t;

static uint8_t *wire;
static size_t wire_cap;
static uint64_t *enum_keys;
static size_t enum_cap;

static cost_t reconcile(rh_store *a, rh_store *b, const rh_schema *sc) {
    cost_t c = {0, 0, 0, 0, 0};
    static segs_t active;
    segs_reserve(&active, 1);
    /* initial_ranges(a) (rbsr/src/protocol.rs:97-102): the whole key space with a's root */
    active.n = 1;
    active.sk[0] = active.ek[0] = 0;
    active.skey[0] = active.ekey[0] = 0;
    CHECK(rh_store_aggregate_keys(a, 0, NULL, 0, NULL, &active.agg[0]));
    int responder_b = 1;
    while (active.n) {
        size_t len = 0;
        CHECK(rh_wire_encode_range_aggregates(sc, RH_FORM_ARRAY, -1, active.sk, active.skey, active.ek, active.ekey,
                                              active.agg, active.n, NULL, 0, &len));
        if (len > wire_cap) {
            wire_cap = 2 * len;
            wire = realloc(wire, wire_cap);
        }
        CHECK(rh_wire_encode_range_aggregates(sc, RH_FORM_ARRAY, -1, active.sk, active.skey, active.ek, active.ekey,
                                              active.agg, active.n, wire, wire_cap, &len));
        c.rounds++;
        c.ranges += active.n;
        c.wire_bytes += len;
        rh_store *resp = responder_b ? b : a;
        const rh_segments in = {active.sk, active.skey, active.ek, active.ekey, active.agg, active.n, active.n};
        rh_segments ch, en;
        rh_round_outcome oc;
        CHECK(rh_store_protocol_round(resp, RH_POLICY_FIXED_FAN_OUT, 16, &in, &ch, &en, &oc));
        segs_copy(&active, &ch);
        c.idlists += en.n;
        /* Enumerate every IDLIST range on the responder (the keys it would ship) */
        const uint8_t *esk = en.start_kinds, *eek = en.end_kinds;
        const uint64_t *eskey = (const uint64_t *)en.start_keys, *eekey = (const uint64_t *)en.end_keys;
        for (size_t j = 0; j < en.n; j++) {
            uint64_t lo = 0, hi = 0, size = 0, q[2], rk[2];
            size_t nq = 0;
            CHECK(rh_store_len(resp, &size));
            hi = size;
            if (esk[j]) q[nq++] = eskey[j];
            if (eek[j]) q[nq++] = eekey[j];
            if (nq) CHECK(rh_store_ranks(resp, q, nq, rk)); /* both bounds' ranks in one question */
            if (esk[j]) lo = rk[0];
            if (eek[j]) hi = rk[nq - 1];
            if (hi > lo) {
                if (hi - lo > enum_cap) {
                    enum_cap = 2 * (hi - lo);
                    enum_keys = realloc(enum_keys, enum_cap * 8);
                }
                CHECK(rh_store_keys(resp, lo, hi, enum_keys));
                c.enumerated += hi - lo;
            }
        }
        responder_b = !responder_b;
    }
    return c;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: rbsr_latency <n> <d> <reps> <host_tier 0|1> [write_rows]\n");
        return 1;
    }
    const uint64_t n = strtoull(argv[1], NULL, 10), d = strtoull(argv[2], NULL, 10);
    const int reps = atoi(argv[3]), tier = atoi(argv[4]);
    const uint64_t wrows = argc > 5 ? strtoull(argv[5], NULL, 10) : 0;
    const rh_schema sc = {RH_KEY_U64, 8, RH_VAL_U64, 8, RH_REC_PLAIN, 0};
    uint64_t *keys = malloc(n * 8), *vals = malloc(n * 8), *hk = malloc(n * 8), *hv = malloc(n * 8);
    if (!keys || !vals || !hk || !hv) return 2;
    uint64_t m = 0;
    for (uint64_t k = 0; k < n; k++) {
        keys[k] = k;
        vals[k] = k * 2654435761ull;
        int missing = 0;
        for (uint64_t i = 1; i <= d && !missing; i++) missing = k == (n / (d + 1)) * i;
        if (!missing) hk[m] = k, hv[m] = vals[k], m++;
    }
    rh_store *a, *b;
    CHECK(rh_store_create(0, &sc, &a));
    CHECK(rh_store_create(0, &sc, &b));
    const rh_columns ca = {keys, NULL, NULL, NULL, NULL, vals}, cb = {hk, NULL, NULL, NULL, NULL, hv};
    CHECK(rh_store_load(a, &ca, n));
    CHECK(rh_store_load(b, &cb, m));
    if (tier) {
        CHECK(rh_store_set_host_tier(a, 1, 0));
        CHECK(rh_store_set_host_tier(b, 1, 0));
    }
    double t0 = now_s();
    cost_t c = reconcile(a, b, &sc); /* the first one (RSOS_HIP_TIER_SYNC=0: the tiers' copies may be in flight) */
    const double first = now_s() - t0;
    CHECK(rh_store_tier_sync(a)); /* then a warm store: the copies have landed */
    CHECK(rh_store_tier_sync(b));
    double *ts = malloc(sizeof(double) * (size_t)(reps > 0 ? reps : 1));
    double *tw = malloc(sizeof(double) * (size_t)(reps > 0 ? reps : 1));
    double total = 0, wtotal = 0;
    uint64_t *wk = malloc(sizeof(uint64_t) * (wrows + 1)), *wv = malloc(sizeof(uint64_t) * (wrows + 1));
    uint8_t *wops = calloc(wrows + 1, 1);
    if (!wk || !wv || !wops) return 2;
    uint64_t next_key = n + 1000, refreshes0 = 0, folds0 = 0;
    CHECK(rh_store_tier_stats(a, NULL, NULL, &refreshes0, &folds0));
    for (int r = 0; r < reps; r++) {
        tw[r] = 0;
        if (wrows) {
            /* fresh keys (the maps hold every key below n): n + a SplitMix64 stream, spread over the
               rest of the key space */
            for (uint64_t j = 0; j < wrows; j++) {
                uint64_t z = (next_key++) * 0x9e3779b97f4a7c15ull;
                z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
                z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
                wk[j] = n + ((z ^ (z >> 31)) >> 2);
                wv[j] = wk[j] * 2654435761ull;
            }
            uint64_t la = 0, lb = 0;
            t0 = now_s();
            for (uint64_t j = 0; j < wrows; j++) {  /* Rsos::insert, one record at a time */
                const rh_columns one = {wk + j, NULL, NULL, NULL, NULL, wv + j};
                CHECK(rh_store_stage(a, &one, wops, 1));
                CHECK(rh_store_stage(b, &one, wops, 1));
            }
            CHECK(rh_store_len(a, &la)); /* each store applies its staged batch on its next question */
            CHECK(rh_store_len(b, &lb));
            tw[r] = now_s() - t0;
            wtotal += tw[r];
        }
        t0 = now_s();
        c = reconcile(a, b, &sc);
        ts[r] = now_s() - t0;
        total += ts[r];
    }
    uint64_t refreshes = 0, folds = 0, tier_delta = 0;
    CHECK(rh_store_tier_stats(a, NULL, &tier_delta, &refreshes, &folds));
    qsort(ts, (size_t)reps, sizeof(double), cmp_d);
    qsort(tw, (size_t)reps, sizeof(double), cmp_d);
    /* per-question costs through the ABI: Rsos::aggregate over a random key range, Rsos::rank */
    const int q = 200000;
    uint64_t x = 12345, sink = 0;
    t0 = now_s();
    for (int i = 0; i < q; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        uint64_t lo = (x >> 11) % n, hi = lo + ((x >> 40) % (n - lo + 1));
        rh_aggregate g;
        CHECK(rh_store_aggregate_keys(a, 1, &lo, 2, &hi, &g));
        sink += g.size;
    }
    const double agg_ns = (now_s() - t0) / q * 1e9;
    t0 = now_s();
    for (int i = 0; i < q; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        uint64_t k = (x >> 11) % (n + 10), r;
        CHECK(rh_store_rank(a, &k, &r));
        sink += r;
    }
    const double rank_ns = (now_s() - t0) / q * 1e9;
    printf("{\"n\": %llu, \"d\": %llu, \"host_tier\": %d, \"reps\": %d, \"rounds\": %llu, \"ranges\": %llu, \"idlists\": %llu, "
           "\"enumerated\": %llu, \"wire_bytes\": %llu, \"first_us\": %.1f, \"mean_us\": %.2f, \"median_us\": %.2f, "
           "\"p10_us\": %.2f, \"p90_us\": %.2f, \"aggregate_ns\": %.1f, \"rank_ns\": %.1f, \"write_rows\": %llu, "
           "\"write_mean_us\": %.2f, \"write_median_us\": %.2f, \"write_p90_us\": %.2f, \"cycle_mean_us\": %.2f, "
           "\"tier_refreshes\": %llu, \"tier_folds\": %llu, \"tier_delta_entries\": %llu, \"sink\": %llu}\n",
           (unsigned long long)n, (unsigned long long)d, tier, reps, (unsigned long long)c.rounds,
           (unsigned long long)c.ranges, (unsigned long long)c.idlists, (unsigned long long)c.enumerated, (unsigned long long)c.wire_bytes,
           first * 1e6, reps ? total / reps * 1e6 : 0.0, reps ? ts[reps / 2] * 1e6 : 0.0, reps ? ts[reps / 10] * 1e6 : 0.0,
           reps ? ts[(reps * 9) / 10] * 1e6 : 0.0, agg_ns, rank_ns, (unsigned long long)wrows,
           reps ? wtotal / reps * 1e6 : 0.0, reps ? tw[reps / 2] * 1e6 : 0.0, reps ? tw[(reps * 9) / 10] * 1e6 : 0.0,
           reps ? (wtotal + total) / reps * 1e6 : 0.0, (unsigned long long)(refreshes - refreshes0),
           (unsigned long long)(folds - folds0), (unsigned long long)tier_delta, (unsigned long long)(sink & 1));
    CHECK(rh_store_destroy(a));
    CHECK(rh_store_destroy(b));
    return 0;
}
