/*
 * sstore_client.c -- a plain C consumer of the sharded store (rh_sstore_*, include/rsos_hip.h):
 * one map over <shards> key-range shards (all on device 0 here: the box has one GPU), checked
 * answer for answer against one rh_store holding the same records, and timed beside it.
 *
 *   sstore_client <shards> <n> [d = 100] [host_tier = 1] [reps = 20]
 *
 * Stores as the reference's protocol bench builds them (benches/protocol.rs:198-232):
 * FingerprintTreeMap<u64, u64>, keys 0..n, values key * 2654435761; the peer lacks d keys
 * scattered at (n / (d + 1)) * i and holds d other keys re-valued.  Checks (exit 1 on any
 * difference): size, root, ranks, selects, key-range and rank-range aggregates, and whole
 * FixedFanOut(16) reconciliations against the peer -- every round's children and enumerations
 * byte for byte -- after the load, after a routed batch (rh_sstore_apply: inserts, overwrites,
 * deletes) and after staged single rows (rh_sstore_stage).  Prints one JSON object with the
 * reconciliation time of the sharded map and of the single store.
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
#define EXPECT(cond, what)                                                               \
    do {                                                                                 \
        if (!(cond)) {                                                                   \
            fprintf(stderr, "mismatch: %s (line %d)\n", what, __LINE__);                 \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint64_t rng_state = 0x243f6a8885a308d3ull;
static uint64_t rnd(void) {
    uint64_t z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

/* the two maps behind one interface: a sharded store or a single store */
typedef struct {
    rh_sstore *ss;
    rh_store *st;
} map_t;

static int m_round(map_t m, const rh_segments *in, rh_segments *ch, rh_segments *en, rh_round_outcome *oc) {
    return m.ss ? rh_sstore_protocol_round(m.ss, RH_POLICY_FIXED_FAN_OUT, 16, in, ch, en, oc)
                : rh_store_protocol_round(m.st, RH_POLICY_FIXED_FAN_OUT, 16, in, ch, en, oc);
}
static uint64_t m_len(map_t m) {
    uint64_t n = 0;
    CHECK(m.ss ? rh_sstore_len(m.ss, &n) : rh_store_len(m.st, &n));
    return n;
}
static uint64_t m_rank(map_t m, uint64_t k) {
    uint64_t r = 0;
    CHECK(m.ss ? rh_sstore_rank(m.ss, &k, &r) : rh_store_rank(m.st, &k, &r));
    return r;
}
static uint64_t m_select(map_t m, uint64_t r) {
    uint64_t k = 0;
    CHECK(m.ss ? rh_sstore_select(m.ss, r, &k) : rh_store_select(m.st, r, &k));
    return k;
}
static rh_aggregate m_agg_keys(map_t m, int lk, uint64_t lo, int hk, uint64_t hi) {
    rh_aggregate a;
    CHECK(m.ss ? rh_sstore_aggregate_keys(m.ss, lk, &lo, hk, &hi, &a) : rh_store_aggregate_keys(m.st, lk, &lo, hk, &hi, &a));
    return a;
}
static rh_aggregate m_agg_ranks(map_t m, uint64_t lo, uint64_t hi) {
    rh_aggregate a;
    CHECK(m.ss ? rh_sstore_aggregates(m.ss, &lo, &hi, 1, &a) : rh_store_aggregates(m.st, &lo, &hi, 1, &a));
    return a;
}

/* one round's output, copied (the store's buffers are valid until its next call) */
typedef struct {
    uint8_t *bytes;
    size_t len, cap;
} blob_t;
static void blob_put(blob_t *b, const void *p, size_t n) {
    if (b->len + n > b->cap) {
        b->cap = 2 * (b->len + n) + 64;
        b->bytes = realloc(b->bytes, b->cap);
        if (!b->bytes) exit(2);
    }
    if (n) memcpy(b->bytes + b->len, p, n);
    b->len += n;
}

/* per-round times of `a`'s rounds in the last timed reconciliation (detail mode) */
#define MAX_ROUNDS 64
static double round_us[MAX_ROUNDS];
static uint64_t round_r[MAX_ROUNDS];
static int n_timed;

/* a whole reconciliation of `a` with the peer; every round's outputs appended to `log` */
static uint64_t reconcile(map_t a, rh_store *peer, blob_t *log) {
    n_timed = 0;
    size_t cap = 16, n = 1;
    uint8_t *sk = calloc(cap, 1), *ek = calloc(cap, 1);
    uint64_t *skey = calloc(cap, 8), *ekey = calloc(cap, 8);
    rh_aggregate *agg = calloc(cap, sizeof(rh_aggregate));
    CHECK(a.ss ? rh_sstore_aggregate_keys(a.ss, 0, NULL, 0, NULL, &agg[0]) : rh_store_aggregate_keys(a.st, 0, NULL, 0, NULL, &agg[0]));
    uint64_t rounds = 0;
    int peer_turn = 1;
    while (n) {
        const rh_segments in = {sk, skey, ek, ekey, agg, n, n};
        rh_segments ch, en;
        rh_round_outcome oc;
        if (peer_turn) CHECK(rh_store_protocol_round(peer, RH_POLICY_FIXED_FAN_OUT, 16, &in, &ch, &en, &oc));
        else {
            const double t0 = now_s();
            CHECK(m_round(a, &in, &ch, &en, &oc));
            if (n_timed < MAX_ROUNDS) round_us[n_timed] = (now_s() - t0) * 1e6, round_r[n_timed++] = n;
        }
        rounds++;
        if (log) {
            blob_put(log, &oc, sizeof oc);
            blob_put(log, ch.start_kinds, ch.n);
            blob_put(log, ch.end_kinds, ch.n);
            blob_put(log, ch.start_keys, ch.n * 8);
            blob_put(log, ch.end_keys, ch.n * 8);
            blob_put(log, ch.aggregates, ch.n * sizeof(rh_aggregate));
            blob_put(log, en.start_kinds, en.n);
            blob_put(log, en.end_kinds, en.n);
            blob_put(log, en.start_keys, en.n * 8);
            blob_put(log, en.end_keys, en.n * 8);
        }
        if (ch.n > cap) {
            cap = 2 * ch.n;
            sk = realloc(sk, cap), ek = realloc(ek, cap);
            skey = realloc(skey, cap * 8), ekey = realloc(ekey, cap * 8);
            agg = realloc(agg, cap * sizeof(rh_aggregate));
            if (!sk || !ek || !skey || !ekey || !agg) exit(2);
        }
        n = ch.n;
        memcpy(sk, ch.start_kinds, n);
        memcpy(ek, ch.end_kinds, n);
        memcpy(skey, ch.start_keys, n * 8);
        memcpy(ekey, ch.end_keys, n * 8);
        memcpy(agg, ch.aggregates, n * sizeof(rh_aggregate));
        peer_turn = !peer_turn;
    }
    free(sk), free(ek), free(skey), free(ekey), free(agg);
    return rounds;
}

static int agg_eq(rh_aggregate x, rh_aggregate y) { return !memcmp(&x, &y, sizeof x); }

/* every answer of the sharded map against the single store */
static uint64_t compare(map_t s, map_t one, rh_store *peer, uint64_t key_space) {
    const uint64_t n = m_len(one);
    EXPECT(m_len(s) == n, "size");
    EXPECT(agg_eq(m_agg_keys(s, 0, 0, 0, 0), m_agg_keys(one, 0, 0, 0, 0)), "root");
    for (int i = 0; i < 2000; i++) {
        const uint64_t k = rnd() % key_space;
        EXPECT(m_rank(s, k) == m_rank(one, k), "rank");
        if (n) {
            const uint64_t r = rnd() % n;
            EXPECT(m_select(s, r) == m_select(one, r), "select");
        }
        const uint64_t a = rnd() % key_space, b = rnd() % key_space;
        const int lk = 1 + (int)(rnd() % 2), hk = 1 + (int)(rnd() % 2);
        EXPECT(agg_eq(m_agg_keys(s, lk, a, hk, b), m_agg_keys(one, lk, a, hk, b)), "key-range aggregate");
        const uint64_t lo = rnd() % (n + 3), hi = rnd() % (n + 3);
        EXPECT(agg_eq(m_agg_ranks(s, lo, hi), m_agg_ranks(one, lo, hi)), "rank-range aggregate");
    }
    blob_t x = {0}, y = {0};
    const uint64_t rounds = reconcile(s, peer, &x);
    EXPECT(reconcile(one, peer, &y) == rounds, "rounds");
    EXPECT(x.len == y.len && !memcmp(x.bytes, y.bytes, x.len), "reconciliation outputs");
    free(x.bytes), free(y.bytes);
    return rounds;
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: sstore_client <shards> <n> [d] [host_tier] [reps]\n");
        return 1;
    }
    const int G = atoi(argv[1]);
    const uint64_t n = strtoull(argv[2], NULL, 10), d = argc > 3 ? strtoull(argv[3], NULL, 10) : 100;
    const int tier = argc > 4 ? atoi(argv[4]) : 1, reps = argc > 5 ? atoi(argv[5]) : 20;
    if (G < 1 || G > 64 || n < 2 * d + 2) return 1;
    const rh_schema sc = {RH_KEY_U64, 8, RH_VAL_U64, 8, RH_REC_PLAIN, 0};
    uint64_t *keys = malloc(n * 8), *vals = malloc(n * 8), *pk = malloc(n * 8), *pv = malloc(n * 8);
    if (!keys || !vals || !pk || !pv) return 2;
    uint64_t m = 0;
    for (uint64_t k = 0; k < n; k++) {
        keys[k] = k;
        vals[k] = k * 2654435761ull;
        int missing = 0;
        for (uint64_t i = 1; i <= d && !missing; i++) missing = k == (n / (d + 1)) * i;
        if (!missing) pk[m] = k, pv[m] = vals[k] ^ (k % (n / d + 1) == 7), m++;  /* d re-valued keys too */
    }
    int *devs = calloc((size_t)G, sizeof(int));  /* every shard on device 0 */
    rh_sstore *ss;
    rh_store *one, *peer;
    CHECK(rh_sstore_create(devs, G, &sc, &ss));
    EXPECT(rh_sstore_shard_count(ss) == G, "shard count");
    CHECK(rh_store_create(0, &sc, &one));
    CHECK(rh_store_create(0, &sc, &peer));
    const rh_columns ca = {keys, NULL, NULL, NULL, NULL, vals}, cp = {pk, NULL, NULL, NULL, NULL, pv};
    CHECK(rh_sstore_load(ss, &ca, n));
    CHECK(rh_store_load(one, &ca, n));
    CHECK(rh_store_load(peer, &cp, m));
    if (tier) {
        CHECK(rh_sstore_set_host_tier(ss, 1, 0));
        CHECK(rh_store_set_host_tier(one, 1, 0));
        CHECK(rh_store_set_host_tier(peer, 1, 0));
    }
    const map_t S = {ss, NULL}, O = {NULL, one};
    /* the load cut at equal counts */
    for (int i = 0; i < G; i++) {
        rh_store *sh;
        uint64_t len;
        CHECK(rh_sstore_shard(ss, i, &sh));
        CHECK(rh_store_len(sh, &len));
        EXPECT(len == n * (uint64_t)(i + 1) / (uint64_t)G - n * (uint64_t)i / (uint64_t)G, "equal-count cut");
    }
    const uint64_t rounds = compare(S, O, peer, n + 1000);
    /* a routed batch: new keys above n, overwrites and deletes of resident keys */
    const uint64_t bm = n / 2 < 20000 ? n / 2 : 20000;
    uint64_t *bk = malloc(bm * 8), *bv = malloc(bm * 8);
    uint8_t *ops = calloc(bm, 1);
    for (uint64_t j = 0; j < bm; j++) {
        const uint64_t u = rnd() % 10;
        bk[j] = u < 6 ? n + j : (j * 7919) % n;  /* distinct: new keys n + j, resident keys by a stride */
        bv[j] = rnd();
        ops[j] = u >= 8;
    }
    const rh_columns cb = {bk, NULL, NULL, NULL, NULL, bv};
    uint64_t c1[3], c2[3];
    CHECK(rh_sstore_apply(ss, &cb, ops, bm, &c1[0], &c1[1], &c1[2]));
    CHECK(rh_store_apply(one, &cb, ops, bm, &c2[0], &c2[1], &c2[2]));
    EXPECT(!memcmp(c1, c2, sizeof c1), "batch counts");
    compare(S, O, peer, n + bm + 1000);
    /* a repeated key is refused and changes nothing */
    bk[5] = bk[9];
    EXPECT(rh_sstore_apply(ss, &cb, ops, bm, NULL, NULL, NULL) == RH_ERR_ARG, "duplicate batch refused");
    /* staged single rows (Rsos::insert / delete) */
    for (int j = 0; j < 3000; j++) {
        const uint64_t k = rnd() % (n + bm + 5000), v = rnd();
        const uint8_t op = (uint8_t)(rnd() % 5 == 0);
        const rh_columns c1r = {&k, NULL, NULL, NULL, NULL, &v};
        CHECK(rh_sstore_stage(ss, &c1r, &op, 1));
        CHECK(rh_store_stage(one, &c1r, &op, 1));
    }
    compare(S, O, peer, n + bm + 6000);
    /* timing: whole reconciliations with the peer, the sharded map and the single store -- warm:
     * every host tier fresh (rh_store_tier_sync: a refresh the writes above started has landed and
     * been swapped in, so no timed question pays it) and eight untimed reconciliations each (a shard base's row prefix forms after 16 device questions) */
    if (tier) {
        for (int i = 0; i < G; i++) {
            rh_store *sh;
            CHECK(rh_sstore_shard(ss, i, &sh));
            CHECK(rh_store_tier_sync(sh));
        }
        CHECK(rh_store_tier_sync(one));
        CHECK(rh_store_tier_sync(peer));
    }
    for (int w = 0; w < 8; w++) {
        reconcile(S, peer, NULL);
        reconcile(O, peer, NULL);
    }
    double ts = 0, to = 0, rs[MAX_ROUNDS] = {0}, ro[MAX_ROUNDS] = {0};
    uint64_t rr[MAX_ROUNDS] = {0};
    int nr = 0;
    for (int r = 0; r < reps; r++) {
        double t0 = now_s();
        reconcile(S, peer, NULL);
        ts += now_s() - t0;
        for (int i = 0; i < n_timed; i++) rs[i] += round_us[i], rr[i] = round_r[i];
        nr = n_timed;
        t0 = now_s();
        reconcile(O, peer, NULL);
        to += now_s() - t0;
        for (int i = 0; i < n_timed; i++) ro[i] += round_us[i];
    }
    const int q = 100000;
    double t0 = now_s();
    uint64_t sink = 0;
    for (int i = 0; i < q; i++) {
        const uint64_t a = rnd() % n, b = a + rnd() % (n - a + 1);
        sink += m_agg_keys(S, 1, a, 2, b).size;
    }
    const double agg_s = (now_s() - t0) / q * 1e9;
    t0 = now_s();
    for (int i = 0; i < q; i++) {
        const uint64_t a = rnd() % n, b = a + rnd() % (n - a + 1);
        sink += m_agg_keys(O, 1, a, 2, b).size;
    }
    const double agg_o = (now_s() - t0) / q * 1e9;
    printf("{\"shards\": %d, \"n\": %llu, \"d\": %llu, \"host_tier\": %d, \"reps\": %d, \"rounds\": %llu, "
           "\"identical\": true, \"drive_us_sharded\": %.1f, \"drive_us_single\": %.1f, "
           "\"aggregate_ns_sharded\": %.1f, \"aggregate_ns_single\": %.1f, \"sink\": %llu}\n",
           G, (unsigned long long)n, (unsigned long long)d, tier, reps, (unsigned long long)rounds,
           reps ? ts / reps * 1e6 : 0.0, reps ? to / reps * 1e6 : 0.0, agg_s, agg_o, (unsigned long long)(sink & 1));
    if (getenv("SSTORE_ROUNDS")) {  /* this map's rounds: segments in, mean us sharded / single */
        for (int i = 0; i < nr; i++)
            printf("{\"round\": %d, \"segments\": %llu, \"us_sharded\": %.1f, \"us_single\": %.1f}\n", i,
                   (unsigned long long)rr[i], reps ? rs[i] / reps : 0.0, reps ? ro[i] / reps : 0.0);
    }
    CHECK(rh_sstore_destroy(ss));
    CHECK(rh_store_destroy(one));
    CHECK(rh_store_destroy(peer));
    free(keys), free(vals), free(pk), free(pv), free(bk), free(bv), free(ops), free(devs);
    return 0;
}
