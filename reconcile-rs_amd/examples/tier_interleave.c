/*
 * tier_interleave.c -- large write batches interleaved with small reconciliations, through the C ABI:
 * the host tier's background refresh under the load that forces it.
 *
 *   tier_interleave <n> <batch_rows> <reps> <host_tier 0|1> <shape u64|c5> [warmup] [small]
 *
 * Two replicas of n records (shape u64: FingerprintTreeMap<u64, u64>, keys 0..n-1 as the
 * reference's protocol bench builds them, benches/protocol.rs:198-232; shape c5: config5's 16-byte
 * keys / 64-byte values, dated) that differ by one key (the second lacks the last).  Each
 * repetition writes one batch of batch_rows fresh random records into both (device-resident
 * columns, rh_store_apply_device: a replica merging a large received batch,
 * src/replica/dispatch.rs:188-196), then drives one whole FixedFanOut(16) reconciliation between
 * them (the reference's reconciliation_drive, benches/protocol.rs:455-520: every round encoded for
 * the wire, answered with rh_store_protocol_round, its IDLIST ranges enumerated).  Writes and drives
 * are timed separately; the JSON line reports their distributions (p50 / p90 / p99 / max), the
 * rounds of the last drive (identical with the tier on or off: tests/test_tier_interleave.py) and
 * the tier's refreshes and folds.  With the tier on, a batch larger than the tier's delta tree
 * takes starts a background refresh; the drives while it is in flight are answered by the device,
 * and writes go on without waiting for it (one refresh per copy time, never one per batch).
 * tier_refreshes counts the refreshes started by the timed batches (the last one landed by an
 * untimed rh_store_tier_sync after the loop); tier_refreshes_landed_in_loop those that landed
 * inside it.  small > 0: after each large batch and its drive, `small` cycles of one row staged
 * into both replicas (rh_store_stage, the Rsos::insert path) and a drive -- the small writes that
 * follow a large merge (with the tier on they fold over the run copy the large batch took); their
 * distributions are reported as small_write_* / small_drive_*.
 */
#define _POSIX_C_SOURCE 199309L
#define __HIP_PLATFORM_AMD__ 1
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "../../include/rsos_hip.h"

#define CHECK(call)                                                                      \
    do {                                                                                 \
        int rc_ = (call);                                                                \
        if (rc_ != RH_OK) {                                                              \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, rh_last_error());        \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)
#define HCHECK(call)                                                                     \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));            \
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

static uint64_t splitmix64(uint64_t i) {
    uint64_t z = (i + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static size_t KL, VL;
static uint64_t STRIDE = 1;
static int DATED;

/* a round's segments, owned by the driver (copied out of the store's buffers) */
typedef struct {
    uint8_t *sk, *ek, *skey, *ekey;
    rh_aggregate *agg;
    size_t n, cap;
} segs_t;

static void segs_reserve(segs_t *s, size_t n) {
    if (n <= s->cap) return;
    s->cap = n * 2;
    s->sk = realloc(s->sk, s->cap);
    s->ek = realloc(s->ek, s->cap);
    s->skey = realloc(s->skey, s->cap * KL);
    s->ekey = realloc(s->ekey, s->cap * KL);
    s->agg = realloc(s->agg, s->cap * sizeof(rh_aggregate));
    if (!s->sk || !s->ek || !s->skey || !s->ekey || !s->agg) {
        fprintf(stderr, "out of memory\n");
        exit(2);
    }
}

typedef struct {
    uint64_t rounds, ranges, idlists, enumerated, wire_bytes;
} cost_t;

static uint8_t *wire, *enum_keys;
static size_t wire_cap, enum_cap;

static cost_t reconcile(rh_store *a, rh_store *b, const rh_schema *sc) {
    cost_t c = {0, 0, 0, 0, 0};
    static segs_t active;
    segs_reserve(&active, 1);
    active.n = 1;
    active.sk[0] = active.ek[0] = 0;
    memset(active.skey, 0, KL);
    memset(active.ekey, 0, KL);
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
        segs_reserve(&active, ch.n + 1);
        active.n = ch.n;
        memcpy(active.sk, ch.start_kinds, ch.n);
        memcpy(active.ek, ch.end_kinds, ch.n);
        memcpy(active.skey, ch.start_keys, ch.n * KL);
        memcpy(active.ekey, ch.end_keys, ch.n * KL);
        memcpy(active.agg, ch.aggregates, ch.n * sizeof(rh_aggregate));
        c.idlists += en.n;
        const uint8_t *esk = en.start_kinds, *eek = en.end_kinds;
        const uint8_t *eskey = (const uint8_t *)en.start_keys, *eekey = (const uint8_t *)en.end_keys;
        for (size_t j = 0; j < en.n; j++) {  /* Enumerate: the keys the responder would ship */
            uint64_t lo = 0, hi = 0, size = 0;
            CHECK(rh_store_len(resp, &size));
            if (esk[j]) CHECK(rh_store_rank(resp, eskey + j * KL, &lo));
            hi = size;
            if (eek[j]) CHECK(rh_store_rank(resp, eekey + j * KL, &hi));
            if (hi > lo) {
                if ((hi - lo) * KL > enum_cap) {
                    enum_cap = 2 * (hi - lo) * KL;
                    enum_keys = realloc(enum_keys, enum_cap);
                }
                CHECK(rh_store_keys(resp, lo, hi, enum_keys));
                c.enumerated += hi - lo;
            }
        }
        responder_b = !responder_b;
    }
    return c;
}

/* row i of a column set: key, value, stamp (fresh = a random key for a write batch) */
static void make_row(uint64_t i, int fresh, uint8_t *key, uint8_t *val, uint64_t *ph, uint32_t *lg, uint64_t *nd) {
    if (KL == 8) {
        const uint64_t k = fresh ? splitmix64(i ^ 0x5bd1e995ull) : i;
        memcpy(key, &k, 8);
    } else {  /* big-endian (i * stride + r), r < stride = 2^64 / n, then 8 bytes of noise: sorted by i,
                 spread over the whole key space as config5's keys are (rsos_hip/synth.py) */
        const uint64_t h = fresh ? splitmix64(i ^ 0x5bd1e995ull) : i * STRIDE + splitmix64(i) % STRIDE;
        for (int b = 0; b < 8; b++) key[b] = (uint8_t)(h >> (56 - 8 * b));
        const uint64_t l = splitmix64(i + 77);
        memcpy(key + 8, &l, 8);
    }
    if (VL == 8) {
        const uint64_t v = (KL == 8 ? *(uint64_t *)key : i) * 2654435761ull;
        memcpy(val, &v, 8);
    } else {
        for (size_t w = 0; w < VL; w += 8) {
            const uint64_t v = splitmix64(i * 131 + w);
            memcpy(val + w, &v, 8);
        }
    }
    if (DATED) {
        *ph = 1700000000000ull + i;
        *lg = 0;
        *nd = 1;
    }
}

typedef struct {
    uint8_t *keys, *vals;
    uint64_t *phys, *node;
    uint32_t *logical;
} host_cols_t;

static void alloc_cols(host_cols_t *c, uint64_t n) {
    c->keys = malloc(n * KL + 16);
    c->vals = malloc(n * VL + 16);
    c->phys = DATED ? malloc(n * 8 + 16) : NULL;
    c->node = DATED ? malloc(n * 8 + 16) : NULL;
    c->logical = DATED ? malloc(n * 4 + 16) : NULL;
    if (!c->keys || !c->vals || (DATED && (!c->phys || !c->node || !c->logical))) {
        fprintf(stderr, "out of host memory\n");
        exit(2);
    }
}

static rh_columns view(const host_cols_t *c) {
    const rh_columns v = {c->keys, c->phys, c->logical, c->node, NULL, c->vals};
    return v;
}

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: tier_interleave <n> <batch_rows> <reps> <host_tier 0|1> <u64|c5> [warmup] [small]\n");
        return 1;
    }
    const uint64_t n = strtoull(argv[1], NULL, 10), m = strtoull(argv[2], NULL, 10);
    const int reps = atoi(argv[3]), tier = atoi(argv[4]), warm = argc > 6 ? atoi(argv[6]) : 2;
    const int small = argc > 7 ? atoi(argv[7]) : 0;
    const int c5 = strcmp(argv[5], "c5") == 0;
    KL = c5 ? 16 : 8;
    STRIDE = n > 1 ? UINT64_MAX / n : 1;
    VL = c5 ? 64 : 8;
    DATED = c5;
    const rh_schema sc = c5 ? (rh_schema){RH_KEY_BYTES, 16, RH_VAL_BYTES, 64, RH_REC_DATED, 0}
                            : (rh_schema){RH_KEY_U64, 8, RH_VAL_U64, 8, RH_REC_PLAIN, 0};
    host_cols_t base;
    alloc_cols(&base, n);
    for (uint64_t i = 0; i < n; i++)
        make_row(i, 0, base.keys + i * KL, base.vals + i * VL, DATED ? base.phys + i : NULL,
                 DATED ? base.logical + i : NULL, DATED ? base.node + i : NULL);
    rh_store *a, *b;
    CHECK(rh_store_create(0, &sc, &a));
    CHECK(rh_store_create(0, &sc, &b));
    if (tier) {
        CHECK(rh_store_set_host_tier(a, 1, 0));
        CHECK(rh_store_set_host_tier(b, 1, 0));
    }
    const rh_columns cb = view(&base);
    CHECK(rh_store_load(a, &cb, n));
    CHECK(rh_store_load(b, &cb, n - 1)); /* b lacks the last key: d = 1 */
    free(base.keys), free(base.vals), free(base.phys), free(base.node), free(base.logical);
    /* capacity for every batch, as config5's bench reserves it: no reallocation in the loop */
    CHECK(rh_store_reserve(a, n + (uint64_t)(reps + warm) * m, m));
    CHECK(rh_store_reserve(b, n + (uint64_t)(reps + warm) * m, m));
    double t0 = now_s();
    cost_t c = reconcile(a, b, &sc); /* the first drive: the tiers' copies are in flight */
    const double first = now_s() - t0;
    /* the write batches' device columns (one set, refilled per repetition, untimed) */
    host_cols_t hb;
    alloc_cols(&hb, m);
    void *dk, *dv, *dph = NULL, *dnd = NULL, *dlg = NULL;
    HCHECK(hipMalloc(&dk, m * KL + 16));
    HCHECK(hipMalloc(&dv, m * VL + 16));
    if (DATED) {
        HCHECK(hipMalloc(&dph, m * 8 + 16));
        HCHECK(hipMalloc(&dnd, m * 8 + 16));
        HCHECK(hipMalloc(&dlg, m * 4 + 16));
    }
    const rh_columns dc = {dk, dph, dlg, dnd, NULL, dv};
    double *tw = malloc(sizeof(double) * (size_t)(reps + 1)), *td = malloc(sizeof(double) * (size_t)(reps + 1));
    double wsum = 0, dsum = 0;
    uint64_t ref0 = 0, fold0 = 0, next = 1;
    const size_t nsm = (size_t)reps * (size_t)small + 1;
    double *sw = malloc(sizeof(double) * nsm), *sd = malloc(sizeof(double) * nsm);
    size_t ns_done = 0;
    host_cols_t one;
    alloc_cols(&one, 1);
    const uint8_t op0 = 0;
    for (int r = -warm; r < reps; r++) {
        if (r == 0) { /* the timed loop starts from settled tiers (untimed) */
            CHECK(rh_store_tier_sync(a));
            CHECK(rh_store_tier_sync(b));
            CHECK(rh_store_tier_stats(a, NULL, NULL, &ref0, &fold0));
        }
        for (uint64_t j = 0; j < m; j++, next++)
            make_row(n + next, 1, hb.keys + j * KL, hb.vals + j * VL, DATED ? hb.phys + j : NULL,
                     DATED ? hb.logical + j : NULL, DATED ? hb.node + j : NULL);
        HCHECK(hipMemcpy(dk, hb.keys, m * KL, hipMemcpyHostToDevice));
        HCHECK(hipMemcpy(dv, hb.vals, m * VL, hipMemcpyHostToDevice));
        if (DATED) {
            HCHECK(hipMemcpy(dph, hb.phys, m * 8, hipMemcpyHostToDevice));
            HCHECK(hipMemcpy(dnd, hb.node, m * 8, hipMemcpyHostToDevice));
            HCHECK(hipMemcpy(dlg, hb.logical, m * 4, hipMemcpyHostToDevice));
        }
        HCHECK(hipDeviceSynchronize());
        t0 = now_s();
        const double tws = t0;
        CHECK(rh_store_apply_device(a, &dc, NULL, m, NULL, NULL, NULL, NULL));
        CHECK(rh_store_apply_device(b, &dc, NULL, m, NULL, NULL, NULL, NULL));
        const double w = now_s() - t0;
        t0 = now_s();
        const double tds = t0;
        c = reconcile(a, b, &sc);
        const double d = now_s() - t0;
        if (r >= 0) {
            tw[r] = w, td[r] = d;
            wsum += w, dsum += d;
            if (getenv("TIER_INTERLEAVE_CYCLES")) {  /* one line per cycle (stderr) */
                uint64_t rf = 0, fo = 0;
                CHECK(rh_store_tier_stats(a, NULL, NULL, &rf, &fo));
                fprintf(stderr, "cycle %d: write %.1f us, drive %.1f us, refreshes %llu, folds %llu (write at %.3f ms, drive at %.3f ms, monotonic)\n",
                        r, w * 1e6, d * 1e6, (unsigned long long)rf, (unsigned long long)fo, tws * 1e3, tds * 1e3);
            }
        }
        for (int k = 0; r >= 0 && k < small; k++) {  /* one staged row into both, then a drive */
            make_row(n + next, 1, one.keys, one.vals, DATED ? one.phys : NULL, DATED ? one.logical : NULL,
                     DATED ? one.node : NULL);
            next++;
            const rh_columns oc = view(&one);
            uint64_t la = 0, lb = 0;
            t0 = now_s();
            CHECK(rh_store_stage(a, &oc, &op0, 1));
            CHECK(rh_store_stage(b, &oc, &op0, 1));
            CHECK(rh_store_len(a, &la)); /* each store applies its staged row on its next question */
            CHECK(rh_store_len(b, &lb));
            sw[ns_done] = now_s() - t0;
            t0 = now_s();
            c = reconcile(a, b, &sc);
            sd[ns_done++] = now_s() - t0;
        }
    }
    uint64_t size = 0, refreshes = 0, folds = 0, loop_refreshes = 0;
    CHECK(rh_store_len(a, &size));
    CHECK(rh_store_tier_stats(a, NULL, NULL, &loop_refreshes, NULL));
    CHECK(rh_store_tier_sync(a)); /* the copy the last batch started lands (untimed) */
    CHECK(rh_store_tier_stats(a, NULL, NULL, &refreshes, &folds));
    qsort(tw, (size_t)reps, sizeof(double), cmp_d);
    qsort(td, (size_t)reps, sizeof(double), cmp_d);
    qsort(sw, ns_done, sizeof(double), cmp_d);
    qsort(sd, ns_done, sizeof(double), cmp_d);
#define SPCT(x, p) (ns_done ? (x)[(size_t)(((ns_done - 1) * (p)) / 100)] * 1e6 : 0.0)
#define PCT(x, p) ((x)[(size_t)(((reps - 1) * (p)) / 100)] * 1e6)
    printf("{\"n\": %llu, \"shape\": \"%s\", \"batch_rows\": %llu, \"host_tier\": %d, \"reps\": %d, \"size\": %llu, "
           "\"rounds\": %llu, \"ranges\": %llu, \"idlists\": %llu, \"enumerated\": %llu, \"wire_bytes\": %llu, "
           "\"first_drive_us\": %.1f, \"drive_mean_us\": %.1f, \"drive_p50_us\": %.1f, \"drive_p90_us\": %.1f, "
           "\"drive_p99_us\": %.1f, \"drive_max_us\": %.1f, \"write_mean_us\": %.1f, \"write_p50_us\": %.1f, "
           "\"write_p99_us\": %.1f, \"write_max_us\": %.1f, \"tier_refreshes\": %llu, \"tier_refreshes_landed_in_loop\": %llu, "
           "\"tier_folds\": %llu, \"small_cycles\": %llu, \"small_write_p50_us\": %.1f, \"small_write_p99_us\": %.1f, "
           "\"small_write_max_us\": %.1f, \"small_drive_p50_us\": %.1f, \"small_drive_p99_us\": %.1f, "
           "\"small_drive_max_us\": %.1f}\n",
           (unsigned long long)n, c5 ? "c5" : "u64", (unsigned long long)m, tier, reps, (unsigned long long)size,
           (unsigned long long)c.rounds, (unsigned long long)c.ranges, (unsigned long long)c.idlists,
           (unsigned long long)c.enumerated, (unsigned long long)c.wire_bytes, first * 1e6, dsum / reps * 1e6,
           PCT(td, 50), PCT(td, 90), PCT(td, 99), td[reps - 1] * 1e6, wsum / reps * 1e6, PCT(tw, 50), PCT(tw, 99),
           tw[reps - 1] * 1e6, (unsigned long long)(refreshes - ref0), (unsigned long long)(loop_refreshes - ref0),
           (unsigned long long)(folds - fold0), (unsigned long long)ns_done, SPCT(sw, 50), SPCT(sw, 99),
           ns_done ? sw[ns_done - 1] * 1e6 : 0.0, SPCT(sd, 50), SPCT(sd, 99), ns_done ? sd[ns_done - 1] * 1e6 : 0.0);
    CHECK(rh_store_destroy(a));
    CHECK(rh_store_destroy(b));
    return 0;
}
