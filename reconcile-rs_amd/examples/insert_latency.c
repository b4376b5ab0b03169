/*
 * insert_latency.c -- the Rust binding's `HipFingerprintMap::insert` path through the C ABI, timed:
 * one rh_store_stage per record (Rsos::insert / FingerprintTreeMap::insert one at a time,
 * rsos/src/fingerprint_tree_map/mutate.rs:23-88; rust/rsos-hip/src/lib.rs `stage`), then one
 * question -- rh_store_aggregate_keys over `..`, the root -- which applies everything staged as one
 * device batch and folds it into the host tier.  The reference's figure for this shape is the
 * single-writer insert throughput of FingerprintTreeMap<u64, u64> with a 100 k prefill:
 * 2,888,103 ops/s = 346 ns per insert (benches/contention.rs, benches/README.md:848-875).
 *
 *   insert_latency <resident> <inserts> <host_tier 0|1> [batches]
 *
 * Resident keys: SplitMix64(i) for i < resident (sorted, de-duplicated); inserted keys:
 * SplitMix64(resident + j) for j < inserts; value = key * 2654435761 (wrapping) -- the same
 * generator tests/test_insert_latency.py restates to check the root against the oracle.
 * batches > 1 splits the inserts into that many stage-then-question rounds.  Prints one JSON object.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/rsos_hip.h"

#define CHECK(call)                                                               \
    do {                                                                          \
        int rc_ = (call);                                                         \
        if (rc_ != RH_OK) {                                                       \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, rh_last_error()); \
            exit(2);                                                              \
        }                                                                         \
    } while (0)

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint64_t splitmix64(uint64_t i) {
    uint64_t z = (i + 1) * 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return (x > y) - (x < y);
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: insert_latency <resident> <inserts> <host_tier 0|1> [batches]\n");
        return 1;
    }
    const uint64_t n = strtoull(argv[1], NULL, 10), m = strtoull(argv[2], NULL, 10);
    const int tier = atoi(argv[3]);
    const uint64_t batches = argc > 4 ? strtoull(argv[4], NULL, 10) : 1;
    const rh_schema sc = {RH_KEY_U64, 8, RH_VAL_U64, 8, RH_REC_PLAIN, 0};
    uint64_t *keys = malloc((n + 1) * 8), *vals = malloc((n + 1) * 8);
    if (!keys || !vals) return 2;
    for (uint64_t i = 0; i < n; i++) keys[i] = splitmix64(i);
    qsort(keys, n, 8, cmp_u64);
    uint64_t nr = 0;
    for (uint64_t i = 0; i < n; i++)
        if (nr == 0 || keys[i] != keys[nr - 1]) keys[nr++] = keys[i];
    for (uint64_t i = 0; i < nr; i++) vals[i] = keys[i] * 2654435761ull;
    rh_store *s;
    CHECK(rh_store_create(0, &sc, &s));
    if (tier) CHECK(rh_store_set_host_tier(s, 1, 0));
    const rh_columns c = {keys, NULL, NULL, NULL, NULL, vals};
    CHECK(rh_store_load(s, &c, nr));
    rh_aggregate root;
    CHECK(rh_store_aggregate_keys(s, 0, NULL, 0, NULL, &root)); /* a warm store: the tier is copied here */
    if (tier) {
        uint64_t r0 = 0;
        CHECK(rh_store_rank(s, &keys[nr / 2], &r0));
        CHECK(rh_store_tier_sync(s)); /* the background copy of the loaded base has landed */
    }
    uint64_t refreshes0 = 0, folds0 = 0;
    CHECK(rh_store_tier_stats(s, NULL, NULL, &refreshes0, &folds0));
    /* the records to insert, generated ahead of the timed loop (the caller owns them) */
    uint64_t *ik = malloc((m + 1) * 8), *iv = malloc((m + 1) * 8);
    if (!ik || !iv) return 2;
    for (uint64_t j = 0; j < m; j++) {
        ik[j] = splitmix64(n + j);
        iv[j] = ik[j] * 2654435761ull;
    }
    const uint8_t op = 0;
    double t_stage = 0, t_apply = 0;
    uint64_t done = 0;
    for (uint64_t b = 0; b < batches; b++) {
        const uint64_t end = (m * (b + 1)) / batches;
        double t0 = now_s();
        for (; done < end; done++) { /* Rsos::insert, one record at a time */
            const rh_columns one = {ik + done, NULL, NULL, NULL, NULL, iv + done};
            CHECK(rh_store_stage(s, &one, &op, 1));
        }
        double t1 = now_s();
        CHECK(rh_store_aggregate_keys(s, 0, NULL, 0, NULL, &root)); /* applies the staged batch */
        if (tier) {  /* and a question the tier answers: the fold is done by then */
            uint64_t r0 = 0;
            CHECK(rh_store_rank(s, &ik[0], &r0));
        }
        double t2 = now_s();
        t_stage += t1 - t0;
        t_apply += t2 - t1;
    }
    uint64_t size = 0, refreshes = 0, folds = 0;
    CHECK(rh_store_len(s, &size));
    CHECK(rh_store_tier_stats(s, NULL, NULL, &refreshes, &folds));
    printf("{\"resident\": %llu, \"inserts\": %llu, \"batches\": %llu, \"host_tier\": %d, \"stage_ns\": %.1f, "
           "\"apply_ns\": %.1f, \"ns_per_insert\": %.1f, \"reference_ns_per_insert\": 346.0, \"size\": %llu, "
           "\"tier_refreshes\": %llu, \"tier_folds\": %llu, \"root\": \"%016llx%016llx%016llx%016llx\"}\n",
           (unsigned long long)nr, (unsigned long long)m, (unsigned long long)batches, tier, t_stage / m * 1e9,
           t_apply / m * 1e9, (t_stage + t_apply) / m * 1e9, (unsigned long long)size, (unsigned long long)(refreshes - refreshes0),
           (unsigned long long)(folds - folds0), (unsigned long long)root.fingerprint[3], (unsigned long long)root.fingerprint[2],
           (unsigned long long)root.fingerprint[1], (unsigned long long)root.fingerprint[0]);
    CHECK(rh_store_destroy(s));
    return 0;
}
