/*
 * abi_client.c -- a plain C consumer of librsos_hip.so, as the reference's FFI (the rsos-hip
 * Rust crate) would bind it: host buffers in, host results out, status codes,
 * no Python and no torch.
 *
 *   abi_client <n> <seed>
 *
 * Builds n FingerprintTreeMap<u64, u64>-shaped records (SplitMix64 keys, sorted, unique; values
 * from the same stream), loads them into a GPU store (rh_store_load), asks the Rsos<K> questions
 * (size, the root aggregate, rank, select, a key-range aggregate), applies an update batch
 * (inserts, an overwrite, a delete), and runs one whole FixedFanOut(16) reconciliation between
 * the updated store and a second store holding the original records (rh_store_protocol_round,
 * ping-pong until no segment is left).  Prints one JSON object; tests/test_abi_client.py checks
 * every number against the oracle.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rsos_hip.h"

static uint64_t sm_state;
static uint64_t splitmix64(void) {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int cmp_u64(const void *a, const void *b) {
    const uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return (x > y) - (x < y);
}

#define CHECK(call)                                                                      \
    do {                                                                                 \
        int rc_ = (call);                                                                \
        if (rc_ != RH_OK) {                                                              \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, rh_last_error());        \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)

static void print_agg(const char *name, const rh_aggregate *a) {
    printf("\"%s\": {\"fp\": [\"%016llx\", \"%016llx\", \"%016llx\", \"%016llx\"], \"size\": %llu}", name,
           (unsigned long long)a->fingerprint[0], (unsigned long long)a->fingerprint[1],
           (unsigned long long)a->fingerprint[2], (unsigned long long)a->fingerprint[3],
           (unsigned long long)a->size);
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: abi_client <n> <seed>\n");
        return 1;
    }
    const size_t n = (size_t)strtoull(argv[1], NULL, 10);
    sm_state = strtoull(argv[2], NULL, 10);
    if (rh_abi_version() != RH_ABI_VERSION) {
        fprintf(stderr, "ABI version mismatch\n");
        return 2;
    }
    /* records: unique sorted keys, values from the same stream */
    uint64_t *keys = malloc(n * 8), *vals = malloc(n * 8);
    for (size_t i = 0; i < n; i++) keys[i] = splitmix64();
    qsort(keys, n, 8, cmp_u64);
    size_t m = 0;
    for (size_t i = 0; i < n; i++)
        if (m == 0 || keys[i] != keys[m - 1]) keys[m++] = keys[i];
    for (size_t i = 0; i < m; i++) vals[i] = splitmix64();

    const rh_schema schema = {RH_KEY_U64, 8, RH_VAL_U64, 8, RH_REC_PLAIN, 0};
    rh_store *a = NULL, *b = NULL;
    CHECK(rh_store_create(0, &schema, &a));
    CHECK(rh_store_create(0, &schema, &b));
    const rh_columns cols = {keys, NULL, NULL, NULL, NULL, vals};
    CHECK(rh_store_load(a, &cols, m));
    CHECK(rh_store_load(b, &cols, m));

    uint64_t size = 0, rank = 0, sel = 0;
    rh_aggregate root, range;
    CHECK(rh_store_len(a, &size));
    CHECK(rh_store_aggregate_keys(a, 0, NULL, 0, NULL, &root));
    const uint64_t probe = keys[m / 3] + 1; /* between two keys */
    CHECK(rh_store_rank(a, &probe, &rank));
    CHECK(rh_store_select(a, m / 2, &sel));
    CHECK(rh_store_aggregate_keys(a, 1, &keys[m / 4], 2, &keys[3 * m / 4], &range)); /* [k, k') */

    /* an update batch on store a: 3 new keys, 1 overwrite, 1 delete */
    uint64_t bk[5] = {probe, splitmix64(), splitmix64(), keys[10], keys[20]};
    uint64_t bv[5] = {7, 8, 9, vals[10] + 1, 0};
    uint8_t ops[5] = {0, 0, 0, 0, 1};
    const rh_columns batch = {bk, NULL, NULL, NULL, NULL, bv};
    uint64_t n_new = 0, n_over = 0, n_del = 0;
    CHECK(rh_store_apply(a, &batch, ops, 5, &n_new, &n_over, &n_del));
    rh_aggregate root2;
    CHECK(rh_store_aggregate_keys(a, 0, NULL, 0, NULL, &root2));

    /* one whole reconciliation: a's root at b, then rounds alternate until no segment is left */
    uint8_t sk0 = 0, ek0 = 0;
    uint64_t zk = 0;
    rh_segments active = {&sk0, &zk, &ek0, &zk, &root2, 1, 1};
    uint8_t *in_sk = NULL, *in_ek = NULL;
    void *in_skeys = NULL, *in_ekeys = NULL;
    rh_aggregate *in_aggs = NULL;
    rh_store *side[2] = {b, a};
    int rounds = 0;
    uint64_t segments = 0, enumerated = 0;
    while (active.n) {
        rh_segments ch, en;
        rh_round_outcome oc;
        segments += active.n;
        CHECK(rh_store_protocol_round(side[rounds % 2], RH_POLICY_FIXED_FAN_OUT, 16, &active, &ch, &en, &oc));
        enumerated += en.n;
        /* the children belong to the answering store until its next call: copy them out */
        free(in_sk); free(in_ek); free(in_skeys); free(in_ekeys); free(in_aggs);
        in_sk = malloc(ch.n + 1); in_ek = malloc(ch.n + 1);
        in_skeys = malloc(8 * ch.n + 8); in_ekeys = malloc(8 * ch.n + 8);
        in_aggs = malloc(sizeof(rh_aggregate) * (ch.n + 1));
        if (ch.n) {
            memcpy(in_sk, ch.start_kinds, ch.n); memcpy(in_ek, ch.end_kinds, ch.n);
            memcpy(in_skeys, ch.start_keys, 8 * ch.n); memcpy(in_ekeys, ch.end_keys, 8 * ch.n);
            memcpy(in_aggs, ch.aggregates, sizeof(rh_aggregate) * ch.n);
        }
        active = (rh_segments){in_sk, in_skeys, in_ek, in_ekeys, in_aggs, ch.n, ch.n};
        rounds++;
    }

    printf("{\"n\": %zu, \"size\": %llu, \"rank_probe\": %llu, \"probe\": %llu, \"select_mid\": %llu, ", m,
           (unsigned long long)size, (unsigned long long)rank, (unsigned long long)probe,
           (unsigned long long)sel);
    print_agg("root", &root);
    printf(", ");
    print_agg("range_q1_q3", &range);
    printf(", \"batch\": {\"new\": %llu, \"overwritten\": %llu, \"deleted\": %llu, \"keys\": [%llu, %llu, %llu, %llu, %llu]}, ",
           (unsigned long long)n_new, (unsigned long long)n_over, (unsigned long long)n_del,
           (unsigned long long)bk[0], (unsigned long long)bk[1], (unsigned long long)bk[2],
           (unsigned long long)bk[3], (unsigned long long)bk[4]);
    print_agg("root_after_batch", &root2);
    printf(", \"reconcile\": {\"rounds\": %d, \"segments\": %llu, \"enumerated\": %llu}}\n", rounds,
           (unsigned long long)segments, (unsigned long long)enumerated);
    free(in_sk); free(in_ek); free(in_skeys); free(in_ekeys); free(in_aggs);
    CHECK(rh_store_destroy(a));
    CHECK(rh_store_destroy(b));
    free(keys);
    free(vals);
    return 0;
}
