/*
 * oracle.h -- CPU restatement of reconcile-rs's fingerprint-hash path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, and only as the checker / the timed CPU
 * baseline.  The product path (reconcile-rs_amd/, librsos_hip.so) never links,
 * loads or calls anything here and fails loudly when its HIP library is missing.
 *
 * What it restates (citations relative to the reference checkout):
 *   - BLAKE3 unkeyed hash, 32-byte output: third-party crate `blake3` 1.8.5
 *     (Cargo.lock:197-200), called from rsos/src/encoding.rs:89-93 (update) and
 *     rsos/src/fingerprint.rs:235,249 (new / finalize).  Restated from the BLAKE3
 *     specification (chunk 1024 B, block 64 B, 7 rounds, CHUNK_START/END/PARENT/ROOT).
 *   - canonical encoding: rsos/src/encoding.rs:17-35 (format table),
 *     :162-169 (put_len / put_variant), rsos/src/encoding/serializer.rs:40-212.
 *   - lift = BLAKE3(canon(k) || canon(v)): rsos/src/fingerprint.rs:270-275;
 *     digest = BLAKE3(canon(v)): rsos/src/fingerprint.rs:288-292.
 *   - Fingerprint add / sub mod 2^256 over LE u64 limbs: rsos/src/fingerprint.rs:145-173.
 *   - Aggregate (size, fingerprint) monoid: rsos/src/aggregate.rs:38-89.
 *   - Record schemas: Entry<Timestamp,V> / State<V> (lww-register/src/entry.rs:24-29,88-94),
 *     Timestamp{Hlc{physical u64, logical u32}, node_id u64} (lww-register/src/clock.rs:143-181).
 *   - FingerprintTreeMap fill (order-6 B-tree, per-node Aggregate cache, one lift per
 *     insert): rsos/src/fingerprint_tree_map/mutate.rs:23-88, node.rs:54-152.
 *
 * Parity pinning: the reference's own golden vectors (rsos/src/fingerprint/tests.rs:68-93,
 * tests/timestamp_wire_format.rs:105-121) and the BLAKE3 spec's published test vectors
 * (tests/golden/), plus an independent pure-Python restatement (oracle/pyref.py).
 */
#ifndef RECONCILE_ORACLE_H
#define RECONCILE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- BLAKE3 ---------------------------------------------------------------------- */
typedef struct {
    uint32_t key[8];
    uint32_t chunk_cv[8];
    uint64_t chunk_counter;
    uint8_t  block[64];
    uint32_t block_len;
    uint32_t blocks_compressed;
    uint32_t cv_stack[54][8];
    uint32_t cv_stack_len;
} or_hasher;

void or_hasher_init(or_hasher *h);
void or_hasher_update(or_hasher *h, const void *data, size_t len);
void or_hasher_finalize(const or_hasher *h, uint8_t out[32]);
void or_blake3(const void *data, size_t len, uint8_t out[32]);

/* ---- schemas (same numbering as include/rsos_hip.h; checked by tests) ------------ */
enum { OR_KEY_UNIT = 0, OR_KEY_U32 = 1, OR_KEY_U64 = 2, OR_KEY_BYTES = 3 };
enum { OR_VAL_UNIT = 0, OR_VAL_U32 = 1, OR_VAL_U64 = 2, OR_VAL_BYTES = 3 };
enum { OR_REC_PLAIN = 0, OR_REC_DATED = 1, OR_REC_PROJECTION = 2 };

typedef struct {
    int32_t  key_kind;
    uint32_t key_len;     /* bytes per key in the key column (4 / 8 / L) */
    int32_t  value_kind;
    uint32_t value_len;   /* bytes per value in the value column */
    int32_t  record_kind;
    uint32_t reserved;
} or_schema;

typedef struct {
    const uint8_t  *keys;     /* n * key_len                                     */
    const uint64_t *phys;     /* n, DATED only: Hlc.physical (ms)                */
    const uint32_t *logical;  /* n, DATED only: Hlc.logical                      */
    const uint64_t *node;     /* n, DATED only: Timestamp.node_id                */
    const uint8_t  *tags;     /* n or NULL: 0 = State::Present, 1 = Tombstone     */
    const uint8_t  *values;   /* n * value_len                                   */
} or_columns;

/* canonical encoding of record i; returns its byte length (buf may be NULL to size it) */
size_t or_encode_record(const or_schema *s, const or_columns *c, size_t i, uint8_t *buf);
/* lift of every record -> 32-byte LE fingerprints, on `threads` host threads */
void or_lift_records(const or_schema *s, const or_columns *c, size_t n, uint8_t *fps, int threads);
/* BLAKE3 of pre-encoded records: record i = bytes[offsets[i] .. offsets[i+1]) */
void or_lift_encoded(const uint8_t *bytes, const uint64_t *offsets, size_t n, uint8_t *fps, int threads);

/* CPU-baseline backends (blake3_simd.c).  or_set_simd(level): the compression every hash above
 * runs -- 0 the portable restatement (the default; what the tests pin), 1 the SSE4.1 row form of
 * the blake3 crate's compress_in_place, 2 its AVX-512VL form; returns the level in effect (the
 * best the CPU supports, at most `level`).  Process-wide: set it before starting any work.
 * or_lift_records_x16: 16 records per AVX-512 vector (not the reference's path: the best batch
 * lift this CPU can do); -1 without AVX-512.                                                    */
int  or_set_simd(int level);
int  or_cpu_has_sse41(void);
int  or_cpu_has_avx512(void);
void or_compress_sse41(const uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t block_len,
                       uint32_t flags, uint32_t out[16]);
void or_compress_avx512vl(const uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t block_len,
                          uint32_t flags, uint32_t out[16]);
int  or_lift_records_x16(const or_schema *s, const or_columns *c, size_t n, uint8_t *fps, int threads);

/* ---- Fingerprint / Aggregate ------------------------------------------------------ */
typedef struct { uint64_t fp[4]; uint64_t size; } or_aggregate;
void or_fp_add(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]);
void or_fp_sub(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]);
/* aggregates of rank ranges [bounds[j], bounds[j+1]) over a fingerprint array */
void or_range_aggregates(const uint8_t *fps, size_t n, const uint64_t *bounds, size_t r,
                         or_aggregate *out);

/* ---- FingerprintTreeMap restatement (reference-faithful serial fill) -------------- */
typedef struct or_ftm or_ftm;
or_ftm *or_ftm_new(const or_schema *s, const or_columns *c);
void    or_ftm_free(or_ftm *t);
/* insert record i of the bound columns (key, value) -> 1 if the key was new, 0 if overwritten */
int     or_ftm_insert(or_ftm *t, size_t i);
/* insert records [lo, hi) serially, in order */
void    or_ftm_fill(or_ftm *t, size_t lo, size_t hi);
size_t  or_ftm_len(const or_ftm *t);
void    or_ftm_root(const or_ftm *t, or_aggregate *out);
/* Aggregate over keys in [lo_key, hi_key) (NULL = unbounded) by the cached-subtree walk */
void    or_ftm_aggregate(const or_ftm *t, const uint8_t *lo_key, const uint8_t *hi_key,
                         or_aggregate *out);
size_t  or_ftm_rank(const or_ftm *t, const uint8_t *key);
/* select(index) -> the record row holding the index-th key; (size_t)-1 if index >= len */
size_t  or_ftm_select(const or_ftm *t, size_t index);
/* a whole FixedFanOut(fan_out) reconciliation between two trees (rbsr protocol rounds, starting
 * from a's root at b); out: rounds, segments answered, IDLIST segments.  -1 if keys > 32 B */
int     or_reconcile_fixed(const or_ftm *a, const or_ftm *b, size_t fan_out, uint64_t out[3]);
/* 0 on success; -1 if the per-node cached aggregates disagree with a recomputation */
int     or_ftm_check(const or_ftm *t);

#ifdef __cplusplus
}
#endif
#endif
