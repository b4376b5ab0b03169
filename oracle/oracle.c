/*
 * oracle.c -- CPU restatement of the reference's fingerprint-hash path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h for who may use it and the citations).
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ================================================================================== */
/* BLAKE3 (restated from the specification; crate blake3 1.8.5 is the reference's    */
/* implementation, Cargo.lock:197-200)                                                */
/* ================================================================================== */

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };
enum { BLOCK_LEN = 64, CHUNK_LEN = 1024 };

static inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static inline void g(uint32_t *v, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
    v[a] = v[a] + v[b] + mx;
    v[d] = rotr(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];
    v[b] = rotr(v[b] ^ v[c], 12);
    v[a] = v[a] + v[b] + my;
    v[d] = rotr(v[d] ^ v[a], 8);
    v[c] = v[c] + v[d];
    v[b] = rotr(v[b] ^ v[c], 7);
}

/* out[16]: full compression output (first 8 words = new chaining value) */
static void compress_portable(const uint32_t cv[8], const uint32_t block[16], uint64_t counter,
                              uint32_t block_len, uint32_t flags, uint32_t out[16]) {
    uint32_t v[16], m[16], t[16];
    for (int i = 0; i < 8; i++) v[i] = cv[i];
    v[8] = IV[0]; v[9] = IV[1]; v[10] = IV[2]; v[11] = IV[3];
    v[12] = (uint32_t)counter; v[13] = (uint32_t)(counter >> 32);
    v[14] = block_len; v[15] = flags;
    memcpy(m, block, sizeof m);
    for (int r = 0; r < 7; r++) {
        g(v, 0, 4, 8, 12, m[0], m[1]);
        g(v, 1, 5, 9, 13, m[2], m[3]);
        g(v, 2, 6, 10, 14, m[4], m[5]);
        g(v, 3, 7, 11, 15, m[6], m[7]);
        g(v, 0, 5, 10, 15, m[8], m[9]);
        g(v, 1, 6, 11, 12, m[10], m[11]);
        g(v, 2, 7, 8, 13, m[12], m[13]);
        g(v, 3, 4, 9, 14, m[14], m[15]);
        if (r < 6) {
            for (int i = 0; i < 16; i++) t[i] = m[PERM[i]];
            memcpy(m, t, sizeof m);
        }
    }
    for (int i = 0; i < 8; i++) {
        out[i] = v[i] ^ v[i + 8];
        out[i + 8] = v[i + 8] ^ cv[i];
    }
}

/* The compression every hash here runs: the portable restatement above unless the CPU
 * baseline selected the crate's SIMD row form (blake3_simd.c, or_set_simd) */
typedef void (*compress_fn)(const uint32_t *, const uint32_t *, uint64_t, uint32_t, uint32_t, uint32_t *);
static compress_fn g_compress = compress_portable;
static inline void compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter, uint32_t block_len,
                            uint32_t flags, uint32_t out[16]) {
    g_compress(cv, block, counter, block_len, flags, out);
}

int or_set_simd(int level) {
    if (level >= 2 && or_cpu_has_avx512()) {
        g_compress = or_compress_avx512vl;
        return 2;
    }
    if (level >= 1 && or_cpu_has_sse41()) {
        g_compress = or_compress_sse41;
        return 1;
    }
    g_compress = compress_portable;
    return 0;
}

static void words_from_bytes(const uint8_t *b, uint32_t w[16]) {
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
               ((uint32_t)b[4 * i + 3] << 24);
}

static void parent_cv(const uint32_t key[8], const uint32_t l[8], const uint32_t r[8],
                      uint32_t flags, uint32_t out8[8]) {
    uint32_t block[16], o[16];
    memcpy(block, l, 32);
    memcpy(block + 8, r, 32);
    compress(key, block, 0, BLOCK_LEN, PARENT | flags, o);
    memcpy(out8, o, 32);
}

void or_hasher_init(or_hasher *h) {
    memset(h, 0, sizeof *h);
    memcpy(h->key, IV, 32);
    memcpy(h->chunk_cv, IV, 32);
}

static size_t chunk_len(const or_hasher *h) {
    return (size_t)h->blocks_compressed * BLOCK_LEN + h->block_len;
}

static void chunk_output_cv(const or_hasher *h, uint32_t flags, uint32_t out16[16]) {
    uint32_t w[16];
    uint8_t blk[64];
    memset(blk, 0, 64);
    memcpy(blk, h->block, h->block_len);
    words_from_bytes(blk, w);
    uint32_t f = CHUNK_END | (h->blocks_compressed == 0 ? CHUNK_START : 0) | flags;
    compress(h->chunk_cv, w, h->chunk_counter, h->block_len, f, out16);
}

static void push_chunk_cv(or_hasher *h, uint32_t cv[8], uint64_t total_chunks) {
    while ((total_chunks & 1) == 0) {
        h->cv_stack_len--;
        parent_cv(h->key, h->cv_stack[h->cv_stack_len], cv, 0, cv);
        total_chunks >>= 1;
    }
    memcpy(h->cv_stack[h->cv_stack_len], cv, 32);
    h->cv_stack_len++;
}

void or_hasher_update(or_hasher *h, const void *data, size_t len) {
    const uint8_t *p = (const uint8_t *)data;
    while (len > 0) {
        if (chunk_len(h) == CHUNK_LEN) {
            /* the chunk is complete and more input follows: it is not the root */
            uint32_t o[16];
            chunk_output_cv(h, 0, o);
            uint64_t total = h->chunk_counter + 1;
            push_chunk_cv(h, o, total);
            memcpy(h->chunk_cv, h->key, 32);
            h->chunk_counter = total;
            h->block_len = 0;
            h->blocks_compressed = 0;
        }
        if (h->block_len == BLOCK_LEN) {
            uint32_t w[16], o[16];
            words_from_bytes(h->block, w);
            uint32_t f = h->blocks_compressed == 0 ? CHUNK_START : 0;
            compress(h->chunk_cv, w, h->chunk_counter, BLOCK_LEN, f, o);
            memcpy(h->chunk_cv, o, 32);
            h->blocks_compressed++;
            h->block_len = 0;
        }
        size_t take = BLOCK_LEN - h->block_len;
        if (take > len) take = len;
        memcpy(h->block + h->block_len, p, take);
        h->block_len += (uint32_t)take;
        p += take;
        len -= take;
    }
}

void or_hasher_finalize(const or_hasher *h, uint8_t out[32]) {
    uint32_t o[16];
    if (h->cv_stack_len == 0) {
        chunk_output_cv(h, ROOT, o);
    } else {
        uint32_t right[8];
        chunk_output_cv(h, 0, o);
        memcpy(right, o, 32);
        for (int i = (int)h->cv_stack_len - 1; i >= 0; i--) {
            uint32_t fl = (i == 0) ? ROOT : 0;
            uint32_t block[16];
            memcpy(block, h->cv_stack[i], 32);
            memcpy(block + 8, right, 32);
            compress(h->key, block, 0, BLOCK_LEN, PARENT | fl, o);
            memcpy(right, o, 32);
        }
    }
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)o[i];
        out[4 * i + 1] = (uint8_t)(o[i] >> 8);
        out[4 * i + 2] = (uint8_t)(o[i] >> 16);
        out[4 * i + 3] = (uint8_t)(o[i] >> 24);
    }
}

void or_blake3(const void *data, size_t len, uint8_t out[32]) {
    or_hasher h;
    or_hasher_init(&h);
    or_hasher_update(&h, data, len);
    or_hasher_finalize(&h, out);
}

/* ================================================================================== */
/* Canonical encoding of the fixed record schemas (rsos/src/encoding.rs:17-35)        */
/* ================================================================================== */

static inline void put_u32(uint8_t *b, size_t *o, uint32_t x) {
    if (b) { b[*o] = (uint8_t)x; b[*o + 1] = (uint8_t)(x >> 8); b[*o + 2] = (uint8_t)(x >> 16); b[*o + 3] = (uint8_t)(x >> 24); }
    *o += 4;
}
static inline void put_u64(uint8_t *b, size_t *o, uint64_t x) {
    put_u32(b, o, (uint32_t)x);
    put_u32(b, o, (uint32_t)(x >> 32));
}
static inline void put_raw(uint8_t *b, size_t *o, const uint8_t *src, size_t n) {
    if (b) memcpy(b + *o, src, n);
    *o += n;
}

/* a key: unit -> nothing; u32/u64 -> fixed LE (serializer.rs:76-84); bytes -> u64 len + bytes
 * ([u8;L] is a serde tuple -> put_len + elements, serializer.rs:176-179; Vec<u8> / String give
 * the same bytes via serialize_seq / serialize_bytes, :105-113,162-174) */
static void put_key(const or_schema *s, const uint8_t *k, uint8_t *b, size_t *o) {
    switch (s->key_kind) {
    case OR_KEY_UNIT: break;
    case OR_KEY_U32: put_raw(b, o, k, 4); break;
    case OR_KEY_U64: put_raw(b, o, k, 8); break;
    default: put_u64(b, o, s->key_len); put_raw(b, o, k, s->key_len); break;
    }
}
static void put_value(const or_schema *s, const uint8_t *v, uint8_t *b, size_t *o) {
    switch (s->value_kind) {
    case OR_VAL_UNIT: break;
    case OR_VAL_U32: put_raw(b, o, v, 4); break;
    case OR_VAL_U64: put_raw(b, o, v, 8); break;
    default: put_u64(b, o, s->value_len); put_raw(b, o, v, s->value_len); break;
    }
}

size_t or_encode_record(const or_schema *s, const or_columns *c, size_t i, uint8_t *buf) {
    size_t o = 0;
    size_t kst = s->key_kind == OR_KEY_U32 ? 4 : s->key_kind == OR_KEY_U64 ? 8 : s->key_len;
    const uint8_t *k = c->keys ? c->keys + i * kst : NULL;
    const uint8_t *v = c->values ? c->values + i * (size_t)s->value_len : NULL;
    put_key(s, k, buf, &o);
    int tomb = c->tags ? (c->tags[i] != 0) : 0;
    switch (s->record_kind) {
    case OR_REC_PLAIN:
        put_value(s, v, buf, &o);
        break;
    case OR_REC_DATED:
        /* Entry { stamp: Timestamp { hlc: Hlc { physical, logical }, node_id }, state } :
         * struct fields in declaration order, newtypes transparent (entry.rs:88-94,
         * clock.rs:143-181, serializer.rs:143-149,210-212) */
        put_u64(buf, &o, c->phys[i]);
        put_u32(buf, &o, c->logical[i]);
        put_u64(buf, &o, c->node[i]);
        /* fallthrough: State<V> */
        /* FALLTHROUGH */
    case OR_REC_PROJECTION:
        /* State::Present(v) = newtype variant 0 ; State::Tombstone = unit variant 1
         * (entry.rs:24-29; serializer.rs:133-141,151-160) */
        if (tomb) {
            put_u32(buf, &o, 1);
        } else {
            put_u32(buf, &o, 0);
            put_value(s, v, buf, &o);
        }
        break;
    }
    return o;
}

static void lift_one(const or_schema *s, const or_columns *c, size_t i, uint8_t out[32]) {
    uint8_t stackbuf[2048];
    size_t len = or_encode_record(s, c, i, NULL);
    uint8_t *buf = len <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(len);
    or_encode_record(s, c, i, buf);
    or_blake3(buf, len, out);
    if (buf != stackbuf) free(buf);
}

typedef struct {
    const or_schema *s;
    const or_columns *c;
    const uint8_t *bytes;
    const uint64_t *offsets;
    size_t lo, hi;
    uint8_t *fps;
} lift_job;

static void *lift_worker(void *arg) {
    lift_job *j = (lift_job *)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        if (j->s)
            lift_one(j->s, j->c, i, j->fps + 32 * i);
        else
            or_blake3(j->bytes + j->offsets[i], (size_t)(j->offsets[i + 1] - j->offsets[i]),
                      j->fps + 32 * i);
    }
    return NULL;
}

static void run_jobs(lift_job proto, size_t n, int threads) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = n ? (int)n : 1;
    pthread_t tid[256];
    lift_job jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (size_t)t / (size_t)threads;
        jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
        if (threads == 1) lift_worker(&jobs[t]);
        else pthread_create(&tid[t], NULL, lift_worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

void or_lift_records(const or_schema *s, const or_columns *c, size_t n, uint8_t *fps, int threads) {
    lift_job p = {s, c, NULL, NULL, 0, 0, fps};
    run_jobs(p, n, threads);
}

void or_lift_encoded(const uint8_t *bytes, const uint64_t *offsets, size_t n, uint8_t *fps, int threads) {
    lift_job p = {NULL, NULL, bytes, offsets, 0, 0, fps};
    run_jobs(p, n, threads);
}

/* ================================================================================== */
/* Fingerprint group (rsos/src/fingerprint.rs:145-173) and Aggregate (aggregate.rs)   */
/* ================================================================================== */

void or_fp_add(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    unsigned __int128 carry = 0;
    for (int i = 0; i < 4; i++) {
        unsigned __int128 s = (unsigned __int128)a[i] + b[i] + carry;
        out[i] = (uint64_t)s;
        carry = s >> 64;
    }
}

void or_fp_sub(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
    uint64_t borrow = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t d = a[i] - b[i] - borrow;
        borrow = (a[i] < b[i]) || (a[i] - b[i] < borrow);
        out[i] = d;
    }
}

static void fp_load(const uint8_t *p, uint64_t f[4]) {
    for (int l = 0; l < 4; l++) {
        uint64_t x = 0;
        for (int b = 7; b >= 0; b--) x = (x << 8) | p[8 * l + b];
        f[l] = x;
    }
}

void or_range_aggregates(const uint8_t *fps, size_t n, const uint64_t *bounds, size_t r,
                         or_aggregate *out) {
    for (size_t j = 0; j < r; j++) {
        uint64_t lo = bounds[j], hi = bounds[j + 1];
        or_aggregate a;
        memset(&a, 0, sizeof a);
        if (hi > n) hi = n;
        for (uint64_t i = lo; i < hi; i++) {
            uint64_t f[4];
            fp_load(fps + 32 * i, f);
            or_fp_add(a.fp, f, a.fp);
            a.size++;
        }
        out[j] = a;
    }
}

/* ================================================================================== */
/* FingerprintTreeMap restatement: order-6 B-tree, per-element fingerprint and       */
/* per-subtree Aggregate cache, one lift per insert (mutate.rs:23-88, node.rs:93-152) */
/* ================================================================================== */

#define FTM_B 6
#define FTM_MAX (2 * FTM_B - 1)

typedef struct ftm_node {
    uint32_t nkeys;
    size_t rec[FTM_MAX];          /* record index: key + value live in the bound columns */
    uint64_t fps[FTM_MAX][4];
    struct ftm_node *child[FTM_MAX + 1];
    int leaf;
    or_aggregate subtree;
} ftm_node;

struct or_ftm {
    or_schema s;
    or_columns c;
    size_t kst;
    ftm_node *root;
};

static ftm_node *node_new(int leaf) {
    ftm_node *n = (ftm_node *)calloc(1, sizeof(ftm_node));
    n->leaf = leaf;
    return n;
}

static void node_free(ftm_node *n) {
    if (!n) return;
    if (!n->leaf)
        for (uint32_t i = 0; i <= n->nkeys; i++) node_free(n->child[i]);
    free(n);
}

/* key order: numeric for u32/u64 (Ord of the integer), memcmp for byte keys ([u8;L] Ord) */
static int key_cmp(const or_ftm *t, const uint8_t *a, const uint8_t *b) {
    switch (t->s.key_kind) {
    case OR_KEY_U32: { uint32_t x, y; memcpy(&x, a, 4); memcpy(&y, b, 4); return (x > y) - (x < y); }
    case OR_KEY_U64: { uint64_t x, y; memcpy(&x, a, 8); memcpy(&y, b, 8); return (x > y) - (x < y); }
    case OR_KEY_UNIT: return 0;
    default: return memcmp(a, b, t->kst);
    }
}

static const uint8_t *rec_key(const or_ftm *t, size_t rec) { return t->c.keys + rec * t->kst; }

or_ftm *or_ftm_new(const or_schema *s, const or_columns *c) {
    or_ftm *t = (or_ftm *)calloc(1, sizeof(or_ftm));
    t->s = *s;
    t->c = *c;
    t->kst = s->key_kind == OR_KEY_U32 ? 4 : s->key_kind == OR_KEY_U64 ? 8 : s->key_len;
    t->root = node_new(1);
    return t;
}

void or_ftm_free(or_ftm *t) {
    if (!t) return;
    node_free(t->root);
    free(t);
}

static void agg_add(or_aggregate *a, uint64_t size, const uint64_t fp[4]) {
    or_fp_add(a->fp, fp, a->fp);
    a->size += size;
}

static void refresh(ftm_node *n) {
    or_aggregate a;
    memset(&a, 0, sizeof a);
    for (uint32_t i = 0; i < n->nkeys; i++) agg_add(&a, 1, n->fps[i]);
    if (!n->leaf)
        for (uint32_t i = 0; i <= n->nkeys; i++) agg_add(&a, n->child[i]->subtree.size, n->child[i]->subtree.fp);
    n->subtree = a;
}

typedef struct {
    int split;
    size_t rec;
    uint64_t fp[4];
    ftm_node *right;
} split_t;

/* Node::insert (node.rs:93-152): insert at `idx`, splitting a full node at mid */
static split_t node_insert(ftm_node *n, uint32_t idx, size_t rec, const uint64_t fp[4],
                           ftm_node *right_child, const uint64_t diff[4]) {
    split_t res = {0, 0, {0, 0, 0, 0}, NULL};
    if (n->nkeys == FTM_MAX) {
        uint32_t mid = n->nkeys / 2;
        ftm_node *sib = node_new(n->leaf);
        sib->nkeys = n->nkeys - (mid + 1);
        memcpy(sib->rec, n->rec + mid + 1, sib->nkeys * sizeof(size_t));
        memcpy(sib->fps, n->fps + mid + 1, sib->nkeys * sizeof(n->fps[0]));
        if (!n->leaf) memcpy(sib->child, n->child + mid + 1, (sib->nkeys + 1) * sizeof(ftm_node *));
        res.split = 1;
        res.rec = n->rec[mid];
        memcpy(res.fp, n->fps[mid], 32);
        n->nkeys = mid;
        split_t inner;
        if (idx <= mid) inner = node_insert(n, idx, rec, fp, right_child, diff);
        else inner = node_insert(sib, idx - mid - 1, rec, fp, right_child, diff);
        (void)inner;
        refresh(n);
        refresh(sib);
        res.right = sib;
        return res;
    }
    memmove(n->rec + idx + 1, n->rec + idx, (n->nkeys - idx) * sizeof(size_t));
    memmove(n->fps + idx + 1, n->fps + idx, (n->nkeys - idx) * sizeof(n->fps[0]));
    n->rec[idx] = rec;
    memcpy(n->fps[idx], fp, 32);
    if (!n->leaf) {
        memmove(n->child + idx + 2, n->child + idx + 1, (n->nkeys - idx) * sizeof(ftm_node *));
        n->child[idx + 1] = right_child;
    }
    n->nkeys++;
    agg_add(&n->subtree, 1, diff);
    return res;
}

/* binary search: returns 1 + sets *idx if found, else 0 + insertion index */
static int node_search(const or_ftm *t, const ftm_node *n, const uint8_t *key, uint32_t *idx) {
    uint32_t lo = 0, hi = n->nkeys;
    while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        int c = key_cmp(t, rec_key(t, n->rec[mid]), key);
        if (c == 0) { *idx = mid; return 1; }
        if (c < 0) lo = mid + 1; else hi = mid;
    }
    *idx = lo;
    return 0;
}

static void ftm_lift(const or_ftm *t, size_t rec, uint64_t fp[4]) {
    uint8_t out[32];
    lift_one(&t->s, &t->c, rec, out);
    fp_load(out, fp);
}

/* FingerprintTreeMap::insert's aux (mutate.rs:23-70) */
static split_t ins_aux(or_ftm *t, ftm_node *n, size_t rec, uint64_t diff[4], int *was_new) {
    uint32_t idx;
    const uint8_t *key = rec_key(t, rec);
    split_t none = {0, 0, {0, 0, 0, 0}, NULL};
    if (node_search(t, n, key, &idx)) {
        uint64_t nf[4];
        ftm_lift(t, rec, nf);
        or_fp_sub(nf, n->fps[idx], diff);
        memcpy(n->fps[idx], nf, 32);
        n->rec[idx] = rec;
        agg_add(&n->subtree, 0, diff);
        *was_new = 0;
        return none;
    }
    if (!n->leaf) {
        split_t s = ins_aux(t, n->child[idx], rec, diff, was_new);
        if (s.split) return node_insert(n, idx, s.rec, s.fp, s.right, diff);
        agg_add(&n->subtree, *was_new ? 1 : 0, diff);
        return none;
    }
    uint64_t fp[4];
    ftm_lift(t, rec, fp);
    memcpy(diff, fp, 32);
    *was_new = 1;
    return node_insert(n, idx, rec, fp, NULL, fp);
}

int or_ftm_insert(or_ftm *t, size_t i) {
    uint64_t diff[4];
    int was_new = 0;
    split_t s = ins_aux(t, t->root, i, diff, &was_new);
    if (s.split) {
        ftm_node *r = node_new(0);
        r->nkeys = 1;
        r->rec[0] = s.rec;
        memcpy(r->fps[0], s.fp, 32);
        r->child[0] = t->root;
        r->child[1] = s.right;
        refresh(r);
        t->root = r;
    }
    return was_new;
}

void or_ftm_fill(or_ftm *t, size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; i++) or_ftm_insert(t, i);
}

size_t or_ftm_len(const or_ftm *t) { return (size_t)t->root->subtree.size; }

void or_ftm_root(const or_ftm *t, or_aggregate *out) { *out = t->root->subtree; }

/* FingerprintTreeMap::aggregate (query.rs:25-76) for a half-open [lo, hi) key range */
static void agg_aux(const or_ftm *t, const ftm_node *n, const uint8_t *lo, const uint8_t *hi,
                    const uint8_t *lb, const uint8_t *ub, or_aggregate *cum) {
    int lo_in = lo == NULL || (lb != NULL && key_cmp(t, lo, lb) < 0);
    int hi_in = hi == NULL || (ub != NULL && key_cmp(t, hi, ub) > 0);
    if (lo_in && hi_in) {
        agg_add(cum, n->subtree.size, n->subtree.fp);
        return;
    }
    uint32_t i = 0;
    while (i < n->nkeys && lo && key_cmp(t, rec_key(t, n->rec[i]), lo) < 0) i++;
    while (i < n->nkeys && (hi == NULL || key_cmp(t, rec_key(t, n->rec[i]), hi) < 0)) {
        const uint8_t *cur = rec_key(t, n->rec[i]);
        if (!n->leaf) agg_aux(t, n->child[i], lo, hi, lb, cur, cum);
        agg_add(cum, 1, n->fps[i]);
        lb = cur;
        i++;
    }
    if (!n->leaf) agg_aux(t, n->child[i], lo, hi, lb, ub, cum);
}

void or_ftm_aggregate(const or_ftm *t, const uint8_t *lo_key, const uint8_t *hi_key,
                      or_aggregate *out) {
    memset(out, 0, sizeof *out);
    if (lo_key && hi_key && key_cmp(t, lo_key, hi_key) >= 0) return;
    agg_aux(t, t->root, lo_key, hi_key, NULL, NULL, out);
}

/* FingerprintTreeMap::rank (query.rs:93-121) */
size_t or_ftm_rank(const or_ftm *t, const uint8_t *key) {
    const ftm_node *n = t->root;
    size_t index = 0;
    while (!n->leaf) {
        uint32_t i;
        int descended = 0;
        for (i = 0; i < n->nkeys; i++) {
            int c = key_cmp(t, rec_key(t, n->rec[i]), key);
            if (c > 0) { n = n->child[i]; descended = 1; break; }
            index += n->child[i]->subtree.size;
            if (c == 0) return index;
            index += 1;
        }
        if (!descended) n = n->child[n->nkeys];
    }
    uint32_t idx;
    node_search(t, n, key, &idx);
    return index + idx;
}

/* select(index): the index-th key (query.rs:142-161).  Returns the record row holding it, or
 * (size_t)-1 when index >= len (the reference panics). */
size_t or_ftm_select(const or_ftm *t, size_t index) {
    const ftm_node *n = t->root;
    if (index >= n->subtree.size) return (size_t)-1;
    while (!n->leaf) {
        const ftm_node *next = n->child[n->nkeys];
        for (uint32_t i = 0; i < n->nkeys; i++) {
            const size_t sub = n->child[i]->subtree.size;
            if (index < sub) { next = n->child[i]; break; }
            index -= sub;
            if (index == 0) return n->rec[i];
            index -= 1;
        }
        n = next;
    }
    return n->rec[index];
}

/* ---- rbsr protocol rounds over two FTMs (the CPU baseline of bench.py --config rbsr) ----------
 * protocol_round_with_policy (rbsr/src/protocol.rs:212-317) under FixedFanOut(b), restated one
 * question at a time as the reference asks them: aggregate(range) (:230), rank of both bounds
 * (protocol/rank.rs:85-125), shared_cutoffs + ceil(span / b) (policy/cutoffs.rs,
 * fixed_fan_out.rs), and per SPLIT child select(cut) + aggregate(child) (:288-313).  Rounds
 * alternate between the two trees until no segment is left, starting from a's root. */
typedef struct {
    uint8_t sk, ek;           /* 0 Unbounded, 1 Included / Excluded */
    uint8_t skey[32], ekey[32];
    or_aggregate agg;
} or_seg;

typedef struct { or_seg *v; size_t n, cap; } seg_vec;

static void seg_push(seg_vec *q, const or_seg *x) {
    if (q->n == q->cap) {
        q->cap = q->cap ? 2 * q->cap : 64;
        q->v = (or_seg *)realloc(q->v, q->cap * sizeof(or_seg));
    }
    q->v[q->n++] = *x;
}

static void seg_bounds(const or_seg *g, const uint8_t **lo, const uint8_t **hi) {
    *lo = g->sk ? g->skey : NULL;
    *hi = g->ek ? g->ekey : NULL;
}

/* one round on tree t: returns the number of IDLIST (enumerated) segments */
static size_t round_fixed(const or_ftm *t, size_t b, const seg_vec *in, seg_vec *out) {
    size_t enumerated = 0;
    const size_t size = t->root->subtree.size;
    for (size_t j = 0; j < in->n; j++) {
        const or_seg *g = &in->v[j];
        const uint8_t *lo, *hi;
        seg_bounds(g, &lo, &hi);
        or_aggregate local;
        or_ftm_aggregate(t, lo, hi, &local);
        const size_t raw_s = lo ? or_ftm_rank(t, lo) : 0, raw_e = hi ? or_ftm_rank(t, hi) : size;
        if (raw_e < raw_s) continue; /* dropped as malformed */
        const size_t si = raw_s < size ? raw_s : size, ei = raw_e < size ? raw_e : size;
        const uint64_t span = local.size, remote = g->agg.size;
        int kind; /* 0 skip, 1 enumerate, 2 split */
        uint64_t stride = 0;
        if (span == remote && !memcmp(local.fp, g->agg.fp, 32)) kind = 0;
        else if (remote == 0) kind = 1;
        else if (span == 0) kind = 2, stride = 1;
        else if (span == 1 && remote == 1) kind = 1;
        else if (span == 1) kind = 2, stride = 1;
        else kind = 2, stride = (span + b - 1) / b;
        if (kind == 2 && span > 1 && stride >= span) kind = 1;
        if (kind == 1) {
            enumerated++;
            if (remote != 0) {
                or_seg c = *g;
                memset(&c.agg, 0, sizeof c.agg);
                seg_push(out, &c);
            }
        } else if (kind == 2) {
            or_seg c = *g;
            size_t cur = si;
            for (;;) {
                const size_t nxt = cur + stride;
                if (!(nxt < ei)) {
                    c.ek = g->ek;
                    memcpy(c.ekey, g->ekey, sizeof c.ekey);
                    if (cur == si) c.agg = local;
                    else {
                        seg_bounds(&c, &lo, &hi);
                        or_ftm_aggregate(t, lo, hi, &c.agg);
                    }
                    seg_push(out, &c);
                    break;
                }
                c.ek = 1;
                memcpy(c.ekey, rec_key(t, or_ftm_select(t, nxt)), t->kst);
                seg_bounds(&c, &lo, &hi);
                or_ftm_aggregate(t, lo, hi, &c.agg);
                seg_push(out, &c);
                c.sk = 1;
                memcpy(c.skey, c.ekey, sizeof c.skey);
                cur = nxt;
            }
        }
    }
    return enumerated;
}

int or_reconcile_fixed(const or_ftm *a, const or_ftm *bt, size_t fan_out, uint64_t out[3]) {
    if (a->kst > 32 || bt->kst > 32) return -1;
    const size_t b = fan_out < 2 ? 2 : fan_out;
    seg_vec cur = {0}, nxt = {0};
    or_seg root;
    memset(&root, 0, sizeof root);
    or_ftm_root(a, &root.agg);
    seg_push(&cur, &root);
    uint64_t rounds = 0, segs = 0, enums = 0;
    while (cur.n) {
        segs += cur.n;
        nxt.n = 0;
        enums += round_fixed(rounds % 2 ? a : bt, b, &cur, &nxt);
        seg_vec t = cur;
        cur = nxt;
        nxt = t;
        rounds++;
    }
    free(cur.v);
    free(nxt.v);
    out[0] = rounds;
    out[1] = segs;
    out[2] = enums;
    return 0;
}

static int check_aux(const ftm_node *n) {
    if (!n->leaf)
        for (uint32_t i = 0; i <= n->nkeys; i++)
            if (check_aux(n->child[i])) return -1;
    or_aggregate a;
    memset(&a, 0, sizeof a);
    for (uint32_t i = 0; i < n->nkeys; i++) agg_add(&a, 1, n->fps[i]);
    if (!n->leaf)
        for (uint32_t i = 0; i <= n->nkeys; i++) agg_add(&a, n->child[i]->subtree.size, n->child[i]->subtree.fp);
    if (a.size != n->subtree.size || memcmp(a.fp, n->subtree.fp, 32) != 0) return -1;
    return 0;
}

int or_ftm_check(const or_ftm *t) { return check_aux(t->root); }
