/*
 * blake3_simd.c -- SIMD BLAKE3 compressions for the CPU baseline (TEST INFRASTRUCTURE ONLY, like
 * the rest of oracle/; see oracle.h).
 *
 * The reference hashes through crate blake3 1.8.5 (Cargo.lock:197-200), which dispatches at run
 * time to SIMD backends it builds with `cc`.  For the short inputs of
 * this path (one record = one BLAKE3 input of 8 .. 1,080 bytes, fed by Hasher::update) the crate
 * compresses one block at a time with its row-vector `compress_in_place` (SSE4.1, or AVX-512VL
 * where present): the 4x4 state in four 128-bit rows, the G function on all four columns at
 * once, diagonalisation by lane shuffles.  `compress_rows_*` restate that form, so the CPU
 * baseline times what the reference's CPU path actually runs rather than a portable C stand-in.
 *
 * `or_lift_records_x16` is NOT the reference's code path: a 16-records-at-a-time AVX-512
 * transposition (one record per 32-bit lane, the layout the GPU kernels use per wavefront),
 * reported separately as the best batch lift this CPU can do.
 *
 * Both are checked bit for bit against the portable restatement (tests/test_oracle.py).
 */
#include "oracle.h"

#include <immintrin.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static const uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                               0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
/* the message word order of each of the 7 rounds (the permutation applied r times) */
static const uint8_t SCHED[7][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8},
    {3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1},
    {10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6},
    {12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4},
    {9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7},
    {11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13},
};
enum { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

/* ---- row form (the crate's compress_in_place) ------------------------------------------------ */

#define ROWS_BODY(ROT16, ROT12, ROT8, ROT7)                                                              \
    __m128i r0 = _mm_loadu_si128((const __m128i *)cv), r1 = _mm_loadu_si128((const __m128i *)(cv + 4)); \
    __m128i r2 = _mm_loadu_si128((const __m128i *)IV);                                                   \
    __m128i r3 = _mm_set_epi32((int)flags, (int)block_len, (int)(uint32_t)(counter >> 32), (int)(uint32_t)counter); \
    for (int r = 0; r < 7; r++) {                                                                        \
        const uint8_t *s = SCHED[r];                                                                     \
        __m128i mx = _mm_set_epi32((int)m[s[6]], (int)m[s[4]], (int)m[s[2]], (int)m[s[0]]);              \
        __m128i my = _mm_set_epi32((int)m[s[7]], (int)m[s[5]], (int)m[s[3]], (int)m[s[1]]);              \
        r0 = _mm_add_epi32(_mm_add_epi32(r0, mx), r1);                                                   \
        r3 = ROT16(_mm_xor_si128(r3, r0));                                                               \
        r2 = _mm_add_epi32(r2, r3);                                                                      \
        r1 = ROT12(_mm_xor_si128(r1, r2));                                                               \
        r0 = _mm_add_epi32(_mm_add_epi32(r0, my), r1);                                                   \
        r3 = ROT8(_mm_xor_si128(r3, r0));                                                                \
        r2 = _mm_add_epi32(r2, r3);                                                                      \
        r1 = ROT7(_mm_xor_si128(r1, r2));                                                                \
        /* diagonalise: lane j of (r0, r1, r2, r3) = (v[j+3], v[4+j], v[8+j+1], v[12+j+2]) (mod 4) */   \
        r0 = _mm_shuffle_epi32(r0, _MM_SHUFFLE(2, 1, 0, 3));                                             \
        r3 = _mm_shuffle_epi32(r3, _MM_SHUFFLE(1, 0, 3, 2));                                             \
        r2 = _mm_shuffle_epi32(r2, _MM_SHUFFLE(0, 3, 2, 1));                                             \
        /* lanes: G(3,4,9,14) G(0,5,10,15) G(1,6,11,12) G(2,7,8,13) */                                  \
        mx = _mm_set_epi32((int)m[s[12]], (int)m[s[10]], (int)m[s[8]], (int)m[s[14]]);                   \
        my = _mm_set_epi32((int)m[s[13]], (int)m[s[11]], (int)m[s[9]], (int)m[s[15]]);                   \
        r0 = _mm_add_epi32(_mm_add_epi32(r0, mx), r1);                                                   \
        r3 = ROT16(_mm_xor_si128(r3, r0));                                                               \
        r2 = _mm_add_epi32(r2, r3);                                                                      \
        r1 = ROT12(_mm_xor_si128(r1, r2));                                                               \
        r0 = _mm_add_epi32(_mm_add_epi32(r0, my), r1);                                                   \
        r3 = ROT8(_mm_xor_si128(r3, r0));                                                                \
        r2 = _mm_add_epi32(r2, r3);                                                                      \
        r1 = ROT7(_mm_xor_si128(r1, r2));                                                                \
        r0 = _mm_shuffle_epi32(r0, _MM_SHUFFLE(0, 3, 2, 1));                                             \
        r3 = _mm_shuffle_epi32(r3, _MM_SHUFFLE(1, 0, 3, 2));                                             \
        r2 = _mm_shuffle_epi32(r2, _MM_SHUFFLE(2, 1, 0, 3));                                             \
    }                                                                                                    \
    const __m128i c0 = _mm_loadu_si128((const __m128i *)cv), c1 = _mm_loadu_si128((const __m128i *)(cv + 4)); \
    _mm_storeu_si128((__m128i *)out, _mm_xor_si128(r0, r2));                                             \
    _mm_storeu_si128((__m128i *)(out + 4), _mm_xor_si128(r1, r3));                                       \
    _mm_storeu_si128((__m128i *)(out + 8), _mm_xor_si128(r2, c0));                                       \
    _mm_storeu_si128((__m128i *)(out + 12), _mm_xor_si128(r3, c1));

__attribute__((target("sse4.1,ssse3"))) static inline __m128i rot16_sse(__m128i x) {
    return _mm_shuffle_epi8(x, _mm_set_epi8(13, 12, 15, 14, 9, 8, 11, 10, 5, 4, 7, 6, 1, 0, 3, 2));
}
__attribute__((target("sse4.1,ssse3"))) static inline __m128i rot8_sse(__m128i x) {
    return _mm_shuffle_epi8(x, _mm_set_epi8(12, 15, 14, 13, 8, 11, 10, 9, 4, 7, 6, 5, 0, 3, 2, 1));
}
#define ROT12_SSE(x) _mm_or_si128(_mm_srli_epi32((x), 12), _mm_slli_epi32((x), 20))
#define ROT7_SSE(x) _mm_or_si128(_mm_srli_epi32((x), 7), _mm_slli_epi32((x), 25))

__attribute__((target("sse4.1,ssse3"))) void or_compress_sse41(const uint32_t cv[8], const uint32_t m[16],
                                                               uint64_t counter, uint32_t block_len, uint32_t flags,
                                                               uint32_t out[16]) {
    ROWS_BODY(rot16_sse, ROT12_SSE, rot8_sse, ROT7_SSE)
}

#define ROT16_VL(x) _mm_ror_epi32((x), 16)
#define ROT12_VL(x) _mm_ror_epi32((x), 12)
#define ROT8_VL(x) _mm_ror_epi32((x), 8)
#define ROT7_VL(x) _mm_ror_epi32((x), 7)
__attribute__((target("avx512f,avx512vl"))) void or_compress_avx512vl(const uint32_t cv[8], const uint32_t m[16],
                                                                      uint64_t counter, uint32_t block_len,
                                                                      uint32_t flags, uint32_t out[16]) {
    ROWS_BODY(ROT16_VL, ROT12_VL, ROT8_VL, ROT7_VL)
}

int or_cpu_has_avx512(void) {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl");
}
int or_cpu_has_sse41(void) {
    __builtin_cpu_init();
    return __builtin_cpu_supports("sse4.1") && __builtin_cpu_supports("ssse3");
}

/* ---- 16 records at a time (AVX-512F, one record per 32-bit lane) ------------------------------ */

#define G16(a, b, c, d, mx, my)                                  \
    do {                                                         \
        a = _mm512_add_epi32(_mm512_add_epi32(a, b), mx);        \
        d = _mm512_ror_epi32(_mm512_xor_si512(d, a), 16);        \
        c = _mm512_add_epi32(c, d);                              \
        b = _mm512_ror_epi32(_mm512_xor_si512(b, c), 12);        \
        a = _mm512_add_epi32(_mm512_add_epi32(a, b), my);        \
        d = _mm512_ror_epi32(_mm512_xor_si512(d, a), 8);         \
        c = _mm512_add_epi32(c, d);                              \
        b = _mm512_ror_epi32(_mm512_xor_si512(b, c), 7);         \
    } while (0)

/* cv[8] <- the first 8 output words of 16 compressions (same counter / length / flags) */
__attribute__((target("avx512f"))) static void compress16(__m512i cv[8], const __m512i m[16], uint64_t counter,
                                                          uint32_t block_len, uint32_t flags) {
    __m512i v[16];
    for (int i = 0; i < 8; i++) v[i] = cv[i];
    for (int i = 0; i < 4; i++) v[8 + i] = _mm512_set1_epi32((int)IV[i]);
    v[12] = _mm512_set1_epi32((int)(uint32_t)counter);
    v[13] = _mm512_set1_epi32((int)(uint32_t)(counter >> 32));
    v[14] = _mm512_set1_epi32((int)block_len);
    v[15] = _mm512_set1_epi32((int)flags);
    for (int r = 0; r < 7; r++) {
        const uint8_t *s = SCHED[r];
        G16(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]);
        G16(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
        G16(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]);
        G16(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
        G16(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]);
        G16(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
        G16(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]);
        G16(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; i++) cv[i] = _mm512_xor_si512(v[i], v[i + 8]);
}

__attribute__((target("avx512f"))) static void parent16(__m512i out[8], const __m512i l[8], const __m512i r[8],
                                                        uint32_t flags) {
    __m512i m[16];
    for (int i = 0; i < 8; i++) m[i] = l[i], m[8 + i] = r[i];
    for (int i = 0; i < 8; i++) out[i] = _mm512_set1_epi32((int)IV[i]);
    compress16(out, m, 0, 64, PARENT | flags);
}

/* BLAKE3 of 16 inputs of the same length `len`, row i at tile + i * stride (stride a multiple of 64,
 * rows zero-padded to it): 16 hashes into out (32 B each) */
__attribute__((target("avx512f"))) static void hash16(const uint8_t *tile, size_t stride, size_t len, uint8_t *out[16]) {
    const __m512i idx = _mm512_mullo_epi32(_mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15),
                                           _mm512_set1_epi32((int)stride));
    const size_t nchunks = len == 0 ? 1 : (len + 1023) / 1024;
    __m512i stack[54][8], cv[8];
    int sp = 0;
    for (size_t c = 0; c < nchunks; c++) {
        const size_t cbeg = c * 1024, clen = len - cbeg < 1024 ? len - cbeg : 1024;
        const size_t nb = clen == 0 ? 1 : (clen + 63) / 64;
        for (int i = 0; i < 8; i++) cv[i] = _mm512_set1_epi32((int)IV[i]);
        for (size_t b = 0; b < nb; b++) {
            const size_t boff = cbeg + 64 * b, blen = len - boff < 64 ? len - boff : 64;
            __m512i m[16];
            for (int w = 0; w < 16; w++)
                m[w] = _mm512_i32gather_epi32(idx, (const void *)(tile + boff + 4 * w), 1);
            uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b + 1 == nb ? CHUNK_END : 0);
            if (nchunks == 1 && b + 1 == nb) flags |= ROOT;
            compress16(cv, m, c, (uint32_t)blen, flags);
        }
        if (c + 1 < nchunks) {
            uint64_t total = c + 1;
            while ((total & 1) == 0) {
                sp--;
                parent16(cv, stack[sp], cv, 0);
                total >>= 1;
            }
            for (int i = 0; i < 8; i++) stack[sp][i] = cv[i];
            sp++;
        }
    }
    for (int s = sp - 1; s >= 0; s--) parent16(cv, stack[s], cv, s == 0 ? ROOT : 0);
    uint32_t t[8][16];
    for (int i = 0; i < 8; i++) _mm512_storeu_si512((void *)t[i], cv[i]);
    for (int j = 0; j < 16; j++)
        for (int i = 0; i < 8; i++) memcpy(out[j] + 4 * i, &t[i][j], 4);
}

typedef struct {
    const or_schema *s;
    const or_columns *c;
    size_t lo, hi;
    uint8_t *fps;
} job16;

__attribute__((target("avx512f"))) static void *worker16(void *arg) {
    job16 *j = (job16 *)arg;
    uint8_t enc[2304];
    size_t maxlen = 0;
    /* the tile: 16 rows of the longest record, padded to 64 B */
    for (size_t i = j->lo; i < j->hi && i < j->lo + 1; i++) maxlen = or_encode_record(j->s, j->c, i, NULL);
    size_t stride = ((maxlen + 63) / 64) * 64 + 64;
    uint8_t *tile = (uint8_t *)aligned_alloc(64, 16 * stride);
    for (size_t g = j->lo; g < j->hi; g += 16) {
        const size_t cnt = j->hi - g < 16 ? j->hi - g : 16;
        size_t len0 = or_encode_record(j->s, j->c, g, NULL);
        int same = cnt == 16 && len0 + 64 <= stride;
        for (size_t k = 1; same && k < cnt; k++) same = or_encode_record(j->s, j->c, g + k, NULL) == len0;
        if (!same) { /* ragged group (tombstones, the tail): one record at a time */
            for (size_t k = 0; k < cnt; k++) {
                const size_t len = or_encode_record(j->s, j->c, g + k, NULL);
                uint8_t *buf = len <= sizeof enc ? enc : (uint8_t *)malloc(len);
                or_encode_record(j->s, j->c, g + k, buf);
                or_blake3(buf, len, j->fps + 32 * (g + k));
                if (buf != enc) free(buf);
            }
            continue;
        }
        uint8_t *outs[16];
        for (size_t k = 0; k < 16; k++) {
            uint8_t *row = tile + k * stride;
            or_encode_record(j->s, j->c, g + k, row);
            memset(row + len0, 0, stride - len0);
            outs[k] = j->fps + 32 * (g + k);
        }
        hash16(tile, stride, len0, outs);
    }
    free(tile);
    return NULL;
}

int or_lift_records_x16(const or_schema *s, const or_columns *c, size_t n, uint8_t *fps, int threads) {
    if (!or_cpu_has_avx512()) return -1;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    job16 jobs[256];
    const size_t groups = (n + 15) / 16;  /* whole groups of 16 rows per thread */
    for (int t = 0; t < threads; t++) {
        const size_t g0 = groups * (size_t)t / (size_t)threads, g1 = groups * (size_t)(t + 1) / (size_t)threads;
        jobs[t] = (job16){s, c, 16 * g0 < n ? 16 * g0 : n, 16 * g1 < n ? 16 * g1 : n, fps};
    }
    for (int t = 0; t < threads; t++) {
        if (threads == 1) worker16(&jobs[t]);
        else pthread_create(&tid[t], NULL, worker16, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    return 0;
}
