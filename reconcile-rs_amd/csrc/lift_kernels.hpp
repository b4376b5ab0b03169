// lift_kernels.hpp -- schema-specialised lift kernels: canonical encoding synthesised in
// registers + BLAKE3, one record per lane, fused with the per-block fingerprint sum.
//
// Reference path being replaced (per record):
//   rsos::lift(&k, &v)                         rsos/src/fingerprint.rs:270-275
//     = BLAKE3(canon(k) || canon(v))           rsos/src/encoding.rs:117-119 (encode_into)
//   with v = Entry<Timestamp, V> / State<V>    lww-register/src/entry.rs:24-29,88-94
//   the per-insert calls in FingerprintTreeMap::insert (mutate.rs:34,61) and the two lifts of
//   Replica::map_insert (src/replica/write.rs:44-45).
//
// Layout in HBM (SoA, row i = record i): keys[n][KL], phys[n] u64, logical[n] u32,
// node[n] u64, tags[n] u8 (optional), values[n][VL]; output fps[n][32] + block_sums[n/256][32].
// Only key / stamp / tag / value bytes are read; every framing byte of the canonical
// encoding (length prefixes, variant indices) is a compile-time constant folded into the
// message words.  All field offsets are multiples of 4 for the instantiated schemas, so the
// message words are whole loaded dwords -- no byte shuffling.
#pragma once
#include "blake3_device.hpp"

namespace rh {

enum { KEY_UNIT = 0, KEY_U32 = 1, KEY_U64 = 2, KEY_BYTES = 3 };
enum { VAL_UNIT = 0, VAL_U32 = 1, VAL_U64 = 2, VAL_BYTES = 3 };
enum { REC_PLAIN = 0, REC_DATED = 1, REC_PROJECTION = 2 };

struct DevCols {
    const uint8_t *keys;
    const uint64_t *phys;
    const uint32_t *logical;
    const uint64_t *node;
    const uint8_t *tags;
    const uint8_t *values;
    // optional: record i's fingerprint goes to row dst[i] of fps (the batch path's sorted slot,
    // written by the key sort that runs before the lift; rows with dst[i] >= n are not written);
    // block sums are not formed then
    const uint32_t *dst = nullptr;
    // optional, with dst: dst[i] is an index into dst2, which holds the row (the bucket sort's
    // two-level positions: each input row's slot in its bucket's stretch, written in input order,
    // and each slot's sorted row, written in slot order -- both whole-line writes)
    const uint32_t *dst2 = nullptr;
};

constexpr int lowbit(int x) { return x & -x; }
constexpr int cmin(int a, int b) { return a < b ? a : b; }

// Byte layout of one canonical record (rsos/src/encoding.rs:17-35).
template <int KK, int KL, int VK, int VL, int RK>
struct Layout {
    static constexpr int KEY_ROW = KK == KEY_UNIT ? 0 : KK == KEY_U32 ? 4 : KK == KEY_U64 ? 8 : KL;
    static constexpr int KEY_ENC = KK == KEY_BYTES ? 8 + KL : KEY_ROW;  // u64 length prefix
    static constexpr int STAMP = RK == REC_DATED ? 20 : 0;              // u64 + u32 + u64
    static constexpr int TAG = RK == REC_PLAIN ? 0 : 4;                 // u32 variant index
    static constexpr int VAL_ROW = VK == VAL_UNIT ? 0 : VK == VAL_U32 ? 4 : VK == VAL_U64 ? 8 : VL;
    static constexpr int VAL_PREFIX = VK == VAL_BYTES ? 8 : 0;          // u64 length prefix
    static constexpr int P = KEY_ENC + STAMP + TAG + VAL_PREFIX;        // bytes before the payload
    static constexpr int LEN = P + VAL_ROW;                             // present record
    static constexpr int LEN_TOMB = KEY_ENC + STAMP + 4;                // State::Tombstone
    static constexpr int PW = P / 4, VW = VAL_ROW / 4;
    static constexpr int ROW_ALIGN = VAL_ROW == 0 ? 16 : cmin(16, lowbit(VAL_ROW));
    // whole message in registers up to 192 B (or when the prefix spills past block 0);
    // otherwise the value is streamed block by block
    static constexpr bool SMALL = LEN <= 192 || P > 64;
    static constexpr bool OK = (KEY_ROW % 4 == 0) && (VAL_ROW % 4 == 0) && (!SMALL || LEN <= 1024);
};

// ---- loads --------------------------------------------------------------------------------

// N consecutive dwords from p, with p known to be ALIGN-byte aligned
template <int N, int ALIGN>
__device__ __forceinline__ void ldw(const uint8_t *p, uint32_t *out) {
    int k = 0;
    if constexpr (ALIGN >= 16) {
#pragma unroll
        for (; k + 4 <= N; k += 4) {
            uint4 v = *reinterpret_cast<const uint4 *>(p + 4 * k);
            out[k] = v.x; out[k + 1] = v.y; out[k + 2] = v.z; out[k + 3] = v.w;
        }
    }
    if constexpr (ALIGN >= 8) {
#pragma unroll
        for (; k + 2 <= N; k += 2) {
            uint2 v = *reinterpret_cast<const uint2 *>(p + 4 * k);
            out[k] = v.x; out[k + 1] = v.y;
        }
    }
#pragma unroll
    for (; k < N; k++) out[k] = *reinterpret_cast<const uint32_t *>(p + 4 * k);
}

// key encoding words: u32 / u64 raw LE; bytes -> [len lo, len hi, bytes...]
template <int KK, int KL, class I = uint64_t>
__device__ __forceinline__ void load_key(const uint8_t *keys, I i, uint32_t *kw) {
    if constexpr (KK == KEY_U32) {
        kw[0] = reinterpret_cast<const uint32_t *>(keys)[i];
    } else if constexpr (KK == KEY_U64) {
        uint2 v = reinterpret_cast<const uint2 *>(keys)[i];
        kw[0] = v.x; kw[1] = v.y;
    } else if constexpr (KK == KEY_BYTES) {
        kw[0] = (uint32_t)KL;
        kw[1] = 0;
        ldw<KL / 4, cmin(16, lowbit(KL))>(keys + i * (I)KL, kw + 2);
    }
}

// Timestamp{hlc{physical u64, logical u32}, node_id u64}: 5 words (clock.rs:143-181)
template <class I = uint64_t>
__device__ __forceinline__ void load_stamp(const DevCols &c, I i, uint32_t *sw) {
    uint64_t ph = c.phys[i], nd = c.node[i];
    sw[0] = (uint32_t)ph; sw[1] = (uint32_t)(ph >> 32);
    sw[2] = c.logical[i];
    sw[3] = (uint32_t)nd; sw[4] = (uint32_t)(nd >> 32);
}

// Build the P/4 prefix words of a present record (or LEN_TOMB/4 words of a tombstone).
template <class L, int KK, int RK>
__device__ __forceinline__ void build_prefix(const uint32_t *kw, const uint32_t *sw, bool tomb,
                                             uint32_t *pw) {
    constexpr int KWN = L::KEY_ENC / 4;
    int o = 0;
#pragma unroll
    for (int j = 0; j < KWN; j++) pw[o++] = kw[j];
    if constexpr (RK == REC_DATED) {
#pragma unroll
        for (int j = 0; j < 5; j++) pw[o++] = sw[j];
    }
    if constexpr (RK != REC_PLAIN) pw[o++] = tomb ? 1u : 0u;  // State variant index
    if constexpr (L::VAL_PREFIX == 8) {
        if (!tomb) { pw[o++] = (uint32_t)L::VAL_ROW; pw[o++] = 0; }
    }
}

// ---- hashing: whole message in registers (LEN <= 1024) -----------------------------------
template <int LEN>
__device__ __forceinline__ void hash_words(const uint32_t *w, uint32_t out[8]) {
    constexpr int NW = LEN / 4;
    constexpr int NB = LEN == 0 ? 1 : (LEN + 63) / 64;
    static_assert(LEN <= CHUNK_LEN, "single chunk only");
    cv_iv(out);
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint32_t m[16];
#pragma unroll
        for (int j = 0; j < 16; j++) m[j] = (16 * b + j < NW) ? w[16 * b + j] : 0u;
        const uint32_t flags = (b == 0 ? CHUNK_START : 0) | (b == NB - 1 ? (CHUNK_END | ROOT) : 0);
        const uint32_t blen = (b == NB - 1) ? (uint32_t)(LEN - 64 * b) : 64u;
        compress(out, m, 0, 0, blen, flags);
    }
}

// ---- hashing: streamed value (LEN > 192, possibly several chunks) ------------------------
// Block 0 = the prefix words + the first value words; the other blocks are pure value bytes
// loaded as they are consumed; chunk boundaries and the CV-stack merges are resolved at
// compile time (template recursion over chunks), so the stack lives in registers.
template <class L>
struct Streamer {
    static constexpr int LEN = L::LEN, PW = L::PW, VW = L::VW;
    static constexpr int NB = (LEN + 63) / 64;
    static constexpr int NC = (LEN + CHUNK_LEN - 1) / CHUNK_LEN;
    static constexpr int MID_ALIGN = cmin(L::ROW_ALIGN, PW == 0 ? 16 : lowbit(4 * PW));
    static constexpr int DEPTH = 4;  // CV stack depth: NC <= 16
    static_assert(NC <= 16, "values above ~16 KiB take the encoded path");

    const uint32_t *pw;
    const uint8_t *vrow;

    __device__ __forceinline__ void block0(uint32_t m[16]) const {
        constexpr int NV = cmin(16 - PW, VW);
#pragma unroll
        for (int j = 0; j < PW; j++) m[j] = pw[j];
        uint32_t v[NV > 0 ? NV : 1];
        if constexpr (NV > 0) ldw<NV, L::ROW_ALIGN>(vrow, v);
#pragma unroll
        for (int j = 0; j < 16 - PW; j++) m[PW + j] = (j < NV) ? v[j] : 0u;
    }
    __device__ __forceinline__ void block_mid(int b, uint32_t m[16]) const {
        ldw<16, MID_ALIGN>(vrow + (64 * b - 4 * PW), m);
    }
    __device__ __forceinline__ void block_last(uint32_t m[16]) const {
        constexpr int first = 16 * (NB - 1) - PW;  // value word index of m[0]
        constexpr int NV = VW - first;
        static_assert(first >= 0 && NV > 0 && NV <= 16, "last block layout");
        constexpr int ALIGN = cmin(L::ROW_ALIGN, lowbit(4 * first) == 0 ? 16 : lowbit(4 * first));
        uint32_t v[NV];
        ldw<NV, ALIGN>(vrow + 4 * first, v);
#pragma unroll
        for (int j = 0; j < 16; j++) m[j] = j < NV ? v[j] : 0u;
    }

    template <int C>
    __device__ __forceinline__ void chunks(uint32_t (&stk)[DEPTH][8], uint32_t out[8]) const {
        uint32_t cv[8];
        cv_iv(cv);
        if constexpr (C == 0) {
            uint32_t m[16];
            block0(m);
            compress(cv, m, 0, 0, 64, CHUNK_START);
        }
        constexpr int b_start = C == 0 ? 1 : 16 * C;
        constexpr int b_end = C == NC - 1 ? NB - 1 : 16 * C + 16;
        // software-pipelined: block b+1's words are in flight while block b is compressed
        uint32_t m[16];
        if (b_start < b_end) block_mid(b_start, m);
#pragma unroll 1
        for (int b = b_start; b < b_end; b++) {
            uint32_t mn[16];
            block_mid(b + 1 < b_end ? b + 1 : b, mn);  // unconditional (stays ahead of the
                                                       // compression); never past the row
            const uint32_t flags = (b == 16 * C ? CHUNK_START : 0u) | (b == 16 * C + 15 ? CHUNK_END : 0u);
            compress(cv, m, (uint32_t)C, 0, 64, flags);
#pragma unroll
            for (int j = 0; j < 16; j++) m[j] = mn[j];
        }
        if constexpr (C == NC - 1) {
            uint32_t m[16];
            block_last(m);
            constexpr uint32_t fl = CHUNK_END | ((NB - 1) == 16 * C ? CHUNK_START : 0u) | (NC == 1 ? ROOT : 0u);
            compress(cv, m, (uint32_t)C, 0, (uint32_t)(LEN - 64 * (NB - 1)), fl);
            if constexpr (NC == 1) {
#pragma unroll
                for (int k = 0; k < 8; k++) out[k] = cv[k];
            } else {
                // fold the stack top-down; the last (bottom) merge is the root
                constexpr int D = __builtin_popcount(NC - 1);
#pragma unroll
                for (int s = D - 1; s >= 0; s--) {
                    uint32_t p[8];
                    parent(p, stk[s], cv, s == 0 ? ROOT : 0u);
#pragma unroll
                    for (int k = 0; k < 8; k++) cv[k] = p[k];
                }
#pragma unroll
                for (int k = 0; k < 8; k++) out[k] = cv[k];
            }
        } else {
            // chunk C complete and more input follows: push its CV, merging while the
            // total chunk count has trailing zero bits (the BLAKE3 incremental tree)
            constexpr int total = C + 1;
            constexpr int depth_before = __builtin_popcount(total - 1);
            constexpr int merges = __builtin_ctz(total);
#pragma unroll
            for (int k = 0; k < merges; k++) {
                uint32_t p[8];
                parent(p, stk[depth_before - 1 - k], cv, 0u);
#pragma unroll
                for (int q = 0; q < 8; q++) cv[q] = p[q];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) stk[depth_before - merges][q] = cv[q];
            chunks<C + 1 < NC ? C + 1 : NC - 1>(stk, out);
        }
    }

    __device__ __forceinline__ void run(uint32_t out[8]) const {
        uint32_t stk[DEPTH][8];
        chunks<0>(stk, out);
    }
};

// lift of one present record of layout L (prefix words built, value row pointer given)
template <class L>
__device__ __forceinline__ void hash_present(const uint32_t *pw, const uint8_t *vrow, uint32_t out[8]) {
    if constexpr (L::SMALL) {
        uint32_t w[L::LEN / 4 > 0 ? L::LEN / 4 : 1];
#pragma unroll
        for (int j = 0; j < L::PW; j++) w[j] = pw[j];
        if constexpr (L::VW > 0) ldw<L::VW, L::ROW_ALIGN>(vrow, w + L::PW);
        hash_words<L::LEN>(w, out);
    } else {
        Streamer<L> s{pw, vrow};
        s.run(out);
    }
}

template <class I = uint64_t>
__device__ __forceinline__ void store_fp(uint8_t *fps, I i, const uint32_t h[8]) {
    uint4 *o = reinterpret_cast<uint4 *>(fps + (I)32 * i);
    o[0] = make_uint4(h[0], h[1], h[2], h[3]);
    o[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

__device__ __forceinline__ void store_sum(uint8_t *dst, uint64_t g, const uint32_t f[8]) {
    uint4 *o = reinterpret_cast<uint4 *>(dst + 32 * g);
    o[0] = make_uint4(f[0], f[1], f[2], f[3]);
    o[1] = make_uint4(f[4], f[5], f[6], f[7]);
}

// A present record and a tombstone of the same key share block 0 up to the State variant word
// (the tombstone's last word), so when the tombstone fits one block the two are hashed with
// one block-0 compression whose words, length and flags are chosen per lane; only present
// lanes go on to the value blocks.  A wave mixing both kinds then runs NB compressions, not
// NB + 1 as two divergent paths would.
template <class L, int KK, int RK>
__device__ __forceinline__ void hash_merged(const uint32_t *kw, const uint32_t *sw, bool tomb, const uint8_t *vrow,
                                            uint32_t h[8]) {
    constexpr int NW = L::LEN / 4, NB = (L::LEN + 63) / 64, TW = L::LEN_TOMB / 4;
    static_assert(L::SMALL && L::LEN_TOMB <= 64 && TW >= 1, "tombstone must fit block 0");
    uint32_t w[NW];
    build_prefix<L, KK, RK>(kw, sw, false, w);  // present words: variant 0 at TW - 1
    if constexpr (L::VW > 0) ldw<L::VW, L::ROW_ALIGN>(vrow, w + L::PW);
    uint32_t m[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const uint32_t pres = j < NW ? w[j] : 0u;
        m[j] = j < TW - 1 ? pres : j == TW - 1 ? (tomb ? 1u : 0u) : (tomb ? 0u : pres);
    }
    cv_iv(h);
    const uint32_t blen0 = tomb ? (uint32_t)L::LEN_TOMB : (uint32_t)(NB == 1 ? L::LEN : 64);
    const uint32_t fl0 = CHUNK_START | ((tomb || NB == 1) ? (CHUNK_END | ROOT) : 0u);
    compress(h, m, 0, 0, blen0, fl0);
    if (!tomb) {
#pragma unroll
        for (int b = 1; b < NB; b++) {
#pragma unroll
            for (int j = 0; j < 16; j++) m[j] = (16 * b + j < NW) ? w[16 * b + j] : 0u;
            const uint32_t flags = b == NB - 1 ? (CHUNK_END | ROOT) : 0u;
            const uint32_t blen = b == NB - 1 ? (uint32_t)(L::LEN - 64 * b) : 64u;
            compress(h, m, 0, 0, blen, flags);
        }
    }
}

// A layout whose value rows are only known to be A-byte aligned (rows read from a staged file)
template <class L, int A>
struct LayoutAligned : L {
    static constexpr int ROW_ALIGN = cmin(L::ROW_ALIGN, A);
};

// lift one record (present or tombstone) of layout L; TAGS: tomb varies per lane
template <class L, int KK, int RK, bool TAGS>
__device__ __forceinline__ void lift_record_l(const uint32_t *kw, const uint32_t *sw, bool tomb,
                                              const uint8_t *vrow, uint32_t h[8]) {
    if constexpr (TAGS && RK != REC_PLAIN && L::SMALL && L::LEN_TOMB <= 64) {
        hash_merged<L, KK, RK>(kw, sw, tomb, vrow, h);
    } else if (RK != REC_PLAIN && tomb) {
        constexpr int TW = L::LEN_TOMB / 4;
        uint32_t w[TW];
        build_prefix<L, KK, RK>(kw, sw, true, w);
        hash_words<L::LEN_TOMB>(w, h);
    } else {
        uint32_t pw[L::PW > 0 ? L::PW : 1];
        build_prefix<L, KK, RK>(kw, sw, false, pw);
        hash_present<L>(pw, vrow, h);
    }
}

// lift one record (present or tombstone) of schema (KK,KL,VK,VL,RK); TAGS: tomb varies per lane
template <int KK, int KL, int VK, int VL, int RK, bool TAGS = true>
__device__ __forceinline__ void lift_record(const uint32_t *kw, const uint32_t *sw, bool tomb,
                                            const uint8_t *vrow, uint32_t h[8]) {
    lift_record_l<Layout<KK, KL, VK, VL, RK>, KK, RK, TAGS>(kw, sw, tomb, vrow, h);
}

constexpr int LIFT_THREADS = 256;

// The lift kernel.  DUAL: RK == DATED, and additionally emit the projection fingerprint
// lift(k, State<V>) from the same loaded record (Replica::map_insert's second lift).
template <int KK, int KL, int VK, int VL, int RK, bool TAGS, bool DUAL>
__global__ __launch_bounds__(LIFT_THREADS) void k_lift(DevCols c, uint64_t n, uint8_t *fps,
                                                       uint8_t *bsums, uint8_t *fps2,
                                                       uint8_t *bsums2) {
    using L = Layout<KK, KL, VK, VL, RK>;
    static_assert(LIFT_THREADS == 256, "block_sum_fps256");
    __shared__ SumTile tile;
    const uint64_t i = (uint64_t)blockIdx.x * LIFT_THREADS + threadIdx.x;
    const bool valid = i < n;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t h2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (valid) {
        // Column pointers rebased to this block in scalar registers, so every per-lane
        // address is a 32-bit offset (global_load ... saddr): no 64-bit VALU address math.
        const uint64_t b0 = (uint64_t)blockIdx.x * LIFT_THREADS;
        const uint32_t t = threadIdx.x;
        DevCols cb;
        cb.keys = c.keys + b0 * L::KEY_ROW;
        cb.phys = c.phys + b0;
        cb.logical = c.logical + b0;
        cb.node = c.node + b0;
        cb.tags = c.tags + b0;
        cb.values = c.values + b0 * L::VAL_ROW;
        uint32_t kw[L::KEY_ENC / 4 > 0 ? L::KEY_ENC / 4 : 1];
        uint32_t sw[5];
        load_key<KK, KL>(cb.keys, t, kw);
        if constexpr (RK == REC_DATED) load_stamp(cb, t, sw);
        const bool tomb = TAGS ? (cb.tags[t] != 0) : false;
        const uint8_t *vrow = cb.values + t * (uint32_t)L::VAL_ROW;
        lift_record<KK, KL, VK, VL, RK, TAGS>(kw, sw, tomb, vrow, h);
        if (c.dst) {
            // bounded: a bucket the key sort could not order leaves its rows' slots unwritten
            // (the sort flags it and the batch is sorted and lifted again)
            const uint32_t r = c.dst2 ? c.dst2[c.dst[i]] : c.dst[i];
            if (r < n) store_fp<uint64_t>(fps, r, h);
        } else {
            store_fp(fps + b0 * 32, t, h);
        }
        if constexpr (DUAL) {
            lift_record<KK, KL, VK, VL, REC_PROJECTION, TAGS>(kw, sw, tomb, vrow, h2);
            store_fp(fps2 + b0 * 32, t, h2);
        }
    }
    if (bsums) {
        uint32_t f[8];
        block_sum_fps256(h, tile, f);  // invalid lanes hold zero
        if (threadIdx.x == 0) store_sum(bsums, blockIdx.x, f);
    }
    if constexpr (DUAL) {
        if (bsums2) {
            uint32_t f[8];
            block_sum_fps256(h2, tile, f);
            if (threadIdx.x == 0) store_sum(bsums2, blockIdx.x, f);
        }
    }
}

}  // namespace rh
