// aggregate_kernels.hip -- the generic (pre-encoded bytes) lift, the 256-bit block reducer,
// the rank-range aggregate query and the cross-shard combine.
//
//   k_lift_encoded      rsos::lift over bytes from rsos::encoding::encode_to_vec (any schema),
//                       rsos/src/fingerprint.rs:270-275, rsos/src/encoding.rs:117-128
//   k_reduce            per-256 sums: the cached subtree Aggregate of node.rs:54-91
//   k_range_query       FingerprintTreeMap::aggregate, query.rs:25-76, over rank ranges
//   k_combine           Aggregate's Add (rsos/src/aggregate.rs:79-89) over gathered shards
#include "internal.hpp"
#include "lift_kernels.hpp"
#include "round_device.hpp"

namespace rh {


// ---- generic encoded-bytes lift -------------------------------------------------------------

// 16 message words of the block starting at byte `addr`, `blen` (0..64) valid bytes; bytes
// past blen are zero.  Dwords at or beyond `limit` (buffer size rounded up to 4) are not read.
__device__ __forceinline__ void load_block_bytes(const uint8_t *base, uint64_t addr, uint32_t blen,
                                                 uint64_t limit, uint32_t m[16]) {
    const uint64_t a4 = addr & ~3ull;
    const uint32_t sh = (uint32_t)(addr & 3) * 8u;
    uint32_t d[17];
#pragma unroll
    for (int k = 0; k < 17; k++) {
        const uint64_t at = a4 + 4ull * k;
        d[k] = (at < limit && (uint32_t)(4 * k) < blen + 4) ? *reinterpret_cast<const uint32_t *>(base + at) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t w = __builtin_amdgcn_alignbit(d[j + 1], d[j], sh);
        const int valid = (int)blen - 4 * j;
        const uint32_t mask = valid >= 4 ? 0xFFFFFFFFu : valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u);
        m[j] = w & mask;
    }
}

// Records of one chunk (<= 1,024 B) -- every K / V pair of ordinary size -- go through a
// lane-refill loop: a wave owns ENC_PER_WAVE consecutive records, every iteration compresses
// one block for each lane, and a lane whose record is done takes the next unclaimed record of
// the wave's range (ballot + lane rank).  Lanes stay busy whatever the mix of record lengths,
// where one record per lane would leave a wave running its longest record's block count.
// Longer records are left to k_lift_encoded_long.
constexpr int ENC_PER_WAVE = 64 * 4;

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

// record i's bytes [start, start + len), clipped to the buffer: offsets that decrease or run
// past `limit` (a caller error) give a wrong fingerprint, never an out-of-bounds read or a loop
// over a wrapped-around length
__device__ __forceinline__ void record_span(const uint64_t *offs, uint64_t i, uint64_t limit, uint64_t &start,
                                            uint64_t &len) {
    uint64_t a = offs[i], b = offs[i + 1];
    if (a > limit) a = limit;
    if (b > limit) b = limit;
    start = a;
    len = b > a ? b - a : 0;
}

// 16 message words of the block at byte `addr` with `blen` valid bytes (bytes past blen are
// zero): 4 x 16-byte + 1 dword loads from the dword-aligned address, then a funnel shift.  Past
// blen: whole words below the boundary word are kept, the boundary word is masked to its valid
// bytes, the rest are zeroed (compares against constants, selects and an AND per word).  A
// uniform skip of the funnel shift for all-aligned waves measured no faster (the branch's
// register copies cost what the 16 shifts did: profiles/r02_s3_encoded_ab.log).
__device__ __forceinline__ void load_block_fast(const uint8_t *base, uint64_t addr, uint32_t blen, bool partial,
                                                uint32_t m[16]) {
    const uint64_t a4 = addr & ~3ull;
    const uint32_t sh = (uint32_t)(addr & 3) * 8u;
    uint32_t d[17];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const u32x4_a4 v = *reinterpret_cast<const u32x4_a4 *>(base + a4 + 16 * q);
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
    }
    d[16] = *reinterpret_cast<const uint32_t *>(base + a4 + 64);
#pragma unroll
    for (int j = 0; j < 16; j++) m[j] = __builtin_amdgcn_alignbit(d[j + 1], d[j], sh);
    if (partial) {
        const uint32_t jb = blen >> 2, bm = (1u << ((blen & 3u) * 8u)) - 1u;
#pragma unroll
        for (int j = 0; j < 16; j++) m[j] = (uint32_t)j < jb ? m[j] : ((uint32_t)j == jb ? (m[j] & bm) : 0u);
    }
}

// bsums: the wave's ENC_PER_WAVE records are whole 256-row blocks, so it forms their block sums at
// the end from the fingerprints just written (its own, and those k_lift_encoded_long wrote before
// this launch) -- L2-resident reads instead of a second pass.
static_assert(ENC_PER_WAVE % 256 == 0, "a wave's records must be whole 256-row blocks");

__global__ __launch_bounds__(256) void k_lift_encoded_short(const uint8_t *bytes, const uint64_t *offs, uint64_t n,
                                                            uint64_t limit, uint8_t *fps, uint8_t *bsums) {
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint64_t w0 = wave * ENC_PER_WAVE;
    if (w0 >= n) return;  // uniform per wave
    const uint64_t w1 = w0 + ENC_PER_WAVE < n ? w0 + ENC_PER_WAVE : n;
    uint64_t next = w0;  // first unclaimed record of the wave's range (same in every lane)
    uint64_t i = 0, start = 0, len = 0;
    uint32_t b = 0, nb = 0, cv[8];
    bool active = false;
    for (;;) {
        // lanes without a record claim the next ones, in order; a multi-chunk record is skipped
        // (k_lift_encoded_long hashes it) and the lane claims again
        bool need = !active;
        for (;;) {
            const uint64_t mask = __ballot(need && next < w1);
            if (!mask) break;
            const uint64_t cand = next + lanes_below(mask);
            next += (uint64_t)__popcll(mask);
            if (need && cand < w1) {
                uint64_t s0, l0;
                record_span(offs, cand, limit, s0, l0);
                if (l0 <= (uint64_t)CHUNK_LEN) {
                    i = cand;
                    start = s0;
                    len = l0;
                    b = 0;
                    nb = l0 == 0 ? 1u : (uint32_t)((l0 + 63) / 64);
                    cv_iv(cv);
                    active = true;
                    need = false;
                }
            } else {
                need = false;
            }
        }
        if (!__ballot(active)) break;
        if (active) {
            const uint64_t boff = 64ull * b;
            const uint32_t blen = (uint32_t)(len - boff < 64 ? len - boff : 64);
            uint32_t m[16];
            if (start + boff + 68 <= limit) load_block_fast(bytes, start + boff, blen, blen < 64, m);
            else load_block_bytes(bytes, start + boff, blen, limit, m);  // the buffer's last bytes
            const uint32_t flags = (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? (CHUNK_END | ROOT) : 0u);
            compress(cv, m, 0u, 0u, blen, flags);
            if (++b == nb) {
                store_fp(fps, i, cv);
                active = false;
            }
        }
    }
    if (!bsums) return;
    __threadfence_block();  // workgroup scope: this wave reads its own stores back (same L2); an agent-scope fence would write back L2
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int blk = 0; blk < ENC_PER_WAVE / 256; blk++) {
        const uint64_t r0 = w0 + 256ull * blk;
        if (r0 >= n) break;  // uniform
        Acc a;
        acc_zero(a);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t r = r0 + lane + 64 * k;
            if (r < n) {
                uint32_t f[8];
                load_fp(fps, r, f);
                acc_add_fp(a, f);
            }
        }
        acc_wave_reduce(a);
        if (lane == 0) {
            uint32_t f[8];
            acc_normalise(a, f);
            store_sum(bsums, r0 / 256, f);
        }
    }
}

// records longer than one chunk: chunk CVs on a stack, parent nodes (one record per lane;
// shorter records return at once)
constexpr int ENC_STACK = 40;

// BLAKE3 of bytes [start, start + len), any length: chunk CVs on a stack, parent nodes
__device__ __forceinline__ void hash_span(const uint8_t *bytes, uint64_t start, uint64_t len, uint64_t limit,
                                          uint32_t cv[8]) {
    const uint64_t nchunks = len == 0 ? 1 : (len + CHUNK_LEN - 1) / CHUNK_LEN;
    uint32_t stk[ENC_STACK][8];
    int sp = 0;
    for (uint64_t c = 0; c < nchunks; c++) {
        const uint64_t cbeg = c * CHUNK_LEN;
        const uint64_t clen = len - cbeg < (uint64_t)CHUNK_LEN ? len - cbeg : (uint64_t)CHUNK_LEN;
        const uint32_t nb = clen == 0 ? 1u : (uint32_t)((clen + 63) / 64);
        cv_iv(cv);
        for (uint32_t b = 0; b < nb; b++) {
            const uint64_t boff = cbeg + 64ull * b;
            const uint32_t blen = (uint32_t)(len - boff < 64 ? len - boff : 64);
            uint32_t m[16];
            if (start + boff + 68 <= limit) load_block_fast(bytes, start + boff, blen, blen < 64, m);
            else load_block_bytes(bytes, start + boff, blen, limit, m);
            uint32_t flags = (b == 0 ? CHUNK_START : 0u) | (b == nb - 1 ? CHUNK_END : 0u);
            if (nchunks == 1 && b == nb - 1) flags |= ROOT;
            compress(cv, m, (uint32_t)c, (uint32_t)(c >> 32), blen, flags);
        }
        if (c + 1 < nchunks) {
            uint64_t total = c + 1;
            while ((total & 1) == 0) {
                sp--;
                uint32_t p[8];
                parent(p, stk[sp], cv, 0u);
                for (int q = 0; q < 8; q++) cv[q] = p[q];
                total >>= 1;
            }
            for (int q = 0; q < 8; q++) stk[sp][q] = cv[q];
            sp++;
        }
    }
    for (int s2 = sp - 1; s2 >= 0; s2--) {
        uint32_t p[8];
        parent(p, stk[s2], cv, s2 == 0 ? ROOT : 0u);
        for (int q = 0; q < 8; q++) cv[q] = p[q];
    }
}

__global__ __launch_bounds__(256) void k_lift_encoded_long(const uint8_t *bytes, const uint64_t *offs,
                                                           uint64_t n, uint64_t limit, uint8_t *fps) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t start, len;
    record_span(offs, i, limit, start, len);
    if (len <= (uint64_t)CHUNK_LEN) return;
    uint32_t cv[8];
    hash_span(bytes, start, len, limit, cv);
    store_fp(fps, i, cv);
}

// ---- fixed-length encodings -------------------------------------------------------------------
// Every record `len` bytes at stride `len` (a K / V pair whose canonical encoding has one length:
// fixed-width integers, arrays, fixed-size structs).  No offsets to read, and every lane of a wave
// runs the same blocks in lockstep.
// ALIGNED (len % 4 == 0): every block starts on a dword, so its words load as they are -- no
// funnel shift -- and the last block's byte count (the same in every lane) masks whole words.
// The workgroup's 256-row block sum is formed on the way out (bsums != nullptr), as the schema
// kernels do, instead of a second pass over the fingerprints.
__device__ __forceinline__ void fixed_epilogue(uint8_t *fps, uint8_t *bsums, uint64_t i, bool live, uint32_t cv[8]) {
    if (live) store_fp(fps, i, cv);
    if (bsums) {  // uniform: every lane reaches the workgroup barriers
        __shared__ SumTile tile;
        uint32_t h[8], f[8];
#pragma unroll
        for (int q = 0; q < 8; q++) h[q] = live ? cv[q] : 0u;
        block_sum_fps256(h, tile, f);
        if (threadIdx.x == 0) store_sum(bsums, blockIdx.x, f);
    }
}

template <bool ALIGNED>
__global__ __launch_bounds__(256) void k_lift_fixed_short(const uint8_t *bytes, uint32_t len, uint64_t n,
                                                          uint64_t limit, uint8_t *fps, uint8_t *bsums) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = i < n;
    const uint64_t start = i * len;
    const uint32_t nb = len == 0 ? 1u : (len + 63) / 64;
    uint32_t cv[8];
    cv_iv(cv);
    for (uint32_t b = 0; live && b < nb; b++) {
        const uint32_t boff = 64u * b;
        const uint32_t blen = len - boff < 64u ? len - boff : 64u;
        uint32_t m[16];
        if (ALIGNED && blen == 64 && start + boff + 64 <= limit) {  // a full block (uniform branch)
            const u32x4_a4 *p = reinterpret_cast<const u32x4_a4 *>(bytes + start + boff);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4_a4 v = p[q];
                m[4 * q] = v.x;
                m[4 * q + 1] = v.y;
                m[4 * q + 2] = v.z;
                m[4 * q + 3] = v.w;
            }
        } else if (ALIGNED && start + boff + 64 <= limit) {
            const u32x4_a4 *p = reinterpret_cast<const u32x4_a4 *>(bytes + start + boff);
            const uint32_t words = blen / 4;  // uniform: whole words only
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const u32x4_a4 v = (uint32_t)(4 * q) < words ? p[q] : u32x4_a4{0u, 0u, 0u, 0u};
                m[4 * q] = (uint32_t)(4 * q) < words ? v.x : 0u;
                m[4 * q + 1] = (uint32_t)(4 * q + 1) < words ? v.y : 0u;
                m[4 * q + 2] = (uint32_t)(4 * q + 2) < words ? v.z : 0u;
                m[4 * q + 3] = (uint32_t)(4 * q + 3) < words ? v.w : 0u;
            }
        } else if (start + boff + 68 <= limit) {
            load_block_fast(bytes, start + boff, blen, blen < 64, m);
        } else {
            load_block_bytes(bytes, start + boff, blen, limit, m);
        }
        const uint32_t flags = (b == 0 ? CHUNK_START : 0u) | (b + 1 == nb ? (CHUNK_END | ROOT) : 0u);
        compress(cv, m, 0u, 0u, blen, flags);
    }
    fixed_epilogue(fps, bsums, i, live, cv);
}

__global__ __launch_bounds__(256) void k_lift_fixed_long(const uint8_t *bytes, uint64_t len, uint64_t n,
                                                         uint64_t limit, uint8_t *fps, uint8_t *bsums) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = i < n;
    uint32_t cv[8];
    if (live) hash_span(bytes, i * len, len, limit, cv);
    fixed_epilogue(fps, bsums, i, live, cv);
}

// Fixed-length records whose length is a compile-time constant: the encoded forms of the shapes
// the schema kernels instantiate (120 B = [u8; 16] key + Entry<Timestamp, Vec<u8>> of 64 B, the
// north_star record; 100 B its projection State<Vec<u8>>; 104 / 80 B the u64-key dated / plain
// 64 B records; 48 B a 16-byte-key tombstone).  The record is loaded whole into registers with
// 32-bit lane offsets off a workgroup-rebased scalar base -- the schema kernels' loads -- and
// hashed by the same compile-time block schedule (hash_words): no per-block loop, branches,
// masks or funnel shifts, which the runtime-length kernel above pays per block.
template <int LEN>
__global__ __launch_bounds__(256) void k_lift_fixed_ct(const uint8_t *bytes, uint64_t n, uint8_t *fps,
                                                       uint8_t *bsums) {
    static_assert(LEN % 4 == 0 && LEN > 0 && LEN <= 192, "whole words, in registers");
    __shared__ SumTile tile;
    const uint64_t b0 = (uint64_t)blockIdx.x * 256;
    const uint32_t t = threadIdx.x;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (b0 + t < n) {
        const uint8_t *base = bytes + b0 * LEN;
        uint32_t w[LEN / 4];
        ldw<LEN / 4, cmin(16, lowbit(LEN))>(base + t * (uint32_t)LEN, w);
        hash_words<LEN>(w, h);
        store_fp(fps + b0 * 32, t, h);
    }
    if (bsums) {  // uniform: every lane reaches the workgroup barriers; absent rows add zero
        uint32_t f[8];
        block_sum_fps256(h, tile, f);
        if (t == 0) store_sum(bsums, blockIdx.x, f);
    }
}

// ---- reductions ------------------------------------------------------------------------------


__global__ __launch_bounds__(256) void k_reduce(const uint8_t *in, uint32_t stride, uint64_t n_in, uint8_t *out) {
    __shared__ SumTile tile;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (i < n_in) load_fp(in, i, h, stride);
    uint32_t f[8];
    block_sum_fps256(h, tile, f);
    if (threadIdx.x == 0) store_sum(out, blockIdx.x, f);
}

__device__ __forceinline__ void acc_span(Acc &a, const uint8_t *src, uint64_t lo, uint64_t hi, uint32_t stride = 32,
                                         const uint32_t *slots = nullptr) {
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        uint32_t f[8];
        load_fp(src, slots ? slots[i] : i, f, stride);  // slots: entry i lives at src[slots[i]]
        acc_add_fp(a, f);
    }
}

// Σ of n 256-bit entries (one workgroup): the root fingerprint of a run from its super-block
// sums, kept on the host so that the whole-map aggregate is O(1) (the root node's cached
// Aggregate, rsos/src/fingerprint_tree_map/query.rs:25-76 with an unbounded range)
__global__ __launch_bounds__(256) void k_total(const uint8_t *in, uint64_t n, uint64_t *out) {
    __shared__ uint64_t lds[4 * 8];
    Acc a;
    acc_zero(a);
    acc_span(a, in, 0, n);
    uint32_t f[8];
    acc_block_reduce<256>(a, lds, f);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < 4; q++) out[q] = (uint64_t)f[2 * q] | ((uint64_t)f[2 * q + 1] << 32);
    }
}

// One workgroup per query.  [lo, hi) = head rows + whole blocks + tail rows, the whole blocks
// = head blocks + whole super-blocks + tail blocks.  Each thread sums at most a few hundred
// entries into carry-save u64 limbs, then one block reduction.
__global__ __launch_bounds__(256) void k_range_query(const uint8_t *fps, uint32_t stride, const uint32_t *slots,
                                                     const uint8_t *bsums, const uint8_t *ssums, uint64_t n,
                                                     const uint64_t *qlo, const uint64_t *qhi,
                                                     uint64_t r, uint64_t *out) {
    __shared__ uint64_t lds[4 * 8];
    const uint64_t j = blockIdx.x;
    if (j >= r) return;  // uniform per block
    uint64_t lo = qlo[j], hi = qhi[j];
    if (hi > n) hi = n;
    if (lo > hi) lo = hi;
    Acc a;
    acc_zero(a);
    const uint64_t B = 256, S = 65536;
    const uint64_t b1 = (lo + B - 1) / B, b2 = hi / B;  // whole blocks [b1, b2)
    if (b1 >= b2 || bsums == nullptr) {
        acc_span(a, fps, lo, hi, stride, slots);
    } else {
        acc_span(a, fps, lo, b1 * B, stride, slots);
        acc_span(a, fps, b2 * B, hi, stride, slots);
        const uint64_t s1 = (b1 + B - 1) / B, s2 = b2 / B;  // whole super-blocks [s1, s2)
        if (s1 >= s2 || ssums == nullptr) {
            acc_span(a, bsums, b1, b2);
        } else {
            acc_span(a, bsums, b1, s1 * B);
            acc_span(a, bsums, s2 * B, b2);
            acc_span(a, ssums, s1, s2);
        }
    }
    (void)S;
    uint32_t f[8];
    acc_block_reduce<256>(a, lds, f);
    if (threadIdx.x == 0) {
        uint64_t *o = out + 5 * j;
        o[0] = (uint64_t)f[0] | ((uint64_t)f[1] << 32);
        o[1] = (uint64_t)f[2] | ((uint64_t)f[3] << 32);
        o[2] = (uint64_t)f[4] | ((uint64_t)f[5] << 32);
        o[3] = (uint64_t)f[6] | ((uint64_t)f[7] << 32);
        o[4] = hi - lo;
    }
}




__global__ __launch_bounds__(256) void k_range_query_wave(const uint8_t *fps, uint32_t stride, const uint8_t *bsums,
                                                          const uint8_t *ssums, uint64_t n, const uint64_t *qlo,
                                                          const uint64_t *qhi, uint64_t r, uint64_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (j >= r) return;  // uniform per wave
    uint64_t lo = qlo[j], hi = qhi[j];
    if (hi > n) hi = n;
    if (lo > hi) lo = hi;
    wave_range_agg(fps, stride, bsums, ssums, lo, hi, lane, out + 5 * j);
}





// Large rounds, step 1 (after the bounds' ranks and local aggregates): every segment's decision;
// hdr gets the RoundOutcome counts (protocol.rs:135-142) -- skipped, enumerated, split,
// children, dropped
__global__ __launch_bounds__(256) void k_round_plan(RoundSegs g, const uint64_t *remote, uint64_t r, uint64_t n,
                                                    int sqrt_policy, uint64_t b, uint64_t *hdr) {
    __shared__ unsigned long long cnt[5];
    if (threadIdx.x < 5) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < r) {
        const RoundSeg d = round_decide(g.lo[j], g.hi[j], g.loc + 5 * j, remote + 5 * j, n, sqrt_policy, b);
        g.kind[j] = (uint8_t)d.kind;
        g.stride[j] = d.stride;
        g.si[j] = d.si;
        g.ei[j] = d.ei;
        g.nch[j] = d.children;
        g.nen[j] = d.enums;
        atomicAdd(&cnt[d.kind == 3 ? 4 : d.kind], 1ull);
        if (d.children) atomicAdd(&cnt[3], (unsigned long long)d.children);
    }
    __syncthreads();
    if (threadIdx.x < 5 && cnt[threadIdx.x]) atomicAdd((unsigned long long *)&hdr[threadIdx.x], cnt[threadIdx.x]);
}

// ---- the large round's plan in three launches (a memset, k_round_plan and two library scans
// were six): decisions and per-256-segment counts; one workgroup scans the parts and writes the
// header; each segment's child / enumeration offsets ---------------------------------------------
__global__ __launch_bounds__(256) void k_round_plan_part(RoundSegs g, const uint64_t *remote, uint64_t r, uint64_t n,
                                                         int sqrt_policy, uint64_t b, uint64_t *part) {
    __shared__ unsigned long long cnt[5];  // skipped, enumerated (= enumerations), split, children, dropped
    if (threadIdx.x < 5) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < r) {
        const RoundSeg d = round_decide(g.lo[j], g.hi[j], g.loc + 5 * j, remote + 5 * j, n, sqrt_policy, b);
        g.kind[j] = (uint8_t)d.kind;
        g.stride[j] = d.stride;
        g.si[j] = d.si;
        g.ei[j] = d.ei;
        g.nch[j] = d.children;
        g.nen[j] = d.enums;
        atomicAdd(&cnt[d.kind == 3 ? 4 : d.kind], 1ull);
        if (d.children) atomicAdd(&cnt[3], (unsigned long long)d.children);
    }
    __syncthreads();
    if (threadIdx.x < 5) part[5 * (uint64_t)blockIdx.x + threadIdx.x] = cnt[threadIdx.x];
}
__global__ __launch_bounds__(1024) void k_round_plan_scan_parts(uint64_t *part, uint64_t np, uint64_t *hdr) {
    __shared__ uint64_t wsum[2][16], tot[2], carry[2];
    __shared__ unsigned long long other[3];  // skipped, split, dropped
    const uint32_t t = threadIdx.x;
    if (t < 2) carry[t] = 0;
    if (t < 3) other[t] = 0;
    __syncthreads();
    for (uint64_t base = 0; base < np; base += blockDim.x) {  // uniform
        const uint64_t i = base + t;
        const bool in = i < np;
        const uint64_t c = in ? part[5 * i + 3] : 0, e = in ? part[5 * i + 1] : 0;
        if (in) {
            atomicAdd(&other[0], (unsigned long long)part[5 * i]);
            atomicAdd(&other[1], (unsigned long long)part[5 * i + 2]);
            atomicAdd(&other[2], (unsigned long long)part[5 * i + 4]);
        }
        const uint64_t co = block_exclusive_scan(c, wsum[0], &tot[0]);
        const uint64_t eo = block_exclusive_scan(e, wsum[1], &tot[1]);
        if (in) part[5 * i + 3] = carry[0] + co, part[5 * i + 1] = carry[1] + eo;  // the part's offsets
        __syncthreads();
        if (t == 0) carry[0] += tot[0], carry[1] += tot[1];
        __syncthreads();
    }
    if (t == 0) {
        hdr[0] = other[0], hdr[1] = carry[1], hdr[2] = other[1], hdr[3] = carry[0], hdr[4] = other[2];
        hdr[5] = hdr[6] = hdr[7] = 0;
    }
}
__global__ __launch_bounds__(256) void k_round_plan_apply(RoundSegs g, uint64_t r, const uint64_t *part) {
    __shared__ uint64_t wsum[2][4], tot[2];
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t c = j < r ? g.nch[j] : 0, e = j < r ? g.nen[j] : 0;
    const uint64_t co = block_exclusive_scan(c, wsum[0], &tot[0]);
    const uint64_t eo = block_exclusive_scan(e, wsum[1], &tot[1]);
    if (j < r) {
        g.choff[j] = part[5 * (uint64_t)blockIdx.x + 3] + co;
        g.enoff[j] = part[5 * (uint64_t)blockIdx.x + 1] + eo;
    }
}

// Every child, one wave each, grid-stride (the count is known on the device only), then the
// enumerations, one thread each
__global__ __launch_bounds__(256) void k_round_emit(const uint64_t *hdr, uint64_t cap, uint64_t r, uint32_t kl,
                                                    RoundIn in, RoundSegs g, uint8_t *out) {
    const uint64_t nc = hdr[3], ne = hdr[1];
    if (nc > cap) return;  // the host grows the buffer and launches again
    const RoundLayout L = round_layout(nc, ne, kl);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nc; c += nw) {
        const uint64_t j = round_owner(g.choff, r, c);
        round_emit_child(c, j, c - g.choff[j], L, kl, lane, in, g, out);
    }
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < r; j += nw * 64)
        if (g.nen[j]) round_emit_enum(j, g.enoff[j], L, kl, in, g, out);
}



// ---- base-only rounds with the base's row prefix (RoundIn::pre): every sum is one difference, so
// a thread per segment and a thread per child do what a wave each did (the wave's head / tail rows
// and block sums, then a 64-lane reduction, for a range of a few rows) ---------------------------
__device__ __forceinline__ void base_pre_agg(const uint8_t *pre, uint64_t lo, uint64_t hi, uint64_t *o) {
    uint32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8];
    if (hi > lo) {
        load_fp(pre, hi, a);
        load_fp(pre, lo, b);
        sub256(a, b);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) o[q] = (uint64_t)a[2 * q] | ((uint64_t)a[2 * q + 1] << 32);
    o[4] = hi > lo ? hi - lo : 0;
}

// every segment's raw rank range and local aggregate, a thread each
__global__ __launch_bounds__(256) void k_round_bounds_pre(const uint32_t *rank, RoundIn in, RoundSegs g, uint64_t r,
                                                          uint64_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= r) return;
    const uint64_t l = in.sk[j] ? (uint64_t)rank[j] : 0ull, h = in.ek[j] ? (uint64_t)rank[r + j] : n;
    g.lo[j] = l;
    g.hi[j] = h;
    uint64_t hi = h < n ? h : n, lo = l;
    if (lo > hi) lo = hi;
    uint64_t o[5];
    base_pre_agg(in.pre, lo, hi, o);
    uint64_t *d = g.loc + 5 * j;
#pragma unroll
    for (int q = 0; q < 5; q++) d[q] = o[q];
}

// every child a thread (its segment by binary search of the child offsets), 256 consecutive
// children a workgroup per pass: staged in LDS, then stored with consecutive lanes on consecutive
// words -- each wave instruction a whole run of lines into the mapped output (a thread storing its
// own child's words, 16-40 B apart lane to lane, took 810 us for a round's 10 MB against the
// wave-per-child kernel's 417); then the enumerations, a thread each
constexpr uint32_t EMIT_CH = 256, EMIT_KW = 8;  // children per pass; key words (kl <= 32)
__global__ __launch_bounds__(EMIT_CH) void k_round_emit_pre(const uint64_t *hdr, uint64_t cap, uint64_t r, uint32_t kl,
                                                             RoundIn in, RoundSegs g, uint8_t *out) {
    __shared__ __align__(16) uint8_t s_sk[EMIT_CH], s_ek[EMIT_CH];
    __shared__ __align__(16) uint32_t s_key[2][EMIT_CH * EMIT_KW];
    __shared__ __align__(16) uint64_t s_agg[EMIT_CH * 5];
    const uint64_t nc = hdr[3], ne = hdr[1];
    if (nc > cap) return;  // the host grows the buffer and launches again
    const RoundLayout L = round_layout(nc, ne, kl);
    const uint32_t t = threadIdx.x, kw = kl / 4;
    for (uint64_t c0 = (uint64_t)blockIdx.x * EMIT_CH; c0 < nc; c0 += (uint64_t)gridDim.x * EMIT_CH) {  // uniform
        const uint64_t c = c0 + t;
        if (c < nc) {
            const uint64_t j = round_owner(g.choff, r, c), k = c - g.choff[j];
            uint8_t skd = in.sk[j], ekd = in.ek[j];
            const uint8_t *skey = skd ? in.skeys + j * kl : nullptr, *ekey = ekd ? in.ekeys + j * kl : nullptr;
            uint64_t o[5];
            const uint64_t ncuts = g.nch[j] - 1;
            const uint8_t kind = g.kind[j];
            if (kind == 1 || ncuts == 0) {
#pragma unroll
                for (int q = 0; q < 5; q++) o[q] = kind == 1 ? 0ull : g.loc[5 * j + q];
            } else {
                const uint64_t st = g.stride[j], s0 = g.si[j];
                const uint64_t lo = s0 + k * st, hi = k == ncuts ? g.ei[j] : s0 + (k + 1) * st;
                if (k) skd = 1, skey = in.bkeys + lo * kl;
                if (k != ncuts) ekd = 1, ekey = in.bkeys + hi * kl;
                base_pre_agg(in.pre, lo, hi, o);
            }
#pragma unroll
            for (int q = 0; q < 5; q++) s_agg[5 * t + q] = o[q];
            s_sk[t] = skd, s_ek[t] = ekd;
            for (uint32_t w = 0; w < kw; w++) {
                s_key[0][t * kw + w] = skey ? reinterpret_cast<const uint32_t *>(skey)[w] : 0u;
                s_key[1][t * kw + w] = ekey ? reinterpret_cast<const uint32_t *>(ekey)[w] : 0u;
            }
        }
        __syncthreads();
        const uint32_t m = nc - c0 < EMIT_CH ? (uint32_t)(nc - c0) : EMIT_CH;
        for (uint32_t i = t; i < m; i += EMIT_CH) out[L.csk + c0 + i] = s_sk[i], out[L.cek + c0 + i] = s_ek[i];
        uint32_t *os = reinterpret_cast<uint32_t *>(out + L.cskeys + c0 * kl);
        uint32_t *oe = reinterpret_cast<uint32_t *>(out + L.cekeys + c0 * kl);
        for (uint32_t i = t; i < m * kw; i += EMIT_CH) os[i] = s_key[0][i], oe[i] = s_key[1][i];
        uint64_t *oa = reinterpret_cast<uint64_t *>(out + L.caggs) + 5 * c0;
        for (uint32_t i = t; i < 5 * m; i += EMIT_CH) oa[i] = s_agg[i];
        __syncthreads();  // the next pass overwrites the staging
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + t; j < r; j += stride)
        if (g.nen[j]) round_emit_enum(j, g.enoff[j], L, kl, in, g, out);
}

// ---- the same over base + delta run when both row prefixes are there (has_row_prefix): a thread
// per segment, a thread per child (its cut places by view_at, its sum their prefixes' difference)
__global__ __launch_bounds__(256) void k_bounds_view_pre(const uint32_t *rank_b, const uint32_t *rank_j,
                                                         const uint8_t *sk, const uint8_t *ek, RoundIn in, RoundRun R,
                                                         uint64_t r, uint32_t ia, uint32_t ib, uint64_t off,
                                                         uint64_t *lo_out, uint64_t *hi_out, uint64_t *agg_out,
                                                         uint64_t *place) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= r) return;
    const uint64_t qs = ia * j, qe = ib * j + off;
    const uint64_t bs = sk[j] ? rank_b[qs] : 0, js = sk[j] ? rank_j[qs] : 0;
    const uint64_t be = ek[j] ? rank_b[qe] : R.nb, je = ek[j] ? rank_j[qe] : R.n;
    const int64_t cs = R.n ? R.cntp[js] : 0, ce = R.n ? R.cntp[je] : 0;
    const uint64_t l = (uint64_t)((int64_t)bs + cs), h = (uint64_t)((int64_t)be + ce);
    uint64_t fp[4] = {0, 0, 0, 0};
    if (h > l) pre_range_fp(in, R, bs, js, be, je, fp);  // an inverted range is ZERO
    lo_out[j] = l;
    hi_out[j] = h;
    if (place) place[4 * j] = bs, place[4 * j + 1] = js, place[4 * j + 2] = be, place[4 * j + 3] = je;
    uint64_t *o = agg_out + 5 * j;
    o[0] = fp[0], o[1] = fp[1], o[2] = fp[2], o[3] = fp[3];
    o[4] = h > l ? h - l : 0;
}
__global__ __launch_bounds__(EMIT_CH) void k_round_emit_view_pre(const uint64_t *hdr, uint64_t cap, uint64_t r,
                                                                  uint32_t kl, RoundIn in, RoundRun R, RoundSegs g,
                                                                  const uint64_t *place, uint8_t *out) {
    __shared__ __align__(16) uint8_t s_sk[EMIT_CH], s_ek[EMIT_CH];
    __shared__ __align__(16) uint32_t s_key[2][EMIT_CH * EMIT_KW];
    __shared__ __align__(16) uint64_t s_agg[EMIT_CH * 5];
    const uint64_t nc = hdr[3], ne = hdr[1];
    if (nc > cap) return;  // the host grows the buffer and launches again
    const RoundLayout L = round_layout(nc, ne, kl);
    const uint32_t t = threadIdx.x, kw = kl / 4;
    for (uint64_t c0 = (uint64_t)blockIdx.x * EMIT_CH; c0 < nc; c0 += (uint64_t)gridDim.x * EMIT_CH) {  // uniform
        const uint64_t c = c0 + t;
        if (c < nc) {
            const uint64_t j = round_owner(g.choff, r, c), k = c - g.choff[j];
            uint8_t skd = in.sk[j], ekd = in.ek[j];
            const uint8_t *skey = skd ? in.skeys + j * kl : nullptr, *ekey = ekd ? in.ekeys + j * kl : nullptr;
            uint64_t o[5];
            const uint64_t ncuts = g.nch[j] - 1;
            const uint8_t kind = g.kind[j];
            if (kind == 1 || ncuts == 0) {
#pragma unroll
                for (int q = 0; q < 5; q++) o[q] = kind == 1 ? 0ull : g.loc[5 * j + q];
            } else {
                const uint64_t st = g.stride[j], s0 = g.si[j];
                const uint64_t lo = s0 + k * st, hi = k == ncuts ? g.ei[j] : s0 + (k + 1) * st;
                ViewPlace a{place[4 * j], place[4 * j + 1], nullptr}, z{place[4 * j + 2], place[4 * j + 3], nullptr};
                if (k) a = view_at(R, in.bkeys, kl, lo), skd = 1, skey = a.key;
                if (k != ncuts) z = view_at(R, in.bkeys, kl, hi), ekd = 1, ekey = z.key;
                uint64_t fp[4];
                pre_range_fp(in, R, a.b, a.j, z.b, z.j, fp);
                o[0] = fp[0], o[1] = fp[1], o[2] = fp[2], o[3] = fp[3], o[4] = hi - lo;
            }
#pragma unroll
            for (int q = 0; q < 5; q++) s_agg[5 * t + q] = o[q];
            s_sk[t] = skd, s_ek[t] = ekd;
            for (uint32_t w = 0; w < kw; w++) {
                s_key[0][t * kw + w] = skey ? reinterpret_cast<const uint32_t *>(skey)[w] : 0u;
                s_key[1][t * kw + w] = ekey ? reinterpret_cast<const uint32_t *>(ekey)[w] : 0u;
            }
        }
        __syncthreads();
        const uint32_t m = nc - c0 < EMIT_CH ? (uint32_t)(nc - c0) : EMIT_CH;
        for (uint32_t i = t; i < m; i += EMIT_CH) out[L.csk + c0 + i] = s_sk[i], out[L.cek + c0 + i] = s_ek[i];
        uint32_t *os = reinterpret_cast<uint32_t *>(out + L.cskeys + c0 * kl);
        uint32_t *oe = reinterpret_cast<uint32_t *>(out + L.cekeys + c0 * kl);
        for (uint32_t i = t; i < m * kw; i += EMIT_CH) os[i] = s_key[0][i], oe[i] = s_key[1][i];
        uint64_t *oa = reinterpret_cast<uint64_t *>(out + L.caggs) + 5 * c0;
        for (uint32_t i = t; i < 5 * m; i += EMIT_CH) oa[i] = s_agg[i];
        __syncthreads();
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + t; j < r; j += stride)
        if (g.nen[j]) round_emit_enum(j, g.enoff[j], L, kl, in, g, out);
}

// every segment's bounds over the view, one wave each
__global__ __launch_bounds__(256) void k_bounds_view(const uint32_t *rank_b, const uint32_t *rank_j, const uint8_t *sk,
                                                     const uint8_t *ek, RoundIn in, RoundRun R, uint64_t r,
                                                     uint32_t ia, uint32_t ib, uint64_t off, uint64_t *lo_out,
                                                     uint64_t *hi_out, uint64_t *agg_out, uint64_t *place) {
    const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= r) return;  // uniform per wave
    bounds_view_one(j, threadIdx.x & 63, rank_b, rank_j, sk, ek, in, R, ia, ib, off, lo_out, hi_out, agg_out, place);
}

// Rank-range aggregates over the view ([lo, hi) clamped as k_range_query_wave clamps), one wave each
__global__ __launch_bounds__(256) void k_range_query_view(RoundIn in, RoundRun R, uint32_t kl, uint64_t nv,
                                                          const uint64_t *qlo, const uint64_t *qhi, uint64_t q,
                                                          uint64_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (j >= q) return;  // uniform per wave
    uint64_t lo = qlo[j], hi = qhi[j];
    if (hi > nv) hi = nv;
    if (lo > hi) lo = hi;
    uint64_t fp[4] = {0, 0, 0, 0};
    if (hi > lo) {
        const ViewPlace a = view_at(R, in.bkeys, kl, lo);
        const ViewPlace z = hi < nv ? view_at(R, in.bkeys, kl, hi) : ViewPlace{R.nb, R.n, nullptr};
        view_range_fp(in, R, a.b, a.j, z.b, z.j, lane, fp);
    }
    if (lane == 0) {
        uint64_t *o = out + 5 * j;
        o[0] = fp[0];
        o[1] = fp[1];
        o[2] = fp[2];
        o[3] = fp[3];
        o[4] = hi - lo;
    }
}

// The view keys of the given ranks (each < nv), one thread each
__global__ void k_select_view(RoundRun R, const uint8_t *bkeys, uint32_t kl, const uint64_t *ranks, uint64_t first,
                              uint64_t m, uint8_t *out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= m) return;
    const ViewPlace p = view_at(R, bkeys, kl, ranks ? ranks[t] : first + t);
    for (uint32_t w = 0; w < kl / 4; w++)
        reinterpret_cast<uint32_t *>(out + t * kl)[w] = reinterpret_cast<const uint32_t *>(p.key)[w];
}


__global__ __launch_bounds__(256) void k_round_emit_view(const uint64_t *hdr, uint64_t cap, uint64_t r, uint32_t kl,
                                                         RoundIn in, RoundRun R, RoundSegs g, const uint64_t *place,
                                                         uint8_t *out) {
    const uint64_t nc = hdr[3], ne = hdr[1];
    if (nc > cap) return;  // the host grows the buffer and launches again
    const RoundLayout L = round_layout(nc, ne, kl);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nc; c += nw) {
        const uint64_t j = round_owner(g.choff, r, c);
        round_emit_child_view(c, j, c - g.choff[j], L, kl, lane, in, R, g, place, out);
    }
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < r; j += nw * 64)
        if (g.nen[j]) round_emit_enum(j, g.enoff[j], L, kl, in, g, out);
}

// A round's output out of device memory into mapped page-locked memory, exactly round_layout's
// bytes (the header says how many) -- no header round trip to the host first.  Children beyond
// cap: the header alone (the host grows the buffer and emits again).  16-byte stores, whole lines
// per wave.
__global__ __launch_bounds__(256) void k_round_copy_out(const uint64_t *hdr, uint64_t cap, uint32_t kl,
                                                        const uint8_t *src, uint8_t *dst, uint64_t max_bytes) {
    const uint64_t nc = hdr[3], ne = hdr[1];
    uint64_t end = nc > cap ? 64 : round_layout(nc, ne, kl).end;
    if (end > max_bytes) end = max_bytes;
    const uint64_t n16 = end / 16;
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        d[i] = s[i];
}

// Every segment's raw rank range and local aggregate, one wave each
__global__ __launch_bounds__(256) void k_round_bounds(const uint32_t *rank, RoundIn in, RoundSegs g, uint64_t r,
                                                      uint64_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (j >= r) return;  // uniform per wave
    const uint64_t l = in.sk[j] ? (uint64_t)rank[j] : 0ull, h = in.ek[j] ? (uint64_t)rank[r + j] : n;
    if (lane == 0) {
        g.lo[j] = l;
        g.hi[j] = h;
    }
    uint64_t hi = h < n ? h : n, lo = l;
    if (lo > hi) lo = hi;
    wave_range_agg(in.fps, 32, in.bsums, in.ssums, lo, hi, lane, g.loc + 5 * j);
}


__global__ __launch_bounds__(1024) void k_round_small(const uint32_t *rank, RoundIn in, RoundSegs g, uint64_t r,
                                                      uint64_t n, int sqrt_policy, uint64_t b, uint64_t cap,
                                                      uint32_t kl, uint8_t *out) {
    __shared__ uint64_t wsum[2][16], tot[2];
    __shared__ unsigned long long cnt[5];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t < 5) cnt[t] = 0;
    const bool mine = t < r;
    if (mine) {
        g.lo[t] = in.sk[t] ? (uint64_t)rank[t] : 0ull;
        g.hi[t] = in.ek[t] ? (uint64_t)rank[r + t] : n;
    }
    __syncthreads();
    for (uint64_t j = w; j < r; j += 16) {
        uint64_t lo = g.lo[j], hi = g.hi[j];
        if (hi > n) hi = n;
        if (lo > hi) lo = hi;
        wave_range_agg(in.fps, 32, in.bsums, in.ssums, lo, hi, lane, g.loc + 5 * j);
    }
    __syncthreads();
    RoundSeg d{3, 0, 0, 0, 0, 0};
    if (mine) {
        d = round_decide(g.lo[t], g.hi[t], g.loc + 5 * t, in.remote + 5 * t, n, sqrt_policy, b);
        g.kind[t] = (uint8_t)d.kind;
        g.stride[t] = d.stride;
        g.si[t] = d.si;
        g.ei[t] = d.ei;
        g.nch[t] = d.children;
        g.nen[t] = d.enums;
        atomicAdd(&cnt[d.kind == 3 ? 4 : d.kind], 1ull);
    }
    const uint64_t co = block_exclusive_scan(d.children, wsum[0], &tot[0]);
    const uint64_t eo = block_exclusive_scan(d.enums, wsum[1], &tot[1]);
    const uint64_t nc = tot[0], ne = tot[1];
    if (mine) {
        g.choff[t] = co;
        g.enoff[t] = eo;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t *hdr = reinterpret_cast<uint64_t *>(out);
        hdr[0] = cnt[0];
        hdr[1] = ne;
        hdr[2] = cnt[2];
        hdr[3] = nc;
        hdr[4] = cnt[4];
    }
    if (nc > cap) return;  // uniform
    const RoundLayout L = round_layout(nc, ne, kl);
    if (mine && d.enums) round_emit_enum(t, eo, L, kl, in, g, out);
    for (uint64_t c = w; c < nc; c += 16) {
        const uint64_t j = round_owner(g.choff, r, c);
        round_emit_child(c, j, c - g.choff[j], L, kl, lane, in, g, out);
    }
}
// A tiny round over base + delta run in one launch after the two searches: k_round_small's
// shape with the view's bounds (bounds_view_one) and children (round_emit_child_view)
__global__ __launch_bounds__(1024) void k_round_small_view(const uint32_t *rank_b, const uint32_t *rank_j, RoundIn in,
                                                           RoundRun R, RoundSegs g, uint64_t *place, uint64_t r,
                                                           uint64_t n, int sqrt_policy, uint64_t b, uint64_t cap,
                                                           uint32_t kl, uint8_t *out) {
    __shared__ uint64_t wsum[2][16], tot[2];
    __shared__ unsigned long long cnt[5];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t < 5) cnt[t] = 0;
    const bool mine = t < r;
    for (uint64_t j = w; j < r; j += 16)
        bounds_view_one<false>(j, lane, rank_b, rank_j, in.sk, in.ek, in, R, 1u, 1u, r, g.lo, g.hi, g.loc, place);
    __syncthreads();
    RoundSeg d{3, 0, 0, 0, 0, 0};
    if (mine) {
        d = round_decide(g.lo[t], g.hi[t], g.loc + 5 * t, in.remote + 5 * t, n, sqrt_policy, b);
        g.kind[t] = (uint8_t)d.kind;
        g.stride[t] = d.stride;
        g.si[t] = d.si;
        g.ei[t] = d.ei;
        g.nch[t] = d.children;
        g.nen[t] = d.enums;
        atomicAdd(&cnt[d.kind == 3 ? 4 : d.kind], 1ull);
    }
    const uint64_t co = block_exclusive_scan(d.children, wsum[0], &tot[0]);
    const uint64_t eo = block_exclusive_scan(d.enums, wsum[1], &tot[1]);
    const uint64_t nc = tot[0], ne = tot[1];
    if (mine) {
        g.choff[t] = co;
        g.enoff[t] = eo;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t *hdr = reinterpret_cast<uint64_t *>(out);
        hdr[0] = cnt[0];
        hdr[1] = ne;
        hdr[2] = cnt[2];
        hdr[3] = nc;
        hdr[4] = cnt[4];
    }
    if (nc > cap) return;  // uniform
    const RoundLayout L = round_layout(nc, ne, kl);
    if (mine && d.enums) round_emit_enum(t, eo, L, kl, in, g, out);
    for (uint64_t c = w; c < nc; c += 16) {
        const uint64_t j = round_owner(g.choff, r, c);
        round_emit_child_view<false>(c, j, c - g.choff[j], L, kl, lane, in, R, g, place, out);
    }
}
__global__ __launch_bounds__(1024) void k_round_plan_scan(RoundIn in, RoundSegs g, uint64_t r, uint64_t n,
                                                          int sqrt_policy, uint64_t b, uint8_t *out) {
    __shared__ uint64_t wsum[2][16], tot[2];
    __shared__ unsigned long long cnt[5];
    const uint32_t t = threadIdx.x;
    if (t < 5) cnt[t] = 0;
    __syncthreads();
    const bool mine = t < r;
    RoundSeg d{3, 0, 0, 0, 0, 0};
    if (mine) {
        d = round_decide(g.lo[t], g.hi[t], g.loc + 5 * t, in.remote + 5 * t, n, sqrt_policy, b);
        g.kind[t] = (uint8_t)d.kind;
        g.stride[t] = d.stride;
        g.si[t] = d.si;
        g.ei[t] = d.ei;
        g.nch[t] = d.children;
        g.nen[t] = d.enums;
        atomicAdd(&cnt[d.kind == 3 ? 4 : d.kind], 1ull);
    }
    const uint64_t co = block_exclusive_scan(d.children, wsum[0], &tot[0]);
    const uint64_t eo = block_exclusive_scan(d.enums, wsum[1], &tot[1]);
    const uint64_t nc = tot[0], ne = tot[1];
    if (mine) {
        g.choff[t] = co;
        g.enoff[t] = eo;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t *hdr = reinterpret_cast<uint64_t *>(out);
        hdr[0] = cnt[0];
        hdr[1] = ne;
        hdr[2] = cnt[2];
        hdr[3] = nc;
        hdr[4] = cnt[4];
    }
}


// out[j] = Σ_p in[p*r + j] over rh_aggregate {u64 fp[4]; u64 size}
__global__ void k_combine(const uint64_t *in, uint64_t parts, uint64_t r, uint64_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= r) return;
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0, sz = 0;
    for (uint64_t p = 0; p < parts; p++) {
        const uint64_t *a = in + 5 * (p * r + j);
        uint64_t t0 = s0 + a[0];
        uint64_t c = t0 < s0;
        uint64_t t1 = s1 + a[1];
        uint64_t c1 = t1 < s1;
        t1 += c;
        c1 |= (t1 < c);
        uint64_t t2 = s2 + a[2];
        uint64_t c2 = t2 < s2;
        t2 += c1;
        c2 |= (t2 < c1);
        uint64_t t3 = s3 + a[3] + c2;
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
        sz += a[4];
    }
    uint64_t *o = out + 5 * j;
    o[0] = s0; o[1] = s1; o[2] = s2; o[3] = s3; o[4] = sz;
}

// ---- launchers --------------------------------------------------------------------------------

hipError_t launch_lift_encoded(const uint8_t *bytes, const uint64_t *offs, uint64_t n, uint64_t limit,
                               uint8_t *fps, uint8_t *bsums, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t waves = (n + ENC_PER_WAVE - 1) / ENC_PER_WAVE;
    // multi-chunk records first: the short kernel's block sums read their fingerprints
    hipLaunchKernelGGL(k_lift_encoded_long, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, bytes, offs, n, limit,
                       fps);
    hipLaunchKernelGGL(k_lift_encoded_short, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, st, bytes, offs, n,
                       limit, fps, bsums);
    return hipGetLastError();
}

// ---- exclusive 256-bit prefix sums (the host tier's per-row prefix) -----------------
// out[i] = Σ in[0..i) mod 2^256 for i in [0, n] (out[n] = the total): one workgroup per chunk of
// 256 entries, a carry-save wave scan (64-bit shuffles of the 8 u32-limb sums, which stay below
// 2^40), the waves' totals through LDS, then the chunk's base -- base[c] = Σ in[0..256 c), from the
// level above (the block sums' prefix for rows, the super-block sums' prefix for blocks).
__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t x, int d) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    lo = __shfl_up(lo, d, 64);
    hi = __shfl_up(hi, d, 64);
    return ((uint64_t)hi << 32) | lo;
}

// grid-stride over the 256-entry chunks: a grid of one workgroup per chunk (launch_prefix), or at
// most PREFIX_WGS workgroups (launch_row_prefix: a row prefix formed beside the store's questions,
// ensure_base_prefix, leaves the CUs' slots to their one-workgroup kernels)
constexpr uint32_t PREFIX_WGS = 1024;
__global__ __launch_bounds__(256) void k_prefix256(const uint8_t *in, uint64_t n, const uint8_t *base,
                                                   uint8_t *out) {
    __shared__ uint64_t wtot[4][8];
    const uint64_t nch = n / 256 + 1;
    for (uint64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
        __syncthreads();  // the previous chunk's wtot reads are done
        const uint64_t i = ch * 256 + threadIdx.x;
        const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        uint32_t f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i < n) load_fp(in, i, f);
        Acc a;
#pragma unroll
        for (int q = 0; q < 8; q++) a.l[q] = f[q];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint64_t y = shfl_up_u64(a.l[q], d);
                if (lane >= (uint32_t)d) a.l[q] += y;
            }
        }
        if (lane == 63) {
#pragma unroll
            for (int q = 0; q < 8; q++) wtot[w][q] = a.l[q];
        }
        __syncthreads();
        uint32_t bf[8];
        load_fp(base, ch, bf);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            uint64_t v = a.l[q] - f[q] + bf[q];  // inclusive -> exclusive, + the chunk's base
            for (uint32_t k = 0; k < w; k++) v += wtot[k][q];
            a.l[q] = v;
        }
        if (i <= n) {
            uint32_t o[8];
            acc_normalise(a, o);
            store_sum(out, i, o);
        }
    }
}

// The top level, one workgroup: out[i] = Σ in[0..i) for i in [0, n], chunk by chunk with the
// running total carried in LDS (n = the super-block count: at most 2^31 / 65536 + 1 entries)
__global__ __launch_bounds__(256) void k_prefix_top(const uint8_t *in, uint64_t n, uint8_t *out) {
    __shared__ uint64_t wtot[4][8];
    __shared__ uint32_t run[8];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 8) run[threadIdx.x] = 0;
    __syncthreads();
    for (uint64_t c0 = 0; c0 <= n; c0 += 256) {
        const uint64_t i = c0 + threadIdx.x;
        uint32_t f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i < n) load_fp(in, i, f);
        Acc a;
#pragma unroll
        for (int q = 0; q < 8; q++) a.l[q] = f[q];
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint64_t y = shfl_up_u64(a.l[q], d);
                if (lane >= (uint32_t)d) a.l[q] += y;
            }
        }
        if (lane == 63) {
#pragma unroll
            for (int q = 0; q < 8; q++) wtot[w][q] = a.l[q];
        }
        __syncthreads();
        Acc e;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            uint64_t v = a.l[q] - f[q] + run[q];
            for (uint32_t k = 0; k < w; k++) v += wtot[k][q];
            e.l[q] = v;
        }
        uint32_t o[8];
        acc_normalise(e, o);
        if (i <= n) store_sum(out, i, o);
        __syncthreads();  // every lane has read run[] and wtot[]
        if (threadIdx.x == 255) {  // the chunk's inclusive total = the next chunk's running base
            Acc t;
#pragma unroll
            for (int q = 0; q < 8; q++) t.l[q] = e.l[q] + f[q];
            uint32_t r[8];
            acc_normalise(t, r);
#pragma unroll
            for (int q = 0; q < 8; q++) run[q] = r[q];
        }
        __syncthreads();
    }
}

// ---- rank-addressed batch merge (the encoded store, rh_estore_apply) ----------------------------
// out[r] for r in [0, n_out): the row of the segment holding r -- seg k covers out rows
// [start[k], start[k + 1]) and reads them from `newf` (src[k] with bit 63 set: the batch's lifted
// fingerprints) or `old` (the previous rank order) from row src[k] & ~bit63 on.  A thread per
// output row, its segment by binary search of the (L2-resident) segment starts; rows of one
// segment are contiguous on both sides, so the 32-B reads and writes stay coalesced.
__global__ __launch_bounds__(256) void k_seg_copy(const uint8_t *old, const uint8_t *newf, const uint64_t *start,
                                                  const uint64_t *src, uint64_t nseg, uint64_t n_out, uint8_t *out) {
    const uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n_out) return;
    uint64_t a = 0, z = nseg;
    while (z - a > 1) {  // the last k with start[k] <= r
        const uint64_t mid = (a + z) >> 1;
        if (start[mid] <= r) a = mid;
        else z = mid;
    }
    const uint64_t sv = src[a], row = (sv & ~(1ull << 63)) + (r - start[a]);
    const uint4 *p = reinterpret_cast<const uint4 *>((sv >> 63 ? newf : old) + 32 * row);
    uint4 *o = reinterpret_cast<uint4 *>(out + 32 * r);
    o[0] = p[0];
    o[1] = p[1];
}

hipError_t launch_seg_copy(const uint8_t *old, const uint8_t *newf, const uint64_t *start, const uint64_t *src,
                           uint64_t nseg, uint64_t n_out, uint8_t *out, hipStream_t st) {
    if (n_out == 0 || nseg == 0) return hipSuccess;
    hipLaunchKernelGGL(k_seg_copy, dim3((uint32_t)((n_out + 255) / 256)), dim3(256), 0, st, old, newf, start, src, nseg,
                       n_out, out);
    return hipGetLastError();
}

hipError_t launch_prefix(const uint8_t *fps, uint64_t n, const uint8_t *bsums, const uint8_t *ssums, uint8_t *spre,
                         uint8_t *bpre, uint8_t *out, hipStream_t st, uint32_t max_wgs) {
    const uint64_t nbk = (n + 255) / 256, ns = (nbk + 255) / 256;
    hipLaunchKernelGGL(k_prefix_top, dim3(1), dim3(256), 0, st, ssums, ns, spre);
    hipLaunchKernelGGL(k_prefix256, dim3((uint32_t)(nbk / 256 + 1)), dim3(256), 0, st, bsums, nbk,
                       (const uint8_t *)spre, bpre);
    const uint64_t g = max_wgs ? std::min<uint64_t>(n / 256 + 1, max_wgs) : n / 256 + 1;
    hipLaunchKernelGGL(k_prefix256, dim3((uint32_t)g), dim3(256), 0, st, fps, n, (const uint8_t *)bpre,
                       out);
    return hipGetLastError();
}

hipError_t launch_row_prefix(const uint8_t *fps, uint64_t n, const uint8_t *bpre, uint8_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_prefix256, dim3((uint32_t)std::min<uint64_t>(n / 256 + 1, PREFIX_WGS)), dim3(256), 0, st, fps, n,
                       bpre, out);
    return hipGetLastError();
}

hipError_t launch_block_prefix(uint64_t n, const uint8_t *bsums, const uint8_t *ssums, uint8_t *spre, uint8_t *bpre,
                               hipStream_t st) {
    const uint64_t nbk = (n + 255) / 256, ns = (nbk + 255) / 256;
    hipLaunchKernelGGL(k_prefix_top, dim3(1), dim3(256), 0, st, ssums, ns, spre);
    hipLaunchKernelGGL(k_prefix256, dim3((uint32_t)(nbk / 256 + 1)), dim3(256), 0, st, bsums, nbk,
                       (const uint8_t *)spre, bpre);
    return hipGetLastError();
}

hipError_t launch_reduce(const uint8_t *in, uint64_t n_in, uint8_t *out, hipStream_t st, uint32_t stride) {
    if (n_in == 0) return hipSuccess;
    const uint64_t g = (n_in + 255) / 256;
    hipLaunchKernelGGL(k_reduce, dim3((uint32_t)g), dim3(256), 0, st, in, stride, n_in, out);
    return hipGetLastError();
}

hipError_t launch_total(const uint8_t *in, uint64_t n, uint64_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_total, dim3(1), dim3(256), 0, st, in, n, out);
    return hipGetLastError();
}

hipError_t launch_lift_fixed(const uint8_t *bytes, uint64_t len, uint64_t n, uint64_t limit, uint8_t *fps,
                             uint8_t *bsums, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const dim3 g((uint32_t)((n + 255) / 256));
    // compile-time lengths: the record is read exactly (n * len <= limit is the caller's check),
    // with loads as wide as the records' alignment allows
    const uint64_t align = len < 16 ? 16 : std::min<uint64_t>(16, len & (~len + 1));
    if (len && n * len <= limit && reinterpret_cast<uintptr_t>(bytes) % align == 0) {
        switch (len) {
#define RH_FIXED_CT(L)                                                                           \
    case L:                                                                                      \
        hipLaunchKernelGGL(k_lift_fixed_ct<L>, g, dim3(256), 0, st, bytes, n, fps, bsums);       \
        return hipGetLastError();
            RH_FIXED_CT(48)
            RH_FIXED_CT(80)
            RH_FIXED_CT(100)
            RH_FIXED_CT(104)
            RH_FIXED_CT(120)
#undef RH_FIXED_CT
            default:
                break;
        }
    }
    if (len <= (uint64_t)CHUNK_LEN && len % 4 == 0)
        hipLaunchKernelGGL(k_lift_fixed_short<true>, g, dim3(256), 0, st, bytes, (uint32_t)len, n, limit, fps, bsums);
    else if (len <= (uint64_t)CHUNK_LEN)
        hipLaunchKernelGGL(k_lift_fixed_short<false>, g, dim3(256), 0, st, bytes, (uint32_t)len, n, limit, fps,
                           bsums);
    else hipLaunchKernelGGL(k_lift_fixed_long, g, dim3(256), 0, st, bytes, len, n, limit, fps, bsums);
    return hipGetLastError();
}

hipError_t launch_range_query(const uint8_t *fps, const uint8_t *bsums, const uint8_t *ssums, uint64_t n,
                              const uint64_t *lo, const uint64_t *hi, uint64_t r, uint64_t *out,
                              hipStream_t st, uint32_t stride, const uint32_t *slots) {
    if (r == 0) return hipSuccess;
    if (bsums && ssums && r >= 64 && !slots) {  // many queries: one wave each
        hipLaunchKernelGGL(k_range_query_wave, dim3((uint32_t)((r + 3) / 4)), dim3(256), 0, st, fps, stride, bsums,
                           ssums, n, lo, hi, r, out);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_range_query, dim3((uint32_t)r), dim3(256), 0, st, fps, stride, slots, bsums, ssums, n, lo, hi,
                       r, out);
    return hipGetLastError();
}

hipError_t launch_round_plan3(const RoundSegs &g, const uint64_t *remote, uint64_t r, uint64_t n, int sqrt_policy,
                              uint64_t b, uint64_t *part, uint64_t *hdr, hipStream_t st) {
    if (r == 0) return hipSuccess;
    const uint64_t np = (r + 255) / 256;
    hipLaunchKernelGGL(k_round_plan_part, dim3((uint32_t)np), dim3(256), 0, st, g, remote, r, n, sqrt_policy, b, part);
    hipLaunchKernelGGL(k_round_plan_scan_parts, dim3(1), dim3(1024), 0, st, part, np, hdr);
    hipLaunchKernelGGL(k_round_plan_apply, dim3((uint32_t)np), dim3(256), 0, st, g, r, (const uint64_t *)part);
    return hipGetLastError();
}

hipError_t launch_round_plan(const RoundSegs &g, const uint64_t *remote, uint64_t r, uint64_t n, int sqrt_policy,
                             uint64_t b, uint64_t *hdr, hipStream_t st) {
    if (r == 0) return hipSuccess;
    hipLaunchKernelGGL(k_round_plan, dim3((uint32_t)((r + 255) / 256)), dim3(256), 0, st, g, remote, r, n,
                       sqrt_policy, b, hdr);
    return hipGetLastError();
}

hipError_t launch_round_emit(const uint64_t *hdr, uint64_t cap, uint64_t r, uint32_t kl, const RoundIn &in,
                             const RoundSegs &g, uint8_t *out, hipStream_t st) {
    if (r == 0) return hipSuccess;
    if (in.pre && kl <= 4 * EMIT_KW) {  // a thread per child
        const uint64_t w = std::min<uint64_t>(std::max<uint64_t>((cap + EMIT_CH - 1) / EMIT_CH, (r + 255) / 256), 8192);
        hipLaunchKernelGGL(k_round_emit_pre, dim3((uint32_t)w), dim3(EMIT_CH), 0, st, hdr, cap, r, kl, in, g, out);
        return hipGetLastError();
    }
    const uint64_t wgs = std::min<uint64_t>(std::max<uint64_t>((cap + 3) / 4, (r + 255) / 256), 4096);
    hipLaunchKernelGGL(k_round_emit, dim3((uint32_t)wgs), dim3(256), 0, st, hdr, cap, r, kl, in, g, out);
    return hipGetLastError();
}

hipError_t launch_round_bounds(const uint32_t *rank, const RoundIn &in, const RoundSegs &g, uint64_t r, uint64_t n,
                               hipStream_t st) {
    if (r == 0) return hipSuccess;
    if (in.pre) {  // a thread per segment
        hipLaunchKernelGGL(k_round_bounds_pre, dim3((uint32_t)((r + 255) / 256)), dim3(256), 0, st, rank, in, g, r, n);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_round_bounds, dim3((uint32_t)((r + 3) / 4)), dim3(256), 0, st, rank, in, g, r, n);
    return hipGetLastError();
}

hipError_t launch_round_bounds_view(const uint32_t *rank_b, const uint32_t *rank_j, const RoundIn &in,
                                    const RoundRun &run, const RoundSegs &g, uint64_t *place, uint64_t r,
                                    hipStream_t st) {
    if (r == 0) return hipSuccess;
    if (in.pre && (run.n == 0 || run.pre)) {  // a thread per segment
        hipLaunchKernelGGL(k_bounds_view_pre, dim3((uint32_t)((r + 255) / 256)), dim3(256), 0, st, rank_b, rank_j, in.sk,
                           in.ek, in, run, r, 1u, 1u, r, g.lo, g.hi, g.loc, place);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_bounds_view, dim3((uint32_t)((r + 3) / 4)), dim3(256), 0, st, rank_b, rank_j, in.sk, in.ek, in,
                       run, r, 1u, 1u, r, g.lo, g.hi, g.loc, place);
    return hipGetLastError();
}

hipError_t launch_resolve_view(const uint32_t *rank_b, const uint32_t *rank_j, const uint8_t *sk, const uint8_t *ek,
                               const RoundIn &in, const RoundRun &run, uint64_t r, uint64_t *lo, uint64_t *hi,
                               uint64_t *aggs, hipStream_t st) {
    if (r == 0) return hipSuccess;
    if (in.pre && (run.n == 0 || run.pre)) {  // a thread per segment
        hipLaunchKernelGGL(k_bounds_view_pre, dim3((uint32_t)((r + 255) / 256)), dim3(256), 0, st, rank_b, rank_j, sk, ek,
                           in, run, r, 2u, 2u, (uint64_t)1, lo, hi, aggs, (uint64_t *)nullptr);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(k_bounds_view, dim3((uint32_t)((r + 3) / 4)), dim3(256), 0, st, rank_b, rank_j, sk, ek, in, run,
                       r, 2u, 2u, (uint64_t)1, lo, hi, aggs, (uint64_t *)nullptr);
    return hipGetLastError();
}

hipError_t launch_range_query_view(const RoundIn &in, const RoundRun &run, uint32_t kl, uint64_t nv,
                                   const uint64_t *lo, const uint64_t *hi, uint64_t q, uint64_t *out, hipStream_t st) {
    if (q == 0) return hipSuccess;
    hipLaunchKernelGGL(k_range_query_view, dim3((uint32_t)((q + 3) / 4)), dim3(256), 0, st, in, run, kl, nv, lo, hi, q,
                       out);
    return hipGetLastError();
}

hipError_t launch_select_view(const RoundRun &run, const uint8_t *bkeys, uint32_t kl, const uint64_t *ranks,
                              uint64_t first, uint64_t m, uint8_t *out, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_select_view, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, st, run, bkeys, kl, ranks, first,
                       m, out);
    return hipGetLastError();
}

hipError_t launch_round_emit_view(const uint64_t *hdr, uint64_t cap, uint64_t r, uint32_t kl, const RoundIn &in,
                                  const RoundRun &run, const RoundSegs &g, const uint64_t *place, uint8_t *out,
                                  hipStream_t st) {
    if (r == 0) return hipSuccess;
    if (in.pre && (run.n == 0 || run.pre) && kl <= 4 * EMIT_KW) {  // a thread per child
        const uint64_t w = std::min<uint64_t>(std::max<uint64_t>((cap + EMIT_CH - 1) / EMIT_CH, (r + 255) / 256), 8192);
        hipLaunchKernelGGL(k_round_emit_view_pre, dim3((uint32_t)w), dim3(EMIT_CH), 0, st, hdr, cap, r, kl, in, run, g,
                           place, out);
        return hipGetLastError();
    }
    const uint64_t wgs = std::min<uint64_t>(std::max<uint64_t>((cap + 3) / 4, (r + 255) / 256), 4096);
    hipLaunchKernelGGL(k_round_emit_view, dim3((uint32_t)wgs), dim3(256), 0, st, hdr, cap, r, kl, in, run, g, place,
                       out);
    return hipGetLastError();
}

// every job's 16-byte units by the whole grid (the tails of jobs not a multiple of 16 bytes by
// single bytes); src and dst 16-byte aligned (device buffers and page-locked allocations are)
__global__ __launch_bounds__(256) void k_copy_to_host(CopyJobs j) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    for (int k = 0; k < j.n; k++) {
        const uint64_t n16 = j.bytes[k] / 16;
        const uint4 *s = reinterpret_cast<const uint4 *>(j.src[k]);
        uint4 *d = reinterpret_cast<uint4 *>(j.dst[k]);
        for (uint64_t i = tid; i < n16; i += nt) d[i] = s[i];
        for (uint64_t i = n16 * 16 + tid; i < j.bytes[k]; i += nt) j.dst[k][i] = j.src[k][i];
    }
}

hipError_t launch_copy_to_host(const CopyJobs &jobs, hipStream_t st, uint32_t max_wgs) {
    uint64_t tot = 0;
    for (int k = 0; k < jobs.n; k++) tot += jobs.bytes[k];
    if (tot == 0) return hipSuccess;
    // one workgroup per CU at most: enough stores in flight for the link, and CUs left for the
    // store's own kernels while a background refresh copies
    const uint64_t wgs = std::min<uint64_t>(max_wgs ? max_wgs : 256, (tot / 16 + 255) / 256 + 1);
    hipLaunchKernelGGL(k_copy_to_host, dim3((uint32_t)wgs), dim3(256), 0, st, jobs);
    return hipGetLastError();
}

hipError_t launch_round_copy_out(const uint64_t *hdr, uint64_t cap, uint32_t kl, const uint8_t *src, uint8_t *dst,
                                 uint64_t worst, hipStream_t st) {
    const uint64_t wgs = std::min<uint64_t>(std::max<uint64_t>(worst / 16 / 256, 1), 1024);
    hipLaunchKernelGGL(k_round_copy_out, dim3((uint32_t)wgs), dim3(256), 0, st, hdr, cap, kl, src, dst, worst);
    return hipGetLastError();
}

uint64_t round_tiny_max() { return ROUND_TINY; }
uint64_t round_small_max() { return ROUND_SMALL; }

hipError_t launch_round_plan_scan(const RoundIn &in, const RoundSegs &g, uint64_t r, uint64_t n, int sqrt_policy,
                                  uint64_t b, uint8_t *out, hipStream_t st) {
    if (r == 0 || r > ROUND_SMALL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_round_plan_scan, dim3(1), dim3(ROUND_SMALL), 0, st, in, g, r, n, sqrt_policy, b, out);
    return hipGetLastError();
}

hipError_t launch_round_small(const uint32_t *rank, const RoundIn &in, const RoundSegs &g, uint64_t r, uint64_t n,
                              int sqrt_policy, uint64_t b, uint64_t cap, uint32_t kl, uint8_t *out, hipStream_t st) {
    if (r == 0 || r > ROUND_TINY) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_round_small, dim3(1), dim3(ROUND_SMALL), 0, st, rank, in, g, r, n, sqrt_policy, b, cap, kl,
                       out);
    return hipGetLastError();
}

hipError_t launch_round_small_view(const uint32_t *rank_b, const uint32_t *rank_j, const RoundIn &in,
                                   const RoundRun &run, const RoundSegs &g, uint64_t *place, uint64_t r, uint64_t n,
                                   int sqrt_policy, uint64_t b, uint64_t cap, uint32_t kl, uint8_t *out,
                                   hipStream_t st) {
    if (r == 0 || r > ROUND_TINY) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_round_small_view, dim3(1), dim3(ROUND_SMALL), 0, st, rank_b, rank_j, in, run, g, place, r, n,
                       sqrt_policy, b, cap, kl, out);
    return hipGetLastError();
}

hipError_t launch_combine(const uint64_t *in, uint64_t parts, uint64_t r, uint64_t *out, hipStream_t st) {
    if (r == 0) return hipSuccess;
    const uint64_t g = (r + 255) / 256;
    hipLaunchKernelGGL(k_combine, dim3((uint32_t)g), dim3(256), 0, st, in, parts, r, out);
    return hipGetLastError();
}

}  // namespace rh
