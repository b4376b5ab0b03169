// blake3_device.hpp -- BLAKE3 compression and the 256-bit fingerprint group on gfx950.
//
// One record per lane.  The compression is pure 32-bit VALU ARX work: each G is
// 2 x v_add3_u32 + 2 x v_add_u32 + 4 x v_xor_b32 + 4 x v_alignbit_b32 (rotations), so a
// compression is 56 G = 672 VALU ops + 8 XORs for the output.  Message words are passed
// as registers and the per-round permutation is resolved at compile time (register
// renaming, no data movement).
//
// Reference semantics: rsos::lift hashes with crate `blake3` 1.8.5 (Cargo.lock:197-200;
// call sites rsos/src/encoding.rs:89-93, rsos/src/fingerprint.rs:235,249).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rh {

constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u, IV3 = 0xA54FF53Au,
                   IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu, IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;
constexpr uint32_t CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8;
constexpr int BLOCK_LEN = 64, CHUNK_LEN = 1024;

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}

#define RH_G(a, b, c, d, mx, my)          \
    do {                                  \
        a = a + b + (mx);                 \
        d = rotr(d ^ a, 16);              \
        c = c + d;                        \
        b = rotr(b ^ c, 12);              \
        a = a + b + (my);                 \
        d = rotr(d ^ a, 8);               \
        c = c + d;                        \
        b = rotr(b ^ c, 7);               \
    } while (0)

// Compress one block.  cv[8] in/out (out = first 8 words of the compression output,
// i.e. the new chaining value, or the root hash when flags has ROOT).
__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16], uint32_t counter_lo,
                                         uint32_t counter_hi, uint32_t block_len, uint32_t flags) {
    uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3];
    uint32_t v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
    uint32_t v8 = IV0, v9 = IV1, v10 = IV2, v11 = IV3;
    uint32_t v12 = counter_lo, v13 = counter_hi, v14 = block_len, v15 = flags;
#define RH_ROUND(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
    RH_G(v0, v4, v8, v12, m[s0], m[s1]);                                          \
    RH_G(v1, v5, v9, v13, m[s2], m[s3]);                                          \
    RH_G(v2, v6, v10, v14, m[s4], m[s5]);                                         \
    RH_G(v3, v7, v11, v15, m[s6], m[s7]);                                         \
    RH_G(v0, v5, v10, v15, m[s8], m[s9]);                                         \
    RH_G(v1, v6, v11, v12, m[s10], m[s11]);                                       \
    RH_G(v2, v7, v8, v13, m[s12], m[s13]);                                        \
    RH_G(v3, v4, v9, v14, m[s14], m[s15]);
    // the message schedule: row r = the BLAKE3 permutation applied r times
    RH_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    RH_ROUND(2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8);
    RH_ROUND(3, 4, 10, 12, 13, 2, 7, 14, 6, 5, 9, 0, 11, 15, 8, 1);
    RH_ROUND(10, 7, 12, 9, 14, 3, 13, 15, 4, 0, 11, 2, 5, 8, 1, 6);
    RH_ROUND(12, 13, 9, 11, 15, 10, 14, 8, 7, 2, 5, 3, 0, 1, 6, 4);
    RH_ROUND(9, 14, 11, 5, 8, 12, 15, 1, 13, 3, 0, 10, 2, 6, 4, 7);
    RH_ROUND(11, 15, 5, 0, 1, 9, 8, 6, 14, 10, 2, 12, 3, 4, 7, 13);
#undef RH_ROUND
    cv[0] = v0 ^ v8;
    cv[1] = v1 ^ v9;
    cv[2] = v2 ^ v10;
    cv[3] = v3 ^ v11;
    cv[4] = v4 ^ v12;
    cv[5] = v5 ^ v13;
    cv[6] = v6 ^ v14;
    cv[7] = v7 ^ v15;
}
#undef RH_G

__device__ __forceinline__ void cv_iv(uint32_t cv[8]) {
    cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
    cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// parent node: cv_out = compress(IV, left || right, 0, 64, PARENT | extra)
__device__ __forceinline__ void parent(uint32_t out[8], const uint32_t l[8], const uint32_t r[8],
                                       uint32_t extra) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; i++) { m[i] = l[i]; m[i + 8] = r[i]; }
    cv_iv(out);
    compress(out, m, 0, 0, BLOCK_LEN, PARENT | extra);
}

// ---- 256-bit fingerprint sums (rsos/src/fingerprint.rs:145-154: add with carry) ----------
//
// Carry-save form: a fingerprint is 8 x u32 limbs (LE, limb 0 least significant).  A sum of
// k < 2^32 fingerprints is held as 8 x u64 per-limb sums (no carry propagation), which is
// associative and commutative like the group itself, and normalised once at the end.
struct Acc {
    uint64_t l[8];
};

__device__ __forceinline__ void acc_zero(Acc &a) {
#pragma unroll
    for (int i = 0; i < 8; i++) a.l[i] = 0;
}

__device__ __forceinline__ void acc_add_fp(Acc &a, const uint32_t f[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) a.l[i] += f[i];
}

__device__ __forceinline__ void acc_add(Acc &a, const Acc &b) {
#pragma unroll
    for (int i = 0; i < 8; i++) a.l[i] += b.l[i];
}

// carry-propagate to 8 x u32 = the fingerprint mod 2^256
__device__ __forceinline__ void acc_normalise(const Acc &a, uint32_t f[8]) {
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t t = a.l[i] + carry;  // a.l[i] < 2^63 by construction, carry < 2^32
        f[i] = (uint32_t)t;
        carry = t >> 32;
    }
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    lo = __shfl_xor(lo, m, 64);
    hi = __shfl_xor(hi, m, 64);
    return ((uint64_t)hi << 32) | lo;
}

// butterfly over the 64-lane wave: every lane ends with the wave total
__device__ __forceinline__ void acc_wave_reduce(Acc &a) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
#pragma unroll
        for (int i = 0; i < 8; i++) a.l[i] += shfl_xor_u64(a.l[i], m);
    }
}

// Block-wide reduction of per-thread carry-save sums.  `lds` must hold (blockDim/64)*8 u64.
// Returns the normalised total in f[] on thread 0 (other threads: unspecified).
template <int NT>
__device__ __forceinline__ void acc_block_reduce(Acc &a, uint64_t *lds, uint32_t f[8]) {
    constexpr int NW = NT / 64;
    acc_wave_reduce(a);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (NW > 1) {
        if (lane < 8) {
            uint64_t mine = 0;
#pragma unroll
            for (int i = 0; i < 8; i++) mine = (lane == i) ? a.l[i] : mine;
            lds[wave * 8 + lane] = mine;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                uint64_t s = 0;
#pragma unroll
                for (int w = 0; w < NW; w++) s += lds[w * 8 + i];
                a.l[i] = s;
            }
        }
    }
    if (threadIdx.x == 0) acc_normalise(a, f);
}

// Sum of one fingerprint per thread over a 256-thread block, via an LDS transpose:
// every thread stores its 8 limbs limb-major, then thread t sums 8 consecutive values of
// limb (t >> 5) into a u64, and 32 lanes finish that limb with 5 shuffle steps.  About 45
// instructions per wave, against ~250 for a per-limb 64-lane butterfly.
// `tile` must hold 8*256 u32 + 8 u64 (the limb totals).  Result on thread 0.
struct SumTile {
    uint32_t limb[8][256];
    uint64_t total[8];
};

__device__ __forceinline__ void block_sum_fps256(const uint32_t h[8], SumTile &t, uint32_t f[8]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < 8; j++) t.limb[j][tid] = h[j];
    __syncthreads();
    const int l = tid >> 5, s = tid & 31;
    const uint4 a = *reinterpret_cast<const uint4 *>(&t.limb[l][s * 8]);
    const uint4 b = *reinterpret_cast<const uint4 *>(&t.limb[l][s * 8 + 4]);
    uint64_t p = (uint64_t)a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
    // butterfly over the 32 lanes of this half-wave: ds_swizzle in bit mode
    // (and_mask 0x1f, xor_mask m) needs no per-lane address arithmetic
#define RH_SWZ(m)                                                                               \
    {                                                                                           \
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)p, ((m) << 10) | 0x1f);        \
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_swizzle((int)(uint32_t)(p >> 32), ((m) << 10) | 0x1f); \
        p += ((uint64_t)hi << 32) | lo;                                                         \
    }
    RH_SWZ(16) RH_SWZ(8) RH_SWZ(4) RH_SWZ(2) RH_SWZ(1)
#undef RH_SWZ
    if (s == 0) t.total[l] = p;
    __syncthreads();
    if (tid == 0) {
        Acc acc;
#pragma unroll
        for (int j = 0; j < 8; j++) acc.l[j] = t.total[j];
        acc_normalise(acc, f);
    }
}

}  // namespace rh
