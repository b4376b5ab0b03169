// snap_lift.hpp -- the fused snapshot reload pass: locate, lift and load 256 entries per
// workgroup straight from the file bytes (included by every per-shape lift translation unit).
//
// Replaces, for a reload into stores, the column decode (k_snap_decode: 1.01 GB of SoA columns
// written for 10 M entries), the lift reading them back, the stores' key copies, their
// sortedness checks and their search-sample passes.  Reference path: Replica::load_snapshot
// replays the snapshot's entries with map_insert (src/snapshot.rs:76-98,
// src/replica/write.rs:44-45): per entry, the dated lift lift(k, Entry<Timestamp, V>) and the
// projection lift lift(k, State<V>) (rsos/src/fingerprint.rs:270-275).
//
// Block b is entries [256 b, 256 b + 256) -- exactly the lift's block, so the block sums come
// out as the store keeps them.  snapshot_locate has placed every segment's first entry
// (start, basev) and the segments holding each block's boundary entries (segq).  The workgroup
// stages those segments' candidate State-variant words in LDS -- entries start on a g-byte grid,
// so only every (g / 4)-th word can be a variant: with g = 8, half the bytes -- and one lane per
// segment re-walks its entries from the true start, listing their file offsets (entry 256 b - 1
// included, for the order check).  Every lane then loads its own entry from the file (the lines
// were just staged through L2) and hashes it.  The small LDS footprint (~17 KiB for 16 B / 64 B
// entries) keeps 8 waves per SIMD on the hashing, like the column lift.  HBM traffic per entry:
// its file bytes once, 32 B per fingerprint written, the key written once per store and the
// stores' search samples (1 u64 per 8 keys).
#pragma once
#include "lift_kernels.hpp"
#include "snap_device.hpp"

namespace rh {

// N consecutive dwords to p, with p known to be ALIGN-byte aligned
template <int N, int ALIGN>
__device__ __forceinline__ void stw(uint8_t *p, const uint32_t *v) {
    int k = 0;
    if constexpr (ALIGN >= 16) {
#pragma unroll
        for (; k + 4 <= N; k += 4) *reinterpret_cast<uint4 *>(p + 4 * k) = make_uint4(v[k], v[k + 1], v[k + 2], v[k + 3]);
    }
    if constexpr (ALIGN >= 8) {
#pragma unroll
        for (; k + 2 <= N; k += 2) *reinterpret_cast<uint2 *>(p + 4 * k) = make_uint2(v[k], v[k + 1]);
    }
#pragma unroll
    for (; k < N; k++) *reinterpret_cast<uint32_t *>(p + 4 * k) = v[k];
}

// MODE 0 dated, 1 projection, 2 both.  R: candidate-word stride (entries start every g bytes,
// R = a power of two dividing g / 4, at most 2); entries are then 4R-byte aligned in the file.
template <int KK, int KL, int VK, int VL, int MODE, int R>
__global__ __launch_bounds__(256) void k_snap_lift(SnapLift a) {
    static_assert(R == 1 || R == 2, "candidate stride");
    constexpr int A = 4 * R;
    using LD = LayoutAligned<Layout<KK, KL, VK, VL, REC_DATED>, A>;
    using LP = LayoutAligned<Layout<KK, KL, VK, VL, REC_PROJECTION>, A>;
    constexpr int KR = LD::KEY_ROW / 4;  // key words in the file
    constexpr int KA = cmin(A, KR > 0 ? cmin(16, lowbit(4 * KR)) : 16);  // key row alignment
    extern __shared__ uint32_t img[];     // the candidate words; later the block-sum tile
    __shared__ uint32_t list[257];        // file offsets (from the range start) of entries q0 ..
    __shared__ uint32_t listed, wsum[4];
    const SnapFmt &f = a.f;
    const uint32_t t = threadIdx.x;
    const uint64_t b = blockIdx.x;
    const uint64_t e0 = b * 256, e1 = std::min<uint64_t>(e0 + 256, a.n);
    const uint64_t q0 = e0 ? e0 - 1 : 0;  // first listed entry
    // the segments to stage (clamped, so a corrupt file -- reported by the caller -- stays in bounds)
    const uint64_t s_lo = std::min<uint64_t>(a.segq[b], a.nseg - 1);
    const uint64_t s_hi = std::min<uint64_t>(std::max<uint64_t>(a.segq[b + 1], s_lo),
                                             std::min<uint64_t>(s_lo + a.nsmax - 1, a.nseg - 1));
    const uint64_t base = snap::seg_start(f, s_lo) & ~15ull;
    const uint64_t end = std::min<uint64_t>(snap::seg_start(f, s_hi + 1) + f.lp, f.len);
    const uint32_t o_var = f.key_pre + f.key_len + 20;
    // candidate words: file word w holds a variant only if w = (f.base + o_var) / 4 (mod R);
    // image word k <-> file word wb + k R.  With R = 2 they are words vb and vb + 2 of every
    // 16-byte chunk (vb = 0 or 1, the same for the whole range), so chunk c lands in image words
    // 2c and 2c + 1.  32-bit offsets from the range start.
    const uint64_t w0 = base >> 2;
    const uint64_t wb = w0 + ((((f.base + o_var) >> 2) - w0) & (R - 1));
    const uint32_t vb = (uint32_t)(wb - w0);
    {
        const uint32_t span = (uint32_t)(end - base);
        const uint32_t avail = (uint32_t)std::min<uint64_t>(f.len - base, 1u << 31);  // file bytes from base
        const uint8_t *src = a.blob + base;
        // every lane's loads in flight before its first LDS store (snap::stage's batching)
        for (uint32_t r0 = 16 * t; r0 < span; r0 += 16 * 256 * snap::STAGE_U) {
            uint4 v[snap::STAGE_U];
#pragma unroll
            for (int u = 0; u < snap::STAGE_U; u++) {
                const uint32_t rel = r0 + 4096 * u;
                if (rel < span)
                    v[u] = rel + 16 <= avail ? *reinterpret_cast<const uint4 *>(src + rel)
                                             : snap::load16(a.blob, f.len, base + rel);
            }
#pragma unroll
            for (int u = 0; u < snap::STAGE_U; u++) {
                const uint32_t rel = r0 + 4096 * u;
                if (rel >= span) continue;
                if constexpr (R == 1) {
                    *reinterpret_cast<uint4 *>(img + (rel >> 2)) = v[u];
                } else {
                    *reinterpret_cast<uint2 *>(img + (rel >> 3)) =
                        vb ? make_uint2(v[u].y, v[u].w) : make_uint2(v[u].x, v[u].z);
                }
            }
        }
    }
    list[t] = 0;
    if (t == 0) {
        list[256] = 0;
        listed = 0;
    }
    __syncthreads();
    const uint32_t ns = (uint32_t)(s_hi - s_lo + 1);
    if (t < ns) {  // one lane per segment lists the block's entries that start in it
        const uint64_t s = s_lo + t;
        const uint32_t x = a.start[s];
        uint64_t i = a.basev[s];
        uint32_t mine = 0;
        if (x != snap::BAD) {
            // 32-bit offsets from the range start
            const uint32_t send = (uint32_t)(snap::seg_start(f, s + 1) - base);
            uint32_t p = (uint32_t)(snap::seg_start(f, s) + (uint64_t)x * f.g - base);
            uint32_t k = (uint32_t)(i - q0);  // list index (wraps below q0: skipped)
            const uint32_t kend = (uint32_t)(e1 - q0);
            while (p < send && (int32_t)k < (int32_t)kend) {
                const uint32_t L = img[(((p + o_var) >> 2) - vb) / R] == 1 ? f.lt : f.lp;
                if ((int32_t)k >= 0) {
                    list[k] = p;
                    mine++;
                }
                if (q0 + k == a.n - 1) a.words[0] = base + p + L;
                p += L;
                k++;
            }
        }
        if (mine) atomicAdd(&listed, mine);
    }
    __syncthreads();
    if (listed != (uint32_t)(e1 - q0)) {  // only for a chain that did not parse (the call fails)
        if (t == 0) {
            atomicOr(a.words + 1, 1ull);
            a.tomb_part[b] = 0;
        }
        return;
    }
    const uint32_t li0 = e0 ? 1 : 0;  // list index of entry e0
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t h2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t tomb_c = 0;
    const bool valid = e0 + t < e1;
    uint32_t kw[LD::KEY_ENC / 4 > 0 ? LD::KEY_ENC / 4 : 1];
    constexpr int K0 = KK == KEY_BYTES ? 2 : 0;
    if constexpr (KK == KEY_BYTES) {
        kw[0] = (uint32_t)KL;
        kw[1] = 0;
    }
    if (valid) {
        // the entry from the file: key, stamp, variant, value (L2-resident since the staging)
        const uint8_t *ep = a.blob + base + list[li0 + t] + f.key_pre;
        if constexpr (KR > 0) ldw<KR, KA>(ep, kw + K0);
        uint32_t sv[6];  // stamp words, variant
        ldw<6, cmin(A, 8)>(ep + 4 * KR, sv);
        const bool tomb = sv[5] == 1;
        const uint8_t *vrow = ep + 4 * KR + 24 + LD::VAL_PREFIX;
        if constexpr (MODE == 1) {
            lift_record_l<LP, KK, REC_PROJECTION, true>(kw, sv, tomb, vrow, h);
        } else {
            lift_record_l<LD, KK, REC_DATED, true>(kw, sv, tomb, vrow, h);
            if constexpr (MODE == 2) lift_record_l<LP, KK, REC_PROJECTION, true>(kw, sv, tomb, vrow, h2);
        }
        store_fp(a.fps + e0 * 32, t, h);
        if constexpr (MODE == 2) store_fp(a.fps2 + e0 * 32, t, h2);
        tomb_c = tomb;
        if constexpr (KR > 0) {  // the block's keys into the store(s)
            stw<KR, KA>(a.keys + (e0 + t) * (4 * KR), kw + K0);
            if (a.keys2) stw<KR, KA>(a.keys2 + (e0 + t) * (4 * KR), kw + K0);
        }
    }
    // the key's leading u64 digit in key order (k_sample's search samples, the order check)
    uint64_t d = 0;
    if constexpr (KK == KEY_BYTES) d = ((uint64_t)__builtin_bswap32(kw[2]) << 32) | __builtin_bswap32(kw[3]);
    else if constexpr (KK == KEY_U64) d = ((uint64_t)kw[1] << 32) | kw[0];
    else if constexpr (KK == KEY_U32) d = kw[0];
    if (valid && t % SMP2_STRIDE == 0) {
        const uint64_t e = e0 + t;
        a.smp2[e / SMP2_STRIDE] = d;
        if (a.smp2_2) a.smp2_2[e / SMP2_STRIDE] = d;
        if (t == 0) {
            a.smp[b] = d;
            if (a.smp_2) a.smp_2[b] = d;
        }
    }
    // strictly increasing keys (k_check_sorted's rule) in the key's Ord -- bytes: memcmp
    // (big-endian words); u32 / u64: numeric.  The previous entry's key from the lane below,
    // or for a wave's first lane, from the file
    {
        uint32_t pk[KR > 0 ? KR : 1];
#pragma unroll
        for (int j = 0; j < KR; j++) pk[j] = __shfl_up(kw[K0 + j], 1, 64);
        if ((t & 63) == 0 && valid && e0 + t > 0) {
            if constexpr (KR > 0) ldw<KR, KA>(a.blob + base + list[li0 + t - 1] + f.key_pre, pk);
        }
        if (valid && e0 + t > 0) {
            int c = 0;  // sign of (previous - mine)
            if constexpr (KK == KEY_BYTES) {
#pragma unroll
                for (int j = 0; j < KR; j++) {
                    const uint32_t x = __builtin_bswap32(pk[j]), y = __builtin_bswap32(kw[K0 + j]);
                    if (c == 0) c = (x > y) - (x < y);
                }
            } else if constexpr (KK == KEY_U64) {
                const uint64_t x = ((uint64_t)pk[1] << 32) | pk[0];
                c = (x > d) - (x < d);
            } else if constexpr (KK == KEY_U32) {
                c = (pk[0] > kw[0]) - (pk[0] < kw[0]);
            }
            if (c >= 0) atomicOr(a.unsorted, 1u);
        }
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) tomb_c += __shfl_xor(tomb_c, k, 64);
    if ((t & 63) == 0) wsum[t >> 6] = tomb_c;
    __syncthreads();  // every read of the candidate words is done: the sum tile reuses them
    if (t == 0) a.tomb_part[b] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    SumTile &tile = *reinterpret_cast<SumTile *>(img);
    uint32_t fs[8];
    block_sum_fps256(h, tile, fs);  // lanes past e1 hold zero
    if (t == 0) store_sum(a.bsums, b, fs);
    if constexpr (MODE == 2) {
        block_sum_fps256(h2, tile, fs);
        if (t == 0) store_sum(a.bsums2, b, fs);
    }
}

// the fused pass for shape (KK, KL, VK, VL): whole-message layouts only (a dated record up to
// 192 B); *supported = false otherwise (the caller decodes columns and lifts them instead)
template <int KK, int KL, int VK, int VL>
hipError_t launch_snap_lift_t(int mode, const SnapLift &a, uint64_t lds, hipStream_t st, bool *supported) {
    using LD = Layout<KK, KL, VK, VL, REC_DATED>;
    if constexpr (!(LD::SMALL && LD::LEN <= 192)) {
        *supported = false;
        return hipSuccess;
    } else {
        *supported = true;
        if (a.n == 0) return hipSuccess;
        if (lds < sizeof(SumTile) || (uint64_t)(a.f.key_len) != (uint64_t)LD::KEY_ROW ||
            a.f.val_len != (uint32_t)LD::VAL_ROW || a.f.val_pre != (uint32_t)LD::VAL_PREFIX)
            return hipErrorInvalidValue;
        const dim3 grid((uint32_t)((a.n + 255) / 256)), block(256);
        const int R = snap_lift_stride(a.f);
#define RH_SL(M, RR) hipLaunchKernelGGL((k_snap_lift<KK, KL, VK, VL, M, RR>), grid, block, (size_t)lds, st, a)
        if (R == 2) {
            if (mode == 0) RH_SL(0, 2);
            else if (mode == 1) RH_SL(1, 2);
            else RH_SL(2, 2);
        } else {
            if (mode == 0) RH_SL(0, 1);
            else if (mode == 1) RH_SL(1, 1);
            else RH_SL(2, 1);
        }
#undef RH_SL
        return hipGetLastError();
    }
}

}  // namespace rh
