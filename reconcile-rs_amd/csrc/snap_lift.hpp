// snap_lift.hpp -- the fused snapshot reload pass: locate, lift and load 256 entries per
// workgroup straight from the file bytes (included by every per-shape lift translation unit).
//
// Replaces, for a reload into stores, the column decode (k_snap_decode: 1.01 GB of SoA columns
// written for 10 M entries), the lift reading them back, the stores' key copies and their
// sortedness checks.  Reference path: Replica::load_snapshot replays the snapshot's entries with
// map_insert (src/snapshot.rs:76-98, src/replica/write.rs:44-45): per entry, the dated lift
// lift(k, Entry<Timestamp, V>) and the projection lift lift(k, State<V>) (fingerprint.rs:270-275).
//
// Workgroup b owns entries [256 b, 256 b + 256) -- exactly the lift's block, so the block sums
// come out as the store keeps them.  snapshot_locate has placed every segment's first entry
// (start, basev) and the segments holding each block's boundary entries (segq).  The workgroup
// stages those segments in LDS (16-byte coalesced loads), one lane per segment re-walks its
// entries from the true start listing their LDS offsets (entry 256 b - 1 included, for the
// order check), then every lane hashes its own entry reading key, stamp, variant and value
// from LDS.  HBM traffic per entry: its file bytes once, 32 B per fingerprint written and the
// key written once per store (with the stores' search samples: 1 u64 per 8 keys).
#pragma once
#include "lift_kernels.hpp"
#include "snap_device.hpp"

namespace rh {

template <int KK, int KL, int VK, int VL, int MODE>  // MODE 0 dated, 1 projection, 2 both
__global__ __launch_bounds__(256) void k_snap_lift(SnapLift a) {
    using LD = LayoutAligned<Layout<KK, KL, VK, VL, REC_DATED>, 4>;
    using LP = LayoutAligned<Layout<KK, KL, VK, VL, REC_PROJECTION>, 4>;
    constexpr int KR = LD::KEY_ROW / 4;  // key words in the file
    extern __shared__ uint32_t img[];
    __shared__ uint32_t list[257];  // LDS byte offsets of entries q0 ..
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
    snap::stage(a.blob, f.len, base, end, img);
    list[t] = 0;
    if (t == 0) {
        list[256] = 0;
        listed = 0;
    }
    __syncthreads();
    const uint32_t ns = (uint32_t)(s_hi - s_lo + 1);
    if (t < ns) {  // one lane per segment lists the block's entries that start in it
        const snap::Img m{img, base};
        const uint64_t s = s_lo + t;
        const uint32_t x = a.start[s];
        uint64_t i = a.basev[s];
        uint32_t mine = 0;
        if (x != snap::BAD) {
            const uint64_t send = snap::seg_start(f, s + 1);
            const uint32_t o_var = f.key_pre + f.key_len + 20;
            uint64_t p = snap::seg_start(f, s) + (uint64_t)x * f.g;
            while (p < send && i < e1) {
                const uint32_t L = m.ld32(p + o_var) == 1 ? f.lt : f.lp;
                if (i >= q0) {
                    list[i - q0] = (uint32_t)(p - base);
                    mine++;
                }
                if (i == a.n - 1) a.words[0] = p + L;
                p += L;
                i++;
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
    const uint32_t kp = f.key_pre >> 2;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t h2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t tomb_c = 0;
    if (e0 + t < e1) {
        const uint32_t *w = img + (list[li0 + t] >> 2) + kp;  // the key's first word
        uint32_t kw[LD::KEY_ENC / 4 > 0 ? LD::KEY_ENC / 4 : 1];
        constexpr int K0 = KK == KEY_BYTES ? 2 : 0;
        if constexpr (KK == KEY_BYTES) {
            kw[0] = (uint32_t)KL;
            kw[1] = 0;
        }
#pragma unroll
        for (int j = 0; j < KR; j++) kw[K0 + j] = w[j];
        uint32_t sw[5];
#pragma unroll
        for (int j = 0; j < 5; j++) sw[j] = w[KR + j];
        const bool tomb = w[KR + 5] == 1;
        const uint8_t *vrow = reinterpret_cast<const uint8_t *>(w + KR + 6 + LD::VAL_PREFIX / 4);
        if constexpr (MODE == 1) {
            lift_record_l<LP, KK, REC_PROJECTION, true>(kw, sw, tomb, vrow, h);
        } else {
            lift_record_l<LD, KK, REC_DATED, true>(kw, sw, tomb, vrow, h);
            if constexpr (MODE == 2) lift_record_l<LP, KK, REC_PROJECTION, true>(kw, sw, tomb, vrow, h2);
        }
        store_fp(a.fps + e0 * 32, t, h);
        if constexpr (MODE == 2) store_fp(a.fps2 + e0 * 32, t, h2);
        tomb_c = tomb;
        // the stores' search samples (k_sample's): the leading u64 digit in key order
        if (t % SMP2_STRIDE == 0) {
            uint64_t d = 0;
            if constexpr (KK == KEY_BYTES) d = ((uint64_t)__builtin_bswap32(w[0]) << 32) | __builtin_bswap32(w[1]);
            else if constexpr (KK == KEY_U64) d = ((uint64_t)w[1] << 32) | w[0];
            else if constexpr (KK == KEY_U32) d = w[0];
            const uint64_t e = e0 + t;
            a.smp2[e / SMP2_STRIDE] = d;
            if (a.smp2_2) a.smp2_2[e / SMP2_STRIDE] = d;
            if (t == 0) {
                a.smp[b] = d;
                if (a.smp_2) a.smp_2[b] = d;
            }
        }
        // strictly increasing keys (k_check_sorted's rule): compare with entry e - 1, in the
        // key's Ord -- bytes: memcmp (big-endian words); u32 / u64: numeric
        if (e0 + t > 0) {
            const uint32_t *pw = img + (list[li0 + t - 1] >> 2) + kp;
            int c = 0;  // sign of (previous - mine)
            if constexpr (KK == KEY_BYTES) {
#pragma unroll
                for (int j = 0; j < KR; j++) {
                    const uint32_t x = __builtin_bswap32(pw[j]), y = __builtin_bswap32(w[j]);
                    if (c == 0) c = (x > y) - (x < y);
                }
            } else if constexpr (KK == KEY_U64) {
                const uint64_t x = ((uint64_t)pw[1] << 32) | pw[0], y = ((uint64_t)w[1] << 32) | w[0];
                c = (x > y) - (x < y);
            } else if constexpr (KK == KEY_U32) {
                c = (pw[0] > w[0]) - (pw[0] < w[0]);
            }
            if (c >= 0) atomicOr(a.unsorted, 1u);
        }
    }
    // the block's keys into the store(s), coalesced
    if constexpr (KR > 0) {
        uint32_t *k1 = reinterpret_cast<uint32_t *>(a.keys) + e0 * KR;
        uint32_t *k2 = a.keys2 ? reinterpret_cast<uint32_t *>(a.keys2) + e0 * KR : nullptr;
        snap::for_dwords((uint32_t)(e1 - e0), KR, [&](uint32_t j, uint32_t e, uint32_t q) {
            const uint32_t v = img[(list[li0 + e] >> 2) + kp + q];
            k1[j] = v;
            if (k2) k2[j] = v;
        });
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) tomb_c += __shfl_xor(tomb_c, k, 64);
    if ((t & 63) == 0) wsum[t >> 6] = tomb_c;
    __syncthreads();  // every read of the staged bytes is done: the sum tile reuses them
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
        if (mode == 0) hipLaunchKernelGGL((k_snap_lift<KK, KL, VK, VL, 0>), grid, block, (size_t)lds, st, a);
        else if (mode == 1) hipLaunchKernelGGL((k_snap_lift<KK, KL, VK, VL, 1>), grid, block, (size_t)lds, st, a);
        else hipLaunchKernelGGL((k_snap_lift<KK, KL, VK, VL, 2>), grid, block, (size_t)lds, st, a);
        return hipGetLastError();
    }
}

}  // namespace rh
