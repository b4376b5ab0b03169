// search_device.hpp -- the store's key order and the sampled lower-bound search, as device
// functions: used by the search kernels (store_kernels.hip) and by the batch path's fused
// lift + search launch (lift_kernels.hpp, k_lift_search), where the VALU-bound lift and the
// latency-bound searches share the CUs.
#pragma once
#include "store_kernels.hpp"

namespace rh {

template <int KK, int KL>
__device__ __forceinline__ int key_cmp(const uint8_t *a, const uint8_t *b) {
    if constexpr (KK == KEY_U32) {
        uint32_t x = *reinterpret_cast<const uint32_t *>(a), y = *reinterpret_cast<const uint32_t *>(b);
        return (x > y) - (x < y);
    } else if constexpr (KK == KEY_U64) {
        uint64_t x = *reinterpret_cast<const uint64_t *>(a), y = *reinterpret_cast<const uint64_t *>(b);
        return (x > y) - (x < y);
    } else {
        static_assert(KL % 8 == 0, "byte keys: multiple of 8 bytes");
        // memcmp order ([u8; L] Ord) = big-endian u64 chunks
#pragma unroll
        for (int o = 0; o < KL; o += 8) {
            uint64_t x = __builtin_bswap64(*reinterpret_cast<const uint64_t *>(a + o));
            uint64_t y = __builtin_bswap64(*reinterpret_cast<const uint64_t *>(b + o));
            if (x != y) return x < y ? -1 : 1;
        }
        return 0;
    }
}

// radix digit d (0 = most significant) of a key, as an unsigned u64 in key order
template <int KK, int KL>
__device__ __forceinline__ uint64_t key_digit(const uint8_t *k, int d) {
    if constexpr (KK == KEY_U32) return *reinterpret_cast<const uint32_t *>(k);
    else if constexpr (KK == KEY_U64) return *reinterpret_cast<const uint64_t *>(k);
    else return __builtin_bswap64(*reinterpret_cast<const uint64_t *>(k + 8 * d));
}

__device__ __forceinline__ uint64_t lower_bound_u64(const uint64_t *a, uint64_t lo, uint64_t hi, uint64_t x) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// narrow [lo, hi) (a window of the key array that holds the lower bound of a key with leading
// digit d) with samples smp[s] = digit of key s * stride, s in [0, ns)
__device__ __forceinline__ void sample_window(const uint64_t *smp, uint64_t ns, uint64_t stride, uint64_t d,
                                              uint64_t &lo, uint64_t &hi) {
    const uint64_t s_lo = lo / stride, s_hi = (hi + stride - 1) / stride < ns ? (hi + stride - 1) / stride : ns;
    const uint64_t a = lower_bound_u64(smp, s_lo, s_hi, d);  // samples < d: those keys are < key
    if (a > s_lo) lo = (a - 1) * stride > lo ? (a - 1) * stride : lo;
    if (a < s_hi) {
        if (smp[a] > d) hi = a * stride < hi ? a * stride : hi;  // that sample's key is > key
        else {  // samples equal to d: up to the first one above
            const uint64_t b = lower_bound_u64(smp, a, s_hi, d + 1);
            if (b < s_hi && d != ~0ull && b * stride < hi) hi = b * stride;
        }
    }
}

// the sampled search of one key (see k_search_sampled): its lower-bound rank in keys[0, n)
// and whether it is present
template <int KK, int KL>
__device__ __forceinline__ void search_sampled_one(const uint8_t *keys, uint64_t n, const uint64_t *smp,
                                                   const uint64_t *smp2, SearchTable tb, const uint8_t *key,
                                                   uint32_t *rank, uint8_t *present) {
    const uint64_t d = key_digit<KK, KL>(key, 0);
    uint64_t lo = 0, hi = n;
    if (tb.tab) {
        // samples in buckets below d's are < d, those from the next bucket on are > d: the lower
        // bound among the samples lies in [tab[h], tab[h + 1]], the key's in the rows around them
        const uint64_t dmin = tb.par[0], sh = tb.par[1], nt = 1ull << tb.bits;
        uint64_t h = d < dmin ? 0 : (d - dmin) >> sh;
        h = h < nt ? h : nt - 1;
        const uint64_t a0 = tb.tab[h], a1 = tb.tab[h + 1];
        lo = a0 ? (a0 - 1) * SMP2_STRIDE : 0;
        hi = a1 * SMP2_STRIDE < n ? a1 * SMP2_STRIDE : n;
        lo = lo < hi ? lo : hi;
    } else {
        sample_window(smp, (n + SMP_STRIDE - 1) / SMP_STRIDE, SMP_STRIDE, d, lo, hi);
    }
    // the samples narrow a window wider than two sample strides (a fine table's window is one
    // or two strides already: the keys are searched directly, one sample line saved)
    if (smp2 && hi - lo > 2 * SMP2_STRIDE) sample_window(smp2, (n + SMP2_STRIDE - 1) / SMP2_STRIDE, SMP2_STRIDE, d, lo, hi);
    // the window's end is n or a sampled row whose digit is above d (from the table or the
    // samples): a lower bound there is not the key, and its line is not fetched to say so; any
    // other lower bound was compared by the search, so its line is in the cache
    const uint64_t end = hi;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (key_cmp<KK, KL>(keys + mid * KL, key) < 0) lo = mid + 1;
        else hi = mid;
    }
    *rank = (uint32_t)lo;
    if (present) *present = (lo < end && key_cmp<KK, KL>(keys + lo * KL, key) == 0) ? 1 : 0;
}

// ---- the same searches by a group of W lanes (W = 16 or 64), for latency-bound questions -------
// A group's W lanes probe W evenly spaced rows of the window at once, so a window of w rows takes
// ceil(log_W w) dependent loads instead of log2 w (a tiny round's or a single rank's critical path).
// The bits of a wave-wide ballot that belong to the calling group (its W lanes, aligned)
template <int W>
__device__ __forceinline__ uint64_t group_ballot(bool p) {
    const uint64_t b = __ballot(p);
    if constexpr (W == 64) return b;
    else return (b >> (threadIdx.x & 63 & ~(W - 1))) & ((1ull << W) - 1);
}

// lower bound of q in keys[lo, n) given that it lies in [lo, hi] and (hi == n or keys[hi] >= q);
// *present: keys[rank] == q.  Every lane of the group returns the same; gl = the lane's index in it.
template <int KK, int KL, int W>
__device__ __forceinline__ uint64_t lower_bound_group(const uint8_t *keys, uint64_t n, uint64_t lo, uint64_t hi,
                                                      const uint8_t *q, uint32_t gl, bool *present) {
    while (hi - lo + 1 > W) {
        const uint64_t step = (hi - lo + W - 1) / W;
        const uint64_t p = lo + gl * step;
        const bool less = p < hi && key_cmp<KK, KL>(keys + p * KL, q) < 0;
        const uint32_t c = __popcll(group_ballot<W>(less));  // the probes below q: a prefix
        if (c == 0) {
            hi = lo;
            break;
        }
        const uint64_t pc = lo + (c - 1) * step;
        lo = pc + 1;
        hi = pc + step < hi ? pc + step : hi;
    }
    const uint64_t p = lo + gl;
    const bool valid = p <= hi && p < n;
    const int c = valid ? key_cmp<KK, KL>(keys + p * KL, q) : 1;
    const uint64_t lt = group_ballot<W>(valid && c < 0), eq = group_ballot<W>(valid && c == 0);
    const uint32_t r = __popcll(lt);
    *present = (eq >> r) & 1;
    return lo + r;
}

// search_sampled_one by a group: the table's window (base runs), else the whole run
template <int KK, int KL, int W>
__device__ __forceinline__ void search_group(const uint8_t *keys, uint64_t n, SearchTable tb, const uint8_t *key,
                                             uint32_t gl, uint32_t *rank, uint8_t *present) {
    uint64_t lo = 0, hi = n;
    if (tb.tab && n) {
        const uint64_t d = key_digit<KK, KL>(key, 0);
        const uint64_t dmin = tb.par[0], sh = tb.par[1], nt = 1ull << tb.bits;
        uint64_t h = d < dmin ? 0 : (d - dmin) >> sh;
        h = h < nt ? h : nt - 1;
        const uint64_t a0 = tb.tab[h], a1 = tb.tab[h + 1];
        lo = a0 ? (a0 - 1) * SMP2_STRIDE : 0;
        hi = a1 * SMP2_STRIDE < n ? a1 * SMP2_STRIDE : n;  // n, or a sampled row whose digit is above d
        lo = lo < hi ? lo : hi;
    }
    bool pr = false;
    const uint64_t r = n ? lower_bound_group<KK, KL, W>(keys, n, lo, hi, key, gl, &pr) : 0;
    *rank = (uint32_t)r;
    if (present) *present = pr ? 1 : 0;
}

}  // namespace rh
