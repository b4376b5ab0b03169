// store_kernels.hip -- device side of the GPU-resident RSOS store: key order, rank search,
// batch sort, the sorted-run merge, and the signed-delta run of the LSM layout.
//
// Store layout in HBM (rank order):
//   base  : keys[nB][KL] + fps[nB][32] + block sums [nB/256][32] + super sums [nB/65536][32]
//   delta : keys[nD][KL] + DeltaRec[nD] (48 B) + block / super sums of the contributions +
//           the count-delta prefix (inclusive per 256-row block + int16 inside each block)
// A DeltaRec for key k says what the batches since the last compaction did to k:
//   contrib = cur_fp - base_fp   (cur_fp = 0 if k is now deleted; base_fp = 0 if k not in base)
//   in_base, live                 (so the count delta is live - in_base, in {-1, 0, +1})
//   brank                         (k's lower-bound rank in the base run)
// so every aggregate over a key range is   base part + Σ contrib over the delta part,
// exactly as FingerprintTreeMap composes signed deltas into its cached aggregates
// (rsos/src/fingerprint_tree_map/mutate.rs:31-41 overwrite delta, :93-154 remove).
// Record payloads are not kept on the device (the host owns K and V, rsos_trait.rs:66-80).
//
// Batched update = FingerprintTreeMap::insert / remove applied to a whole batch at once
// (mutate.rs:23-154): sort the batch by key, find every key in base and delta, build the
// batch's DeltaRecs, merge them into the delta run (O(m + nD), one pass that also writes the
// run's sums); when the delta run passes nB / 8 it is merged into the base the same way
// (O(nB)) -- amortised, and on demand before rank / select.
#include <atomic>
#include <cstdlib>
#include <type_traits>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "internal.hpp"
#include "store_kernels.hpp"
#include "search_device.hpp"
#include "fp_device.hpp"
#include "round_tiny.hpp"

namespace rh {

namespace {
inline dim3 g1(uint64_t m) { return dim3((uint32_t)((m + 255) / 256)); }
}

// ---- key order ----------------------------------------------------------------------------

// copy N bytes (N a multiple of 4) with the widest aligned accesses
template <int N>
__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src) {
    if constexpr (N % 16 == 0) {
#pragma unroll
        for (int o = 0; o < N; o += 16) *reinterpret_cast<uint4 *>(dst + o) = *reinterpret_cast<const uint4 *>(src + o);
    } else if constexpr (N % 8 == 0) {
#pragma unroll
        for (int o = 0; o < N; o += 8) *reinterpret_cast<uint2 *>(dst + o) = *reinterpret_cast<const uint2 *>(src + o);
    } else {
#pragma unroll
        for (int o = 0; o < N; o += 4) *reinterpret_cast<uint32_t *>(dst + o) = *reinterpret_cast<const uint32_t *>(src + o);
    }
}

template <int KK, int KL>
__device__ __forceinline__ uint64_t lower_bound_keys(const uint8_t *keys, uint64_t n, const uint8_t *key) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (key_cmp<KK, KL>(keys + mid * KL, key) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint64_t lower_bound_u32(const uint32_t *a, uint64_t lo, uint64_t hi, uint64_t x) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// ---- batch sort ------------------------------------------------------------------------------

template <int KK, int KL>
__global__ void k_digit(const uint8_t *keys, const uint32_t *perm, uint64_t m, int d, uint64_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) out[j] = key_digit<KK, KL>(keys + (uint64_t)perm[j] * KL, d);
}

__global__ void k_iota(uint32_t *p, uint64_t m) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) p[j] = (uint32_t)j;
}

// gather the batch into key order; flags |= 1 on adjacent duplicates, and (msd_only) |= 2 when
// adjacent keys share their most significant digit (order not final)
template <int KK, int KL>
__global__ void k_gather(const uint8_t *keys, const uint8_t *fps, const uint8_t *ops, const uint32_t *perm,
                         uint64_t m, uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *pos, uint32_t *flags,
                         int msd_only) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t s = perm[j];
    copy_bytes<KL>(skeys + j * KL, keys + s * KL);
    if (fps) copy_bytes<32>(sfps + 32 * j, fps + 32 * s);
    else pos[s] = (uint32_t)j;
    sops[j] = ops ? ops[s] : 0;
    if (j > 0) {
        const uint8_t *prev = keys + (uint64_t)perm[j - 1] * KL;
        if (key_cmp<KK, KL>(keys + s * KL, prev) == 0) atomicOr(flags, 1u);
        else if (msd_only && key_digit<KK, KL>(keys + s * KL, 0) == key_digit<KK, KL>(prev, 0)) atomicOr(flags, 2u);
    }
}

// ---- batch sort: coarse MSD buckets + a per-bucket sort in LDS ---------------------------------
// For the update batches (m <= CS_MAX_M).  The most significant u64 digit d of each key maps to
// a bucket index B = (d - min) >> shift of CB + 8 bits (shift chosen from the batch's digit
// range, so random and dense key ranges both spread): the high CB bits pick one of C = 2^CB
// coarse buckets (~1,000 keys each), the low 8 bits a fine bucket inside it.
//   k_cs_minmax      per-workgroup digit min / max (every later kernel folds the partials); in
//                    apply_device_many the previous batch's k_lift_search computes them instead
//   k_cs_hist        per-workgroup coarse histograms
//   k_cs_colscan     each workgroup's offset inside each coarse bucket and the bucket totals;
//                    its last workgroup scans the totals into the buckets' starts (and (min,
//                    shift) once); *flags |= 4 if a bucket is larger than CS_CAP
//   k_cs_scatter     (whole key, row) pairs into coarse-bucket order
//   k_cs_sort        one workgroup per coarse bucket: fine buckets in LDS, each key ranked inside
//                    its fine bucket by (digit, whole key, row) -- so the result is the stable
//                    sort by key -- then the keys and ops written in order from the bucket's
//                    stretch, and either each row's sorted position (the batch path: the lift
//                    runs after the sort and writes each fingerprint in place) or the
//                    fingerprints gathered into place (a load)
// The per-key passes use 8,192-key workgroups of 1,024 lanes (8 keys per lane, loads issued
// together); an earlier form with 16 K buckets (a 16 MB histogram matrix) and one wave per
// ~61-key bucket gathering 16- and 32-byte rows from random input rows took 139 us per 1 M
// batch, the round-2 form (digits scattered, keys and fingerprints gathered) ~93, this one ~65.
constexpr int CS_TILE = 8192, CS_WG = 1024;         // keys / lanes per minmax / hist / scatter workgroup
constexpr int CS_FINE_BITS = 8, CS_FINE = 1 << CS_FINE_BITS;
constexpr int CS_CAP = 2048;                        // largest coarse bucket ordered in LDS
constexpr uint32_t CS_MAX_C = 4096;                 // coarse buckets at most
constexpr uint64_t CS_MAX_M = SORT_BUCKET_MAX;

// block-wide min / max (every lane gets the result); lo / hi: one slot per wave
__device__ __forceinline__ void minmax_block(uint64_t &a, uint64_t &b, uint64_t *lo, uint64_t *hi) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t a2 = __shfl_xor(a, o, 64), b2 = __shfl_xor(b, o, 64);
        a = a2 < a ? a2 : a;
        b = b2 > b ? b2 : b;
    }
    if ((threadIdx.x & 63) == 0) {
        lo[threadIdx.x >> 6] = a;
        hi[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    for (uint32_t w = 0; w < blockDim.x / 64; w++) {
        a = lo[w] < a ? lo[w] : a;
        b = hi[w] > b ? hi[w] : b;
    }
    __syncthreads();  // lo / hi may be reused
}

template <int KK, int KL>
__global__ __launch_bounds__(CS_WG) void k_cs_minmax(const uint8_t *keys, uint64_t m, uint64_t *part) {
    __shared__ uint64_t lo[CS_WG / 64], hi[CS_WG / 64];
    uint64_t a = ~0ull, b = 0;
    const uint64_t i0 = (uint64_t)blockIdx.x * CS_TILE;
#pragma unroll
    for (int k = 0; k < CS_TILE / CS_WG; k++) {
        const uint64_t i = i0 + CS_WG * k + threadIdx.x;
        if (i < m) {
            const uint64_t d = key_digit<KK, KL>(keys + i * KL, 0);
            a = d < a ? d : a;
            b = d > b ? d : b;
        }
    }
    minmax_block(a, b, lo, hi);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
}

// (min digit, shift) from the nwg per-workgroup partials, so that (d - min) >> shift < 2^bbits;
// every workgroup of the next kernels folds the (~m / 8192) partials itself
__device__ __forceinline__ void cs_params(const uint64_t *part, uint32_t nwg, uint32_t bbits, uint64_t *mn,
                                          uint32_t *shift) {
    __shared__ uint64_t lo[16], hi[16];
    uint64_t a = ~0ull, b = 0;
    for (uint32_t w = threadIdx.x; w < nwg; w += blockDim.x) {
        a = part[2 * w] < a ? part[2 * w] : a;
        b = part[2 * w + 1] > b ? part[2 * w + 1] : b;
    }
    minmax_block(a, b, lo, hi);
    const uint64_t range = b - a;
    const uint32_t bits = range ? 64u - (uint32_t)__clzll(range) : 0u;
    *mn = a;
    *shift = bits > bbits ? bits - bbits : 0u;
}

template <int KK, int KL>
__global__ __launch_bounds__(CS_WG) void k_cs_hist(const uint8_t *keys, uint64_t m, const uint64_t *part, uint32_t npart,
                                                   uint32_t bbits, uint32_t C, uint32_t *hist, uint32_t *flags,
                                                   uint32_t *ticket) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // no memsets of the sort's own: the flags and the scan's ticket
        *flags = 0;
        *ticket = 0;
    }
    __shared__ uint32_t h[CS_MAX_C];
    uint64_t mn;
    uint32_t sh;
    cs_params(part, npart, bbits, &mn, &sh);
    for (uint32_t b = threadIdx.x; b < C; b += CS_WG) h[b] = 0;
    __syncthreads();
    const uint64_t i0 = (uint64_t)blockIdx.x * CS_TILE;
    uint64_t d[CS_TILE / CS_WG];
#pragma unroll
    for (int k = 0; k < CS_TILE / CS_WG; k++) {
        const uint64_t i = i0 + CS_WG * k + threadIdx.x;
        d[k] = i < m ? key_digit<KK, KL>(keys + i * KL, 0) : 0;
    }
#pragma unroll
    for (int k = 0; k < CS_TILE / CS_WG; k++)
        if (i0 + CS_WG * k + threadIdx.x < m) atomicAdd(&h[(uint32_t)((d[k] - mn) >> sh) >> CS_FINE_BITS], 1u);
    __syncthreads();
    uint32_t *o = hist + (uint64_t)blockIdx.x * C;
    for (uint32_t b = threadIdx.x; b < C; b += CS_WG) o[b] = h[b];
}

// per coarse bucket: each workgroup's running offset within the bucket (in place), and the
// total.  64 buckets per workgroup (one per lane of a wave, so the row reads are coalesced),
// 16 lanes per bucket: lane q sums a sixteenth of the rows, the parts' sums are exchanged in LDS,
// then each lane writes its part's offsets.  The last workgroup to finish (an agent-scope ticket
// after agent-scope stores of the totals; MI355X_MICROARCH.md, inter-workgroup visibility) then
// scans the C totals into the buckets' starts (C <= 4 * 1024) and folds the minmax partials once
// into params = (min, shift) for the scatter and the bucket sorts: one launch where the column
// scan and the bucket scan were two.  *ticket: 0 on entry (k_cs_minmax zeroes it).
__global__ __launch_bounds__(1024) void k_cs_colscan(uint32_t *hist, uint32_t nwg, uint32_t C, uint32_t *total,
                                                     uint32_t *ticket, uint32_t *start, uint32_t *flags,
                                                     const uint64_t *part_mm, uint32_t npart, uint32_t bbits,
                                                     uint64_t *params) {
    constexpr uint32_t Q = 16;
    __shared__ uint32_t part[Q][64];
    __shared__ uint32_t last;
    const uint32_t lb = threadIdx.x & 63, qt = threadIdx.x >> 6, b = blockIdx.x * 64 + lb;
    const bool live = b < C;
    const uint32_t per = (nwg + Q - 1) / Q, w0 = qt * per < nwg ? qt * per : nwg, w1 = w0 + per < nwg ? w0 + per : nwg;
    uint32_t sum = 0;
    if (live)
        for (uint32_t w = w0; w < w1; w++) sum += hist[(uint64_t)w * C + b];
    part[qt][lb] = sum;
    __syncthreads();
    uint32_t run = 0;
    for (uint32_t q = 0; q < qt; q++) run += part[q][lb];
    if (live) {
        if (qt == Q - 1) __hip_atomic_store(total + b, run + sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t w = w0; w < w1; w++) {
            const uint32_t v = hist[(uint64_t)w * C + b];
            hist[(uint64_t)w * C + b] = run;
            run += v;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1 ? 1u
                                                                                                              : 0u;
    __syncthreads();
    if (!last) return;  // uniform
    // the bucket scan (exclusive, over the C totals)
    __shared__ uint32_t ws[16];
    const uint32_t t = threadIdx.x, pc = (C + 1023) / 1024;
    uint64_t mn;
    uint32_t sh;
    cs_params(part_mm, npart, bbits, &mn, &sh);
    if (t == 0) {
        params[0] = mn;
        params[1] = sh;
        *ticket = 0u;
    }
    uint32_t v[4] = {0, 0, 0, 0}, s = 0;
    bool big = false;
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        if (k < pc && pc * t + k < C) {
            v[k] = __hip_atomic_load(total + pc * t + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            big |= v[k] > (uint32_t)CS_CAP;
            s += v[k];
        }
    }
    uint32_t x = s;  // inclusive wave scan of the lane sums
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((t & 63) >= (uint32_t)o) x += y;
    }
    if ((t & 63) == 63) ws[t >> 6] = x;
    __syncthreads();
    uint32_t r = x - s;
    for (uint32_t q = 0; q < (t >> 6); q++) r += ws[q];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        if (k < pc && pc * t + k < C) {
            start[pc * t + k] = r;
            r += v[k];
        }
    }
    if (__ballot(big) && (t & 63) == 0) atomicOr(flags, 4u);
}

// a key's KL bytes as dwords (widest aligned accesses), and back
template <int KL>
__device__ __forceinline__ void key_words_load(const uint8_t *p, uint32_t *w) {
    if constexpr (KL % 16 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 16) {
            const uint4 v = *reinterpret_cast<const uint4 *>(p + o);
            w[o / 4] = v.x; w[o / 4 + 1] = v.y; w[o / 4 + 2] = v.z; w[o / 4 + 3] = v.w;
        }
    } else if constexpr (KL % 8 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 8) {
            const uint2 v = *reinterpret_cast<const uint2 *>(p + o);
            w[o / 4] = v.x; w[o / 4 + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int o = 0; o < KL; o += 4) w[o / 4] = *reinterpret_cast<const uint32_t *>(p + o);
    }
}
template <int KL>
__device__ __forceinline__ void key_words_store(uint8_t *p, const uint32_t *w) {
    if constexpr (KL % 16 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 16)
            *reinterpret_cast<uint4 *>(p + o) = make_uint4(w[o / 4], w[o / 4 + 1], w[o / 4 + 2], w[o / 4 + 3]);
    } else if constexpr (KL % 8 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 8) *reinterpret_cast<uint2 *>(p + o) = make_uint2(w[o / 4], w[o / 4 + 1]);
    } else {
#pragma unroll
        for (int o = 0; o < KL; o += 4) *reinterpret_cast<uint32_t *>(p + o) = w[o / 4];
    }
}
// the leading digit (key_digit d = 0) of a key held as dwords
template <int KK, int KL>
__device__ __forceinline__ uint64_t digit_of_words(const uint32_t *w) {
    if constexpr (KK == KEY_U32) return w[0];
    else if constexpr (KK == KEY_U64) return ((uint64_t)w[1] << 32) | w[0];
    else return __builtin_bswap64(((uint64_t)w[1] << 32) | w[0]);
}

// (key, row) pairs into coarse-bucket order: the whole key travels, so the per-bucket sort
// reads its keys from one contiguous stretch instead of gathering them from the input rows
// oidx (nullable): each slot's input row (for the ops and a stable order of equal keys); islot
// (nullable): each input row's slot, in input order (the first level of the two-level positions)
template <int KK, int KL>
__global__ __launch_bounds__(CS_WG) void k_cs_scatter(const uint8_t *keys, uint64_t m, const uint64_t *params,
                                                      uint32_t C, const uint32_t *hist, const uint32_t *start,
                                                      uint8_t *okey, uint32_t *oidx, uint32_t *islot) {
    __shared__ uint32_t cur[CS_MAX_C];
    const uint64_t mn = params[0], sh = params[1];
    const uint32_t *h = hist + (uint64_t)blockIdx.x * C;
    for (uint32_t b = threadIdx.x; b < C; b += CS_WG) cur[b] = start[b] + h[b];
    __syncthreads();
    const uint64_t i0 = (uint64_t)blockIdx.x * CS_TILE;
    // four keys per lane at a time, each group's loads before its stores (eight at once spill)
    auto group = [&](int k0) {
        constexpr int W = KL / 4;
        uint32_t kw[4][W];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t i = i0 + CS_WG * (k0 + k) + threadIdx.x;
            if (i < m) key_words_load<KL>(keys + i * KL, kw[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t i = i0 + CS_WG * (k0 + k) + threadIdx.x;
            if (i < m) {
                const uint64_t d = digit_of_words<KK, KL>(kw[k]);
                const uint32_t pos = atomicAdd(&cur[(uint32_t)((d - mn) >> sh) >> CS_FINE_BITS], 1u);
                key_words_store<KL>(okey + (uint64_t)pos * KL, kw[k]);
                if (oidx) oidx[pos] = (uint32_t)i;
                if (islot) islot[i] = pos;
            }
        }
    };
    static_assert(CS_TILE / CS_WG == 8, "two groups of four keys per lane");
    group(0);
    group(4);
}

// rows 256 (K0 + k) + lane, k < 4, of a bucket's sorted order: the key from the bucket's stretch
// of scattered keys, the op (and, with fps, the fingerprint) from the input row; pos (when given):
// pos[input row] = its sorted row, for a lift that runs after the sort
// (s2o: pos[input row] is its slot, written by the scatter; here s2o[slot] = its sorted row)
template <int KL, int K0>
__device__ __forceinline__ void cs_gather(const uint16_t *sx, const uint32_t *tx, const uint16_t *tl, uint32_t n,
                                          uint32_t s0, const uint8_t *okey, const uint8_t *fps, const uint8_t *ops,
                                          uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *pos, uint32_t *s2o) {
    static_assert(KL % 4 == 0, "keys: whole dwords");
    const uint32_t t = threadIdx.x;
    uint32_t kw[4][KL / 4], ov[4], xr[4];
    uint4 f0[4], f1[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t j = 256 * (K0 + k) + t;
        const uint32_t q = j < n ? sx[j] : 0;  // slot 0 stands in past n (not stored)
        const uint64_t src = tx[q];
        xr[k] = s2o ? s0 + (uint32_t)tl[q] : (uint32_t)src;
        key_words_load<KL>(okey + (uint64_t)(s0 + tl[q]) * KL, kw[k]);
        if (fps) {
            f0[k] = reinterpret_cast<const uint4 *>(fps + 32 * src)[0];
            f1[k] = reinterpret_cast<const uint4 *>(fps + 32 * src)[1];
        }
        ov[k] = ops ? ops[src] : 0u;
    }
    // written out per row: a loop here is rotated into a variable trip count, which indexes the
    // arrays dynamically and puts them in scratch memory
    auto put = [&](int k, const uint32_t *w, uint4 a, uint4 b, uint32_t op, uint32_t x) {
        const uint32_t j = 256 * (K0 + k) + t;
        if (j >= n) return;
        const uint64_t o = (uint64_t)s0 + j;
        key_words_store<KL>(skeys + o * KL, w);
        if (fps) {
            reinterpret_cast<uint4 *>(sfps + 32 * o)[0] = a;
            reinterpret_cast<uint4 *>(sfps + 32 * o)[1] = b;
        }
        if (s2o) s2o[x] = (uint32_t)o;  // x: the row's slot
        else if (pos) pos[x] = (uint32_t)o;
        sops[o] = (uint8_t)op;
    };
    put(0, kw[0], f0[0], f1[0], ov[0], xr[0]);
    put(1, kw[1], f0[1], f1[1], ov[1], xr[1]);
    put(2, kw[2], f0[2], f1[2], ov[2], xr[2]);
    put(3, kw[3], f0[3], f1[3], ov[3], xr[3]);
}

// one workgroup per coarse bucket (n <= CS_CAP keys, CS_CAP / 256 per lane, held in registers)
template <int KK, int KL>
__global__ __launch_bounds__(256) void k_cs_sort(const uint8_t *okey, const uint32_t *idx, const uint32_t *start,
                                                 const uint32_t *total, const uint64_t *params, const uint8_t *fps,
                                                 const uint8_t *ops, uint8_t *skeys, uint8_t *sfps, uint8_t *sops,
                                                 uint32_t *pos, uint32_t *flags, uint32_t *s2o) {
    constexpr int D = KK == KEY_BYTES ? KL / 8 : 1, PER = CS_CAP / 256;
    static_assert(CS_FINE == 256, "one fine bucket per lane");
    // fine-bucket order: td digit, tx input row, tl index in the bucket's stretch; sx: sorted
    // position -> slot of that order
    __shared__ uint64_t td[CS_CAP];
    __shared__ uint32_t tx[CS_CAP];
    __shared__ uint16_t tl[CS_CAP], sx[CS_CAP];
    static_assert(CS_CAP <= 65536, "16-bit slots");
    __shared__ uint32_t fst[CS_FINE], fcur[CS_FINE], wsum[4];
    const uint32_t b = blockIdx.x, t = threadIdx.x, n = total[b], s0 = start[b];
    if (n == 0 || n > (uint32_t)CS_CAP) return;  // uniform; too large: flagged by k_cs_colscan
    const uint64_t mn = params[0], sh = params[1];
    const uint8_t *bk = okey + (uint64_t)s0 * KL;
    uint64_t d[PER];
    uint32_t x[PER], f[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t i = 256 * k + t;
        d[k] = i < n ? key_digit<KK, KL>(bk + (uint64_t)i * KL, 0) : 0;
        x[k] = i < n ? (idx ? idx[s0 + i] : i) : 0;  // without idx: the slot (ties then by slot)
        f[k] = (uint32_t)((d[k] - mn) >> sh) & (CS_FINE - 1);
    }
    fcur[t] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++)
        if (256 * k + t < n) atomicAdd(&fcur[f[k]], 1u);
    __syncthreads();
    // exclusive scan of the fine counts, lane t holding bucket t
    const uint32_t c = fcur[t];
    uint32_t y = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t z = __shfl_up(y, o, 64);
        if ((t & 63) >= (uint32_t)o) y += z;
    }
    if ((t & 63) == 63) wsum[t >> 6] = y;
    __syncthreads();
    uint32_t before = y - c;
    for (uint32_t q = 0; q < (t >> 6); q++) before += wsum[q];
    fst[t] = before;
    fcur[t] = before;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++) {
        if (256 * k + t < n) {
            const uint32_t p = atomicAdd(&fcur[f[k]], 1u);
            td[p] = d[k];
            tx[p] = x[k];
            tl[p] = (uint16_t)(256 * k + t);
        }
    }
    __syncthreads();
    // fine bucket g spans [fst[g], fcur[g]); rank each key inside it by (digit, key, row)
    bool dup = false;
    for (uint32_t p = t; p < n; p += 256) {
        const uint64_t dp = td[p];
        const uint32_t xp = tx[p], g = (uint32_t)((dp - mn) >> sh) & (CS_FINE - 1);
        const uint32_t lo = fst[g], hi = fcur[g];
        uint32_t r = lo;
        for (uint32_t q = lo; q < hi; q++) {
            const uint64_t dq = td[q];
            if (dq != dp) {
                r += dq < dp ? 1u : 0u;
            } else if (q != p) {
                const uint32_t xq = tx[q];
                const int cmp =
                    D == 1 ? 0 : key_cmp<KK, KL>(bk + (uint64_t)tl[q] * KL, bk + (uint64_t)tl[p] * KL);
                if (cmp == 0) dup = true;
                r += (cmp < 0 || (cmp == 0 && xq < xp)) ? 1u : 0u;
            }
        }
        sx[r] = (uint16_t)p;
    }
    __syncthreads();
    // gather key / op (/ fingerprint) of the sorted rows, 4 per lane at a time with all of the
    // group's loads before its stores
    cs_gather<KL, 0>(sx, tx, tl, n, s0, okey, fps, ops, skeys, sfps, sops, pos, s2o);
    if (n > 4 * 256) cs_gather<KL, 4>(sx, tx, tl, n, s0, okey, fps, ops, skeys, sfps, sops, pos, s2o);
    if (__ballot(dup) && (t & 63) == 0) atomicOr(flags, 1u);
}

// ---- search ---------------------------------------------------------------------------------

// lower_bound rank of each query key in a sorted key array; present = key at rank equals
template <int KK, int KL>
__global__ void k_search(const uint8_t *keys, uint64_t n, const uint8_t *q, uint64_t m, uint32_t *rank,
                         uint8_t *present) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint8_t *key = q + j * KL;
    const uint64_t lo = lower_bound_keys<KK, KL>(keys, n, key);
    rank[j] = (uint32_t)lo;
    if (present) present[j] = (lo < n && key_cmp<KK, KL>(keys + lo * KL, key) == 0) ? 1 : 0;
}

// Sampled search: smp[s] = the leading u64 digit of keys[SMP_STRIDE * s].  The digit's place
// among the samples bounds the key's rank to one stride-wide window (more when samples tie),
// so a query touches the small, cache-resident sample array and then a few lines of one
// window, instead of ~log2(n) scattered lines of the whole run.
// A second level (every SMP2_STRIDE-th key; 8 B per 8 keys) narrows the window to one line of
// 16-byte keys (the key lines are what a batch of searches pays for: 2.4 -> ~1.9 distinct lines
// per query against a 100 M-row base).

uint64_t sample2_entries(uint64_t n) { return (n + SMP2_STRIDE - 1) / SMP2_STRIDE + 2; }

template <int KK, int KL>
__global__ void k_sample(const uint8_t *keys, uint64_t n, uint64_t stride, uint64_t *smp) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s * stride < n) smp[s] = key_digit<KK, KL>(keys + s * stride * KL, 0);
}

// Search table over a run's stride-16 samples (the large base run): tab[h] = the first sample
// whose digit is >= min + (h << shift), h in [0, 2^bits], with (min, shift) in par[0..1] and the
// shift chosen from the samples' digit range so that ~4 samples fall in each bucket.  A key's
// bucket then brackets its lower bound to one or two lines of samples at the cost of one table
// line, where the stride-256 samples took a ~19-step binary search (the deeper steps missing the
// caches once per query).
__device__ __forceinline__ void table_params(const uint64_t *smp2, uint64_t ns2, uint32_t bits, uint64_t &dmin,
                                             uint32_t &sh) {
    dmin = smp2[0];
    const uint64_t range = smp2[ns2 - 1] - dmin;
    const uint32_t rb = range ? 64u - (uint32_t)__clzll(range) : 0u;
    sh = rb > bits ? rb - bits : 0u;
}

// built from the samples in one pass: sample s opens buckets (h(s - 1), h(s)] (h(-1) = -1), and
// the last sample closes the rest; bucket h's value is the first sample at or above it.  A gap of
// more than 256 buckets (keys bunched in a corner of their digit range: one thread would write
// millions of entries -- 10 ms for a 2^24-entry table) is left to k_search_table_gaps, told by
// par[2] = gen (this build's number)
__global__ void k_search_table(const uint64_t *smp2, uint64_t ns2, uint32_t bits, uint32_t *tab, uint64_t *par,
                               uint64_t gen) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = 1ull << bits;
    if (s > ns2) return;
    uint64_t dmin;
    uint32_t sh;
    table_params(smp2, ns2, bits, dmin, sh);
    if (s == 0) {
        par[0] = dmin;
        par[1] = sh;
    }
    // h(s) = the bucket of sample s's digit (samples are sorted, so h is non-decreasing)
    auto h = [&](uint64_t q) -> uint64_t {
        const uint64_t v = (smp2[q] - dmin) >> sh;
        return v < nt ? v : nt - 1;
    };
    const uint64_t lo = s == 0 ? 0 : h(s - 1) + 1, hi = s == ns2 ? nt : h(s);
    if (hi >= lo && hi - lo >= 256) {
        par[2] = gen;
        return;
    }
    for (uint64_t b = lo; b <= hi && b <= nt; b++) tab[b] = (uint32_t)s;
}

// after a build with a long gap: every bucket's value by a binary search of the samples (the
// buckets of one gap all follow the same path, so it stays in cache); otherwise nothing
__global__ void k_search_table_gaps(const uint64_t *smp2, uint64_t ns2, uint32_t bits, uint32_t *tab,
                                    const uint64_t *par, uint64_t gen) {
    if (par[2] != gen) return;
    const uint64_t nt = 1ull << bits, dmin = par[0];
    const uint32_t sh = (uint32_t)par[1];
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= nt; b += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t lo = 0, hi = ns2;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            const uint64_t v = (smp2[mid] - dmin) >> sh;
            if ((v < nt ? v : nt - 1) >= b) hi = mid;
            else lo = mid + 1;
        }
        tab[b] = (uint32_t)lo;
    }
}

template <int KK, int KL>
__global__ void k_search_sampled(const uint8_t *keys, uint64_t n, const uint64_t *smp, const uint64_t *smp2,
                                 SearchTable tb, const uint8_t *q, uint64_t m, uint32_t *rank, uint8_t *present) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    search_sampled_one<KK, KL>(keys, n, smp, smp2, tb, q + j * KL, rank + j, present ? present + j : nullptr);
}

// 1 if keys are not strictly increasing
template <int KK, int KL>
__global__ void k_check_sorted(const uint8_t *keys, uint64_t n, uint32_t *bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i < n && key_cmp<KK, KL>(keys + (i - 1) * KL, keys + i * KL) >= 0) atomicOr(bad, 1u);
}

// rank bounds of a key range in a sorted key array (std::ops::Bound: 0 unbounded, 1 included,
// 2 excluded); an inverted range gives an empty one (rbsr/src/protocol.rs:230-232)
// dedup_last: keep[j] = 1 unless row j + 1 has the same key
template <int KK, int KL>
__global__ void k_last_flags(const uint8_t *keys, uint64_t n, uint32_t *keep) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    keep[j] = (j + 1 == n || key_cmp<KK, KL>(keys + j * KL, keys + (j + 1) * KL) != 0) ? 1u : 0u;
}

template <int KL>
__global__ void k_dedup_scatter(const uint8_t *keys, const uint8_t *fps, const uint32_t *keep, const uint32_t *pos,
                                uint64_t n, uint8_t *okeys, uint8_t *ofps, uint64_t *counts) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    if (keep[j]) {
        copy_bytes<KL>(okeys + (uint64_t)pos[j] * KL, keys + j * KL);
        copy_bytes<32>(ofps + 32ull * pos[j], fps + 32 * j);
    }
    if (j + 1 == n) counts[0] = (uint64_t)pos[j] + keep[j];
}

template <int KK, int KL>
__global__ void k_keep_last(const uint8_t *skeys, const uint32_t *pos, const uint32_t *s2o, uint64_t m,
                            uint32_t *keep) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > m) return;
    if (i == m) {
        keep[m] = 0;
        return;
    }
    const uint64_t j = s2o ? s2o[pos[i]] : pos[i];
    keep[i] = (j + 1 < m && key_cmp<KK, KL>(skeys + j * KL, skeys + (j + 1) * KL) == 0) ? 0u : 1u;
}

__global__ void k_compact_rows(const uint8_t *src, uint32_t row, const uint32_t *keep, const uint32_t *dst, uint64_t m,
                               uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m || !keep[i]) return;
    const uint8_t *s = src + i * row;
    uint8_t *d = out + (uint64_t)dst[i] * row;
    if (row % 4 == 0) {
        for (uint32_t o = 0; o < row; o += 4) *reinterpret_cast<uint32_t *>(d + o) = *reinterpret_cast<const uint32_t *>(s + o);
    } else {
        for (uint32_t o = 0; o < row; o++) d[o] = s[o];
    }
}

template <int KK, int KL>
__global__ void k_bounds(const uint8_t *keys, uint64_t n, const uint8_t *lo_key, int lo_kind, const uint8_t *hi_key,
                         int hi_kind, uint64_t *qlo, uint64_t *qhi) {
    if (threadIdx.x != 0) return;
    uint64_t a = 0, b = n;
    if (lo_kind) {
        a = lower_bound_keys<KK, KL>(keys, n, lo_key);
        if (lo_kind == 2 && a < n && key_cmp<KK, KL>(keys + a * KL, lo_key) == 0) a++;
    }
    if (hi_kind) {
        b = lower_bound_keys<KK, KL>(keys, n, hi_key);
        if (hi_kind == 1 && b < n && key_cmp<KK, KL>(keys + b * KL, hi_key) == 0) b++;
    }
    if (b < a) b = a;
    *qlo = a;
    *qhi = b;
}

// ---- the delta run ------------------------------------------------------------------------

// Build the batch's DeltaRecs (key order) from its fingerprints, what base and delta hold for
// each key, and the op; dops: 0 = upsert into the delta run, 1 = drop the key's delta entry.
// counts (vs the merged view): [0] new keys, [1] overwritten, [2] deleted.
// part[7 g + k], workgroup g: k = 0 new, 1 overwritten, 2 deleted (vs the merged view), and for
// the merge into the delta run 3 upserts (dops 0), 4 keys the run holds (present_d), 5 both,
// 6 the change of the run's count total (int32); dsum[4 g ..] the change of its contribution total
// (Σ new entries' contrib − Σ replaced entries' contrib, mod 2^256)
// 512-row workgroups (~2,000 partials per 1 M batch): at 1,024 lanes the 256-bit accumulators
// of the totals spilled to scratch (a 128-VGPR cap)
constexpr int DB_PARTS = 7, DB_WG = 512, DP_WG = 512, PU = 8;

__global__ __launch_bounds__(DB_WG) void k_delta_build(const uint8_t *sfps, const uint8_t *sops, uint64_t m,
                                                     const uint32_t *rank_b, const uint8_t *present_b,
                                                     const uint8_t *base_fps, const uint32_t *rank_d,
                                                     const uint8_t *present_d, const uint32_t *dslot,
                                                     const uint8_t *heap, uint8_t *bpay, uint8_t *dops,
                                                     uint32_t *part, uint64_t *dsum) {
    __shared__ uint64_t lds[(DB_WG / 64) * 8];
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool c_new = false, c_over = false, c_del = false, c_up = false, c_pr = false;
    int32_t dcnt = 0;
    uint32_t dfp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (j < m) {
        const bool isdel = sops[j] != 0, in_b = present_b[j], in_d = present_d[j];
        bool was_live = in_b;
        const DeltaRec *old_rec = in_d ? reinterpret_cast<const DeltaRec *>(heap) + dslot[rank_d[j]] : nullptr;
        if (in_d) was_live = (old_rec->flags & DeltaRec::LIVE) != 0;
        uint32_t base[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (in_b) fp_load(base_fps + 32ull * rank_b[j], base);
        DeltaRec r;
        r.flags = (in_b ? DeltaRec::IN_BASE : 0u);
        r.brank = rank_b[j];
        uint32_t cur[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (!isdel) {
            fp_load(sfps + 32 * j, cur);
            r.flags |= DeltaRec::LIVE;
            c_new = !was_live;
            c_over = was_live;
        } else {
            c_del = was_live;
        }
        fp_sub(cur, base, r.contrib);
        // deleting a key the base does not hold needs no entry (drop any delta entry it has)
        const bool drop = isdel && !in_b;
        dops[j] = drop ? 1 : 0;
        c_up = !drop;
        c_pr = in_d;
        reinterpret_cast<DeltaRec *>(bpay)[j] = r;
        // what this row changes in the run's totals: its new entry in, the entry it replaces out
        if (!drop) dcnt += (isdel ? 0 : 1) - (in_b ? 1 : 0);
        uint32_t nc[8], oc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 8; k++) nc[k] = drop ? 0u : r.contrib[k];
        if (in_d) {
            const uint2 *op = reinterpret_cast<const uint2 *>(old_rec);
            uint32_t w[10];
#pragma unroll
            for (int k = 0; k < 5; k++) words_of(op[k], w + 2 * k);
#pragma unroll
            for (int k = 0; k < 8; k++) oc[k] = w[k];
            dcnt -= ((w[9] & DeltaRec::LIVE) ? 1 : 0) - ((w[9] & DeltaRec::IN_BASE) ? 1 : 0);
        }
        fp_sub(nc, oc, dfp);
    }
    {
        Acc a;
        acc_zero(a);
        acc_add_fp(a, dfp);
        uint32_t f[8];
        acc_block_reduce<DB_WG>(a, lds, f);
        if (threadIdx.x == 0) {
#pragma unroll
            for (int q = 0; q < 4; q++) dsum[4ull * blockIdx.x + q] = (uint64_t)f[2 * q] | ((uint64_t)f[2 * q + 1] << 32);
        }
    }
    // per-workgroup counts (same-address atomics from every wave would serialise in L2);
    // k_delta_parts adds them up
    __shared__ uint32_t wc[DB_WG / 64][DB_PARTS];
    const unsigned long long b[DB_PARTS] = {__ballot(c_new), __ballot(c_over), __ballot(c_del), __ballot(c_up),
                                            __ballot(c_pr), __ballot(c_up && c_pr)};
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < DB_PARTS; k++) wc[threadIdx.x >> 6][k] = (uint32_t)__popcll(b[k]);
    __syncthreads();
    if (threadIdx.x < DB_PARTS - 1) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) t += wc[w][threadIdx.x];
        part[(uint64_t)DB_PARTS * blockIdx.x + threadIdx.x] = t;
    }
    // the count change: a block sum of small signed ints
    int32_t y = dcnt;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) y += __shfl_xor(y, o, 64);
    __shared__ int32_t wd[DB_WG / 64];
    if ((threadIdx.x & 63) == 0) wd[threadIdx.x >> 6] = y;
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t tsum = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) tsum += wd[w];
        part[(uint64_t)DB_PARTS * blockIdx.x + DB_PARTS - 1] = (uint32_t)tsum;
    }
}

// one workgroup over the G = ceil(m / DB_WG) partials: the batch counts (counts3), the merge counts
// (mcnt: [0] inserts, [1] overwrites, [2] removals, [3] upserts U, [4] present R; out3 the first
// three) and each workgroup's exclusive (U, R) offsets for k_delta_lists (off[2 g], off[2 g + 1])
// (dsum / dtot, optional: the per-workgroup contribution changes and their total; dcnt: the count
// change's total)
__global__ __launch_bounds__(DP_WG) void k_delta_parts(const uint32_t *__restrict__ part, uint64_t G,
                                                      uint64_t *__restrict__ counts3, uint64_t *__restrict__ mcnt,
                                                      uint64_t *__restrict__ out3, uint32_t *__restrict__ off,
                                                      const uint64_t *__restrict__ dsum, uint64_t *__restrict__ dtot,
                                                      int64_t *__restrict__ dcnt) {
    // counts are < 2^31 (the store's row limit): 32-bit sums throughout
    constexpr uint32_t NW = DP_WG / 64;
    __shared__ uint32_t w[NW][DB_PARTS];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint64_t chunk = (G + DP_WG - 1) / DP_WG, g0 = t * chunk < G ? t * chunk : G,
                   g1 = g0 + chunk < G ? g0 + chunk : G;
    uint32_t sum[DB_PARTS] = {0, 0, 0, 0, 0, 0, 0};
    // a thread's partials are read 8 workgroups at a time, every load issued before the adds: the
    // loop was one load latency per workgroup (87 us for a 12.5 M-row compaction's 24 k partials)
    // (a batch's ~2 k partials give each thread 4: the 4-wide stage)
    uint64_t g = g0;
    for (; g + PU <= g1; g += PU) {
        uint32_t v[PU][DB_PARTS];
#pragma unroll
        for (int i = 0; i < PU; i++)
#pragma unroll
            for (int k = 0; k < DB_PARTS; k++) v[i][k] = part[DB_PARTS * (g + i) + k];
#pragma unroll
        for (int i = 0; i < PU; i++)
#pragma unroll
            for (int k = 0; k < DB_PARTS; k++) sum[k] += v[i][k];  // slot 6: int32 bits, wraps right
    }
    for (; g + PU / 2 <= g1; g += PU / 2) {
        uint32_t v[PU / 2][DB_PARTS];
#pragma unroll
        for (int i = 0; i < PU / 2; i++)
#pragma unroll
            for (int k = 0; k < DB_PARTS; k++) v[i][k] = part[DB_PARTS * (g + i) + k];
#pragma unroll
        for (int i = 0; i < PU / 2; i++)
#pragma unroll
            for (int k = 0; k < DB_PARTS; k++) sum[k] += v[i][k];
    }
    for (; g < g1; g++)
#pragma unroll
        for (int k = 0; k < DB_PARTS; k++) sum[k] += part[DB_PARTS * g + k];
    if (dsum) {  // the contribution change (a uniform branch: every lane joins the block reduction)
        __shared__ uint64_t lds[NW * 8];
        Acc a;
        acc_zero(a);
        uint64_t g2 = g0;
        for (; g2 + PU / 2 <= g1; g2 += PU / 2) {  // loads first, as above
            uint64_t v[PU / 2][4];
#pragma unroll
            for (int i = 0; i < PU / 2; i++)
#pragma unroll
                for (int q = 0; q < 4; q++) v[i][q] = dsum[4 * (g2 + i) + q];
#pragma unroll
            for (int i = 0; i < PU / 2; i++) {
                uint32_t f[8];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    f[2 * q] = (uint32_t)v[i][q];
                    f[2 * q + 1] = (uint32_t)(v[i][q] >> 32);
                }
                acc_add_fp(a, f);
            }
        }
        for (; g2 < g1; g2++) {
            uint32_t f[8];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint64_t v = dsum[4 * g2 + q];
                f[2 * q] = (uint32_t)v;
                f[2 * q + 1] = (uint32_t)(v >> 32);
            }
            acc_add_fp(a, f);
        }
        uint32_t f[8];
        acc_block_reduce<DP_WG>(a, lds, f);
        if (t == 0) {
#pragma unroll
            for (int q = 0; q < 4; q++) dtot[q] = (uint64_t)f[2 * q] | ((uint64_t)f[2 * q + 1] << 32);
        }
    }
    // U (3) and R (4): inclusive wave scans; the others: wave totals
    uint32_t xu = sum[3], xr = sum[4];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yu = __shfl_up(xu, o, 64), yr = __shfl_up(xr, o, 64);
        if (lane >= (uint32_t)o) {
            xu += yu;
            xr += yr;
        }
    }
    uint32_t tot[DB_PARTS];
#pragma unroll
    for (int k = 0; k < DB_PARTS; k++) {
        uint32_t v = k == 3 ? xu : k == 4 ? xr : sum[k];
        if (k != 3 && k != 4) {
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        } else {
            v = __shfl(v, 63, 64);
        }
        tot[k] = v;
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < DB_PARTS; k++) w[wv][k] = tot[k];
    }
    __syncthreads();
    uint32_t u = xu - sum[3], r = xr - sum[4];
    for (uint32_t q = 0; q < wv; q++) {
        u += w[q][3];
        r += w[q][4];
    }
    for (g = g0; g + PU <= g1; g += PU) {
        uint32_t pu[PU], pr[PU];
#pragma unroll
        for (int i = 0; i < PU; i++) {
            pu[i] = part[DB_PARTS * (g + i) + 3];
            pr[i] = part[DB_PARTS * (g + i) + 4];
        }
#pragma unroll
        for (int i = 0; i < PU; i++) {
            off[2 * (g + i)] = u;
            off[2 * (g + i) + 1] = r;
            u += pu[i];
            r += pr[i];
        }
    }
    for (; g + PU / 2 <= g1; g += PU / 2) {
        uint32_t pu[PU / 2], pr[PU / 2];
#pragma unroll
        for (int i = 0; i < PU / 2; i++) {
            pu[i] = part[DB_PARTS * (g + i) + 3];
            pr[i] = part[DB_PARTS * (g + i) + 4];
        }
#pragma unroll
        for (int i = 0; i < PU / 2; i++) {
            off[2 * (g + i)] = u;
            off[2 * (g + i) + 1] = r;
            u += pu[i];
            r += pr[i];
        }
    }
    for (; g < g1; g++) {
        off[2 * g] = u;
        off[2 * g + 1] = r;
        u += part[DB_PARTS * g + 3];
        r += part[DB_PARTS * g + 4];
    }
    if (t == 0) {
        uint64_t T[DB_PARTS];
#pragma unroll
        for (int k = 0; k < DB_PARTS; k++) {
            T[k] = 0;
            for (uint32_t q = 0; q < NW; q++) T[k] += w[q][k];
        }
        if (dcnt) {
            int64_t d = 0;
            for (uint32_t q = 0; q < NW; q++) d += (int32_t)w[q][DB_PARTS - 1];
            *dcnt = d;
        }
        if (counts3) {
            counts3[0] = T[0];
            counts3[1] = T[1];
            counts3[2] = T[2];
        }
        const uint64_t U = T[3], R = T[4], ov = T[5];
        mcnt[0] = U - ov;
        mcnt[1] = ov;
        mcnt[2] = R - ov;
        mcnt[3] = U;
        mcnt[4] = R;
        if (out3) {
            out3[0] = U - ov;
            out3[1] = ov;
            out3[2] = R - ov;
        }
    }
}

// the merge lists from the workgroup offsets: upos / usrc for the upserts, rlist
// for the batch keys the run holds
__global__ __launch_bounds__(DB_WG) void k_delta_lists(const uint8_t *dops, const uint8_t *present,
                                                       const uint32_t *rank, const uint32_t *off, uint64_t m,
                                                       uint32_t *upos, uint32_t *usrc, uint32_t *rlist) {
    __shared__ uint32_t wu[DB_WG / 64], wr[DB_WG / 64];
    const uint64_t j = (uint64_t)blockIdx.x * DB_WG + threadIdx.x;
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const bool up = j < m && dops[j] == 0, pr = j < m && present[j] != 0;
    const unsigned long long bu = __ballot(up), br = __ballot(pr);
    const uint32_t lu = __builtin_amdgcn_mbcnt_hi((uint32_t)(bu >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bu, 0u));
    const uint32_t lr = __builtin_amdgcn_mbcnt_hi((uint32_t)(br >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)br, 0u));
    if (lane == 0) {
        wu[wv] = (uint32_t)__popcll(bu);
        wr[wv] = (uint32_t)__popcll(br);
    }
    __syncthreads();
    uint32_t U = off[2 * blockIdx.x] + lu, R = off[2 * blockIdx.x + 1] + lr;
    for (uint32_t q = 0; q < wv; q++) {
        U += wu[q];
        R += wr[q];
    }
    if (up) {
        upos[U] = rank[j] + U - R;
        usrc[U] = (uint32_t)j;
    }
    if (pr) rlist[R] = rank[j];
}

constexpr int MT = 2048;  // output rows per workgroup (8 blocks of 256; 2,048 measured best of 1,024 / 2,048 / 4,096)

// The merge's tiles' bounds in the upsert list, formed once per merge instead of searched by every
// tile: tileU[t] = the upserts placed before output row t * MT, for t in [0, tiles].  Thread U
// writes the tiles that start after upsert U - 1's row and at or before upsert U's (thread U of U
// upserts: the tiles after the last one); upos is strictly increasing.
__global__ void k_tile_bounds(const uint32_t *upos, const uint64_t *counts, uint64_t m, uint64_t tiles, uint32_t *tileU) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, U = counts[3];
    if (j > U || j > m) return;
    const uint64_t lo = j == 0 ? 0 : (uint64_t)upos[j - 1] / MT + 1;
    const uint64_t hi = j < U ? (uint64_t)upos[j] / MT : tiles;
    for (uint64_t t = lo; t <= hi && t <= tiles; t++) tileU[t] = (uint32_t)j;
}

// compaction input: cur fp = contrib + base fp, op = live ? upsert : delete, and the key's
// place in the base (no search: brank was recorded when the entry was built); plus the
// per-1024-row partials of k_delta_parts (slots 3 upserts, 4 keys the base holds, 5 both)
__global__ __launch_bounds__(DB_WG) void k_delta_cur(const uint32_t *dslot, const uint8_t *heap, uint64_t n,
                                                     const uint8_t *base_fps, uint8_t *fps, uint8_t *ops,
                                                     uint32_t *rank, uint8_t *present, uint32_t *part) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool up = false, pr = false;
    if (i < n) {
        // the 40-byte record as five 8-byte loads (it is 8-byte aligned), all issued at once
        const uint2 *rp = reinterpret_cast<const uint2 *>(heap + sizeof(DeltaRec) * (uint64_t)dslot[i]);
        uint2 q[5];
#pragma unroll
        for (int k = 0; k < 5; k++) q[k] = rp[k];
        const uint32_t contrib[8] = {q[0].x, q[0].y, q[1].x, q[1].y, q[2].x, q[2].y, q[3].x, q[3].y};
        const uint32_t brank = q[4].x, flags = q[4].y;  // DeltaRec words 8, 9
        const bool in_b = (flags & DeltaRec::IN_BASE) != 0;
        uint32_t base[8] = {0, 0, 0, 0, 0, 0, 0, 0}, cur[8];
        if (in_b) fp_load(base_fps + 32ull * brank, base);
        fp_add(contrib, base, cur);
        fp_store(fps + 32 * i, cur);
        up = (flags & DeltaRec::LIVE) != 0;
        pr = in_b;
        ops[i] = up ? 0 : 1;
        rank[i] = brank;
        present[i] = in_b ? 1 : 0;
    }
    __shared__ uint32_t wc[DB_WG / 64][3];
    const unsigned long long bu = __ballot(up), br = __ballot(pr), bo = __ballot(up && pr);
    if ((threadIdx.x & 63) == 0) {
        wc[threadIdx.x >> 6][0] = (uint32_t)__popcll(bu);
        wc[threadIdx.x >> 6][1] = (uint32_t)__popcll(br);
        wc[threadIdx.x >> 6][2] = (uint32_t)__popcll(bo);
    }
    __syncthreads();
    if (threadIdx.x < DB_PARTS) {
        uint32_t t = 0;
        if (threadIdx.x >= 3 && threadIdx.x < 6)
            for (uint32_t w = 0; w < blockDim.x / 64; w++) t += wc[w][threadIdx.x - 3];
        part[(uint64_t)DB_PARTS * blockIdx.x + threadIdx.x] = t;
    }
}

// Σ count deltas of delta rows [0, i]: the super-block prefix, the blocks before i's inside its
// super-block, and the rows up to i inside its block
__device__ __forceinline__ int64_t cnt_through(const CntPrefix &c, uint64_t i) {
    const uint64_t b = i / 256;
    return (int64_t)c.sblk[b / 256] + ((b % 256) ? c.blk[b - 1] : 0) + c.inb[i];
}

// The delta run's block sums (of the contributions) and count prefixes, formed on the first
// question after a batch that needs them (a key-range aggregate or a rank): the records gathered
// through the slots, one workgroup per 256-row block; k_delta_finish then forms the upper levels.
__global__ __launch_bounds__(256) void k_delta_sums(const uint32_t *dslot, const uint8_t *heap, uint64_t n,
                                                    uint8_t *obs, int32_t *ocnt, int16_t *oinb) {
    __shared__ SumTile tile;
    __shared__ int32_t wsum[4];
    const uint32_t t = threadIdx.x;
    const uint64_t blk = blockIdx.x, i = blk * 256 + t;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int32_t c = 0;
    if (i < n) {
        const uint2 *hp = reinterpret_cast<const uint2 *>(heap + (uint64_t)dslot[i] * sizeof(DeltaRec));
        uint32_t w[10];
#pragma unroll
        for (int k = 0; k < 5; k++) words_of(hp[k], w + 2 * k);
#pragma unroll
        for (int k = 0; k < 8; k++) h[k] = w[k];
        c = ((w[9] & DeltaRec::LIVE) ? 1 : 0) - ((w[9] & DeltaRec::IN_BASE) ? 1 : 0);
    }
    uint32_t f8[8];
    block_sum_fps256(h, tile, f8);
    if (t == 0) store_sum(obs, blk, f8);
    int32_t y = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t z = __shfl_up(y, o, 64);
        if ((t & 63) >= (uint32_t)o) y += z;
    }
    if ((t & 63) == 63) wsum[t >> 6] = y;
    __syncthreads();
    int32_t before = 0;
    for (uint32_t w = 0; w < (t >> 6); w++) before += wsum[w];
    if (i < n) oinb[i] = (int16_t)(before + y);
    if (t == 255) ocnt[blk] = before + y;
}

hipError_t launch_delta_sums(const uint32_t *dslot, const uint8_t *heap, uint64_t n, uint8_t *obs, int32_t *ocnt,
                             int16_t *oinb, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_delta_sums, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, dslot, heap, n, obs, ocnt,
                       oinb);
    return hipGetLastError();
}

// After a merge into a delta buffer (k_merge_run wrote its block sums and block count totals):
// the count prefix's upper levels, the super-block sums and the run's totals in one launch of one
// workgroup per super-block.
//   blk[b]   block b's count-delta total -> the inclusive prefix inside b's super-block
//   ssums[s] super-block s's contribution sum;  scnt[s] its count total
// and the workgroup that finishes last: sblk[s] = Σ scnt[0..s), *total = Σ scnt, fp_total = Σ
// ssums.  The hand-off to it: sc1 (agent) stores of ssums / scnt, each storing wave's vmcnt wait, a
// barrier, one agent-scope ticket add per workgroup; the last one reads them with sc1 loads
// (MI355X_MICROARCH.md, inter-workgroup visibility, row 1).  *ticket is 0 on entry and on exit.
__global__ __launch_bounds__(256) void k_delta_finish(const uint8_t *bsums, int32_t *blk, uint64_t nbk, uint8_t *ssums,
                                                      int32_t *scnt, int32_t *sblk, uint32_t *ticket, int32_t *total,
                                                      uint64_t *fp_total) {
    __shared__ SumTile tile;
    __shared__ uint64_t lds[4 * 8];
    __shared__ int32_t wsum[4];
    __shared__ uint32_t last;
    const uint32_t t = threadIdx.x;
    const uint64_t sb = blockIdx.x, b = sb * 256 + t;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int32_t c = 0;
    if (b < nbk) {
        fp_load(bsums + 32 * b, h);
        c = blk[b];
    }
    uint32_t f[8];
    block_sum_fps256(h, tile, f);  // on lane 0
    int32_t y = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t z = __shfl_up(y, o, 64);
        if ((t & 63) >= (uint32_t)o) y += z;
    }
    if ((t & 63) == 63) wsum[t >> 6] = y;
    __syncthreads();
    int32_t before = 0;
    for (uint32_t w = 0; w < (t >> 6); w++) before += wsum[w];
    if (b < nbk) blk[b] = before + y;
    if (t == 0) {
        uint64_t *o = reinterpret_cast<uint64_t *>(ssums + 32 * sb);
#pragma unroll
        for (int q = 0; q < 4; q++)
            __hip_atomic_store(o + q, (uint64_t)f[2 * q] | ((uint64_t)f[2 * q + 1] << 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 255) __hip_atomic_store(scnt + sb, before + y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0)
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1 ? 1u
                                                                                                              : 0u;
    __syncthreads();
    if (!last) return;  // uniform
    const uint32_t ns = gridDim.x;
    Acc a;
    acc_zero(a);
    for (uint32_t q = t; q < ns; q += 256) {
        const uint64_t *p = reinterpret_cast<const uint64_t *>(ssums + 32ull * q);
        uint32_t g[8];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t v = __hip_atomic_load(p + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            g[2 * k] = (uint32_t)v;
            g[2 * k + 1] = (uint32_t)(v >> 32);
        }
        acc_add_fp(a, g);
    }
    acc_block_reduce<256>(a, lds, f);
    if (t == 0) {
#pragma unroll
        for (int q = 0; q < 4; q++) fp_total[q] = (uint64_t)f[2 * q] | ((uint64_t)f[2 * q + 1] << 32);
    }
    // exclusive scan of the super-block counts: a contiguous chunk per lane
    const uint32_t chunk = (ns + 255) / 256, q0 = t * chunk < ns ? t * chunk : ns,
                   q1 = q0 + chunk < ns ? q0 + chunk : ns;
    int32_t run = 0;
    for (uint32_t q = q0; q < q1; q++) run += __hip_atomic_load(scnt + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    int32_t x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t z = __shfl_up(x, o, 64);
        if ((t & 63) >= (uint32_t)o) x += z;
    }
    __syncthreads();  // wsum reuse
    if ((t & 63) == 63) wsum[t >> 6] = x;
    __syncthreads();
    int32_t pre = x - run;
    for (uint32_t w = 0; w < (t >> 6); w++) pre += wsum[w];
    for (uint32_t q = q0; q < q1; q++) {
        sblk[q] = pre;
        pre += __hip_atomic_load(scnt + q, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 255) *total = pre;
    if (t == 0) *ticket = 0u;
}

hipError_t launch_delta_finish(const uint8_t *bsums, int32_t *blk, uint64_t nbk, uint8_t *ssums, int32_t *scnt,
                               int32_t *sblk, uint32_t *ticket, int32_t *total, uint64_t *fp_total, hipStream_t st) {
    const uint64_t ns = nbk ? (nbk + 255) / 256 : 1;
    hipLaunchKernelGGL(k_delta_finish, dim3((uint32_t)ns), dim3(256), 0, st, bsums, blk, nbk, ssums, scnt, sblk,
                       ticket, total, fp_total);
    return hipGetLastError();
}

// aggregate over a key range of the merged view = base part + delta part; the delta part's
// size is the sum of its count deltas (prefix difference), not its entry count
__global__ void k_agg_merge(const uint64_t *base_agg, const uint64_t *delta_agg, const uint64_t *dlo,
                            const uint64_t *dhi, CntPrefix cp, uint64_t *out) {
    if (threadIdx.x != 0) return;
    const uint64_t lo = *dlo, hi = *dhi;
    const int64_t c = (hi ? cnt_through(cp, hi - 1) : 0) - (lo ? cnt_through(cp, lo - 1) : 0);
    uint64_t carry = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint64_t a = base_agg[i], b = delta_agg[i];
        const uint64_t s = a + b;
        const uint64_t s2 = s + carry;
        carry = (s < a ? 1u : 0u) | (s2 < s ? 1u : 0u);
        out[i] = s2;
    }
    out[4] = (uint64_t)((int64_t)base_agg[4] + c);
}

// rank in the merged view = rank in base + Σ count deltas of the delta keys below
__global__ void k_rank_merge(const uint32_t *rank_b, const uint32_t *rank_d, CntPrefix cp, uint64_t m,
                             uint64_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t rd = rank_d ? rank_d[j] : 0;
    out[j] = (uint64_t)((int64_t)rank_b[j] + (rd ? cnt_through(cp, rd - 1) : 0));
}

// ---- protocol-round helpers (rbsr/src/protocol.rs:225-317) ------------------------------------
// A segment's bounds as a rank range of the base run: Unbounded start -> 0, Included(k) ->
// rank(k); Unbounded end -> n, Excluded(k) -> rank(k) (BoundedRange::parse, protocol/rank.rs).
// rank[2j] / rank[2j + 1] are the searched ranks of the start / end keys.
__global__ void k_resolve_bounds(const uint32_t *rank, const uint8_t *skind, const uint8_t *ekind, uint64_t r,
                                 uint64_t n, uint64_t *lo, uint64_t *hi) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= r) return;
    lo[j] = skind[j] ? (uint64_t)rank[2 * j] : 0ull;
    hi[j] = ekind[j] ? (uint64_t)rank[2 * j + 1] : n;
}

// out[i] = keys[sel[i]]: the select() cuts of every SPLIT in a round, one dword per lane
__global__ void k_gather_keys(const uint8_t *keys, uint32_t kl, const uint64_t *sel, uint64_t m, uint8_t *out) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t words = kl / 4;
    if (t >= m * words) return;
    const uint64_t i = t / words, w = t % words;
    reinterpret_cast<uint32_t *>(out)[i * words + w] =
        reinterpret_cast<const uint32_t *>(keys + sel[i] * kl)[w];
}

// ---- run merge: the merged run and its block sums in one pass ----------------------------------
// Merging a key-sorted batch into a sorted run A (rank / present: each batch key's lower bound
// in A and whether A holds it; op 0 upsert, 1 drop):
//   an upsert u lands at    pos_u = rank + U_before - R_before
//   (U: upserts, R: batch keys present in A -- overwritten or dropped A rows), and the A rows
//   that survive fill the remaining output slots in order.
// k_delta_parts / k_delta_lists list the upserts' positions and the removed A ranks (from
// per-1,024-row counts and one scan of them); k_merge_run then owns MT output rows per workgroup: it marks the upserts' slots, fills the
// free slots with A survivors (the q-th survivor is A row s + k, k = #removed ranks before it,
// found by a binary search over rank - index), copies each row once, and emits the 256-row
// block sums of the payload's leading fingerprint -- and, for the delta run, each block's
// count-delta total and every row's in-block count prefix.  This replaces a row-move pass, a
// batch-scatter pass and a re-read of the whole run for its sums.
// (MT, the output rows per workgroup: with k_tile_bounds above)

// The first index in [lo, hi) whose predicate holds (hi if none), for a predicate that is false
// then true along the range, searched by one whole wave: each step probes 64 evenly spaced
// positions at once and keeps the 1/64 of the range between the last false and the first true
// probe -- ~4 dependent loads for a million entries where a one-lane binary search makes ~20.
// Every lane of the wave calls it and gets the result.
template <typename Pred>
__device__ __forceinline__ uint64_t wave_partition_point(uint64_t lo, uint64_t hi, Pred pred) {
    const uint32_t lane = threadIdx.x & 63;
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        uint64_t p = lo + (lane + 1) * step - 1;
        p = p < hi ? p : hi - 1;
        const uint32_t n = (uint32_t)__popcll(__ballot(!pred(p)));  // probes before the boundary
        const uint64_t nlo = lo + n * step, nhi = lo + (n + 1) * step;
        lo = nlo < hi ? nlo : hi;
        hi = nhi < hi ? nhi : hi;
    }
    const uint64_t p = lo + lane;
    return lo + (uint64_t)__popcll(__ballot(p < hi && !pred(p)));
}

// smallest k in [lo, hi] with k == R or rlist[k] - k > s: the number of removed A rows before
// the s-th survivor
__device__ __forceinline__ uint64_t survivor_k(const uint32_t *rlist, uint64_t R, uint64_t lo, uint64_t hi, uint64_t s) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (mid >= R || (int64_t)rlist[mid] - (int64_t)mid > (int64_t)s) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}


// HEAP (the delta run): a row's payload is the 4-byte slot of its DeltaRec in the record heap
// (A rows: apay; batch row j: heap_base + j), and a merge moves key + slot only: the run's block
// sums and count prefixes are formed by k_delta_sums on the first question that needs them, and
// its totals are kept per batch by k_delta_build / k_delta_parts.
template <int KK, int KL, int P, bool COUNTS, bool HEAP>
__global__ __launch_bounds__(256) void k_merge_run(const uint8_t *akeys, const uint8_t *apay, uint64_t nA,
                                                   const uint8_t *bkeys, const uint8_t *bpay, uint64_t m,
                                                   const uint32_t *upos, const uint32_t *usrc, const uint32_t *rlist,
                                                   const uint64_t *counts, uint8_t *okeys, uint8_t *opay,
                                                   uint8_t *obs, int32_t *ocnt, int16_t *oinb, uint64_t nbk,
                                                   uint64_t *osmp, uint64_t *osmp2, const uint8_t *heap,
                                                   uint32_t heap_base, const uint32_t *tileU) {
    static_assert(HEAP ? (P == 4 && COUNTS) : (P % 8 == 0 && P >= 32), "payload: a slot, or a leading fingerprint");
    using V = typename std::conditional<P % 16 == 0, uint4, uint2>::type;  // widest aligned unit
    constexpr int NV = P / (int)sizeof(V) > 0 ? P / (int)sizeof(V) : 1;
    static_assert(MT % SMP_STRIDE == 0 && SMP_STRIDE % SMP2_STRIDE == 0, "whole sample strides per tile");
    __shared__ int32_t src[MT];  // A row, or -2 - batch row, or -1
    __shared__ uint64_t smp_t[MT / SMP2_STRIDE];
    __shared__ uint64_t prm[6];
    __shared__ uint32_t wsum[4];
    __shared__ SumTile tile;
    const uint32_t t = threadIdx.x;
    const uint64_t U = counts[3], R = counts[4];
    const uint64_t nC = nA + U - R;  // <= nA + m
    const uint64_t o0 = (uint64_t)blockIdx.x * MT;
    if (t < 64) {  // the tile's bounds in the upsert and removed-row lists: wave 0 searches them
        uint64_t o1 = o0, ju0 = 0, ju1 = 0, s0 = 0, k0 = 0, k1 = 0;
        if (o0 < nC) {
            o1 = o0 + MT < nC ? o0 + MT : nC;
            if (tileU) {  // k_tile_bounds (the last tile's end: every upsert lies before nC)
                ju0 = tileU[blockIdx.x];
                ju1 = o1 == nC ? U : tileU[blockIdx.x + 1];
            } else {
                ju0 = wave_partition_point(0, U, [&](uint64_t i) { return (uint64_t)upos[i] >= o0; });
                ju1 = wave_partition_point(ju0, U, [&](uint64_t i) { return (uint64_t)upos[i] >= o1; });
            }
            s0 = o0 >= ju0 ? o0 - ju0 : 0;
            const uint64_t s1 = o1 >= ju1 ? o1 - ju1 : 0;
            // survivor_k's predicate: k == R or rlist[k] - k > s, over k in [lo, R]
            auto gone = [&](uint64_t s_) {
                return [=](uint64_t k) { return k >= R || (int64_t)rlist[k] - (int64_t)k > (int64_t)s_; };
            };
            k0 = wave_partition_point(0, R, gone(s0));
            k1 = wave_partition_point(k0, R, gone(s1));
        }
        if (t == 0) {
            prm[0] = o1 - o0; prm[1] = ju0; prm[2] = ju1; prm[3] = s0; prm[4] = k0; prm[5] = k1;
        }
    }
    for (uint32_t q = t; q < MT; q += 256) src[q] = -1;
    __syncthreads();
    const uint32_t nrows = (uint32_t)prm[0];
    const uint64_t ju0 = prm[1], ju1 = prm[2], s0 = prm[3], k0 = prm[4], k1 = prm[5];
    for (uint64_t u = ju0 + t; u < ju1; u += 256) {
        const uint64_t p = (uint64_t)upos[u] - o0;
        const uint32_t j = usrc[u];
        if (p < nrows && j < m) src[p] = -2 - (int32_t)j;
    }
    __syncthreads();
    // free slots (MT / 256 per lane) in order -> the tile's A survivors
    constexpr int SPL = MT / 256;
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < SPL; k++) cnt += (SPL * t + k < nrows && src[SPL * t + k] == -1) ? 1u : 0u;
    uint32_t x = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((t & 63) >= (uint32_t)o) x += y;
    }
    if ((t & 63) == 63) wsum[t >> 6] = x;
    __syncthreads();
    uint32_t q = x - cnt;
    for (uint32_t w = 0; w < (t >> 6); w++) q += wsum[w];
#pragma unroll
    for (int k = 0; k < SPL; k++) {
        const uint32_t slot = SPL * t + k;
        if (slot < nrows && src[slot] == -1) {
            const uint64_t sidx = s0 + q;
            const uint64_t i = sidx + survivor_k(rlist, R, k0, k1, sidx);
            if (i < nA) src[slot] = (int32_t)i;
            q++;
        }
    }
    __syncthreads();
    // copy + block sums: lane t moves row b * 256 + t of each of the tile's 4 blocks
    for (int b = 0; b < MT / 256; b++) {
        const uint32_t o = b * 256 + t;
        uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int32_t c = 0;
        const int32_t sr = o < nrows ? src[o] : -1;
        if (sr != -1) {
            const bool fromA = sr >= 0;
            const uint64_t r = fromA ? (uint64_t)sr : (uint64_t)(-2 - sr);
            const uint8_t *ks = (fromA ? akeys : bkeys) + r * KL;
            const uint64_t od = o0 + o;
            copy_bytes<KL>(okeys + od * KL, ks);
            // the merged run's search samples (k_sample's, without re-reading the run), staged in
            // LDS and written as whole lines after the copy
            if (osmp2 && (o % SMP2_STRIDE) == 0) smp_t[o / SMP2_STRIDE] = key_digit<KK, KL>(ks, 0);
            if constexpr (HEAP) {
                const uint32_t slot = fromA ? reinterpret_cast<const uint32_t *>(apay)[r] : heap_base + (uint32_t)r;
                reinterpret_cast<uint32_t *>(opay)[od] = slot;
            } else {
                const V *ps = reinterpret_cast<const V *>((fromA ? apay : bpay) + r * P);
                V pv[NV];
#pragma unroll
                for (int k = 0; k < NV; k++) pv[k] = ps[k];
                V *pd = reinterpret_cast<V *>(opay + od * P);
#pragma unroll
                for (int k = 0; k < NV; k++) pd[k] = pv[k];
                uint32_t w[P / 4];
#pragma unroll
                for (int k = 0; k < NV; k++) words_of(pv[k], w + k * (int)(sizeof(V) / 4));
#pragma unroll
                for (int k = 0; k < 8; k++) h[k] = w[k];
                if constexpr (COUNTS) {
                    static_assert(P == sizeof(DeltaRec), "delta payload");
                    const uint32_t f = w[9];  // DeltaRec::flags
                    c = ((f & DeltaRec::LIVE) ? 1 : 0) - ((f & DeltaRec::IN_BASE) ? 1 : 0);
                }
            }
        }
        if constexpr (HEAP) continue;  // no sums: k_delta_sums forms them when a question needs them
        const uint64_t blk = o0 / 256 + b;
        uint32_t f8[8];
        block_sum_fps256(h, tile, f8);
        if (t == 0 && blk < nbk) store_sum(obs, blk, f8);
        if constexpr (COUNTS) {
            int32_t y = c;
#pragma unroll
            for (int o2 = 1; o2 < 64; o2 <<= 1) {
                const int32_t z = __shfl_up(y, o2, 64);
                if ((t & 63) >= (uint32_t)o2) y += z;
            }
            __syncthreads();
            if ((t & 63) == 63) wsum[t >> 6] = (uint32_t)y;
            __syncthreads();
            int32_t before = 0;
            for (uint32_t w = 0; w < (t >> 6); w++) before += (int32_t)wsum[w];
            if (o < nrows) oinb[o0 + o] = (int16_t)(before + y);
            if (t == 255 && blk < nbk) ocnt[blk] = before + y;
        }
    }
    if (osmp2) {
        __syncthreads();
        constexpr uint32_t R = SMP_STRIDE / SMP2_STRIDE;
        for (uint32_t e = t; e < MT / SMP2_STRIDE; e += 256) {
            if (e * SMP2_STRIDE >= nrows) break;
            osmp2[o0 / SMP2_STRIDE + e] = smp_t[e];
            if (osmp && e % R == 0) osmp[o0 / SMP_STRIDE + e / R] = smp_t[e];
        }
    }
}

template <int KK, int KL, int P, bool COUNTS, bool HEAP = false>
hipError_t merge_kernel_t(const uint8_t *akeys, const uint8_t *apay, uint64_t nA, const uint8_t *bkeys,
                          const uint8_t *bpay, uint64_t m, const uint32_t *upos, const uint32_t *usrc,
                          const uint32_t *rlist, const uint64_t *counts, uint8_t *okeys, uint8_t *opay, uint8_t *obs,
                          int32_t *ocnt, int16_t *oinb, uint64_t nbk, uint64_t *osmp, uint64_t *osmp2, hipStream_t st,
                          const uint8_t *heap = nullptr, uint32_t heap_base = 0, const uint32_t *tileU = nullptr) {
    const uint64_t tiles = (nA + m + MT - 1) / MT;
    if (tiles)
        hipLaunchKernelGGL((k_merge_run<KK, KL, P, COUNTS, HEAP>), dim3((uint32_t)tiles), dim3(256), 0, st, akeys,
                           apay, nA, bkeys, bpay, m, upos, usrc, rlist, counts, okeys, opay, obs, ocnt, oinb, nbk, osmp,
                           osmp2, heap, heap_base, tileU);
    return hipGetLastError();
}

// the merge kernel alone, for lists and counts made by the caller: payload 32 = fingerprint rows
// (the base run), payload 4 with a heap = slot rows (the delta run)
hipError_t launch_merge_kernel(int kk, int kl, int payload, const uint8_t *akeys, const uint8_t *apay, uint64_t nA,
                               const uint8_t *bkeys, const uint8_t *bpay, uint64_t m, const uint32_t *upos,
                               const uint32_t *usrc, const uint32_t *rlist, const uint64_t *counts, uint8_t *okeys,
                               uint8_t *opay, uint8_t *obs, int32_t *ocnt, int16_t *oinb, uint64_t nbk,
                               uint64_t *osmp, uint64_t *osmp2, hipStream_t st, const uint8_t *heap = nullptr,
                               uint32_t heap_base = 0, const uint32_t *tileU = nullptr) {
    if (osmp && !osmp2) return hipErrorInvalidValue;
#define RH_MK(KKV, KLV)                                                                                            \
    if (kk == KKV && kl == KLV) {                                                                                  \
        if (payload == 32)                                                                                         \
            return merge_kernel_t<KKV, KLV, 32, false>(akeys, apay, nA, bkeys, bpay, m, upos, usrc, rlist, counts,  \
                                                       okeys, opay, obs, ocnt, oinb, nbk, osmp, osmp2, st,         \
                                                       nullptr, 0, tileU);                                         \
        if (payload == 4 && heap)                                                                                  \
            return merge_kernel_t<KKV, KLV, 4, true, true>(akeys, apay, nA, bkeys, bpay, m, upos, usrc, rlist,     \
                                                           counts, okeys, opay, obs, ocnt, oinb, nbk, osmp, osmp2,  \
                                                           st, heap, heap_base, tileU);                            \
    }
    RH_MK(KEY_U32, 4) RH_MK(KEY_U64, 8) RH_MK(KEY_BYTES, 8) RH_MK(KEY_BYTES, 16) RH_MK(KEY_BYTES, 32)
#undef RH_MK
    return hipErrorInvalidValue;
}

// ---- host-side drivers --------------------------------------------------------------------------


template <int KK, int KL>
struct KeyOps final : StoreKeyOps {
    static constexpr int D = KK == KEY_BYTES ? KL / 8 : 1;
    static constexpr int BITS = KK == KEY_U32 ? 32 : 64;

    hipError_t sort_batch(const uint8_t *keys, const uint8_t *fps, const uint8_t *ops, uint64_t m, Scratch &s,
                          uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *flags, bool full,
                          hipStream_t st, uint32_t *pos, const uint64_t *pre_part, uint32_t pre_npart,
                          uint32_t *s2o) override {
        hipError_t e;
        if (!fps == !pos) return hipErrorInvalidValue;  // exactly one of: gather fps, emit positions
        uint32_t *perm = s.u32(0, m), *perm2 = s.u32(1, m);
        uint64_t *dig = s.u64(0, m), *dig2 = s.u64(1, m);
        if (s.err) return s.err;
        auto pass = [&](int d) -> hipError_t {
            hipError_t e2;
            hipLaunchKernelGGL((k_digit<KK, KL>), g1(m), dim3(256), 0, st, keys, perm, m, d, dig);
            size_t tb = 0;
            if ((e2 = rocprim::radix_sort_pairs(nullptr, tb, dig, dig2, perm, perm2, m, 0, BITS, st))) return e2;
            void *tmp = s.bytes(tb);
            if (s.err) return s.err;
            if ((e2 = rocprim::radix_sort_pairs(tmp, tb, dig, dig2, perm, perm2, m, 0, BITS, st))) return e2;
            std::swap(perm, perm2);
            return hipSuccess;
        };
        if (!full && m <= CS_MAX_M)
            return sort_batch_buckets(keys, fps, ops, m, s, skeys, sfps, sops, flags, st, pos, pre_part, pre_npart,
                                      pos ? s2o : nullptr);
        if ((e = hipMemsetAsync(flags, 0, 4, st))) return e;
        hipLaunchKernelGGL(k_iota, g1(m), dim3(256), 0, st, perm, m);
        // multi-digit keys: the most significant digit alone orders random and spread keys
        // (k_gather reports a tie); the LSD sort (least significant digit first, stable passes)
        // is the fallback
        const int lo_digit = (full || D == 1) ? D - 1 : 0;
        for (int d = lo_digit; d >= 0; d--)
            if ((e = pass(d))) return e;
        hipLaunchKernelGGL((k_gather<KK, KL>), g1(m), dim3(256), 0, st, keys, fps, ops, perm, m, skeys, sfps, sops,
                           pos, flags, (full || D == 1) ? 0 : 1);
        return hipGetLastError();
    }

    hipError_t sort_batch_buckets(const uint8_t *keys, const uint8_t *fps, const uint8_t *ops, uint64_t m, Scratch &s,
                                  uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *flags, hipStream_t st,
                                  uint32_t *pos, const uint64_t *pre_part, uint32_t pre_npart, uint32_t *s2o) {
        uint32_t cb = 0;
        while ((1ull << cb) * 1024 < m) cb++;  // ~1,000 keys per coarse bucket
        const uint32_t C = 1u << cb, nwg = (uint32_t)((m + CS_TILE - 1) / CS_TILE), bbits = cb + CS_FINE_BITS;
        uint64_t *part = s.u64(2, 2ull * nwg + 3);
        uint8_t *okey = reinterpret_cast<uint8_t *>(s.u64(0, (m * KL + 7) / 8));
        uint32_t *hist = s.u32(15, (uint64_t)nwg * C), *idx = s.u32(0, m), *total = s.u32(1, C);
        uint32_t *start = s.u32(2, C);
        if (s.err) return s.err;
        uint64_t *params = part + 2ull * nwg;
        uint32_t *ticket = reinterpret_cast<uint32_t *>(part + 2ull * nwg + 2);
        // the digit min / max partials: precomputed (k_lift_search of the previous batch) or here
        const uint64_t *mm = pre_part ? pre_part : part;
        const uint32_t npart = pre_part ? pre_npart : nwg;
        if (!pre_part) hipLaunchKernelGGL((k_cs_minmax<KK, KL>), dim3(nwg), dim3(CS_WG), 0, st, keys, m, part);
        hipLaunchKernelGGL((k_cs_hist<KK, KL>), dim3(nwg), dim3(CS_WG), 0, st, keys, m, mm, npart, bbits, C, hist, flags,
                           ticket);
        hipLaunchKernelGGL(k_cs_colscan, dim3((C + 63) / 64), dim3(1024), 0, st, hist, nwg, C, total, ticket, start,
                           flags, mm, npart, bbits, params);
        // the slots' input rows only where something needs them (the ops, the fingerprints of the
        // gather mode, a stable order of equal keys: always there when ops are)
        uint32_t *sidx = (ops || fps || !s2o) ? idx : nullptr;
        hipLaunchKernelGGL((k_cs_scatter<KK, KL>), dim3(nwg), dim3(CS_WG), 0, st, keys, m, params, C, hist, start,
                           okey, sidx, s2o ? pos : nullptr);
        hipLaunchKernelGGL((k_cs_sort<KK, KL>), dim3(C), dim3(256), 0, st, okey, sidx, start, total, params, fps, ops,
                           skeys, sfps, sops, s2o ? nullptr : pos, flags, s2o);
        return hipGetLastError();
    }

    hipError_t search(const uint8_t *keys, uint64_t n, const uint8_t *q, uint64_t m, uint32_t *rank, uint8_t *present,
                      hipStream_t st) override {
        if (m == 0) return hipSuccess;
        hipLaunchKernelGGL((k_search<KK, KL>), g1(m), dim3(256), 0, st, keys, n, q, m, rank, present);
        return hipGetLastError();
    }

    hipError_t sample(const uint8_t *keys, uint64_t n, uint64_t *smp, uint64_t *smp2, hipStream_t st) override {
        const uint64_t ns = (n + SMP_STRIDE - 1) / SMP_STRIDE, ns2 = (n + SMP2_STRIDE - 1) / SMP2_STRIDE;
        if (ns == 0) return hipSuccess;
        hipLaunchKernelGGL((k_sample<KK, KL>), g1(ns), dim3(256), 0, st, keys, n, SMP_STRIDE, smp);
        if (smp2) hipLaunchKernelGGL((k_sample<KK, KL>), g1(ns2), dim3(256), 0, st, keys, n, SMP2_STRIDE, smp2);
        return hipGetLastError();
    }

    hipError_t search_sampled(const uint8_t *keys, uint64_t n, const uint64_t *smp, const uint64_t *smp2,
                              const uint8_t *q, uint64_t m, uint32_t *rank, uint8_t *present, hipStream_t st,
                              SearchTable tb) override {
        if (m == 0) return hipSuccess;
        if (!smp2 || n == 0) tb = SearchTable{};
        hipLaunchKernelGGL((k_search_sampled<KK, KL>), g1(m), dim3(256), 0, st, keys, n, smp, smp2, tb, q, m, rank,
                           present);
        return hipGetLastError();
    }

    hipError_t check_sorted(const uint8_t *keys, uint64_t n, uint32_t *bad, hipStream_t st) override {
        if (n < 2) return hipSuccess;
        hipLaunchKernelGGL((k_check_sorted<KK, KL>), g1(n), dim3(256), 0, st, keys, n, bad);
        return hipGetLastError();
    }

    hipError_t dedup_last(const uint8_t *keys, const uint8_t *fps, uint64_t n, Scratch &s, uint8_t *okeys,
                          uint8_t *ofps, uint64_t *counts, hipStream_t st) override {
        if (n == 0) return hipMemsetAsync(counts, 0, 8, st);
        hipError_t e;
        uint32_t *keep = s.u32(11, n), *pos = s.u32(12, n);
        if (s.err) return s.err;
        hipLaunchKernelGGL((k_last_flags<KK, KL>), g1(n), dim3(256), 0, st, keys, n, keep);
        size_t tb = 0;
        if ((e = rocprim::exclusive_scan(nullptr, tb, keep, pos, 0u, n, rocprim::plus<uint32_t>(), st))) return e;
        void *tmp = s.bytes(tb);
        if (s.err) return s.err;
        if ((e = rocprim::exclusive_scan(tmp, tb, keep, pos, 0u, n, rocprim::plus<uint32_t>(), st))) return e;
        hipLaunchKernelGGL((k_dedup_scatter<KL>), g1(n), dim3(256), 0, st, keys, fps, keep, pos, n, okeys, ofps, counts);
        return hipGetLastError();
    }

    hipError_t bounds(const uint8_t *keys, uint64_t n, const uint8_t *lo_key, int lo_kind, const uint8_t *hi_key,
                      int hi_kind, uint64_t *qlo, uint64_t *qhi, hipStream_t st) override {
        hipLaunchKernelGGL((k_bounds<KK, KL>), dim3(1), dim3(64), 0, st, keys, n, lo_key, lo_kind, hi_key, hi_kind, qlo,
                           qhi);
        return hipGetLastError();
    }

    hipError_t keep_last_rows(const uint8_t *skeys, const uint32_t *pos, const uint32_t *s2o, uint64_t m,
                              uint32_t *keep, hipStream_t st) override {
        hipLaunchKernelGGL((k_keep_last<KK, KL>), g1(m + 1), dim3(256), 0, st, skeys, pos, s2o, m, keep);
        return hipGetLastError();
    }

    hipError_t sample_stride(const uint8_t *keys, uint64_t n, uint64_t stride, uint64_t *smp, hipStream_t st) override {
        const uint64_t ns = (n + stride - 1) / stride;
        if (ns == 0) return hipSuccess;
        hipLaunchKernelGGL((k_sample<KK, KL>), g1(ns), dim3(256), 0, st, keys, n, stride, smp);
        return hipGetLastError();
    }

    hipError_t query_tiny(const QueryTiny &a, hipStream_t st) override {
        if (a.m > QUERY_TINY || (a.mode == 2 && a.m != 1)) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_query_tiny<KK, KL>), dim3(1), dim3(1024), 0, st, a);
        return hipGetLastError();
    }

    hipError_t round_tiny(const RoundTiny &a, hipStream_t st) override {
        if (a.r == 0 || a.r > ROUND_TINY) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_round_tiny<KK, KL>), dim3(1), dim3(ROUND_TINY_THREADS), 0, st, a);
        return hipGetLastError();
    }

    int compare_keys_host(const uint8_t *a, const uint8_t *b) const override {
        if constexpr (KK == KEY_U32) {
            uint32_t x, y;
            memcpy(&x, a, 4); memcpy(&y, b, 4);
            return (x > y) - (x < y);
        } else if constexpr (KK == KEY_U64) {
            uint64_t x, y;
            memcpy(&x, a, 8); memcpy(&y, b, 8);
            return (x > y) - (x < y);
        } else {
            return memcmp(a, b, KL);
        }
    }
};

StoreKeyOps *store_key_ops(int kk, int kl) {
    static KeyOps<KEY_U32, 4> u32;
    static KeyOps<KEY_U64, 8> u64;
    static KeyOps<KEY_BYTES, 16> b16;
    static KeyOps<KEY_BYTES, 32> b32;
    static KeyOps<KEY_BYTES, 8> b8;
    if (kk == KEY_U32 && kl == 4) return &u32;
    if (kk == KEY_U64 && kl == 8) return &u64;
    if (kk == KEY_BYTES && kl == 16) return &b16;
    if (kk == KEY_BYTES && kl == 32) return &b32;
    if (kk == KEY_BYTES && kl == 8) return &b8;
    return nullptr;
}

// ---- delta launchers (key-type independent) -------------------------------------------------

// k_tile_bounds for a merge of m rows into a run (nA + m rows at most), into scratch slot u32(8);
// nullptr (the merge searches its bounds itself) when switched off for an A/B
static uint32_t *merge_tile_bounds(const uint32_t *upos, const uint64_t *counts, uint64_t m, uint64_t rows, Scratch &s,
                                   hipStream_t st) {
    const char *sw = getenv("RSOS_HIP_TILE_SEARCH");  // read per merge: a test toggles it
    if (sw && *sw == '1') return nullptr;
    const uint64_t tiles = (rows + MT - 1) / MT;
    // a thread fills the tiles between two upserts: with few upserts per tile on average (a tiny
    // batch into a large run) the tiles search their bounds themselves
    if (tiles > 16 * (m + 1)) return nullptr;
    uint32_t *tileU = s.u32(8, tiles + 1);
    if (!tileU) return nullptr;
    hipLaunchKernelGGL(k_tile_bounds, g1(m + 1), dim3(256), 0, st, upos, counts, m, tiles, tileU);
    return tileU;
}

hipError_t launch_delta_apply(int kk, int kl, const uint8_t *sfps, const uint8_t *sops, uint64_t m,
                              const uint32_t *rank_b, const uint8_t *present_b, const uint8_t *base_fps,
                              const uint32_t *rank_d, const uint8_t *present_d, const uint8_t *dkeys,
                              const uint32_t *dslot, uint64_t nd, uint8_t *heap, uint64_t heap_base,
                              const uint8_t *skeys, uint8_t *dops, uint64_t *counts3, Scratch &s, uint8_t *okeys,
                              uint32_t *oslot, uint8_t *obs, int32_t *ocnt, int16_t *oinb, uint64_t nbk,
                              uint64_t *mcnt, uint64_t *out3, uint64_t *osmp, uint64_t *osmp2, uint64_t *dtot,
                              int64_t *dcnt, hipStream_t st) {
    if (m == 0 || heap_base + m >= (1ull << 32)) return hipErrorInvalidValue;
    const uint64_t G = (m + DB_WG - 1) / DB_WG;
    uint32_t *part = s.u32(13, G * DB_PARTS), *off = s.u32(6, 2 * G);
    uint64_t *dsum = s.u64(7, 4 * G);
    uint32_t *upos = s.u32(3, m + 1), *usrc = s.u32(4, m + 1), *rlist = s.u32(5, m + 1);
    if (s.err) return s.err;
    // the batch's records go straight to the heap, at slots heap_base + j
    uint8_t *bpay = heap + heap_base * sizeof(DeltaRec);
    hipLaunchKernelGGL(k_delta_build, dim3((uint32_t)G), dim3(DB_WG), 0, st, sfps, sops, m, rank_b, present_b,
                       base_fps, rank_d, present_d, dslot, heap, bpay, dops, part, dsum);
    hipLaunchKernelGGL(k_delta_parts, dim3(1), dim3(DP_WG), 0, st, part, G, counts3, mcnt, out3, off, dsum, dtot, dcnt);
    hipLaunchKernelGGL(k_delta_lists, dim3((uint32_t)G), dim3(DB_WG), 0, st, dops, present_d, rank_d, off, m, upos,
                       usrc, rlist);
    uint32_t *tileU = merge_tile_bounds(upos, mcnt, m, nd + m, s, st);
    if (s.err) return s.err;
    return launch_merge_kernel(kk, kl, 4, dkeys, reinterpret_cast<const uint8_t *>(dslot), nd, skeys, nullptr, m, upos,
                               usrc, rlist, mcnt, okeys, reinterpret_cast<uint8_t *>(oslot), nullptr, nullptr, nullptr,
                               nbk, osmp, osmp2, st, heap, (uint32_t)heap_base, tileU);
}

hipError_t launch_delta_merge(int kk, int kl, const uint8_t *dkeys, const uint32_t *dslot, uint64_t nd,
                              const uint8_t *skeys, uint64_t m, const uint32_t *upos, const uint32_t *usrc,
                              const uint32_t *rlist, const uint64_t *mcnt, uint8_t *okeys, uint32_t *oslot,
                              uint64_t nbk, uint64_t *osmp, uint64_t *osmp2, const uint8_t *heap, uint64_t heap_base,
                              hipStream_t st) {
    if (m == 0 || heap_base + m >= (1ull << 32)) return hipErrorInvalidValue;
    // a few rows into the run: every tile finds its bounds in the short lists itself
    return launch_merge_kernel(kk, kl, 4, dkeys, reinterpret_cast<const uint8_t *>(dslot), nd, skeys, nullptr, m, upos,
                               usrc, rlist, mcnt, okeys, reinterpret_cast<uint8_t *>(oslot), nullptr, nullptr, nullptr,
                               nbk, osmp, osmp2, st, heap, (uint32_t)heap_base, nullptr);
}

// The host tier's run copy (host_tier.hpp HostTier::Run): delta row i's DeltaRec, read through its
// slot, as columns -- the contribution (32 B), the count delta live - in_base (cnt[n] = 0 closes
// the array for the exclusive scan that follows), the flags and the base rank
// One workgroup per 256-entry block: with bsums, the block's contribution sum too (the pass a
// k_reduce over the written contributions took).
__global__ __launch_bounds__(256) void k_tier_run(const uint32_t *slot, const uint8_t *heap, uint64_t n,
                                                  uint8_t *contrib, uint32_t *cnt, uint8_t *flags, uint32_t *brank,
                                                  uint8_t *bsums) {
    __shared__ SumTile tile;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (i < n) {
        const DeltaRec *r = reinterpret_cast<const DeltaRec *>(heap) + slot[i];
        const uint4 *c = reinterpret_cast<const uint4 *>(r->contrib);
        const uint4 a = c[0], b = c[1];
        reinterpret_cast<uint4 *>(contrib + 32 * i)[0] = a;
        reinterpret_cast<uint4 *>(contrib + 32 * i)[1] = b;
        h[0] = a.x, h[1] = a.y, h[2] = a.z, h[3] = a.w, h[4] = b.x, h[5] = b.y, h[6] = b.z, h[7] = b.w;
        const uint32_t f = r->flags;
        cnt[i] = (uint32_t)(((f & DeltaRec::LIVE) ? 1 : 0) - ((f & DeltaRec::IN_BASE) ? 1 : 0));
        flags[i] = (uint8_t)f;
        brank[i] = r->brank;
    } else if (i == n) {
        cnt[n] = 0;
    }
    if (!bsums || (uint64_t)blockIdx.x * 256 >= n) return;  // uniform
    uint32_t sum[8];
    block_sum_fps256(h, tile, sum);  // lanes past the end hold zero
    if (threadIdx.x == 0) store_sum(bsums, blockIdx.x, sum);
}

hipError_t launch_tier_run(const uint32_t *slot, const uint8_t *heap, uint64_t n, uint8_t *contrib, uint32_t *cnt,
                           uint8_t *flags, uint32_t *brank, hipStream_t st, uint8_t *bsums) {
    hipLaunchKernelGGL(k_tier_run, g1(n + 1), dim3(256), 0, st, slot, heap, n, contrib, cnt, flags, brank, bsums);
    return hipGetLastError();
}

// select's index over the run copy: G(64 k) = live keys <= entry 64 k = brank + count prefix + live
__global__ void k_tier_gsamp(const uint32_t *brank, const uint32_t *cntp, const uint8_t *flags, uint64_t n,
                             uint64_t *gsamp) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, j = k * 64;
    if (j >= n) return;
    gsamp[k] = (uint64_t)((int64_t)brank[j] + (int32_t)cntp[j] + ((flags[j] & DeltaRec::LIVE) ? 1 : 0));
}

hipError_t launch_tier_gsamp(const uint32_t *brank, const uint32_t *cntp, const uint8_t *flags, uint64_t n,
                             uint64_t *gsamp, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_tier_gsamp, g1((n + 63) / 64), dim3(256), 0, st, brank, cntp, flags, n, gsamp);
    return hipGetLastError();
}

// The delta run's columns for a short run in one launch of one workgroup (1,024 lanes, four
// consecutive entries each): the entries as k_tier_run reads them; one workgroup scan gives the
// contributions' row prefix and the count deltas' prefix; then the block sums and block /
// super-block prefixes are differences and entries of the row prefix, and G(64 k) as
// k_tier_gsamp.  A run of one batch's few rows (a 1-row write before a question) paid ~70 us of
// host launches and in-stream gaps for the eight kernels this replaces.
constexpr uint32_t RUNCOL_THREADS = 1024, RUNCOL_PER = 4;
static_assert(RUNCOL_SMALL < (uint64_t)RUNCOL_THREADS * RUNCOL_PER, "k_run_columns_small: n + 1 entries");
__global__ __launch_bounds__(RUNCOL_THREADS) void k_run_columns_small(const uint32_t *slot, const uint8_t *heap,
                                                                       uint64_t n, RunCols o) {
    __shared__ uint64_t wacc[RUNCOL_THREADS / 64][8];
    __shared__ int32_t wcnt[RUNCOL_THREADS / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    int32_t c[RUNCOL_PER];
    Acc s;
    acc_zero(s);
    int32_t cs = 0;
#pragma unroll
    for (uint32_t q = 0; q < RUNCOL_PER; q++) {
        const uint64_t i = (uint64_t)t * RUNCOL_PER + q;
        c[q] = 0;
        if (i < n) {
            const DeltaRec *r = reinterpret_cast<const DeltaRec *>(heap) + slot[i];
            const uint4 *cp = reinterpret_cast<const uint4 *>(r->contrib);
            const uint4 a = cp[0], b = cp[1];
            const uint32_t f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            reinterpret_cast<uint4 *>(o.contrib + 32 * i)[0] = a;
            reinterpret_cast<uint4 *>(o.contrib + 32 * i)[1] = b;
            const uint32_t fl = r->flags;
            c[q] = ((fl & DeltaRec::LIVE) ? 1 : 0) - ((fl & DeltaRec::IN_BASE) ? 1 : 0);
            o.cnt[i] = (uint32_t)c[q];
            o.flags[i] = (uint8_t)fl;
            o.brank[i] = r->brank;
            acc_add_fp(s, f);
            cs += c[q];
        } else if (i == n) {
            o.cnt[n] = 0;
        }
    }
    // inclusive scans of the lanes' sums in the wave, then across the waves
    Acc inc = s;
    int32_t ic = cs;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint64_t y = __shfl_up((unsigned long long)inc.l[k], d);
            if (lane >= (uint32_t)d) inc.l[k] += y;
        }
        const int32_t y = __shfl_up(ic, d);
        if (lane >= (uint32_t)d) ic += y;
    }
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < 8; k++) wacc[w][k] = inc.l[k];
        wcnt[w] = ic;
    }
    __syncthreads();
    Acc e;
    int32_t ec = ic - cs;
#pragma unroll
    for (int k = 0; k < 8; k++) e.l[k] = inc.l[k] - s.l[k];
    for (uint32_t v = 0; v < w; v++) {
#pragma unroll
        for (int k = 0; k < 8; k++) e.l[k] += wacc[v][k];
        ec += wcnt[v];
    }
#pragma unroll
    for (uint32_t q = 0; q < RUNCOL_PER; q++) {
        const uint64_t i = (uint64_t)t * RUNCOL_PER + q;
        if (i <= n) {
            uint32_t g[8];
            acc_normalise(e, g);
            store_sum(o.pre, i, g);
            o.cntp[i] = (uint32_t)ec;
        }
        if (i < n) {  // this lane's own contribution, written above (read back: no registers held over the scan)
            uint32_t f[8];
            load_fp(o.contrib, i, f);
            acc_add_fp(e, f), ec += c[q];
        }
    }
    __syncthreads();  // the row prefix is written (the workgroup's own global stores)
    const uint64_t nbk = (n + 255) / 256;
    for (uint64_t k = t; k <= nbk; k += RUNCOL_THREADS) {
        const uint64_t lo = k * 256 < n ? k * 256 : n, hi = (k + 1) * 256 < n ? (k + 1) * 256 : n;
        uint32_t a[8], b[8];
        load_fp(o.pre, lo, b);
        store_sum(o.bpre, k, b);  // bpre[nbk] = pre[n], the total
        if (k < nbk) {
            load_fp(o.pre, hi, a);
            sub256(a, b);
            store_sum(o.bsums, k, a);
        }
    }
    if (t == 0) {  // one super-block (n < 65536): its sum and prefix
        uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tot[8];
        load_fp(o.pre, n, tot);
        if (n) store_sum(o.ssums, 0, tot);
        store_sum(o.spre, 0, z);
        store_sum(o.spre, 1, tot);
    }
    for (uint64_t k = t; k * 64 < n; k += RUNCOL_THREADS) {
        const uint64_t j = k * 64;
        o.gsamp[k] = (uint64_t)((int64_t)o.brank[j] + (int32_t)o.cntp[j] + ((o.flags[j] & DeltaRec::LIVE) ? 1 : 0));
    }
}

hipError_t launch_run_columns_small(const uint32_t *slot, const uint8_t *heap, uint64_t n, const RunCols &o,
                                    hipStream_t st) {
    if (n == 0 || n > RUNCOL_SMALL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_run_columns_small, dim3(1), dim3(RUNCOL_THREADS), 0, st, slot, heap, n, o);
    return hipGetLastError();
}

hipError_t launch_compact_rows(const uint8_t *src, uint32_t row_bytes, const uint32_t *keep, const uint32_t *dst,
                               uint64_t m, uint8_t *out, hipStream_t st) {
    if (m == 0 || row_bytes == 0 || !src) return hipSuccess;
    hipLaunchKernelGGL(k_compact_rows, g1(m), dim3(256), 0, st, src, row_bytes, keep, dst, m, out);
    return hipGetLastError();
}

hipError_t launch_exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, Scratch &s, hipStream_t st) {
    size_t tb = 0;
    hipError_t e;
    if ((e = rocprim::exclusive_scan(nullptr, tb, in, out, 0u, n, rocprim::plus<uint32_t>(), st))) return e;
    void *tmp = s.bytes(tb);
    if (s.err) return s.err;
    return rocprim::exclusive_scan(tmp, tb, in, out, 0u, n, rocprim::plus<uint32_t>(), st);
}

hipError_t launch_compact(int kk, int kl, const uint8_t *bkeys, const uint8_t *bfps, uint64_t nb, const uint8_t *dkeys,
                          const uint32_t *dslot, const uint8_t *heap, uint64_t nd, Scratch &s, uint8_t *cfps,
                          uint8_t *cops, uint8_t *okeys, uint8_t *ofps,
                          uint8_t *obs, uint64_t nbk, uint64_t *mcnt, uint64_t *osmp, uint64_t *osmp2,
                          hipStream_t st) {
    if (nd == 0) return hipErrorInvalidValue;
    const uint64_t G = (nd + DB_WG - 1) / DB_WG;
    uint32_t *part = s.u32(13, G * DB_PARTS), *off = s.u32(6, 2 * G), *crank = s.u32(14, nd);
    uint32_t *upos = s.u32(3, nd + 1), *usrc = s.u32(4, nd + 1), *rlist = s.u32(5, nd + 1);
    uint8_t *cpres = s.u8(4, nd);
    if (s.err) return s.err;
    hipLaunchKernelGGL(k_delta_cur, dim3((uint32_t)G), dim3(DB_WG), 0, st, dslot, heap, nd, bfps, cfps, cops, crank,
                       cpres, part);
    hipLaunchKernelGGL(k_delta_parts, dim3(1), dim3(DP_WG), 0, st, part, G, nullptr, mcnt, nullptr, off, nullptr,
                       nullptr, nullptr);
    hipLaunchKernelGGL(k_delta_lists, dim3((uint32_t)G), dim3(DB_WG), 0, st, cops, cpres, crank, off, nd, upos, usrc,
                       rlist);
    uint32_t *tileU = merge_tile_bounds(upos, mcnt, nd, nb + nd, s, st);
    if (s.err) return s.err;
    return launch_merge_kernel(kk, kl, 32, bkeys, bfps, nb, dkeys, cfps, nd, upos, usrc, rlist, mcnt, okeys, ofps, obs,
                               nullptr, nullptr, nbk, osmp, osmp2, st, nullptr, 0, tileU);
}

hipError_t launch_agg_merge(const uint64_t *base_agg, const uint64_t *delta_agg, const uint64_t *dlo,
                            const uint64_t *dhi, CntPrefix cp, uint64_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_agg_merge, dim3(1), dim3(64), 0, st, base_agg, delta_agg, dlo, dhi, cp, out);
    return hipGetLastError();
}

hipError_t launch_resolve_bounds(const uint32_t *rank, const uint8_t *skind, const uint8_t *ekind, uint64_t r,
                                 uint64_t n, uint64_t *lo, uint64_t *hi, hipStream_t st) {
    if (r == 0) return hipSuccess;
    hipLaunchKernelGGL(k_resolve_bounds, g1(r), dim3(256), 0, st, rank, skind, ekind, r, n, lo, hi);
    return hipGetLastError();
}

uint32_t search_table_bits(uint64_t n, bool base) {
    const uint64_t ns2 = (n + SMP2_STRIDE - 1) / SMP2_STRIDE;
    // the base run: ~one sample per bucket (a table line, then one or two lines of keys: no
    // sample line); a delta run (rebuilt every batch): ~8 samples (one line of them) per bucket,
    // a table small enough to stay in the caches -- one sample per bucket there measured slower
    // (profiles/r03s2_c5_fine_dtab_ab.txt)
    const uint64_t per = base ? 1 : 8;
    const uint32_t cap = base ? 25 : 24;
    uint32_t b = 0;
    while ((1ull << b) * per < ns2 && b < cap) b++;
    return b;
}

hipError_t launch_search_table(const uint64_t *smp2, uint64_t n, uint32_t *tab, uint64_t *par, hipStream_t st,
                               bool base) {
    const uint64_t ns2 = (n + SMP2_STRIDE - 1) / SMP2_STRIDE;
    if (ns2 == 0) return hipSuccess;
    const uint32_t bits = search_table_bits(n, base);
    static std::atomic<uint64_t> builds{0};
    const uint64_t gen = ++builds;
    hipLaunchKernelGGL(k_search_table, g1(ns2 + 1), dim3(256), 0, st, smp2, ns2, bits, tab, par, gen);
    const uint64_t nt = 1ull << bits;
    // a small grid: without a long gap (the usual case) it only reads par[2] and exits (~1 us)
    hipLaunchKernelGGL(k_search_table_gaps, dim3((uint32_t)std::min<uint64_t>((nt + 1 + 255) / 256, 128)), dim3(256), 0,
                       st, smp2, ns2, bits, tab, (const uint64_t *)par, gen);
    return hipGetLastError();
}

hipError_t reserve_merge_scratch(Scratch &s, uint64_t plan, uint64_t batch, uint64_t base_rows) {
    // the slots the compaction (plan rows) and a batch (batch rows) take
    (void)s.u32(3, plan + 1), (void)s.u32(4, plan + 1), (void)s.u32(5, plan + 1);
    (void)s.u32(14, plan), (void)s.u8(4, plan);
    const uint64_t G = (std::max(plan, batch) + DB_WG - 1) / DB_WG;  // launch_delta_apply / launch_compact partials
    (void)s.u32(13, G * DB_PARTS), (void)s.u32(6, 2 * G), (void)s.u64(7, 4 * G);
    (void)s.u32(9, batch), (void)s.u32(10, batch), (void)s.u8(2, batch), (void)s.u8(3, batch);
    (void)s.i32(0, batch);  // the bucket sort's slot -> sorted row
    // merge_tile_bounds' tiles over a compaction's output (the base grows with every compaction:
    // a slot grown then frees the old one, and hipFree waits for every copy in flight)
    (void)s.u32(8, (std::max(base_rows, plan) + MT - 1) / MT + 1);
    // the library scans' temporary storage (one shared slot): a delta run's count scan
    // (run_columns, up to plan rows) and the u64 scans over up to a base
    size_t t32 = 0, t64 = 0;
    const uint64_t big = std::max(base_rows, plan) + 2;
    if (rocprim::exclusive_scan(nullptr, t32, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u, plan + 2,
                                rocprim::plus<uint32_t>(), (hipStream_t)0) != hipSuccess)
        t32 = 0;
    if (rocprim::exclusive_scan(nullptr, t64, (const uint64_t *)nullptr, (uint64_t *)nullptr, (uint64_t)0, big,
                                rocprim::plus<uint64_t>(), (hipStream_t)0) != hipSuccess)
        t64 = 0;
    (void)hipGetLastError();
    if (std::max(t32, t64)) (void)s.bytes(std::max(t32, t64));
    return s.err;
}

hipError_t launch_exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, Scratch &s, hipStream_t st) {
    if (n == 0) return hipSuccess;
    size_t tb = 0;
    hipError_t e;
    if ((e = rocprim::exclusive_scan(nullptr, tb, in, out, (uint64_t)0, n, rocprim::plus<uint64_t>(), st))) return e;
    void *tmp = s.bytes(tb);
    if (s.err) return s.err;
    return rocprim::exclusive_scan(tmp, tb, in, out, (uint64_t)0, n, rocprim::plus<uint64_t>(), st);
}

hipError_t launch_gather_keys(const uint8_t *keys, uint32_t kl, const uint64_t *sel, uint64_t m, uint8_t *out,
                              hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_keys, g1(m * (kl / 4)), dim3(256), 0, st, keys, kl, sel, m, out);
    return hipGetLastError();
}

hipError_t launch_rank_merge(const uint32_t *rank_b, const uint32_t *rank_d, CntPrefix cp, uint64_t m,
                             uint64_t *out, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rank_merge, g1(m), dim3(256), 0, st, rank_b, rank_d, cp, m, out);
    return hipGetLastError();
}

}  // namespace rh
