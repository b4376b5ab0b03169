// store_kernels.hip -- device side of the GPU-resident RSOS store: key order, rank search,
// batch sort, the sorted-run merge, and the signed-delta run of the LSM layout.
//
// Store layout in HBM (rank order):
//   base  : keys[nB][KL] + fps[nB][32] + block sums [nB/256][32] + super sums [nB/65536][32]
//   delta : keys[nD][KL] + DeltaRec[nD] (48 B) + block / super sums of the contributions +
//           an inclusive prefix of the count deltas
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
// batch's DeltaRecs, merge them into the delta run (O(m + nD)); when the delta run passes
// nB / 8 it is merged into the base (O(nB)) -- amortised, and on demand before rank / select.
#include <type_traits>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "internal.hpp"
#include "store_kernels.hpp"

namespace rh {

// ---- key order ----------------------------------------------------------------------------

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

// ---- 256-bit helpers (the Fingerprint group, rsos/src/fingerprint.rs:145-173) ----------------

__device__ __forceinline__ void fp_load(const uint8_t *p, uint32_t f[8]) {
    const uint4 a = reinterpret_cast<const uint4 *>(p)[0], b = reinterpret_cast<const uint4 *>(p)[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void fp_store(uint8_t *p, const uint32_t f[8]) {
    reinterpret_cast<uint4 *>(p)[0] = make_uint4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<uint4 *>(p)[1] = make_uint4(f[4], f[5], f[6], f[7]);
}
__device__ __forceinline__ void fp_add(const uint32_t a[8], const uint32_t b[8], uint32_t o[8]) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)a[i] + b[i] + c;
        o[i] = (uint32_t)t;
        c = t >> 32;
    }
}
__device__ __forceinline__ void fp_sub(const uint32_t a[8], const uint32_t b[8], uint32_t o[8]) {
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)a[i] - b[i] - br;
        o[i] = (uint32_t)t;
        br = (t >> 63) & 1;  // borrow out
    }
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
                         uint64_t m, uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *flags, int msd_only) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t s = perm[j];
    copy_bytes<KL>(skeys + j * KL, keys + s * KL);
    copy_bytes<32>(sfps + 32 * j, fps + 32 * s);
    sops[j] = ops ? ops[s] : 0;
    if (j > 0) {
        const uint8_t *prev = keys + (uint64_t)perm[j - 1] * KL;
        if (key_cmp<KK, KL>(keys + s * KL, prev) == 0) atomicOr(flags, 1u);
        else if (msd_only && key_digit<KK, KL>(keys + s * KL, 0) == key_digit<KK, KL>(prev, 0)) atomicOr(flags, 2u);
    }
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

// ---- sorted-run merge (payload P bytes per row) ------------------------------------------

// classify: op 0 = upsert, 1 = delete.  INS = upsert of an absent key, DEL = delete of a
// present key; an upsert of a present key overwrites its payload; deleting an absent key is a
// no-op (FingerprintTreeMap::remove returns None).
__global__ void k_classify(const uint8_t *sops, const uint8_t *present, uint64_t m, uint32_t *ins, uint32_t *del) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const bool p = present[j], isdel = sops[j] != 0;
    ins[j] = (!isdel && !p) ? 1u : 0u;
    del[j] = (isdel && p) ? 1u : 0u;
}

// compact the ranks of inserts and deletes (both come out sorted: the batch is key-sorted)
__global__ void k_compact(const uint32_t *rank, const uint32_t *ins, const uint32_t *del, const uint32_t *cum_ins,
                          const uint32_t *cum_del, uint64_t m, uint32_t *ins_rank, uint32_t *del_rank) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    if (ins[j]) ins_rank[cum_ins[j]] = rank[j];
    if (del[j]) del_rank[cum_del[j]] = rank[j];
}

// counts[0] = inserts, counts[2] = deletes (counts[1], overwrites, by k_count_ovr)
__global__ void k_counts(const uint32_t *ins, const uint32_t *del, const uint32_t *cum_ins, const uint32_t *cum_del,
                         uint64_t m, uint64_t *counts) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    counts[0] = m ? (uint64_t)cum_ins[m - 1] + ins[m - 1] : 0;
    counts[1] = 0;
    counts[2] = m ? (uint64_t)cum_del[m - 1] + del[m - 1] : 0;
}

__global__ void k_count_ovr(const uint8_t *sops, const uint8_t *present, uint64_t m, unsigned long long *ovr) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool o = j < m && sops[j] == 0 && present[j];
    const unsigned long long b = __ballot(o);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(ovr, (unsigned long long)__popcll(b));
}

// Survivors move to i + #inserts(rank <= i) - #deletes(rank < i); deleted rows are skipped.
// One workgroup covers MOVE_TILE consecutive rows: one lane finds the slice of the (sorted)
// insert / delete rank lists that falls inside the tile, every row binary-searches only that
// slice for its shift (kept in LDS), and then the tile's key and payload bytes are copied as
// flat dword streams -- consecutive lanes read consecutive dwords of the source run and write
// consecutive dwords of the destination (a shifted memmove between insert / delete points).
// No n-sized scratch arrays, no n-sized scan.
constexpr int MOVE_TILE = 1024;

template <int B>
struct Unit {  // the widest access that divides a B-byte row
    static constexpr int SIZE = B % 16 == 0 ? 16 : B % 8 == 0 ? 8 : 4;
    using T = typename std::conditional<SIZE == 16, uint4, typename std::conditional<SIZE == 8, uint2, uint32_t>::type>::type;
};

// rows [i0, i0 + rows) of a B-byte-row run to row i + shift[i - i0] of dst, as a flat stream of
// the widest units (consecutive lanes: consecutive source units)
template <int B>
__device__ __forceinline__ void move_rows(const uint8_t *src, uint8_t *dst, uint64_t i0, uint32_t rows,
                                          const int32_t *shift, uint64_t cap) {
    using U = typename Unit<B>::T;
    constexpr int NU = B / Unit<B>::SIZE;
    const U *s = reinterpret_cast<const U *>(src) + i0 * NU;
    U *d = reinterpret_cast<U *>(dst);
    for (uint32_t w = threadIdx.x; w < rows * NU; w += blockDim.x) {
        const uint32_t r = w / NU;
        const int32_t sh = shift[r];
        const uint64_t pos = (uint64_t)((int64_t)(i0 + r) + sh);
        // pos < cap always holds for a key-sorted batch; the guard keeps a speculative merge of
        // a batch whose order was not final (re-run by the caller) inside the output run
        if (sh != INT32_MIN && pos < cap) d[pos * NU + (w - r * NU)] = s[w];
    }
}

template <int KL, int P>
__global__ __launch_bounds__(256) void k_move_tiles(const uint8_t *keys, const uint8_t *pay, uint64_t n,
                                                    const uint32_t *ins_rank, const uint32_t *del_rank,
                                                    const uint64_t *counts, uint8_t *okeys, uint8_t *opay,
                                                    uint64_t cap) {
    static_assert(KL % 4 == 0 && P % 4 == 0, "dword rows");
    __shared__ uint64_t bounds[4];
    __shared__ int32_t shift[MOVE_TILE];  // pos - i, or INT32_MIN for a deleted row
    const uint64_t i0 = (uint64_t)blockIdx.x * MOVE_TILE;
    if (threadIdx.x == 0) {
        const uint64_t a = counts[0], d = counts[2];  // list lengths: #inserts, #deletes
        bounds[0] = lower_bound_u32(ins_rank, 0, a, i0);              // inserts with rank < i0
        bounds[1] = lower_bound_u32(ins_rank, 0, a, i0 + MOVE_TILE);  // ... < tile end
        bounds[2] = lower_bound_u32(del_rank, 0, d, i0);
        bounds[3] = lower_bound_u32(del_rank, 0, d, i0 + MOVE_TILE);
    }
    __syncthreads();
    const uint64_t ia = bounds[0], ib = bounds[1], da = bounds[2], db = bounds[3];
    const uint32_t rows = (uint32_t)(n - i0 < (uint64_t)MOVE_TILE ? n - i0 : MOVE_TILE);
    for (uint32_t r = threadIdx.x; r < rows; r += 256) {
        const uint64_t i = i0 + r;
        const uint64_t ins_le = lower_bound_u32(ins_rank, ia, ib, i + 1);  // rank <= i
        const uint64_t del_lt = lower_bound_u32(del_rank, da, db, i);      // rank < i
        const bool gone = del_lt < db && del_rank[del_lt] == i;
        shift[r] = gone ? INT32_MIN : (int32_t)((int64_t)ins_le - (int64_t)del_lt);
    }
    __syncthreads();
    move_rows<KL>(keys, okeys, i0, rows, shift, cap);
    move_rows<P>(pay, opay, i0, rows, shift, cap);
}

// inserts and overwrites land at r + (#inserts before j) - (#deletes before j): for an insert
// that is its slot; for an overwrite it is where its surviving row moved (the inserts with
// rank <= r and the deletes with rank < r are exactly the batch entries before j in key order)
template <int KL, int P>
__global__ void k_scatter(const uint8_t *skeys, const uint8_t *spay, const uint8_t *present, const uint8_t *sops,
                          const uint32_t *rank, const uint32_t *cum_ins, const uint32_t *cum_del, uint64_t m,
                          uint8_t *okeys, uint8_t *opay, uint64_t cap) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m || sops[j] != 0) return;
    const uint64_t pos = (uint64_t)rank[j] + cum_ins[j] - cum_del[j];
    if (pos >= cap) return;  // only for a batch whose order was not final (see move_rows)
    if (!present[j]) copy_bytes<KL>(okeys + pos * KL, skeys + j * KL);
    copy_bytes<P>(opay + (uint64_t)P * pos, spay + (uint64_t)P * j);
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
__global__ void k_delta_build(const uint8_t *sfps, const uint8_t *sops, uint64_t m, const uint32_t *rank_b,
                              const uint8_t *present_b, const uint8_t *base_fps, const uint32_t *rank_d,
                              const uint8_t *present_d, const uint8_t *dpay, uint8_t *bpay, uint8_t *dops,
                              uint32_t *part) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool c_new = false, c_over = false, c_del = false;
    if (j < m) {
        const bool isdel = sops[j] != 0, in_b = present_b[j], in_d = present_d[j];
        bool was_live = in_b;
        if (in_d) was_live = (reinterpret_cast<const DeltaRec *>(dpay)[rank_d[j]].flags & DeltaRec::LIVE) != 0;
        uint32_t base[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (in_b) fp_load(base_fps + 32ull * rank_b[j], base);
        DeltaRec r;
        r.flags = (in_b ? DeltaRec::IN_BASE : 0u);
        r.brank = rank_b[j];
        r.pad[0] = r.pad[1] = 0;
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
        dops[j] = (isdel && !in_b) ? 1 : 0;
        reinterpret_cast<DeltaRec *>(bpay)[j] = r;
    }
    // per-workgroup counts (same-address atomics from every wave would serialise in L2);
    // k_sum_parts3 adds them up
    __shared__ uint32_t wc[4][3];
    const unsigned long long bn = __ballot(c_new), bo = __ballot(c_over), bd = __ballot(c_del);
    if ((threadIdx.x & 63) == 0) {
        wc[threadIdx.x >> 6][0] = (uint32_t)__popcll(bn);
        wc[threadIdx.x >> 6][1] = (uint32_t)__popcll(bo);
        wc[threadIdx.x >> 6][2] = (uint32_t)__popcll(bd);
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) t += wc[w][threadIdx.x];
        part[3ull * blockIdx.x + threadIdx.x] = t;
    }
}

// counts[k] = Σ_g part[3 g + k], one workgroup
__global__ __launch_bounds__(1024) void k_sum_parts3(const uint32_t *part, uint64_t groups, uint64_t *counts) {
    __shared__ unsigned long long w[16][3];
    unsigned long long t[3] = {0, 0, 0};
    for (uint64_t g = threadIdx.x; g < groups; g += blockDim.x) {
        t[0] += part[3 * g];
        t[1] += part[3 * g + 1];
        t[2] += part[3 * g + 2];
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const uint32_t lo = __shfl_xor((uint32_t)t[k], m, 64), hi = __shfl_xor((uint32_t)(t[k] >> 32), m, 64);
            t[k] += ((unsigned long long)hi << 32) | lo;
        }
        if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6][k] = t[k];
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        unsigned long long s = 0;
        for (uint32_t q = 0; q < blockDim.x / 64; q++) s += w[q][threadIdx.x];
        counts[threadIdx.x] = s;
    }
}

// one pass over the delta run: the 256-row block sums of the contributions and each entry's
// count delta (live - in_base), which the caller then prefix-sums
__global__ __launch_bounds__(256) void k_delta_sums(const uint8_t *dpay, uint64_t n_max, uint64_t nd_old,
                                                    const uint64_t *merge_counts, uint8_t *bsums, int32_t *cnt) {
    __shared__ SumTile tile;
    const uint64_t n = nd_old + merge_counts[0] - merge_counts[2];
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (i < n_max) cnt[i] = 0;
    if (i < n) {
        const DeltaRec &r = reinterpret_cast<const DeltaRec *>(dpay)[i];
        fp_load(reinterpret_cast<const uint8_t *>(r.contrib), h);
        const uint32_t f = r.flags;
        cnt[i] = (int32_t)((f & DeltaRec::LIVE) ? 1 : 0) - (int32_t)((f & DeltaRec::IN_BASE) ? 1 : 0);
    }
    uint32_t f8[8];
    block_sum_fps256(h, tile, f8);
    if (threadIdx.x == 0) store_sum(bsums, blockIdx.x, f8);
}

// compaction input: cur fp = contrib + base fp, op = live ? upsert : delete, and the key's
// place in the base (no search: brank was recorded when the entry was built)
__global__ void k_delta_cur(const uint8_t *dpay, uint64_t n, const uint8_t *base_fps, uint8_t *fps, uint8_t *ops,
                            uint32_t *rank, uint8_t *present) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const DeltaRec &r = reinterpret_cast<const DeltaRec *>(dpay)[i];
    const bool in_b = (r.flags & DeltaRec::IN_BASE) != 0;
    uint32_t base[8] = {0, 0, 0, 0, 0, 0, 0, 0}, cur[8];
    if (in_b) fp_load(base_fps + 32ull * r.brank, base);
    fp_add(r.contrib, base, cur);
    fp_store(fps + 32 * i, cur);
    ops[i] = (r.flags & DeltaRec::LIVE) ? 0 : 1;
    rank[i] = r.brank;
    present[i] = in_b ? 1 : 0;
}

// aggregate over a key range of the merged view = base part + delta part; the delta part's
// size is the sum of its count deltas (prefix difference), not its entry count
__global__ void k_agg_merge(const uint64_t *base_agg, const uint64_t *delta_agg, const uint64_t *dlo,
                            const uint64_t *dhi, const int32_t *cnt_prefix, uint64_t *out) {
    if (threadIdx.x != 0) return;
    const uint64_t lo = *dlo, hi = *dhi;
    const int64_t c = (int64_t)(hi ? cnt_prefix[hi - 1] : 0) - (int64_t)(lo ? cnt_prefix[lo - 1] : 0);
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
__global__ void k_rank_merge(const uint32_t *rank_b, const uint32_t *rank_d, const int32_t *cnt_prefix, uint64_t m,
                             uint64_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t rd = rank_d ? rank_d[j] : 0;
    out[j] = (uint64_t)((int64_t)rank_b[j] + (rd ? cnt_prefix[rd - 1] : 0));
}

// ---- host-side drivers --------------------------------------------------------------------------

namespace {
inline dim3 g1(uint64_t m) { return dim3((uint32_t)((m + 255) / 256)); }
}

template <int KK, int KL>
struct KeyOps final : StoreKeyOps {
    static constexpr int D = KK == KEY_BYTES ? KL / 8 : 1;
    static constexpr int BITS = KK == KEY_U32 ? 32 : 64;

    hipError_t sort_batch(const uint8_t *keys, const uint8_t *fps, const uint8_t *ops, uint64_t m, Scratch &s,
                          uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *flags, bool full,
                          hipStream_t st) override {
        hipError_t e;
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
        hipLaunchKernelGGL(k_iota, g1(m), dim3(256), 0, st, perm, m);
        // multi-digit keys: the most significant digit alone orders random and spread keys
        // (k_gather reports a tie); the LSD sort (least significant digit first, stable passes)
        // is the fallback
        const int lo_digit = (full || D == 1) ? D - 1 : 0;
        for (int d = lo_digit; d >= 0; d--)
            if ((e = pass(d))) return e;
        hipLaunchKernelGGL((k_gather<KK, KL>), g1(m), dim3(256), 0, st, keys, fps, ops, perm, m, skeys, sfps, sops,
                           flags, (full || D == 1) ? 0 : 1);
        return hipGetLastError();
    }

    hipError_t search(const uint8_t *keys, uint64_t n, const uint8_t *q, uint64_t m, uint32_t *rank, uint8_t *present,
                      hipStream_t st) override {
        if (m == 0) return hipSuccess;
        hipLaunchKernelGGL((k_search<KK, KL>), g1(m), dim3(256), 0, st, keys, n, q, m, rank, present);
        return hipGetLastError();
    }

    template <int P>
    hipError_t merge_p(const uint8_t *keys, const uint8_t *pay, uint64_t n, const uint8_t *skeys, const uint8_t *spay,
                       const uint8_t *sops, uint64_t m, Scratch &s, uint8_t *okeys, uint8_t *opay, uint64_t *counts,
                       hipStream_t st, const uint32_t *rank_in, const uint8_t *present_in) {
        hipError_t e;
        uint32_t *ins = s.u32(3, m), *del = s.u32(4, m);
        uint32_t *cins = s.u32(5, m), *cdel = s.u32(6, m), *ins_rank = s.u32(7, m), *del_rank = s.u32(8, m);
        const uint32_t *rank = rank_in;
        const uint8_t *present = present_in;
        if (!rank_in || !present_in) {  // where each batch key sits in the run
            uint32_t *r = s.u32(2, m);
            uint8_t *pr = s.u8(0, m);
            if (s.err) return s.err;
            if ((e = search(keys, n, skeys, m, r, pr, st))) return e;
            rank = r;
            present = pr;
        }
        if (s.err) return s.err;
        hipLaunchKernelGGL(k_classify, g1(m), dim3(256), 0, st, sops, present, m, ins, del);
        size_t tb = 0;
        if ((e = rocprim::exclusive_scan(nullptr, tb, ins, cins, 0u, m, rocprim::plus<uint32_t>(), st))) return e;
        void *tmp = s.bytes(tb);
        if (s.err) return s.err;
        if ((e = rocprim::exclusive_scan(tmp, tb, ins, cins, 0u, m, rocprim::plus<uint32_t>(), st))) return e;
        if ((e = rocprim::exclusive_scan(tmp, tb, del, cdel, 0u, m, rocprim::plus<uint32_t>(), st))) return e;
        hipLaunchKernelGGL(k_compact, g1(m), dim3(256), 0, st, rank, ins, del, cins, cdel, m, ins_rank, del_rank);
        // list lengths (counts[0], counts[2]) are read by the tile kernel on the device
        hipLaunchKernelGGL(k_counts, dim3(1), dim3(64), 0, st, ins, del, cins, cdel, m, counts);
        if (n) {
            const uint64_t tiles = (n + MOVE_TILE - 1) / MOVE_TILE;
            hipLaunchKernelGGL((k_move_tiles<KL, P>), dim3((uint32_t)tiles), dim3(256), 0, st, keys, pay, n, ins_rank,
                               del_rank, counts, okeys, opay, n + m);
        }
        hipLaunchKernelGGL((k_scatter<KL, P>), g1(m), dim3(256), 0, st, skeys, spay, present, sops, rank, cins, cdel,
                           m, okeys, opay, n + m);
        hipLaunchKernelGGL(k_count_ovr, g1(m), dim3(256), 0, st, sops, present, m,
                           reinterpret_cast<unsigned long long *>(counts + 1));
        return hipGetLastError();
    }

    hipError_t merge(const uint8_t *keys, const uint8_t *pay, uint64_t n, const uint8_t *skeys, const uint8_t *spay,
                     const uint8_t *sops, uint64_t m, int payload, Scratch &s, uint8_t *okeys, uint8_t *opay,
                     uint64_t *counts, hipStream_t st, const uint32_t *rank, const uint8_t *present) override {
        if (m == 0) return hipMemsetAsync(counts, 0, 24, st);
        if (payload == 32)
            return merge_p<32>(keys, pay, n, skeys, spay, sops, m, s, okeys, opay, counts, st, rank, present);
        if (payload == (int)sizeof(DeltaRec))
            return merge_p<sizeof(DeltaRec)>(keys, pay, n, skeys, spay, sops, m, s, okeys, opay, counts, st, rank,
                                             present);
        return hipErrorInvalidValue;
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

hipError_t launch_delta_build(const uint8_t *sfps, const uint8_t *sops, uint64_t m, const uint32_t *rank_b,
                              const uint8_t *present_b, const uint8_t *base_fps, const uint32_t *rank_d,
                              const uint8_t *present_d, const uint8_t *dpay, uint8_t *bpay, uint8_t *dops,
                              uint64_t *counts, Scratch &s, hipStream_t st) {
    if (m == 0) return hipMemsetAsync(counts, 0, 24, st);
    const uint64_t groups = (m + 255) / 256;
    uint32_t *part = s.u32(13, groups * 3);
    if (s.err) return s.err;
    hipLaunchKernelGGL(k_delta_build, g1(m), dim3(256), 0, st, sfps, sops, m, rank_b, present_b, base_fps, rank_d,
                       present_d, dpay, bpay, dops, part);
    hipLaunchKernelGGL(k_sum_parts3, dim3(1), dim3(1024), 0, st, part, groups, counts);
    return hipGetLastError();
}

hipError_t launch_delta_sums(const uint8_t *dpay, uint64_t n_max, uint64_t nd_old, const uint64_t *merge_counts,
                             uint8_t *bsums, int32_t *cnt, Scratch &s, hipStream_t st) {
    const uint64_t n = n_max;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_delta_sums, g1(n), dim3(256), 0, st, dpay, n_max, nd_old, merge_counts, bsums, cnt);
    size_t tb = 0;
    hipError_t e;
    if ((e = rocprim::inclusive_scan(nullptr, tb, cnt, cnt, n, rocprim::plus<int32_t>(), st))) return e;
    void *tmp = s.bytes(tb);
    if (s.err) return s.err;
    return rocprim::inclusive_scan(tmp, tb, cnt, cnt, n, rocprim::plus<int32_t>(), st);
}

hipError_t launch_delta_cur(const uint8_t *dpay, uint64_t n, const uint8_t *base_fps, uint8_t *fps, uint8_t *ops,
                            uint32_t *rank, uint8_t *present, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_delta_cur, g1(n), dim3(256), 0, st, dpay, n, base_fps, fps, ops, rank, present);
    return hipGetLastError();
}

hipError_t launch_agg_merge(const uint64_t *base_agg, const uint64_t *delta_agg, const uint64_t *dlo,
                            const uint64_t *dhi, const int32_t *cnt_prefix, uint64_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_agg_merge, dim3(1), dim3(64), 0, st, base_agg, delta_agg, dlo, dhi, cnt_prefix, out);
    return hipGetLastError();
}

hipError_t launch_rank_merge(const uint32_t *rank_b, const uint32_t *rank_d, const int32_t *cnt_prefix, uint64_t m,
                             uint64_t *out, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rank_merge, g1(m), dim3(256), 0, st, rank_b, rank_d, cnt_prefix, m, out);
    return hipGetLastError();
}

}  // namespace rh
