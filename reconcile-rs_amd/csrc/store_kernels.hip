// store_kernels.hip -- device side of the GPU-resident RSOS store: key order, rank search,
// batch sort, and the batched insert / overwrite / delete merge.
//
// Store layout in HBM (rank order): keys[n][KL] + fps[n][32] + block sums [n/256][32] +
// super-block sums [n/65536][32].  Record payloads are not kept on the device: a record's
// only role after its lift is its fingerprint (the host owns K and V, as the reference's
// map does -- rsos_trait.rs:70-80 returns borrows into host memory).
//
// Batched update = FingerprintTreeMap::insert / remove applied to a whole batch at once
// (rsos/src/fingerprint_tree_map/mutate.rs:23-154):
//   sort batch by key -> rank of each batch key in the store -> classify INS / OVR / DEL
//   -> positions by prefix sums -> move survivors + scatter inserts / overwrites
//   -> recompute block / super-block sums.
// An overwrite replaces the fingerprint (new - old delta, mutate.rs:31-41); a delete removes
// the element (its fingerprint leaves every enclosing sum, mutate.rs:93-154); re-delivering
// an identical record changes nothing (btreemap_oracle.rs:195-231).
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

template <int KK, int KL>
__device__ __forceinline__ void copy_key(uint8_t *dst, const uint8_t *src) {
    if constexpr (KL % 16 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 16) *reinterpret_cast<uint4 *>(dst + o) = *reinterpret_cast<const uint4 *>(src + o);
    } else if constexpr (KL % 8 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 8) *reinterpret_cast<uint2 *>(dst + o) = *reinterpret_cast<const uint2 *>(src + o);
    } else {
#pragma unroll
        for (int o = 0; o < KL; o += 4) *reinterpret_cast<uint32_t *>(dst + o) = *reinterpret_cast<const uint32_t *>(src + o);
    }
}

__device__ __forceinline__ void copy_fp(uint8_t *dst, const uint8_t *src) {
    const uint4 *s = reinterpret_cast<const uint4 *>(src);
    uint4 *d = reinterpret_cast<uint4 *>(dst);
    d[0] = s[0];
    d[1] = s[1];
}

// ---- kernels --------------------------------------------------------------------------------

template <int KK, int KL>
__global__ void k_digit(const uint8_t *keys, const uint32_t *perm, uint64_t m, int d, uint64_t *out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) out[j] = key_digit<KK, KL>(keys + (uint64_t)perm[j] * KL, d);
}

__global__ void k_iota(uint32_t *p, uint64_t m) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) p[j] = (uint32_t)j;
}

// gather the batch into key order; flag adjacent duplicates
template <int KK, int KL>
__global__ void k_gather(const uint8_t *keys, const uint8_t *fps, const uint8_t *ops, const uint32_t *perm,
                         uint64_t m, uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *dup) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t s = perm[j];
    copy_key<KK, KL>(skeys + j * KL, keys + s * KL);
    copy_fp(sfps + 32 * j, fps + 32 * s);
    sops[j] = ops ? ops[s] : 0;
    if (j > 0 && key_cmp<KK, KL>(keys + s * KL, keys + (uint64_t)perm[j - 1] * KL) == 0) atomicOr(dup, 1u);
}

// lower_bound rank of each query key in the sorted store keys; present = key at rank equals
template <int KK, int KL>
__global__ void k_search(const uint8_t *keys, uint64_t n, const uint8_t *q, uint64_t m, uint32_t *rank,
                         uint8_t *present) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint8_t *key = q + j * KL;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (key_cmp<KK, KL>(keys + mid * KL, key) < 0) lo = mid + 1;
        else hi = mid;
    }
    rank[j] = (uint32_t)lo;
    if (present) present[j] = (lo < n && key_cmp<KK, KL>(keys + lo * KL, key) == 0) ? 1 : 0;
}

// classify: op 0 = insert-or-overwrite, 1 = delete.  ins/del as 0/1 for the scans.
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

__device__ __forceinline__ uint64_t lower_bound_u32(const uint32_t *a, uint64_t lo, uint64_t hi, uint64_t x) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Survivors move to i + #inserts(rank <= i) - #deletes(rank < i); deleted rows are skipped.
// One workgroup covers MOVE_TILE consecutive rows: one lane finds the slice of the (sorted)
// insert / delete rank lists that falls inside the tile, then every row binary-searches only
// that slice -- no n-sized scratch arrays, no n-sized scan.
constexpr int MOVE_TILE = 1024;
template <int KK, int KL>
__global__ __launch_bounds__(256) void k_move_tiles(const uint8_t *keys, const uint8_t *fps, uint64_t n,
                                                    const uint32_t *ins_rank, const uint32_t *del_rank,
                                                    const uint64_t *counts, uint8_t *okeys, uint8_t *ofps) {
    __shared__ uint64_t bounds[4];
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
#pragma unroll
    for (int k = 0; k < MOVE_TILE / 256; k++) {
        const uint64_t i = i0 + threadIdx.x + 256 * k;
        if (i >= n) break;
        const uint64_t ins_le = lower_bound_u32(ins_rank, ia, ib, i + 1);  // rank <= i
        const uint64_t del_lt = lower_bound_u32(del_rank, da, db, i);      // rank < i
        if (del_lt < db && del_rank[del_lt] == i) continue;                 // deleted
        const uint64_t pos = i + ins_le - del_lt;
        copy_key<KK, KL>(okeys + pos * KL, keys + i * KL);
        copy_fp(ofps + 32 * pos, fps + 32 * i);
    }
}

// inserts and overwrites land at r + (#inserts before j) - (#deletes before j): for an insert
// that is its slot; for an overwrite it is where its surviving element moved (the inserts with
// rank <= r and the deletes with rank < r are exactly the batch entries before j in key order)
template <int KK, int KL>
__global__ void k_scatter(const uint8_t *skeys, const uint8_t *sfps, const uint8_t *present, const uint8_t *sops,
                          const uint32_t *rank, const uint32_t *cum_ins, const uint32_t *cum_del, uint64_t m,
                          uint8_t *okeys, uint8_t *ofps) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m || sops[j] != 0) return;
    const uint64_t pos = (uint64_t)rank[j] + cum_ins[j] - cum_del[j];
    if (!present[j]) copy_key<KK, KL>(okeys + pos * KL, skeys + j * KL);
    copy_fp(ofps + 32 * pos, sfps + 32 * j);
}

// counts[0..3] = inserted, overwritten, deleted, (dup flag is separate)
__global__ void k_counts(const uint32_t *ins, const uint32_t *del, const uint32_t *cum_ins, const uint32_t *cum_del,
                         const uint8_t *sops, const uint8_t *present, uint64_t m, uint64_t *counts) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    counts[0] = m ? (uint64_t)cum_ins[m - 1] + ins[m - 1] : 0;
    counts[2] = m ? (uint64_t)cum_del[m - 1] + del[m - 1] : 0;
}

__global__ void k_count_ovr(const uint8_t *sops, const uint8_t *present, uint64_t m, unsigned long long *ovr) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool o = j < m && sops[j] == 0 && present[j];
    const unsigned long long b = __ballot(o);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(ovr, (unsigned long long)__popcll(b));
}

// 1 if keys are not strictly increasing
template <int KK, int KL>
__global__ void k_check_sorted(const uint8_t *keys, uint64_t n, uint32_t *bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (i < n && key_cmp<KK, KL>(keys + (i - 1) * KL, keys + i * KL) >= 0) atomicOr(bad, 1u);
}

// rank bounds of a key range (std::ops::Bound kinds 0 unbounded / 1 included / 2 excluded)
template <int KK, int KL>
__global__ void k_bounds(const uint8_t *keys, uint64_t n, const uint8_t *lo_key, int lo_kind, const uint8_t *hi_key,
                         int hi_kind, uint64_t *qlo, uint64_t *qhi) {
    if (threadIdx.x != 0) return;
    auto lb = [&](const uint8_t *k) {
        uint64_t lo = 0, hi = n;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (key_cmp<KK, KL>(keys + mid * KL, k) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    auto present = [&](uint64_t r, const uint8_t *k) { return r < n && key_cmp<KK, KL>(keys + r * KL, k) == 0; };
    uint64_t a = 0, b = n;
    if (lo_kind) {
        a = lb(lo_key);
        if (lo_kind == 2 && present(a, lo_key)) a++;
    }
    if (hi_kind) {
        b = lb(hi_key);
        if (hi_kind == 1 && present(b, hi_key)) b++;
    }
    if (b < a) b = a;  // inverted range -> ZERO (rbsr/src/protocol.rs:230-232)
    *qlo = a;
    *qhi = b;
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
                          uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *dup, hipStream_t st) override {
        hipError_t e;
        uint32_t *perm = s.u32(0, m), *perm2 = s.u32(1, m);
        uint64_t *dig = s.u64(0, m), *dig2 = s.u64(1, m);
        hipLaunchKernelGGL(k_iota, g1(m), dim3(256), 0, st, perm, m);
        for (int d = D - 1; d >= 0; d--) {  // LSD: least significant digit first, stable passes
            hipLaunchKernelGGL((k_digit<KK, KL>), g1(m), dim3(256), 0, st, keys, perm, m, d, dig);
            size_t tb = 0;
            if ((e = rocprim::radix_sort_pairs(nullptr, tb, dig, dig2, perm, perm2, m, 0, BITS, st))) return e;
            void *tmp = s.bytes(tb);
            if ((e = rocprim::radix_sort_pairs(tmp, tb, dig, dig2, perm, perm2, m, 0, BITS, st))) return e;
            std::swap(perm, perm2);
        }
        hipLaunchKernelGGL((k_gather<KK, KL>), g1(m), dim3(256), 0, st, keys, fps, ops, perm, m, skeys, sfps, sops, dup);
        return hipGetLastError();
    }

    hipError_t search(const uint8_t *keys, uint64_t n, const uint8_t *q, uint64_t m, uint32_t *rank, uint8_t *present,
                      hipStream_t st) override {
        if (m == 0) return hipSuccess;
        hipLaunchKernelGGL((k_search<KK, KL>), g1(m), dim3(256), 0, st, keys, n, q, m, rank, present);
        return hipGetLastError();
    }

    hipError_t merge(const uint8_t *keys, const uint8_t *fps, uint64_t n, const uint8_t *skeys, const uint8_t *sfps,
                     const uint8_t *sops, uint64_t m, Scratch &s, uint8_t *okeys, uint8_t *ofps, uint64_t *counts,
                     hipStream_t st) override {
        hipError_t e;
        uint32_t *rank = s.u32(2, m), *ins = s.u32(3, m), *del = s.u32(4, m);
        uint32_t *cins = s.u32(5, m), *cdel = s.u32(6, m), *ins_rank = s.u32(7, m), *del_rank = s.u32(8, m);
        uint8_t *present = s.u8(0, m);
        if (s.err) return s.err;
        if ((e = search(keys, n, skeys, m, rank, present, st))) return e;
        hipLaunchKernelGGL(k_classify, g1(m), dim3(256), 0, st, sops, present, m, ins, del);
        size_t tb = 0;
        if ((e = rocprim::exclusive_scan(nullptr, tb, ins, cins, 0u, m, rocprim::plus<uint32_t>(), st))) return e;
        void *tmp = s.bytes(tb);
        if ((e = rocprim::exclusive_scan(tmp, tb, ins, cins, 0u, m, rocprim::plus<uint32_t>(), st))) return e;
        if ((e = rocprim::exclusive_scan(tmp, tb, del, cdel, 0u, m, rocprim::plus<uint32_t>(), st))) return e;
        hipLaunchKernelGGL(k_compact, g1(m), dim3(256), 0, st, rank, ins, del, cins, cdel, m, ins_rank, del_rank);
        // totals of inserts / deletes (counts[0], counts[2]) are read by the tile kernel on the device
        hipLaunchKernelGGL(k_counts, dim3(1), dim3(64), 0, st, ins, del, cins, cdel, sops, present, m, counts);
        if (n) {
            const uint64_t tiles = (n + MOVE_TILE - 1) / MOVE_TILE;
            hipLaunchKernelGGL((k_move_tiles<KK, KL>), dim3((uint32_t)tiles), dim3(256), 0, st, keys, fps, n, ins_rank,
                               del_rank, counts, okeys, ofps);
        }
        hipLaunchKernelGGL((k_scatter<KK, KL>), g1(m), dim3(256), 0, st, skeys, sfps, present, sops, rank, cins, cdel,
                           m, okeys, ofps);
        if ((e = hipMemsetAsync(counts + 1, 0, 8, st))) return e;
        hipLaunchKernelGGL(k_count_ovr, g1(m), dim3(256), 0, st, sops, present, m,
                           reinterpret_cast<unsigned long long *>(counts + 1));
        return hipGetLastError();
    }

    hipError_t check_sorted(const uint8_t *keys, uint64_t n, uint32_t *bad, hipStream_t st) override {
        if (n < 2) return hipSuccess;
        hipLaunchKernelGGL((k_check_sorted<KK, KL>), g1(n), dim3(256), 0, st, keys, n, bad);
        return hipGetLastError();
    }

    hipError_t bounds(const uint8_t *keys, uint64_t n, const uint8_t *lo_key, int lo_kind, const uint8_t *hi_key,
                      int hi_kind, uint64_t *qlo, uint64_t *qhi, hipStream_t st) override {
        hipLaunchKernelGGL((k_bounds<KK, KL>), dim3(1), dim3(64), 0, st, keys, n, lo_key, lo_kind, hi_key, hi_kind, qlo,
                           qhi);
        return hipGetLastError();
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

}  // namespace rh
