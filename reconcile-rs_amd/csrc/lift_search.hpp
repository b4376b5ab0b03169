// lift_search.hpp -- the batch path's fused launch: the lift of an update batch into its sorted
// rows and the two lower-bound searches of its sorted keys (base run, delta run), as one grid.
//
// The lift is VALU-bound (two BLAKE3 compressions per 120-byte record, streaming reads) and the
// searches are bound by dependent random lines (a table line, then one or two key lines per
// query), so run back to back each leaves the other's resource idle.  Here every third
// workgroup lifts 256 records and the other two search 256 keys, so the CUs interleave both
// kinds of waves: the searches' load latency is hidden behind the lift's ALU work.
// Both depend only on the key sort (the positions and the sorted keys); the batch's delta records
// (k_delta_build) need both.  Reference: the per-insert lift and descent of
// FingerprintTreeMap::insert (rsos/src/fingerprint_tree_map/mutate.rs:23-88), for a whole batch.
#pragma once
#include "lift_kernels.hpp"
#include "search_device.hpp"

namespace rh {

// The next batch's digit min / max for its key sort (apply_device_many): where the batch path
// already knows the next batch, the workgroups after the lift and search ones each reduce
// MINMAX_TILE of its keys' leading digits to one (min, max) pair, which the next sort takes in
// place of its own k_cs_minmax launch (NextMinmax, store_kernels.hpp).
// grid: 3 * ceil(n / 256) workgroups, then ceil(nx.m / MINMAX_TILE); block b < 3 ceil(n / 256)
// lifts (b % 3 == 0) or searches the base (1) or the delta run (2), for rows [256 (b / 3), +256)
// of the batch; c.dst: each record's sorted row.  The blocks after them: nx's min / max partials.
template <int KK, int KL, int VK, int VL, int RK, bool TAGS>
__global__ __launch_bounds__(LIFT_THREADS) void k_lift_search(DevCols c, uint64_t n, uint8_t *fps, const uint8_t *q,
                                                              SearchJob jb, SearchJob jd, NextMinmax nx) {
    using L = Layout<KK, KL, VK, VL, RK>;
    const uint32_t t = threadIdx.x;
    const uint64_t nblk3 = 3 * ((n + LIFT_THREADS - 1) / LIFT_THREADS);
    if (blockIdx.x >= nblk3) {  // uniform: the next batch's digit min / max
        static_assert(MINMAX_TILE % LIFT_THREADS == 0, "whole keys per lane");
        __shared__ uint64_t lo[LIFT_THREADS / 64], hi[LIFT_THREADS / 64];
        const uint64_t w = blockIdx.x - nblk3, k0 = w * MINMAX_TILE;
        uint64_t a = ~0ull, b = 0;
#pragma unroll
        for (int k = 0; k < (int)(MINMAX_TILE / LIFT_THREADS); k++) {
            const uint64_t r = k0 + (uint64_t)LIFT_THREADS * k + t;
            if (r < nx.m) {
                const uint64_t d = key_digit<KK, KL>(nx.keys + r * KL, 0);
                a = d < a ? d : a;
                b = d > b ? d : b;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint64_t a2 = __shfl_xor(a, o, 64), b2 = __shfl_xor(b, o, 64);
            a = a2 < a ? a2 : a;
            b = b2 > b ? b2 : b;
        }
        if ((t & 63) == 0) {
            lo[t >> 6] = a;
            hi[t >> 6] = b;
        }
        __syncthreads();
        if (t == 0) {
            for (uint32_t v = 1; v < LIFT_THREADS / 64; v++) {
                a = lo[v] < a ? lo[v] : a;
                b = hi[v] > b ? hi[v] : b;
            }
            nx.part[2 * w] = a;
            nx.part[2 * w + 1] = b;
        }
        return;
    }
    const uint32_t role = blockIdx.x % 3;
    const uint64_t b0 = (uint64_t)(blockIdx.x / 3) * LIFT_THREADS, i = b0 + t;
    if (i >= n) return;
    if (role == 0) {
        // as k_lift: column pointers rebased to this block (32-bit lane offsets)
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
        uint32_t h[8];
        lift_record<KK, KL, VK, VL, RK, TAGS>(kw, sw, tomb, vrow, h);
        const uint32_t r = c.dst2 ? c.dst2[c.dst[i]] : c.dst[i];
        if (r < n) store_fp<uint64_t>(fps, r, h);  // bounded as in k_lift
    } else {
        const SearchJob &j = role == 1 ? jb : jd;
        search_sampled_one<KK, KL>(j.keys, j.n, j.smp, j.smp2, j.tb, q + i * KL, j.rank + i, j.present + i);
    }
}

}  // namespace rh
