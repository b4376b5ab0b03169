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

// grid: 3 * ceil(n / 256) workgroups; block b lifts (b % 3 == 0) or searches the base (1) or the
// delta run (2), for rows [256 (b / 3), +256) of the batch.  c.dst: each record's sorted row.
template <int KK, int KL, int VK, int VL, int RK, bool TAGS>
__global__ __launch_bounds__(LIFT_THREADS) void k_lift_search(DevCols c, uint64_t n, uint8_t *fps, const uint8_t *q,
                                                              SearchJob jb, SearchJob jd) {
    using L = Layout<KK, KL, VK, VL, RK>;
    const uint32_t role = blockIdx.x % 3, t = threadIdx.x;
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
        const uint32_t r = c.dst[i];
        if (r < n) store_fp(fps, r, h);  // bounded as in k_lift
    } else {
        const SearchJob &j = role == 1 ? jb : jd;
        search_sampled_one<KK, KL>(j.keys, j.n, j.smp, j.smp2, j.tb, q + i * KL, j.rank + i, j.present + i);
    }
}

}  // namespace rh
