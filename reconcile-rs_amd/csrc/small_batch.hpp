// small_batch.hpp -- the store's small-batch path: a few rows into a large map (a replica's network
// merge, src/replica/dispatch.rs:188-196, or one staged Rsos::insert) in one workgroup, one launch.
//
// The large-batch path (rsos_hip_abi.hip apply_device) is built for a million rows: a bucket sort
// over the whole device (four launches), the fused lift + search grid, the delta front (three
// launches) and the merge -- about a dozen commands, each a few microseconds of launch latency
// whatever the batch size, plus copies.  For m <= small_batch_max(kl) rows one workgroup does
// everything before the merge, with the keys and fingerprints held in LDS:
//   1. the batch's keys into LDS; a bitonic sort of row indices by (key, input row) -- a stable
//      sort, so the last row of a repeated key is the last of its run;
//   2. duplicates: with last_wins, every row but the last of each key is dropped (the result of
//      applying the rows in order: Replica::just_insert_bulk, src/replica/write.rs:107-121);
//      otherwise they are reported (flags bit 1) and the caller commits nothing;
//   3. every kept row lifted (lift_record, as k_lift) into its sorted slot in LDS, and every kept
//      key searched in the base and the delta run (search_sampled_one, as k_lift_search) -- for a
//      batch of up to 320 rows by three groups of waves at once (the launch is then 3 x the rows,
//      rounded to waves): the lift's VALU work and the two searches' chains of dependent loads
//      overlap instead of following one another in each thread;
//   4. the batch's DeltaRecs into the record heap and the merge lists, exactly as k_delta_build /
//      k_delta_parts / k_delta_lists form them (FingerprintTreeMap::insert / remove's signed
//      deltas, rsos/src/fingerprint_tree_map/mutate.rs:23-154), the counts and totals by block
//      reductions, the result block and (optionally) the host tier's fold rows written straight to
//      page-locked host memory mapped into the device's address space -- no copy command; every
//      thread's writes made visible to the host (a system-scope fence), then the block's sequence
//      word, which the host polls instead of waiting for the stream.
// Then the delta merge (k_merge_run<HEAP>) is the second and last launch of the batch.
#pragma once
#include "fp_device.hpp"
#include "lift_kernels.hpp"
#include "search_device.hpp"

namespace rh {

// the largest batch the one-workgroup path takes.  LDS per workgroup (k_small_batch's arrays):
// SBM * (KL + 32 + 3 * 2 + 2 * 4 + 2) bytes + ~1.5 KiB of reductions -- 67 KB for 16-byte keys
// (1,024 rows), 42 KB for 32-byte keys (512 rows): within gfx950's 160 KiB per workgroup, not
// within the 64 KiB of earlier CDNA parts (checked per instantiation below, small_batch_lds)
__host__ __device__ constexpr uint32_t small_batch_max(int kl) { return kl <= 16 ? 1024u : 512u; }
__host__ __device__ constexpr uint32_t small_batch_lds(int kl) {
    return small_batch_max(kl) * (uint32_t)(kl + 32 + 3 * 2 + 2 * 4 + 2) + 16 * 4 * 2 + 16 * 5 * 4 + 16 * 4 + 16 * 8 * 8;
}
constexpr uint32_t LDS_BYTES_GFX950 = 160u * 1024u;

// result block words (res): [0..2] new / overwritten / deleted rows vs the merged view, [3..5] the
// merge's inserts / overwrites / removals in the delta run, [6] flags (1: duplicate keys, not
// merged), [7] the change of the delta run's count total (int64), [8..11] the change of its
// contribution total (mod 2^256), [12] rows kept, [13] the batch's sequence number, written last
constexpr int SMALL_RES_WORDS = 14;

// threads of the launch for m rows: three groups of whole waves while they fit one workgroup
__host__ __device__ constexpr uint32_t small_batch_threads(uint32_t m) {
    const uint32_t r = ((m + 63) / 64) * 64;
    return 3 * r <= 1024 ? 3 * r : r;
}

struct SmallBatch {
    DevCols c;             // the batch's columns (device memory or mapped host memory), input order
    const uint8_t *ops;    // 0 upsert, 1 delete (nullptr: every row an upsert)
    uint32_t m;
    int last_wins;         // 1: keep the last row of each repeated key; 0: report duplicates
    SearchJob jb, jd;      // the base and delta runs (rank / present unused)
    const uint8_t *base_fps;
    const uint32_t *dslot;
    uint8_t *heap;
    uint32_t heap_base;
    uint8_t *skeys;        // out: the kept keys in key order (the merge's batch rows)
    uint32_t *upos, *usrc, *rlist;
    uint64_t *mcnt;        // out (device): [0] inserts, [1] overwrites, [2] removals, [3] upserts, [4] present
    uint64_t *res;         // out: the result block (SMALL_RES_WORDS words)
    uint64_t seq;          // written to res[13] after everything else is visible to the host
    // the host tier's fold rows, in key order (each nullable): the kept keys, their DeltaRecs and
    // drop flags (folds against the device's base), their fingerprints and ops (folds against the
    // tier's own base copy)
    uint8_t *fkeys, *frecs, *fdrop, *ffps, *fops;
};

// KL key bytes with the widest aligned word accesses (key rows are KL-aligned; KL a multiple of 4)
template <int KL>
__device__ __forceinline__ void copy_key_words(uint8_t *d, const uint8_t *s) {
    if constexpr (KL % 16 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 16) *reinterpret_cast<uint4 *>(d + o) = *reinterpret_cast<const uint4 *>(s + o);
    } else if constexpr (KL % 8 == 0) {
#pragma unroll
        for (int o = 0; o < KL; o += 8) *reinterpret_cast<uint2 *>(d + o) = *reinterpret_cast<const uint2 *>(s + o);
    } else {
#pragma unroll
        for (int o = 0; o < KL; o += 4) *reinterpret_cast<uint32_t *>(d + o) = *reinterpret_cast<const uint32_t *>(s + o);
    }
}

template <int KK, int KL>
__device__ __forceinline__ bool sb_less(const uint8_t *K, uint32_t x, uint32_t y, uint32_t m) {
    if (x >= m || y >= m) return x < m ? true : (y < m ? false : x < y);  // padding sorts last
    const int c = key_cmp<KK, KL>(K + x * KL, K + y * KL);
    return c < 0 || (c == 0 && x < y);
}

// exclusive scans of two flags over the block's threads (NW waves); totals on every thread
__device__ __forceinline__ void sb_scan2(uint32_t a, uint32_t b, uint32_t *wa, uint32_t *wb, uint32_t &ea,
                                         uint32_t &eb, uint32_t &ta, uint32_t &tb) {
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6, NW = blockDim.x >> 6;
    uint32_t x = a, y = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t px = __shfl_up(x, o, 64), py = __shfl_up(y, o, 64);
        if (lane >= (uint32_t)o) {
            x += px;
            y += py;
        }
    }
    if (lane == 63) {
        wa[wv] = x;
        wb[wv] = y;
    }
    __syncthreads();
    ea = x - a;
    eb = y - b;
    ta = 0;
    tb = 0;
    for (uint32_t w = 0; w < NW; w++) {
        if (w < wv) {
            ea += wa[w];
            eb += wb[w];
        }
        ta += wa[w];
        tb += wb[w];
    }
    __syncthreads();  // wa / wb reusable
}

template <int KK, int KL, int VK, int VL, int RK, bool TAGS>
__global__ __launch_bounds__(1024) void k_small_batch(SmallBatch a) {
    using L = Layout<KK, KL, VK, VL, RK>;
    constexpr uint32_t SBM = small_batch_max(KL);
    static_assert(small_batch_lds(KL) <= LDS_BYTES_GFX950, "k_small_batch's LDS exceeds a gfx950 workgroup's 160 KiB");
    __shared__ __attribute__((aligned(16))) uint8_t K[SBM * KL];
    __shared__ __attribute__((aligned(16))) uint32_t F[SBM * 8];
    __shared__ uint16_t sidx[SBM], kidx[SBM], posof[SBM];
    __shared__ uint32_t srb[SBM], srd[SBM];  // each sorted kept row's base / delta rank
    __shared__ uint8_t sib[SBM], sid[SBM];   // and whether its key is there
    __shared__ uint32_t wa[16], wb[16];
    __shared__ uint32_t wcnt[16][5];
    __shared__ int32_t wdc[16];
    __shared__ uint64_t wacc[16 * 8];
    const uint32_t t = threadIdx.x, NT = blockDim.x, lane = t & 63, wv = t >> 6, NW = NT >> 6;
    const uint32_t m = a.m;
    // 1. keys into LDS, sort (bitonic over the next power of two; padding sorts last)
    if (t < m) copy_key_words<KL>(K + t * KL, a.c.keys + (uint64_t)t * KL);
    uint32_t NP = 1;
    while (NP < m) NP <<= 1;
    for (uint32_t i = t; i < NP; i += NT) sidx[i] = (uint16_t)i;
    __syncthreads();
    for (uint32_t k = 2; k <= NP; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < NP; i += NT) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint32_t x = sidx[i], y = sidx[l];
                    const bool up = (i & k) == 0;
                    if (up ? sb_less<KK, KL>(K, y, x, m) : sb_less<KK, KL>(K, x, y, m)) {
                        sidx[i] = (uint16_t)y;
                        sidx[l] = (uint16_t)x;
                    }
                }
            }
            __syncthreads();
        }
    }
    // 2. duplicates: sorted row t keeps its key unless the next sorted row has the same key
    const bool real = t < m;
    const bool dup = real && t + 1 < m && key_cmp<KK, KL>(K + sidx[t] * KL, K + sidx[t + 1] * KL) == 0;
    const int anydup = __syncthreads_or(dup ? 1 : 0);
    const bool keep = real && !(a.last_wins && dup);
    uint32_t jn, unused_e, m2, unused_t;
    sb_scan2(keep ? 1u : 0u, 0u, wa, wb, jn, unused_e, m2, unused_t);
    if (real) posof[sidx[t]] = keep ? (uint16_t)jn : (uint16_t)0xFFFF;
    if (keep) kidx[jn] = sidx[t];
    __syncthreads();
    // 3. with three groups (G threads each): group 0 lifts, group 1 searches the base, group 2 the
    // delta run; otherwise every thread does all three for its row
    const uint32_t G = (m + 63) & ~63u;
    const bool split = NT >= 3 * G;
    const uint32_t role = split ? t / G : 3u, row = split ? t - role * G : t;
    // 3a. the lift of input row t into its sorted slot (the key from LDS)
    if ((role == 0 || role == 3) && row < m && posof[row] != 0xFFFF) {
        uint32_t kw[L::KEY_ENC / 4 > 0 ? L::KEY_ENC / 4 : 1];
        uint32_t sw[5];
        load_key<KK, KL, uint32_t>(K, t, kw);
        if constexpr (RK == REC_DATED) load_stamp<uint32_t>(a.c, t, sw);
        const bool tomb = TAGS ? (a.c.tags[t] != 0) : false;
        const uint8_t *vrow = a.c.values + (uint64_t)t * L::VAL_ROW;
        uint32_t h[8];
        lift_record<KK, KL, VK, VL, RK, TAGS>(kw, sw, tomb, vrow, h);
        uint32_t *o = F + 8 * posof[t];
#pragma unroll
        for (int q = 0; q < 8; q++) o[q] = h[q];
    }
    // 3b. sorted kept row `row`: where its key is in the base and the delta run
    if (row < m2 && role != 0) {
        const uint8_t *key = K + kidx[row] * KL;
        uint32_t rk = 0, rk2 = 0;
        uint8_t in = 0, in2 = 0;
        if (role != 2) {
            search_sampled_one<KK, KL>(a.jb.keys, a.jb.n, a.jb.smp, a.jb.smp2, a.jb.tb, key, &rk, &in);
            srb[row] = rk;
            sib[row] = in;
            copy_key_words<KL>(a.skeys + (uint64_t)row * KL, key);
        }
        if (role != 1) {
            search_sampled_one<KK, KL>(a.jd.keys, a.jd.n, a.jd.smp, a.jd.smp2, a.jd.tb, key, &rk2, &in2);
            srd[row] = rk2;
            sid[row] = in2;
        }
    }
    __syncthreads();  // F, the ranks complete
    const bool act = t < m2;
    const uint32_t src = act ? kidx[t] : 0u;
    const uint8_t *key = K + src * KL;
    const uint32_t rank_b = act ? srb[t] : 0u, rank_d = act ? srd[t] : 0u;
    const uint8_t in_b = act ? sib[t] : 0, in_d = act ? sid[t] : 0;
    // 4. the row's DeltaRec (k_delta_build's rule)
    bool c_new = false, c_over = false, c_del = false, c_up = false, c_pr = false;
    int32_t dcnt = 0;
    uint32_t dfp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    DeltaRec r;
    bool drop = false, isdel = false;
    if (act) {
        isdel = a.ops ? a.ops[src] != 0 : false;
        bool was_live = in_b;
        const DeltaRec *old_rec = in_d ? reinterpret_cast<const DeltaRec *>(a.heap) + a.dslot[rank_d] : nullptr;
        if (in_d) was_live = (old_rec->flags & DeltaRec::LIVE) != 0;
        uint32_t base[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (in_b) fp_load(a.base_fps + 32ull * rank_b, base);
        r.flags = in_b ? DeltaRec::IN_BASE : 0u;
        r.brank = rank_b;
        uint32_t cur[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (!isdel) {
#pragma unroll
            for (int q = 0; q < 8; q++) cur[q] = F[8 * t + q];
            r.flags |= DeltaRec::LIVE;
            c_new = !was_live;
            c_over = was_live;
        } else {
            c_del = was_live;
        }
        fp_sub(cur, base, r.contrib);
        drop = isdel && !in_b;  // deleting a key the base does not hold: no entry
        c_up = !drop;
        c_pr = in_d;
        reinterpret_cast<DeltaRec *>(a.heap)[a.heap_base + t] = r;
        if (!drop) dcnt += (isdel ? 0 : 1) - (in_b ? 1 : 0);
        uint32_t nc[8], oc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 8; q++) nc[q] = drop ? 0u : r.contrib[q];
        if (in_d) {
            const uint2 *op = reinterpret_cast<const uint2 *>(old_rec);
            uint32_t w[10];
#pragma unroll
            for (int q = 0; q < 5; q++) words_of(op[q], w + 2 * q);
#pragma unroll
            for (int q = 0; q < 8; q++) oc[q] = w[q];
            dcnt -= ((w[9] & DeltaRec::LIVE) ? 1 : 0) - ((w[9] & DeltaRec::IN_BASE) ? 1 : 0);
        }
        fp_sub(nc, oc, dfp);
        if (a.fkeys) copy_key_words<KL>(a.fkeys + (uint64_t)t * KL, key);
        if (a.frecs) reinterpret_cast<DeltaRec *>(a.frecs)[t] = r;
        if (a.fdrop) a.fdrop[t] = drop ? 1 : 0;
        if (a.ffps) fp_store(a.ffps + 32ull * t, cur);
        if (a.fops) a.fops[t] = isdel ? 1 : 0;
    }
    // the merge lists (k_delta_lists): upsert U lands at rank + U - R (U upserts, R run rows replaced
    // before it); the run rows the batch replaces, in order
    uint32_t ub, rb, U, R;
    sb_scan2(c_up ? 1u : 0u, c_pr ? 1u : 0u, wa, wb, ub, rb, U, R);
    if (c_up) {
        a.upos[ub] = rank_d + ub - rb;
        a.usrc[ub] = t;
    }
    if (c_pr) a.rlist[rb] = rank_d;
    // totals: the counts, the count change and the contribution change
    const unsigned long long bl[5] = {__ballot(c_new), __ballot(c_over), __ballot(c_del), __ballot(c_up && c_pr),
                                      0ull};
    int32_t y = dcnt;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) y += __shfl_xor(y, o, 64);
    Acc acc;
    acc_zero(acc);
    acc_add_fp(acc, dfp);
    acc_wave_reduce(acc);
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 4; q++) wcnt[wv][q] = (uint32_t)__popcll(bl[q]);
        wdc[wv] = y;
    }
    if (lane < 8) {
        uint64_t mine = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) mine = (lane == (uint32_t)q) ? acc.l[q] : mine;
        wacc[wv * 8 + lane] = mine;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t T[4] = {0, 0, 0, 0};
        int64_t dc = 0;
        Acc s;
        acc_zero(s);
        for (uint32_t w = 0; w < NW; w++) {
#pragma unroll
            for (int q = 0; q < 4; q++) T[q] += wcnt[w][q];
            dc += wdc[w];
#pragma unroll
            for (int q = 0; q < 8; q++) s.l[q] += wacc[w * 8 + q];
        }
        uint32_t f[8];
        acc_normalise(s, f);
        const uint64_t ov = T[3];
        a.mcnt[0] = U - ov;
        a.mcnt[1] = ov;
        a.mcnt[2] = R - ov;
        a.mcnt[3] = U;
        a.mcnt[4] = R;
        uint64_t *o = a.res;
        o[0] = T[0];
        o[1] = T[1];
        o[2] = T[2];
        o[3] = U - ov;
        o[4] = ov;
        o[5] = R - ov;
        o[6] = (anydup && !a.last_wins) ? 1u : 0u;
        o[7] = (uint64_t)dc;
#pragma unroll
        for (int q = 0; q < 4; q++) o[8 + q] = (uint64_t)f[2 * q] | ((uint64_t)f[2 * q + 1] << 32);
        o[12] = m2;
    }
    // every thread's host-visible writes (the fold rows, the result block) before the sequence word
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(a.res + 13, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace rh
