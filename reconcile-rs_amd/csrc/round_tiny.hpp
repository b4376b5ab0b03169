// round_tiny.hpp -- a tiny rbsr protocol round (r <= ROUND_TINY segments) in ONE launch, over the
// base run and any pending delta run (protocol_round_with_policy, rbsr/src/protocol.rs:212-317).
//
// One workgroup of 8 waves: the segments come in from the kernel's arguments into LDS (no PCIe
// round trip, every thread loading a word); the 2r bound keys are searched in the base run
// (a 16-lane group per key: table, then W-way probes of the window, search_device.hpp) and in the
// delta run at once;
// a wave per segment forms its view rank range, places and local sum (view_range_fp); wave 0
// decides the segments, a lane each, and scans their children / enumeration counts; then a wave per child
// cuts it (select over base + run, view_at) and sums it, and the round is written in round_layout()
// straight into mapped page-locked memory.  Every per-segment array lives in LDS.  The host waits
// for a sequence word stored last, after a system-scope fence (as k_small_batch's), not for the
// stream's completion signal.  The same kernel serves a store with no delta run (run.n == 0).
// Replaces, for tiny rounds, two search launches and k_round_small(_view) (three launches, the
// per-segment arrays in global memory): VERDICT r04 item 5.
#pragma once
#include "round_device.hpp"
#include "search_device.hpp"

namespace rh {


// 512 lanes (8 waves): 1,024 would cap a lane at 128 VGPRs and spill the emission's state to scratch
constexpr uint32_t ROUND_TINY_THREADS = 512;
template <int KK, int KL>
__global__ __launch_bounds__(ROUND_TINY_THREADS) void k_round_tiny(RoundTiny a) {
    constexpr uint32_t RT = ROUND_TINY;
    __shared__ __align__(16) uint8_t keys[2 * RT * KL];
    __shared__ uint8_t sk[RT], ek[RT], kind[RT];
    __shared__ uint64_t rem[5 * RT], loc[5 * RT], place[4 * RT];
    __shared__ uint32_t rb[2 * RT], rj[2 * RT];
    __shared__ uint64_t lo[RT], hi[RT], stride[RT], si[RT], ei[RT], nch[RT], choff[RT], nen[RT], enoff[RT];
    __shared__ uint64_t tot[2];
    __shared__ uint64_t cpb[ROUND_TINY_THREADS / 16], cpj[ROUND_TINY_THREADS / 16];  // cut places
    __shared__ __align__(16) uint8_t ckey[ROUND_TINY_THREADS / 16 * KL];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t r = (uint32_t)a.r;
    const RoundRun &R = a.run;
    // phase clocks (the 100 MHz real-time counter, a read; stored by a vector store) when asked
    auto clock = [&](int k) {
        if (a.dbg && t == 0) a.dbg[k] = __builtin_amdgcn_s_memrealtime();
    };
    clock(0);
    // the segments into LDS from the kernel's arguments: kinds, bound keys (4-byte words), the
    // peer's aggregates
    static_assert(RT == ROUND_TINY_SEGS && KL <= (int)ROUND_TINY_KL, "RoundTiny's inline segments");
    {
        const uint32_t nk = 2 * r * KL / 4;
        const uint32_t *src = reinterpret_cast<const uint32_t *>(a.ikeys);
        for (uint32_t i = t; i < nk; i += blockDim.x) reinterpret_cast<uint32_t *>(keys)[i] = src[i];
        if (t < r) sk[t] = a.isk[t], ek[t] = a.iek[t];
        for (uint32_t i = t; i < 5 * r; i += blockDim.x) rem[i] = a.irem[i];
    }
    __syncthreads();
    clock(1);
    // the bound keys' lower bounds, a 16-lane group each (search_group: W-way probes), all at once:
    // groups 0..31 in the base run, 32..63 in the delta run; row q < r is segment q's start, row
    // r + j segment j's end; an unbounded side is not searched
    {
        const uint32_t grp = t >> 4, gl = t & 15, ngrp = ROUND_TINY_THREADS / 16;
        for (uint32_t job = grp; job < 4 * r; job += ngrp) {  // uniform per group
            const bool in_run = job >= 2 * r;
            const uint32_t q = in_run ? job - 2 * r : job;
            const bool bounded = q < r ? sk[q] : ek[q - r];
            uint32_t rank = 0;
            if (bounded && !in_run) search_group<KK, KL, 16>(a.in.bkeys, R.nb, a.btab, keys + q * KL, gl, &rank, nullptr);
            if (bounded && in_run && R.n) search_group<KK, KL, 16>(R.keys, R.n, SearchTable{}, keys + q * KL, gl, &rank, nullptr);
            if (gl == 0) (in_run ? rj : rb)[q] = rank;
        }
    }
    __syncthreads();
    clock(2);
    // segment j's view rank range, places and local sum: with the row prefixes a lane each (two
    // rounds of loads: the count prefix, then the prefixes' difference), else a wave each
    constexpr uint32_t NW = ROUND_TINY_THREADS / 64;
    const bool fast = has_row_prefix(a.in, R);  // uniform
    if (fast) {
        if (t < r) {
            const uint32_t j = t;
            const uint64_t bs = sk[j] ? rb[j] : 0, js = sk[j] ? rj[j] : 0;
            const uint64_t be = ek[j] ? rb[r + j] : R.nb, je = ek[j] ? rj[r + j] : R.n;
            const int64_t cs = R.n ? R.cntp[js] : 0, ce = R.n ? R.cntp[je] : 0;
            const uint64_t l = (uint64_t)((int64_t)bs + cs), h = (uint64_t)((int64_t)be + ce);
            uint64_t fp[4] = {0, 0, 0, 0};
            if (h > l) pre_range_fp(a.in, R, bs, js, be, je, fp);  // inverted: ZERO
            lo[j] = l, hi[j] = h;
            place[4 * j] = bs, place[4 * j + 1] = js, place[4 * j + 2] = be, place[4 * j + 3] = je;
            loc[5 * j] = fp[0], loc[5 * j + 1] = fp[1], loc[5 * j + 2] = fp[2], loc[5 * j + 3] = fp[3];
            loc[5 * j + 4] = h > l ? h - l : 0;
        }
    } else {
        for (uint32_t j = w; j < r; j += NW) {
            const uint64_t bs = sk[j] ? rb[j] : 0, js = sk[j] ? rj[j] : 0;
            const uint64_t be = ek[j] ? rb[r + j] : R.nb, je = ek[j] ? rj[r + j] : R.n;
            const int64_t cs = R.n ? R.cntp[js] : 0, ce = R.n ? R.cntp[je] : 0;
            const uint64_t l = (uint64_t)((int64_t)bs + cs), h = (uint64_t)((int64_t)be + ce);
            uint64_t fp[4] = {0, 0, 0, 0};
            if (h > l) view_range_fp(a.in, R, bs, js, be, je, lane, fp);  // uniform; inverted: ZERO
            if (lane == 0) {
                lo[j] = l, hi[j] = h;
                place[4 * j] = bs, place[4 * j + 1] = js, place[4 * j + 2] = be, place[4 * j + 3] = je;
                loc[5 * j] = fp[0], loc[5 * j + 1] = fp[1], loc[5 * j + 2] = fp[2], loc[5 * j + 3] = fp[3];
                loc[5 * j + 4] = h > l ? h - l : 0;
            }
        }
    }
    __syncthreads();
    clock(3);
    // the decisions, offsets and header: wave 0, a lane per segment, the child and enumeration
    // offsets by a wave scan (a single thread's ~1,000-cycle decisions in series were 5 us a round)
    static_assert(RT <= 64, "a tiny round's segments fit one wave");
    if (w == 0) {
        const bool mine = t < r;
        RoundSeg d{3, 0, 0, 0, 0, 0};
        if (mine) d = round_decide(lo[t], hi[t], loc + 5 * t, rem + 5 * t, a.n, a.sqrt_policy, a.b);
        unsigned long long cs = d.children, es = d.enums;  // inclusive scans
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long x = __shfl_up(cs, o), y = __shfl_up(es, o);
            if (lane >= (uint32_t)o) cs += x, es += y;
        }
        if (mine) {
            kind[t] = (uint8_t)d.kind, stride[t] = d.stride, si[t] = d.si, ei[t] = d.ei;
            nch[t] = d.children, nen[t] = d.enums, choff[t] = cs - d.children, enoff[t] = es - d.enums;
        }
        const uint64_t skipped = __popcll(__ballot(mine && d.kind == 0));
        const uint64_t split = __popcll(__ballot(mine && d.kind == 2));
        const uint64_t dropped = __popcll(__ballot(mine && d.kind == 3));
        const uint64_t nc = __shfl(cs, 63), ne = __shfl(es, 63);
        if (t == 0) {
            tot[0] = nc, tot[1] = ne;
            uint64_t *hdr = reinterpret_cast<uint64_t *>(a.out);
            hdr[0] = skipped, hdr[1] = ne, hdr[2] = split, hdr[3] = nc, hdr[4] = dropped;
        }
        if (nc > a.cap && mine) {  // the host emits again from global copies of the arrays
            const uint32_t j = t;
            a.g.kind[j] = (uint8_t)d.kind, a.g.lo[j] = lo[j], a.g.hi[j] = hi[j], a.g.stride[j] = d.stride;
            a.g.si[j] = d.si, a.g.ei[j] = d.ei, a.g.nch[j] = d.children, a.g.choff[j] = cs - d.children;
            a.g.nen[j] = d.enums, a.g.enoff[j] = es - d.enums;
            for (int q = 0; q < 5; q++) a.g.loc[5 * j + q] = loc[5 * j + q];
            for (int q = 0; q < 4; q++) a.gplace[4 * j + q] = place[4 * j + q];
        }
    }
    __syncthreads();
    clock(4);
    const uint64_t nc = tot[0], ne = tot[1];
    if (nc <= a.cap) {  // uniform
        const RoundLayout L = round_layout(nc, ne, KL);
        // the emit helpers read the segments and their arrays from LDS
        RoundIn il = a.in;
        il.sk = sk, il.ek = ek, il.skeys = keys, il.ekeys = keys + r * KL;
        const RoundSegs gl{kind, lo, hi, loc, stride, si, ei, nch, choff, nen, enoff};
        if (t < r && nen[t]) round_emit_enum(t, enoff[t], L, KL, il, gl, a.out);
        if (fast) {
            // CH children a pass: a 16-lane group per cut place (select over base + run, the key
            // into LDS), then a lane per child (the places' prefix difference, its keys and sum)
            constexpr uint32_t NG = ROUND_TINY_THREADS / 16, CH = NG - 1;
            for (uint64_t c0 = 0; c0 < nc; c0 += CH) {  // uniform
                {
                    const uint32_t grp = t >> 4, g16 = t & 15;
                    const uint64_t c = c0 + grp;  // place grp: child c's start
                    if (c < nc) {                 // uniform per group
                        const uint32_t j = (uint32_t)round_owner(choff, r, c);
                        const uint64_t k = c - choff[j];
                        if (kind[j] == 2 && nch[j] > 1 && k > 0) {
                            const ViewPlace p = view_at_group<16>(R, a.in.bkeys, KL, si[j] + k * stride[j], g16);
                            if (g16 == 0) cpb[grp] = p.b, cpj[grp] = p.j;
                            if (g16 < KL / 4)
                                reinterpret_cast<uint32_t *>(ckey + grp * KL)[g16] =
                                    reinterpret_cast<const uint32_t *>(p.key)[g16];
                        }
                    }
                }
                __syncthreads();
                const uint64_t c = c0 + t;
                if (t < CH && c < nc) {
                    const uint32_t j = (uint32_t)round_owner(choff, r, c);
                    const uint64_t k = c - choff[j], ncuts = nch[j] - 1;
                    uint8_t skd = sk[j], ekd = ek[j];
                    const uint8_t *skey = keys + j * KL, *ekey = keys + (r + j) * KL;
                    uint64_t ag[5];
                    if (kind[j] == 1 || ncuts == 0) {
                        for (int q = 0; q < 5; q++) ag[q] = kind[j] == 1 ? 0ull : loc[5 * j + q];
                    } else {
                        const uint64_t st = stride[j], s0 = si[j];
                        const uint64_t l = s0 + k * st, h = k == ncuts ? ei[j] : s0 + (k + 1) * st;
                        uint64_t b0 = place[4 * j], j0 = place[4 * j + 1], b1 = place[4 * j + 2], j1 = place[4 * j + 3];
                        if (k) b0 = cpb[t], j0 = cpj[t], skd = 1, skey = ckey + t * KL;
                        if (k != ncuts) b1 = cpb[t + 1], j1 = cpj[t + 1], ekd = 1, ekey = ckey + (t + 1) * KL;
                        uint64_t fp[4];
                        pre_range_fp(a.in, R, b0, j0, b1, j1, fp);
                        ag[0] = fp[0], ag[1] = fp[1], ag[2] = fp[2], ag[3] = fp[3], ag[4] = h - l;
                    }
                    uint64_t *agg = reinterpret_cast<uint64_t *>(a.out + L.caggs) + 5 * c;
                    for (int q = 0; q < 5; q++) agg[q] = ag[q];
                    a.out[L.csk + c] = skd;
                    a.out[L.cek + c] = ekd;
                    uint32_t *os = reinterpret_cast<uint32_t *>(a.out + L.cskeys + c * KL);
                    uint32_t *oe = reinterpret_cast<uint32_t *>(a.out + L.cekeys + c * KL);
                    for (uint32_t q = 0; q < KL / 4; q++) {
                        os[q] = skd ? reinterpret_cast<const uint32_t *>(skey)[q] : 0u;
                        oe[q] = ekd ? reinterpret_cast<const uint32_t *>(ekey)[q] : 0u;
                    }
                }
                __syncthreads();  // the next pass's places overwrite these
            }
        } else {
            for (uint64_t c = w; c < nc; c += NW) {
                uint32_t j = 0;
                while (j + 1 < r && choff[j + 1] <= c) j++;  // the segment that owns child c
                round_emit_child_view(c, j, c - choff[j], L, KL, lane, il, R, gl, place, a.out);
            }
        }
    }
    __syncthreads();
    clock(5);
    // every thread's host-visible writes before the sequence word
    __threadfence_system();
    __syncthreads();
    clock(6);
    if (t == 0) __hip_atomic_store(reinterpret_cast<uint64_t *>(a.out) + 7, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The small questions of a store whose host tier is off or stale (rank, select, aggregate over a
// key range), each one launch: the keys searched in both runs at once (waves 0 and 1), the view's
// rank b + cntp[j] of a place (b base rows, j run entries) below the key, select by view_at, the
// sum between two places by view_range_fp -- where these took two to five launches, copies both
// ways and a stream wait.  A key's place "after" it (an Included upper or Excluded lower bound) is
// (rank_b + in base, rank_j + in run): the sum between the two places is the key's current
// fingerprint, or ZERO when the run deletes it.
template <int KK, int KL>
__global__ __launch_bounds__(1024) void k_query_tiny(QueryTiny a) {
    __shared__ __align__(16) uint8_t keys[QUERY_TINY * KL];
    __shared__ uint32_t rb[QUERY_TINY], rj[QUERY_TINY];
    __shared__ uint8_t pb[QUERY_TINY], pj[QUERY_TINY];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    const RoundRun &R = a.run;
    const uint32_t m = (uint32_t)a.m;
    const uint32_t grp = t >> 4, gl = t & 15;  // 64 groups of 16 lanes
    if (a.mode == 1) {  // selects: a group each (view_at_group)
        for (uint32_t q = grp; q < m; q += 64) {
            const ViewPlace p = view_at_group<16>(R, a.base.bkeys, KL, a.in[q], gl);
            if (gl < KL / 4) reinterpret_cast<uint32_t *>(a.out + q * KL)[gl] = reinterpret_cast<const uint32_t *>(p.key)[gl];
        }
    } else {
        const uint32_t nq = a.mode == 0 ? m : 2;
        for (uint32_t i = t; i < nq * KL / 4; i += blockDim.x)
            reinterpret_cast<uint32_t *>(keys)[i] = reinterpret_cast<const uint32_t *>(a.in)[i];
        static_assert(KL <= (int)ROUND_TINY_KL, "QueryTiny's inline keys");
        __syncthreads();
        // every key searched in both runs, a 16-lane group per (key, run)
        for (uint32_t job = grp; job < 2 * nq; job += 64) {
            const bool in_run = job >= nq;
            const uint32_t q = in_run ? job - nq : job;
            const bool bounded = a.mode == 0 || (q == 0 ? a.lo_kind : a.hi_kind);
            uint32_t rank = 0;
            uint8_t present = 0;
            if (bounded && !in_run) search_group<KK, KL, 16>(a.base.bkeys, R.nb, a.btab, keys + q * KL, gl, &rank, &present);
            if (bounded && in_run && R.n) search_group<KK, KL, 16>(R.keys, R.n, SearchTable{}, keys + q * KL, gl, &rank, &present);
            if (gl == 0) (in_run ? rj : rb)[q] = rank, (in_run ? pj : pb)[q] = present;
        }
        __syncthreads();
        if (a.mode == 0) {
            if (t < m) reinterpret_cast<uint64_t *>(a.out)[t] = (uint64_t)((int64_t)rb[t] + (R.n ? R.cntp[rj[t]] : 0));
        } else if (w == 0) {
            uint64_t b0 = 0, j0 = 0, b1 = R.nb, j1 = R.n;
            if (a.lo_kind) b0 = rb[0] + (a.lo_kind == 2 ? pb[0] : 0), j0 = rj[0] + (a.lo_kind == 2 ? pj[0] : 0);
            if (a.hi_kind) b1 = rb[1] + (a.hi_kind == 1 ? pb[1] : 0), j1 = rj[1] + (a.hi_kind == 1 ? pj[1] : 0);
            const int64_t l = (int64_t)b0 + (R.n ? R.cntp[j0] : 0), h = (int64_t)b1 + (R.n ? R.cntp[j1] : 0);
            uint64_t fp[4] = {0, 0, 0, 0};
            if (h > l) view_range_fp(a.base, R, b0, j0, b1, j1, lane, fp);  // uniform; inverted: ZERO
            if (lane == 0) {
                uint64_t *o = reinterpret_cast<uint64_t *>(a.out);
                o[0] = fp[0], o[1] = fp[1], o[2] = fp[2], o[3] = fp[3];
                o[4] = h > l ? (uint64_t)(h - l) : 0;
            }
        }
    }
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(a.seq_word, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace rh
