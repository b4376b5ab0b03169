// snapshot_kernels.hip -- snapshot reload on the device: locate every entry of an RCNL v1
// snapshot's bincode `Vec<(K, Entry<Timestamp, V>)>` and decode the entries into SoA columns.
//
// The file (src/snapshot.rs:30-58) is "RCNL" | u32 version | bincode 1.3.3 (fixint, LE) of
// PersistedState (lww-register/src/persistence.rs:62-70), whose first field is the entry Vec
// (:32): u64 count, then the entries back to back.  An entry's length depends on its State
// variant (a tombstone carries no value), so entry i's offset depends on every variant before
// it -- a serial chain through the whole file.  It is broken up like this:
//   1. the body is cut into segments of `seg` bytes (~16 entries).  Entry starts are multiples
//      of g = gcd(tombstone len, present len) past the body start, and the first entry starting
//      in a segment lies within one present-entry length of the segment start, so there are
//      only P = lp / g candidate positions.  A workgroup stages a run of segments in LDS
//      (16-byte coalesced loads) and one lane per (segment, candidate) walks its segment in LDS,
//      recording where the chain leaves the segment and how many entries it crossed (or that
//      no valid entry starts there: bad variant, wrong Vec length, past the end of the file);
//   2. the per-segment transfer functions are composed up a tree (fan-out 32; a node stages
//      its children's tables in LDS and chains through them there) and the true first-entry
//      position and entry index of every segment are pushed back down from the file's first
//      entry;
//   3. a workgroup stages a run of segments in LDS again, one lane per segment re-walks it from
//      the true position listing entry offsets in LDS, and the workgroup writes its contiguous
//      range of entries into every column with coalesced stores (the AoS -> SoA transpose).
//      A reload into stores takes the fused pass instead (snap_lift.hpp): the same listing,
//      then the lifts and the key rows straight from the staged bytes, no columns.
// HBM traffic: the body is read twice (steps 1 and 3) and the columns written once; step 2
// touches P words per segment.
#include <algorithm>
#include <vector>

#include "snap_device.hpp"
#include "snapshot_kernels.hpp"

namespace rh {

namespace {

constexpr uint32_t SNAP_BAD = snap::BAD;
constexpr uint32_t SNAP_FAN = 32;
constexpr uint32_t SNAP_TREE_LDS = 24576;  // a tree node's staged child tables
constexpr uint32_t SNAP_LDS = 32768;  // staged bytes per workgroup
using snap::Img;
using snap::entry_len;
using snap::for_dwords;
using snap::seg_start;
using snap::stage;

// step 1: transfer function of every (segment, candidate first-entry position); G segments
// per workgroup, lane = segment * P + candidate
__global__ __launch_bounds__(256) void k_snap_walk(const uint8_t *blob, SnapFmt f, uint64_t nseg, uint32_t G,
                                                   uint32_t *ex, uint32_t *cnt) {
    extern __shared__ uint32_t lds[];
    const uint64_t s0 = (uint64_t)blockIdx.x * G;
    const uint32_t nG = (uint32_t)std::min<uint64_t>(G, nseg - s0);
    const uint64_t a = seg_start(f, s0) & ~15ull;
    const uint64_t b = std::min<uint64_t>(seg_start(f, s0 + nG) + f.lp, f.len);
    stage(blob, f.len, a, b, lds);
    __syncthreads();
    const uint32_t gs = threadIdx.x / f.phases, ph = threadIdx.x - gs * f.phases;
    if (gs >= nG) return;
    const Img m{lds, a};
    const uint64_t s = s0 + gs, end = seg_start(f, s + 1);
    uint64_t p = seg_start(f, s) + (uint64_t)ph * f.g;
    uint32_t c = 0, x;
    for (;;) {
        if (p >= end) {
            x = (uint32_t)((p - end) / f.g);
            break;
        }
        const uint32_t L = entry_len(m, f, p);
        if (!L) {
            x = SNAP_BAD;
            break;
        }
        p += L;
        c++;
    }
    ex[s * f.phases + ph] = x;
    cnt[s * f.phases + ph] = c;
}

// step 2 (up): compose the transfer functions of F consecutive groups; one 64-lane workgroup per
// parent stages its children's tables in LDS (coalesced), then lane x chains candidate x
// through them -- F dependent LDS reads instead of F dependent global loads
template <class CIn>
__global__ __launch_bounds__(64) void k_snap_up(const uint32_t *ex, const CIn *cnt, uint64_t nin, uint32_t P,
                                                uint32_t F, uint32_t *ex_out, uint64_t *cnt_out) {
    extern __shared__ uint64_t tab[];  // F * P counts, then F * P exits
    uint64_t *sc = tab;
    uint32_t *sx = reinterpret_cast<uint32_t *>(tab + (uint64_t)F * P);
    const uint64_t g = blockIdx.x, c0 = g * F;
    const uint32_t nc = (uint32_t)std::min<uint64_t>(F, nin - c0);
    for (uint32_t j = threadIdx.x; j < nc * P; j += blockDim.x) {
        sx[j] = ex[c0 * P + j];
        sc[j] = cnt[c0 * P + j];
    }
    __syncthreads();
    for (uint32_t x0 = threadIdx.x; x0 < P; x0 += blockDim.x) {
        uint32_t x = x0;
        uint64_t c = 0;
        for (uint32_t j = 0; j < nc; j++) {
            const uint32_t i = j * P + x;
            c += sc[i];
            x = sx[i];
            if (x == SNAP_BAD) break;
        }
        ex_out[g * P + x0] = x;
        cnt_out[g * P + x0] = c;
    }
}

// step 2 (down): true entry position and entry index at the start of every child of a parent
// (one workgroup per parent, its children's tables in LDS, one lane follows the chain).  At
// level 0 with segq given (the fused reload): segq[b] = the segment holding entry
// min(256 b, n) - 1 for b in [1, ceil(n / 256)] -- the first and last segments a 256-entry
// block of the lift reads (segq[0] = 0 is set by k_snap_init)
template <class CIn>
__global__ __launch_bounds__(64) void k_snap_down(const uint32_t *ex, const CIn *cnt, uint64_t nl, uint32_t P,
                                                  uint32_t F, const uint32_t *start_up, const uint64_t *base_up,
                                                  uint32_t *start, uint64_t *basev, uint32_t *segq, uint64_t n) {
    extern __shared__ uint64_t tab[];  // F * P counts, F * P exits, then F chain positions
    uint64_t *sc = tab;
    uint64_t *qc = tab + (uint64_t)F * P;      // entry index at each child's start (F + 1)
    uint32_t *sx = reinterpret_cast<uint32_t *>(qc + F + 1);
    uint32_t *qx = sx + (uint64_t)F * P;        // position at each child's start
    const uint64_t g = blockIdx.x, c0 = g * F;
    const uint32_t nc = (uint32_t)std::min<uint64_t>(F, nl - c0);
    for (uint32_t j = threadIdx.x; j < nc * P; j += blockDim.x) {
        sx[j] = ex[c0 * P + j];
        sc[j] = cnt[c0 * P + j];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x = start_up[g];
        uint64_t c = base_up[g];
        for (uint32_t j = 0; j < nc; j++) {
            qx[j] = x;
            qc[j] = c;
            if (x != SNAP_BAD) {
                const uint32_t i = j * P + x;
                c += sc[i];
                x = sx[i];
            }
        }
        qc[nc] = c;
    }
    __syncthreads();
    const uint64_t nblk = (n + 255) / 256;
    for (uint32_t j = threadIdx.x; j < nc; j += blockDim.x) {
        const uint64_t s = c0 + j;
        start[s] = qx[j];
        basev[s] = qc[j];
        const uint64_t c = qc[j], c1 = qc[j + 1];  // entries [c, c1) start in segment s
        if (segq && qx[j] != SNAP_BAD && c < n) {
            for (uint64_t b = std::max<uint64_t>(1, (c + 256) / 256); b < nblk && 256 * b - 1 < c1; b++)
                segq[b] = (uint32_t)s;
            if (n - 1 < c1) segq[nblk] = (uint32_t)s;
        }
    }
}

// the chain enters the top group at candidate 0 (the body's first entry) with 0 entries before
// it; words zeroed, words[3] = the entries on the chain (the top group's count for candidate 0);
// the caller's flag word (the fused pass's out-of-order flag) zeroed
__global__ void k_snap_init(uint32_t *start_top, uint64_t *base_top, const void *cnt_top, int top_u64,
                            unsigned long long *words, uint32_t *segq, uint32_t *flag) {
    if (threadIdx.x != 0) return;
    *start_top = 0;
    *base_top = 0;
    for (int k = 0; k < 8; k++) words[k] = 0;
    words[3] = top_u64 ? *static_cast<const uint64_t *>(cnt_top) : *static_cast<const uint32_t *>(cnt_top);
    if (segq) segq[0] = 0;
    if (flag) *flag = 0;
}

// step 3: G segments per workgroup -> their entries [r0, r1) into the columns.
// res[0] = end of entry n-1, res[1] = inconsistency flag, res[2] = tombstones
__global__ __launch_bounds__(256) void k_snap_decode(const uint8_t *blob, SnapFmt f, uint64_t nseg, uint32_t G,
                                                     uint32_t list_cap, const uint32_t *start, const uint64_t *basev,
                                                     uint64_t n, uint32_t *keys, uint32_t *phys, uint32_t *logical,
                                                     uint32_t *node, uint8_t *tags, uint32_t *values,
                                                     unsigned long long *res, uint32_t *tomb_part) {
    extern __shared__ uint32_t lds[];
    const uint64_t s0 = (uint64_t)blockIdx.x * G;
    const uint32_t nG = (uint32_t)std::min<uint64_t>(G, nseg - s0);
    const uint64_t r0 = basev[s0];
    if (start[s0] == SNAP_BAD || r0 >= n) {  // the whole group is past entry n-1
        if (threadIdx.x == 0) tomb_part[blockIdx.x] = 0;
        return;
    }
    const uint64_t r1 = std::min<uint64_t>(s0 + nG < nseg ? basev[s0 + nG] : n, n);
    const uint64_t a = seg_start(f, s0) & ~15ull;
    const uint64_t b = std::min<uint64_t>(seg_start(f, s0 + nG) + f.lp, f.len);
    const uint32_t img_words = (uint32_t)(((b - a) + 15) / 16 * 4);
    uint32_t *list = lds + img_words;  // entry offsets relative to a
    stage(blob, f.len, a, b, lds);
    __syncthreads();
    const Img m{lds, a};
    __shared__ uint32_t bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    if (threadIdx.x < nG) {  // one lane per segment lists its entries (nG <= blockDim)
        // The chain was validated by k_snap_walk; here only the State variant picks the length.
        // (For a corrupt file the chain is short -- the call reports it -- and this walk stays
        // inside the segment and the LDS image whatever it reads.)
        const uint64_t s = s0 + threadIdx.x;
        const uint32_t x = start[s];
        uint64_t i = basev[s];
        if (x != SNAP_BAD) {
            const uint64_t end = seg_start(f, s + 1);
            const uint32_t o_var = f.key_pre + f.key_len + 20;
            uint64_t p = seg_start(f, s) + (uint64_t)x * f.g;
            while (p < end && i < r1) {
                if (i - r0 >= list_cap) {
                    atomicOr(res + 1, 1ull);
                    bad = 1;
                    break;
                }
                const uint32_t L = m.ld32(p + o_var) == 1 ? f.lt : f.lp;
                list[i - r0] = (uint32_t)(p - a);
                if (i == n - 1) res[0] = p + L;
                p += L;
                i++;
            }
        }
    }
    __syncthreads();
    if (bad) {
        if (threadIdx.x == 0) tomb_part[blockIdx.x] = 0;
        return;
    }
    const uint32_t cnt = (uint32_t)(r1 - r0);
    const uint32_t K4 = f.key_len / 4, V4 = f.val_len / 4;
    const uint32_t o_key = f.key_pre, o_stamp = f.key_pre + f.key_len, o_var = o_stamp + 20, o_val = f.lt + f.val_pre;
    // every column's rows [r0, r1) are contiguous: lane j writes dword j of the range
    for_dwords(cnt, K4, [&](uint32_t j, uint32_t e, uint32_t q) { keys[r0 * K4 + j] = lds[(list[e] + o_key) / 4 + q]; });
    for_dwords(cnt, 2, [&](uint32_t j, uint32_t e, uint32_t q) {
        const uint32_t b4 = (list[e] + o_stamp) / 4 + q;
        phys[r0 * 2 + j] = lds[b4];
        node[r0 * 2 + j] = lds[b4 + 3];
    });
    uint32_t my_tomb = 0;
    for (uint32_t e = threadIdx.x; e < cnt; e += blockDim.x) {
        const uint32_t b4 = (list[e] + o_stamp) / 4;
        logical[r0 + e] = lds[b4 + 2];
        const uint32_t v = lds[b4 + 5];
        tags[r0 + e] = (uint8_t)v;
        my_tomb += v;
    }
    for_dwords(cnt, V4, [&](uint32_t j, uint32_t e, uint32_t q) {
        const uint32_t base = list[e];
        values[r0 * V4 + j] = lds[(base + o_var) / 4] == 0 ? lds[(base + o_val) / 4 + q] : 0u;
    });
    // per-workgroup tombstone count (a same-address atomic per workgroup would serialise
    // ~10^5 workgroups in the L2 atomic unit); summed by k_snap_sum
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) my_tomb += __shfl_xor(my_tomb, k, 64);
    __shared__ uint32_t wsum[4];
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = my_tomb;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < (blockDim.x + 63) / 64; w++) t += wsum[w];
        tomb_part[blockIdx.x] = t;
    }
}

// res[2] += Σ part[0 .. m): a grid-stride pass, one atomic per workgroup (gridDim <= 256)
__global__ __launch_bounds__(1024) void k_snap_sum(const uint32_t *part, uint64_t m, unsigned long long *res) {
    __shared__ unsigned long long w[16];
    unsigned long long t = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x)
        t += part[i];
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)t, k, 64), hi = __shfl_xor((uint32_t)(t >> 32), k, 64);
        t += ((unsigned long long)hi << 32) | lo;
    }
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (uint32_t k = 0; k < blockDim.x / 64; k++) s += w[k];
        if (s) atomicAdd(res + 2, s);
    }
}

}  // namespace

// step 1 and the up-sweep of step 2 (independent of the entry count: a reload starts them before
// it has read the file's header back)
hipError_t snapshot_walk(const SnapFmt &f, const uint8_t *blob, Scratch &s, hipStream_t st, SnapTables *t) {
    const uint32_t P = f.phases;
    if (P > 256 || f.seg + f.lp + 32 > SNAP_LDS) return hipErrorInvalidValue;
    const uint64_t body = f.len > f.base ? f.len - f.base : 0;
    const uint64_t nseg = std::max<uint64_t>(1, (body + f.seg - 1) / f.seg);
    // tree fan-out: a node stages its children's tables (F * P * 12 B) in LDS
    const uint32_t F = std::max<uint32_t>(8, std::min<uint32_t>(SNAP_FAN, SNAP_TREE_LDS / (12 * P)));
    t->sizes.assign(1, nseg);
    while (t->sizes.back() > 1) t->sizes.push_back((t->sizes.back() + F - 1) / F);
    const size_t L = t->sizes.size();
    if (L > 12) return hipErrorInvalidValue;
    t->ex.assign(L, nullptr);
    t->cnt.assign(L, nullptr);  // level 0: u32 per segment, above: u64
    t->lstart.assign(L, nullptr);
    t->lbase.assign(L, nullptr);
    for (size_t l = 0; l < L; l++) {
        t->ex[l] = static_cast<uint32_t *>(s.get(64 + 4 * l, t->sizes[l] * P * 4));
        t->cnt[l] = s.get(65 + 4 * l, t->sizes[l] * P * (l ? 8 : 4));
        t->lstart[l] = static_cast<uint32_t *>(s.get(66 + 4 * l, t->sizes[l] * 4));
        t->lbase[l] = static_cast<uint64_t *>(s.get(67 + 4 * l, t->sizes[l] * 8));
    }
    t->words = static_cast<unsigned long long *>(s.get(97, 64));
    if (s.err) return s.err;
    t->F = F;
    t->nseg = nseg;
    const auto &sizes = t->sizes;
    const auto &ex = t->ex;
    const auto &cnt = t->cnt;
    // staged bytes of a run of G segments: G * seg + lp (+ 16 for the aligned start)
    auto img_bytes = [&](uint32_t G) { return ((uint64_t)G * f.seg + f.lp + 16 + 15) / 16 * 16; };
    // 1. transfer functions.  Small workgroups (one wave when P <= 64) keep the LDS stage small,
    // so many workgroups per CU overlap their dependent walks
    {
        const uint32_t bd = P <= 64 ? 64 : 256;
        uint32_t G = std::max<uint32_t>(1, bd / P);
        while (G > 1 && img_bytes(G) > SNAP_LDS) G--;
        const uint64_t groups = (nseg + G - 1) / G;
        hipLaunchKernelGGL(k_snap_walk, dim3((uint32_t)groups), dim3(bd), (size_t)img_bytes(G), st, blob, f, nseg, G,
                           ex[0], static_cast<uint32_t *>(cnt[0]));
    }
    // 2 (up). compose up to one group
    const size_t up_lds = (size_t)F * P * 12;
    for (size_t l = 0; l + 1 < L; l++) {
        if (l == 0)
            hipLaunchKernelGGL(k_snap_up<uint32_t>, dim3((uint32_t)sizes[1]), dim3(64), up_lds, st, ex[0],
                               static_cast<const uint32_t *>(cnt[0]), sizes[0], P, F, ex[1],
                               static_cast<uint64_t *>(cnt[1]));
        else
            hipLaunchKernelGGL(k_snap_up<uint64_t>, dim3((uint32_t)sizes[l + 1]), dim3(64), up_lds, st, ex[l],
                               static_cast<const uint64_t *>(cnt[l]), sizes[l], P, F, ex[l + 1],
                               static_cast<uint64_t *>(cnt[l + 1]));
    }
    return hipGetLastError();
}

// the down-sweep of step 2 (after snapshot_walk on the same stream): every segment's true first
// entry, and with segq the fused pass's per-block segments; words zeroed, words[3] = entries on
// the chain; *flag zeroed
hipError_t snapshot_place(const SnapFmt &f, uint64_t n, bool with_segq, Scratch &s, hipStream_t st, SnapTables *t,
                          uint32_t *flag) {
    const uint32_t P = f.phases, F = t->F;
    const auto &sizes = t->sizes;
    const auto &ex = t->ex;
    const auto &cnt = t->cnt;
    const auto &start = t->lstart;
    const auto &basev = t->lbase;
    const size_t L = sizes.size();
    const uint64_t nblk = (n + 255) / 256;
    uint32_t *segq = with_segq ? static_cast<uint32_t *>(s.get(99, (nblk + 1) * 4)) : nullptr;
    if (s.err) return s.err;
    const size_t down_lds = (size_t)F * P * 12 + 8ull * (F + 1) + 4ull * F;
    hipLaunchKernelGGL(k_snap_init, dim3(1), dim3(64), 0, st, start[L - 1], basev[L - 1], cnt[L - 1], L > 1 ? 1 : 0,
                       t->words, segq, flag);
    // entries on the chain from the file's first entry are checked against n by the caller: a
    // short chain only leaves rows unwritten, every access stays inside the blob and the outputs
    for (size_t l = L - 1; l-- > 0;) {
        if (l == 0)
            hipLaunchKernelGGL(k_snap_down<uint32_t>, dim3((uint32_t)sizes[1]), dim3(64), down_lds, st, ex[0],
                               static_cast<const uint32_t *>(cnt[0]), sizes[0], P, F, start[1], basev[1], start[0],
                               basev[0], segq, n);
        else
            hipLaunchKernelGGL(k_snap_down<uint64_t>, dim3((uint32_t)sizes[l + 1]), dim3(64), down_lds, st, ex[l],
                               static_cast<const uint64_t *>(cnt[l]), sizes[l], P, F, start[l + 1], basev[l + 1],
                               start[l], basev[l], nullptr, 0);
    }
    t->start = start[0];
    t->basev = basev[0];
    t->segq = segq;
    return hipGetLastError();
}

hipError_t snapshot_locate(const SnapFmt &f, const uint8_t *blob, uint64_t n, bool with_segq, Scratch &s,
                           hipStream_t st, SnapTables *t, uint32_t *flag) {
    hipError_t e = snapshot_walk(f, blob, s, st, t);
    return e ? e : snapshot_place(f, n, with_segq, s, st, t, flag);
}

// LDS of one fused-reload workgroup: the candidate words of the run of segments holding 257
// consecutive entries (or the block-sum tile, which reuses it).  A segment holds at least
// floor(seg / lp) entry starts, so 257 entries span at most 257 / that + 2 segments.  0 when
// that exceeds 64 KiB (or 256 walker lanes).
uint64_t snap_lift_lds_bytes(const SnapFmt &f, uint32_t *nsmax) {
    const uint64_t per = f.lp ? f.seg / f.lp : 0;
    if (per == 0) return 0;
    const uint64_t ns = 257 / per + 2;
    const uint64_t words = (ns * f.seg + f.lp + 16 + 3) / 4 / snap_lift_stride(f) + 8;
    const uint64_t bytes = std::max<uint64_t>((4 * words + 15) / 16 * 16, sizeof(SumTile));
    if (ns > 256 || bytes > 65536) return 0;
    *nsmax = (uint32_t)ns;
    return bytes;
}

hipError_t snapshot_sum_tombstones(const uint32_t *part, uint64_t groups, unsigned long long *words, hipStream_t st) {
    const uint32_t sum_grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(256, (groups + 1023) / 1024));
    hipLaunchKernelGGL(k_snap_sum, dim3(sum_grid), dim3(1024), 0, st, part, groups, words);
    return hipGetLastError();
}

hipError_t snapshot_decode(const SnapFmt &f, const uint8_t *blob, uint64_t n, uint8_t *keys, uint64_t *phys,
                           uint32_t *logical, uint64_t *node, uint8_t *tags, uint8_t *values, Scratch &s,
                           hipStream_t st, SnapResult *res, int *corrupt) {
    *res = SnapResult{};
    *corrupt = 0;
    if (n == 0) {
        res->entries_end = f.base;
        return hipSuccess;
    }
    hipError_t e;
    SnapTables t;
    if ((e = snapshot_locate(f, blob, n, false, s, st, &t))) return e;
    auto img_bytes = [&](uint32_t G) { return ((uint64_t)G * f.seg + f.lp + 16 + 15) / 16 * 16; };
    // 3. list + scatter: one wave per run of G segments (G walker lanes, then all 64 lanes scatter)
    {
        uint32_t G = 4;
        auto lds_bytes = [&](uint32_t g) {
            const uint64_t cap = (uint64_t)g * (f.seg / f.lt + 1);
            return img_bytes(g) + cap * 4;
        };
        while (G > 1 && lds_bytes(G) > SNAP_LDS) G--;
        const uint32_t cap = G * (uint32_t)(f.seg / f.lt + 1);
        const uint64_t groups = (t.nseg + G - 1) / G;
        uint32_t *part = static_cast<uint32_t *>(s.get(98, groups * 4));
        if (s.err) return s.err;
        hipLaunchKernelGGL(k_snap_decode, dim3((uint32_t)groups), dim3(64), (size_t)lds_bytes(G), st, blob, f, t.nseg,
                           G, cap, t.start, t.basev, n, reinterpret_cast<uint32_t *>(keys),
                           reinterpret_cast<uint32_t *>(phys), logical, reinterpret_cast<uint32_t *>(node), tags,
                           reinterpret_cast<uint32_t *>(values), t.words, part);
        if ((e = snapshot_sum_tombstones(part, groups, t.words, st))) return e;
    }
    unsigned long long w[4] = {0, 0, 0, 0};
    if ((e = hipMemcpyAsync(w, t.words, 32, hipMemcpyDeviceToHost, st))) return e;
    if ((e = hipStreamSynchronize(st))) return e;
    res->parsed = w[3];
    if (w[3] < n) {  // the file ends, or stops parsing, before entry n
        *corrupt = 1;
        return hipSuccess;
    }
    if (w[1]) {  // cannot happen for a chain that parsed in step 1
        *corrupt = 2;
        return hipSuccess;
    }
    res->entries_end = w[0];
    res->tombstones = w[2];
    return hipSuccess;
}

}  // namespace rh
