// internal.hpp -- declarations shared by the kernel translation units and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rh {

struct DevCols;


// Schema-specialised lift; returns hipErrorInvalidValue-free status, or sets *supported = false
// when no instantiation matches (the caller then reports RH_ERR_UNSUPPORTED).
hipError_t launch_lift_schema(int kk, int kl, int vk, int vl, int rk, bool tags, bool dual,
                              const DevCols &c, uint64_t n, uint8_t *fps, uint8_t *bsums,
                              uint8_t *fps2, uint8_t *bsums2, hipStream_t st, bool *supported);
bool schema_instantiated(int kk, int kl, int vk, int vl);

hipError_t launch_lift_encoded(const uint8_t *bytes, const uint64_t *offs, uint64_t n, uint64_t limit,
                               uint8_t *fps, uint8_t *bsums, hipStream_t st);
// fixed-length records: record i = bytes[i * len, (i + 1) * len), read limit `limit`
hipError_t launch_lift_fixed(const uint8_t *bytes, uint64_t len, uint64_t n, uint64_t limit, uint8_t *fps,
                             uint8_t *bsums, hipStream_t st);
// stride: bytes between consecutive level-0 entries (32 = a fingerprint array)
hipError_t launch_reduce(const uint8_t *in, uint64_t n_in, uint8_t *out, hipStream_t st, uint32_t stride = 32);
// out[0..3] = Σ of n 256-bit entries (n small: one workgroup)
hipError_t launch_total(const uint8_t *in, uint64_t n, uint64_t *out, hipStream_t st);
// Exclusive prefix sums of n fingerprints: out[i] = Σ fps[0..i) for i in [0, n] (n + 1 entries),
// from the run's block sums (ceil(n/256)) and super-block sums (ceil(n/65536)); scratch: spre
// (ceil(n/65536) + 1 entries), bpre (ceil(n/256) + 1 entries), 32 B each.  max_wgs > 0: the row
// level on at most that many workgroups (grid-stride), for a scan beside latency-bound work
hipError_t launch_prefix(const uint8_t *fps, uint64_t n, const uint8_t *bsums, const uint8_t *ssums, uint8_t *spre,
                         uint8_t *bpre, uint8_t *out, hipStream_t st, uint32_t max_wgs = 0);
// launch_prefix's last level only: out[i] = Σ fps [0, i) for i in [0, n], from bpre
hipError_t launch_row_prefix(const uint8_t *fps, uint64_t n, const uint8_t *bpre, uint8_t *out, hipStream_t st);
// launch_prefix's first two levels only: bpre[k] = Σ block sums [0, k), k in [0, ceil(n / 256)]
hipError_t launch_block_prefix(uint64_t n, const uint8_t *bsums, const uint8_t *ssums, uint8_t *spre, uint8_t *bpre,
                               hipStream_t st);
// Rank-addressed merge: out row r of segment k (start[k] <= r < start[k + 1]) is row
// (src[k] & ~2^63) + r - start[k] of `newf` if src[k] has bit 63 set, else of `old`
hipError_t launch_seg_copy(const uint8_t *old, const uint8_t *newf, const uint64_t *start, const uint64_t *src,
                           uint64_t nseg, uint64_t n_out, uint8_t *out, hipStream_t st);
// slots (optional): row i's entry is fps + stride * slots[i] (the store's delta records live in a heap)
hipError_t launch_range_query(const uint8_t *fps, const uint8_t *bsums, const uint8_t *ssums, uint64_t n,
                              const uint64_t *lo, const uint64_t *hi, uint64_t r, uint64_t *out,
                              hipStream_t st, uint32_t stride = 32, const uint32_t *slots = nullptr);

// One rbsr protocol round's output, read back in one copy: a 64-byte header (u64 skipped,
// enumerated, split, children, dropped), then the children (start kinds, end kinds, start keys,
// end keys, aggregates) and the enumerations (kinds and keys), each array 16-byte aligned.
struct RoundLayout {
    uint64_t csk, cek, cskeys, cekeys, caggs, esk, eek, eskeys, eekeys, end;
};
__host__ __device__ inline RoundLayout round_layout(uint64_t nc, uint64_t ne, uint64_t kl) {
    auto pad = [](uint64_t x) { return (x + 15) & ~15ull; };
    RoundLayout o;
    uint64_t p = 64;
    o.csk = p, p += pad(nc);
    o.cek = p, p += pad(nc);
    o.cskeys = p, p += pad(nc * kl);
    o.cekeys = p, p += pad(nc * kl);
    o.caggs = p, p += pad(nc * 40);
    o.esk = p, p += pad(ne);
    o.eek = p, p += pad(ne);
    o.eskeys = p, p += pad(ne * kl);
    o.eekeys = p, p += pad(ne * kl);
    o.end = p;
    return o;
}
// A round's per-segment device arrays: kind (0 skip, 1 IDLIST, 2 SPLIT, 3 dropped), raw rank
// range, local aggregate (5 u64), stride, clamped rank range, children / enumeration counts and
// their exclusive offsets
struct RoundSegs {
    uint8_t *kind;
    uint64_t *lo, *hi, *loc, *stride, *si, *ei, *nch, *choff, *nen, *enoff;
};
// The round's segments as they came in (device: bound kinds, bound keys, remote aggregates) and
// the store's base run
struct RoundIn {
    const uint8_t *sk, *ek, *skeys, *ekeys;
    const uint64_t *remote;
    const uint8_t *bkeys, *fps, *bsums, *ssums;
    // nullable: the base's exclusive prefix over its block sums (launch_block_prefix), which makes
    // any range sum the head and tail rows plus one difference (wave_range_fp_pre)
    const uint8_t *bpre = nullptr;
    // nullable: the base's exclusive prefix over its rows (pre[i] = Σ fps [0, i), n + 1 entries):
    // any range sum is one difference, two loads a lane can take alone (pre_range_fp)
    const uint8_t *pre = nullptr;
};
// A round over the base + the delta run as they stand (no compaction first): the run's entries in
// key order as columns (k_tier_run, the host tier's run copy) -- the contributions (cur - base)
// with their block and super-block sums, the exclusive prefix sums of the count deltas
// (live - in_base), the DeltaRec flags, the base ranks and G(64 k) = live keys <= entry 64 k.  A
// place in the view is (b base rows, j run entries) below it: view rank b + cntp[j]; the sum
// between two places is Σ base[b0, b1) + Σ contrib[j0, j1).
struct RoundRun {
    uint64_t n = 0;
    const uint8_t *keys = nullptr;
    const uint8_t *contrib = nullptr, *bsums = nullptr, *ssums = nullptr;
    const int32_t *cntp = nullptr;
    const uint8_t *flags = nullptr;
    const uint32_t *brank = nullptr;
    const uint64_t *gsamp = nullptr;
    uint64_t nb = 0;
    const uint8_t *bpre = nullptr;  // nullable: the contributions' block prefix (as RoundIn::bpre)
    const uint8_t *pre = nullptr;   // nullable: the contributions' row prefix (as RoundIn::pre)
};
// every segment's view rank range, its places (place[4 j ..]: start b, start j, end b, end j)
// and local aggregate, from the bound keys' base ranks (rank_b) and run ranks (rank_j)
hipError_t launch_round_bounds_view(const uint32_t *rank_b, const uint32_t *rank_j, const RoundIn &in,
                                    const RoundRun &run, const RoundSegs &g, uint64_t *place, uint64_t r,
                                    hipStream_t st);
// a tiny round (r <= round_tiny_max()) over the view in one launch after the two searches
hipError_t launch_round_small_view(const uint32_t *rank_b, const uint32_t *rank_j, const RoundIn &in,
                                   const RoundRun &run, const RoundSegs &g, uint64_t *place, uint64_t r, uint64_t n,
                                   int sqrt_policy, uint64_t b, uint64_t cap, uint32_t kl, uint8_t *out,
                                   hipStream_t st);
// the two-call path's step 1 over the view: bound keys interleaved (row 2 j start, 2 j + 1 end)
hipError_t launch_resolve_view(const uint32_t *rank_b, const uint32_t *rank_j, const uint8_t *sk, const uint8_t *ek,
                               const RoundIn &in, const RoundRun &run, uint64_t r, uint64_t *lo, uint64_t *hi,
                               uint64_t *aggs, hipStream_t st);
// rank-range aggregates over the view (in: only bkeys, fps, bsums, ssums are read)
hipError_t launch_range_query_view(const RoundIn &in, const RoundRun &run, uint32_t kl, uint64_t nv,
                                   const uint64_t *lo, const uint64_t *hi, uint64_t q, uint64_t *out, hipStream_t st);
// select over the view: the keys of ranks[t] (ranks NULL: first + t), each < nv
hipError_t launch_select_view(const RoundRun &run, const uint8_t *bkeys, uint32_t kl, const uint64_t *ranks,
                              uint64_t first, uint64_t m, uint8_t *out, hipStream_t st);
// k_round_emit over the view: cut keys by select over base + run, children's sums over both
hipError_t launch_round_emit_view(const uint64_t *hdr, uint64_t cap, uint64_t r, uint32_t kl, const RoundIn &in,
                                  const RoundRun &run, const RoundSegs &g, const uint64_t *place, uint8_t *out,
                                  hipStream_t st);
// large rounds: decisions (g.lo / g.hi / g.loc filled) -> hdr (zeroed by the caller) gets the
// outcome counts; after the offsets are scanned, children and enumerations into `out`
// (round_layout(hdr children, hdr enumerated, kl)), nothing when the children outnumber cap
// the plan, the child / enumeration offsets and the header in three launches (part: 5 u64 per 256
// segments)
hipError_t launch_round_plan3(const RoundSegs &g, const uint64_t *remote, uint64_t r, uint64_t n, int sqrt_policy,
                              uint64_t b, uint64_t *part, uint64_t *hdr, hipStream_t st);
hipError_t launch_round_plan(const RoundSegs &g, const uint64_t *remote, uint64_t r, uint64_t n, int sqrt_policy,
                             uint64_t b, uint64_t *hdr, hipStream_t st);
hipError_t launch_round_emit(const uint64_t *hdr, uint64_t cap, uint64_t r, uint32_t kl, const RoundIn &in,
                             const RoundSegs &g, uint8_t *out, hipStream_t st);
// the round (round_layout bytes, per the header at hdr; the header alone when the children
// outnumber cap) from src into dst, mapped page-locked memory of at least `worst` bytes
// Device -> host copies as a kernel's 16-byte stores into mapped page-locked memory (dst: the
// mapped buffers' device addresses): ~52 GB/s over PCIe, where the copy engine moves ~30 GB/s
// (microbench/pcie_copy.hip, profiles/r04_pcie_copy.jsonl).  Up to 8 (src, dst, bytes) jobs.
struct CopyJobs {
    const uint8_t *src[8];
    uint8_t *dst[8];
    uint64_t bytes[8];
    int n;
};
// max_wgs: the grid cap (256, one per CU, when the stores cross PCIe beside other work; more
// for a copy within HBM)
hipError_t launch_copy_to_host(const CopyJobs &jobs, hipStream_t st, uint32_t max_wgs = 256);
hipError_t launch_round_copy_out(const uint64_t *hdr, uint64_t cap, uint32_t kl, const uint8_t *src, uint8_t *dst,
                                 uint64_t worst, hipStream_t st);
// every segment's raw rank range (from the searched bound ranks) and local aggregate
hipError_t launch_round_bounds(const uint32_t *rank, const RoundIn &in, const RoundSegs &g, uint64_t r, uint64_t n,
                               hipStream_t st);
// medium rounds (r <= round_small_max()): decisions, offsets and the header in one workgroup
uint64_t round_small_max();
hipError_t launch_round_plan_scan(const RoundIn &in, const RoundSegs &g, uint64_t r, uint64_t n, int sqrt_policy,
                                  uint64_t b, uint8_t *out, hipStream_t st);
// tiny rounds (r <= round_tiny_max()): from the searched bound ranks to `out` in one launch
uint64_t round_tiny_max();
hipError_t launch_round_small(const uint32_t *rank, const RoundIn &in, const RoundSegs &g, uint64_t r, uint64_t n,
                              int sqrt_policy, uint64_t b, uint64_t cap, uint32_t kl, uint8_t *out, hipStream_t st);
hipError_t launch_combine(const uint64_t *in, uint64_t parts, uint64_t r, uint64_t *out, hipStream_t st);

}  // namespace rh
