// store_kernels.hpp -- interface between the store (rsos_hip_abi.hip) and its device kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "internal.hpp"
#include "lift_kernels.hpp"

namespace rh {

// Growable device scratch buffers in numbered slots, reused across calls.  Growing a slot
// drains `stream` first, so no in-flight kernel still reads the freed buffer.
struct Scratch {
    hipStream_t stream = nullptr;
    struct Slot {
        void *p = nullptr;
        size_t bytes = 0;
    };
    std::vector<Slot> slots;
    hipError_t err = hipSuccess;

    void *get(size_t idx, size_t bytes) {
        if (slots.size() <= idx) slots.resize(idx + 1);
        Slot &s = slots[idx];
        bytes = std::max<size_t>(bytes, 256);
        if (s.bytes < bytes) {
            static const bool dbg = getenv("RSOS_HIP_ALLOC_DBG") != nullptr;  // every regrowth, to stderr
            if (dbg && s.p) fprintf(stderr, "rsos_hip: scratch slot %zu grows %zu -> %zu bytes\n", idx, s.bytes, bytes);
            if (s.p) {
                (void)hipStreamSynchronize(stream);
                (void)hipFree(s.p);
            }
            s.p = nullptr;
            s.bytes = 0;
            const size_t want = (bytes + (bytes >> 3) + 255) & ~size_t(255);  // +12.5% headroom
            hipError_t e = hipMalloc(&s.p, want);
            if (e != hipSuccess) {
                err = e;
                return nullptr;
            }
            s.bytes = want;
        }
        return s.p;
    }
    uint32_t *u32(int k, size_t n) { return static_cast<uint32_t *>(get(0 + k, n * 4)); }
    uint64_t *u64(int k, size_t n) { return static_cast<uint64_t *>(get(16 + k, n * 8)); }
    uint8_t *u8(int k, size_t n) { return static_cast<uint8_t *>(get(32 + k, n)); }
    int32_t *i32(int k, size_t n) { return static_cast<int32_t *>(get(48 + k, n * 4)); }
    void *bytes(size_t n) { return get(63, n); }
    void release() {
        (void)hipStreamSynchronize(stream);
        for (auto &s : slots)
            if (s.p) (void)hipFree(s.p);
        slots.clear();
    }
};

// One entry of the store's delta run (40 B): what the batches since the last compaction did to
// a key.  contrib = cur - base (mod 2^256); count delta = live - in_base.  brank is the key's
// lower-bound rank in the base run: the base does not change until the next compaction, so it
// locates the base fingerprint (cur = base_fps[brank] + contrib) and the key's slot in the
// compaction merge without searching again.
// Rows are moved as five 8-byte words (no padding to 48: the delta merge and the compaction
// move 56 instead of 64 bytes per row).
struct alignas(8) DeltaRec {
    enum : uint32_t { IN_BASE = 1, LIVE = 2 };
    uint32_t contrib[8];
    uint32_t brank;
    uint32_t flags;
};
static_assert(sizeof(DeltaRec) == 40, "DeltaRec layout (k_merge_run reads flags as word 9)");

// a run's search samples: the leading key digit of every SMP_STRIDE-th and SMP2_STRIDE-th row
constexpr uint64_t SMP_STRIDE = 256, SMP2_STRIDE = 8;  // 8 x 16-byte keys = one 128-byte line
// entries of a run's second-level (stride SMP2_STRIDE) sample array for n rows, with slack
uint64_t sample2_entries(uint64_t n);
// A run's search table (k_search_table): tab has 2^bits + 1 entries, par = (min digit, shift).
struct SearchTable {
    const uint32_t *tab = nullptr;
    const uint64_t *par = nullptr;
    uint32_t bits = 0;
};
// one sampled search over a sorted run (k_search_sampled; the batch path's fused lift + search,
// lift_search.hpp): the lower-bound rank and presence of each query key
struct SearchJob {
    const uint8_t *keys;
    uint64_t n;
    const uint64_t *smp, *smp2;
    SearchTable tb;
    uint32_t *rank;
    uint8_t *present;
};
// the next batch's keys whose leading-digit (min, max) partials a k_lift_search also forms:
// ceil(m / MINMAX_TILE) pairs into part (keys == nullptr: none)
struct NextMinmax {
    const uint8_t *keys = nullptr;
    uint64_t m = 0;
    uint64_t *part = nullptr;
};
// table size for a run of n rows, and its build from the run's second-level samples
// (base: the base run's fine table, ~1 sample per bucket; otherwise a delta run's, ~8)
uint32_t search_table_bits(uint64_t n, bool base = true);
hipError_t launch_search_table(const uint64_t *smp2, uint64_t n, uint32_t *tab, uint64_t *par, hipStream_t st,
                               bool base = true);

// largest batch the bucket sort orders (larger ones take the LSD radix sort)
constexpr uint64_t SORT_BUCKET_MAX = 2ull << 20;
// keys per workgroup of k_lift_search's digit min / max role (its partials replace k_cs_minmax's)
constexpr uint64_t MINMAX_TILE = 2048;

// Key-type-specialised device operations of the store.
// A tiny protocol round in one launch (round_tiny.hpp k_round_tiny): the segments, the base and
// delta runs with their search samples, where the round goes
constexpr uint32_t ROUND_TINY_SEGS = 16, ROUND_TINY_KL = 32;  // = ROUND_TINY; the widest key
struct RoundTiny {
    // the segments, inline in the kernel's arguments: the kernel reads them where the runtime put
    // them (in device memory), not over PCIe from page-locked memory -- 2.9 us a round as mapped input
    uint64_t irem[5 * ROUND_TINY_SEGS];               // the peer's aggregates
    uint8_t ikeys[2 * ROUND_TINY_SEGS * ROUND_TINY_KL];  // start keys, then end keys (kl bytes each)
    uint8_t isk[ROUND_TINY_SEGS], iek[ROUND_TINY_SEGS];
    RoundIn in;  // sk, ek, skeys, ekeys, remote: the mapped copy (unread); bkeys, fps, sums: the base
    RoundRun run;  // run.n == 0: no delta run (run.nb = the base rows either way)
    const uint64_t *bsmp, *bsmp2;  // the base run's search samples and table
    SearchTable btab;
    const uint64_t *dsmp, *dsmp2;  // the delta run's (its keys: run.keys)
    RoundSegs g;                   // global copies of the per-segment arrays, written only when the
    uint64_t *gplace;              // children outnumber cap (the host then emits again from them)
    uint64_t r, n;                 // segments; live keys of base + run
    int sqrt_policy;
    uint64_t b, cap;
    uint8_t *out;                  // round_layout (mapped page-locked)
    uint64_t seq;                  // stored to out word 7 last
    uint64_t *dbg;                 // nullable: per-phase real-time clocks (RSOS_HIP_ROUND_DBG)
};

// The small questions in one launch (round_tiny.hpp k_query_tiny), over the base run and any delta
// run (as columns, RoundRun; run.n == 0: none): mode 0, the ranks of m <= QUERY_TINY keys; mode 1,
// the keys of m <= QUERY_TINY ranks (select); mode 2, one key-range aggregate.  The question in
// the kernel's arguments, the answer in mapped page-locked memory with a sequence word stored last.
constexpr uint32_t QUERY_TINY = 64;
struct QueryTiny {
    // the question, inline in the kernel's arguments (as RoundTiny's segments): mode 0, m keys;
    // 1, m u64 ranks (each < the view's size); 2, lo key, hi key
    uint64_t in[QUERY_TINY * ROUND_TINY_KL / 8];
    int mode;
    uint64_t m;
    int lo_kind, hi_kind;  // mode 2: 0 unbounded, 1 included, 2 excluded (std::ops::Bound)
    RoundIn base;          // bkeys, fps, bsums, ssums
    RoundRun run;
    const uint64_t *bsmp, *bsmp2;
    SearchTable btab;
    const uint64_t *dsmp, *dsmp2;
    uint8_t *out;          // mode 0: m u64; 1: m keys; 2: one rh_aggregate
    uint64_t *seq_word;
    uint64_t seq;
};

struct StoreKeyOps {
    virtual ~StoreKeyOps() = default;
    // sort a batch by key (stable) and gather keys / fingerprints / ops into key order; with
    // fps == nullptr, pos[input row] = its sorted row instead (exactly one of fps / pos given),
    // for the batch path's lift, which runs after the sort and writes each fingerprint in place.
    // pre_part (bucket sort only): pre_npart (min, max) pairs of the keys' leading digits already
    // computed (k_lift_search of the previous batch), in place of the sort's own min / max pass.
    // full = false: coarse buckets of the most significant u64 digit + a sort of each bucket in
    // LDS (ties on that digit broken by the whole key); *flags |= 4 if the digits are too skewed
    // for the buckets, and (multi-digit keys past the bucket path's size) |= 2 if two keys share
    // the digit: the order is then not final -- sort again with full = true, the LSD radix over
    // every digit.  *flags |= 1 if two batch keys are equal.  *flags is zeroed first (in stream
    // order) by the sort itself.
    // s2o (bucket sort with pos only): the positions in two levels -- pos[input row] = its slot in
    // its bucket's stretch (written by the scatter in input order), s2o[slot] = its sorted row
    // (written by the bucket sort in slot order): whole-line writes both, where one level is a
    // 4-byte store per row scattered over the whole batch.  The full sort ignores it (one level).
    // Without ops, equal keys are ordered by slot rather than input row (they only reject the batch).
    virtual hipError_t sort_batch(const uint8_t *keys, const uint8_t *fps, const uint8_t *ops, uint64_t m,
                                  Scratch &s, uint8_t *skeys, uint8_t *sfps, uint8_t *sops, uint32_t *flags,
                                  bool full, hipStream_t st, uint32_t *pos = nullptr,
                                  const uint64_t *pre_part = nullptr, uint32_t pre_npart = 0,
                                  uint32_t *s2o = nullptr) = 0;
    // lower-bound rank of each query key (and whether it is present)
    virtual hipError_t search(const uint8_t *keys, uint64_t n, const uint8_t *q, uint64_t m, uint32_t *rank,
                              uint8_t *present, hipStream_t st) = 0;
    // smp[s] = leading digit of keys[256 s] (ceil(n / 256) entries), smp2 (optional) the same
    // for every 8th key, and the lower-bound search through them (same results as search)
    virtual hipError_t sample(const uint8_t *keys, uint64_t n, uint64_t *smp, uint64_t *smp2, hipStream_t st) = 0;
    // (tb: the run's search table, which replaces the stride-256 level; needs smp2)
    virtual hipError_t search_sampled(const uint8_t *keys, uint64_t n, const uint64_t *smp, const uint64_t *smp2,
                                      const uint8_t *q, uint64_t m, uint32_t *rank, uint8_t *present,
                                      hipStream_t st, SearchTable tb = SearchTable{}) = 0;
    virtual hipError_t check_sorted(const uint8_t *keys, uint64_t n, uint32_t *bad, hipStream_t st) = 0;
    // keep the last row of every run of equal keys of a key-sorted run (a stable sort keeps
    // input order within a run, so this is "the last insert wins"); counts[0] = rows kept
    virtual hipError_t dedup_last(const uint8_t *keys, const uint8_t *fps, uint64_t n, Scratch &s, uint8_t *okeys,
                                  uint8_t *ofps, uint64_t *counts, hipStream_t st) = 0;
    virtual hipError_t bounds(const uint8_t *keys, uint64_t n, const uint8_t *lo_key, int lo_kind,
                              const uint8_t *hi_key, int hi_kind, uint64_t *qlo, uint64_t *qhi, hipStream_t st) = 0;
    // keep[i] (i < m) = 1 unless input row i's sorted successor has its key; keep[m] = 0
    virtual hipError_t keep_last_rows(const uint8_t *skeys, const uint32_t *pos, const uint32_t *s2o, uint64_t m,
                                      uint32_t *keep, hipStream_t st) = 0;
    // keys[64 j] leading digits, j < ceil(n / stride): the host tier's sample array
    virtual hipError_t sample_stride(const uint8_t *keys, uint64_t n, uint64_t stride, uint64_t *smp, hipStream_t st) = 0;
    // the key type's Ord on the host (for argument checks)
    virtual int compare_keys_host(const uint8_t *a, const uint8_t *b) const = 0;
    // a whole tiny round (a.r <= ROUND_TINY segments) in one launch of one workgroup
    virtual hipError_t round_tiny(const RoundTiny &a, hipStream_t st) = 0;
    // ranks, selects or a key-range aggregate (QueryTiny) in one launch of one workgroup
    virtual hipError_t query_tiny(const QueryTiny &a, hipStream_t st) = 0;
};

// Σ count deltas of delta rows [0, i] = sblk[i / 65536] (exclusive super-block prefix)
// + blk[i / 256 - 1] (inclusive block prefix inside the super-block; 0 for its first block)
// + inb[i] (inclusive prefix inside the row's 256-row block)
struct CntPrefix {
    const int32_t *sblk;
    const int32_t *blk;
    const int16_t *inb;
};
// after a delta merge: blk -> in-super-block prefixes, super-block sums, sblk, the count and
// contribution totals (one launch; scnt: ns scratch ints, *ticket 0 on entry and exit)
hipError_t launch_delta_finish(const uint8_t *bsums, int32_t *blk, uint64_t nbk, uint8_t *ssums, int32_t *scnt,
                               int32_t *sblk, uint32_t *ticket, int32_t *total, uint64_t *fp_total, hipStream_t st);


// delta-run kernels (store_kernels.hip)
// The batch path after the searches.  The delta run is rows of (key, slot): a slot indexes the
// record heap, where every batch appends its DeltaRecs (heap_base + j for sorted batch row j);
// a merge moves keys and slots and gathers the records only for the block sums and count
// prefixes.  This launch: the batch's DeltaRecs (from its sorted fingerprints / ops and what
// base and delta hold for each key; dops 0 = upsert into the delta run, 1 = drop the key's
// entry), its counts vs the merged view (counts3: new, overwritten, deleted), the merge lists,
// and the merge into the delta run's other buffer: keys, slots and search samples (obs / ocnt /
// oinb unused: the run's sums are formed lazily, launch_delta_sums); mcnt: [0]
// inserts, [1] overwrites, [2] removals, [3] upserts, [4] batch keys the run held; out3 the first
// three.
hipError_t launch_delta_apply(int kk, int kl, const uint8_t *sfps, const uint8_t *sops, uint64_t m,
                              const uint32_t *rank_b, const uint8_t *present_b, const uint8_t *base_fps,
                              const uint32_t *rank_d, const uint8_t *present_d, const uint8_t *dkeys,
                              const uint32_t *dslot, uint64_t nd, uint8_t *heap, uint64_t heap_base,
                              const uint8_t *skeys, uint8_t *dops, uint64_t *counts3, Scratch &s, uint8_t *okeys,
                              uint32_t *oslot, uint8_t *obs, int32_t *ocnt, int16_t *oinb, uint64_t nbk,
                              uint64_t *mcnt, uint64_t *out3, uint64_t *osmp, uint64_t *osmp2, uint64_t *dtot,
                              int64_t *dcnt, hipStream_t st);
// the delta run's block sums and count prefixes (what launch_delta_finish completes), formed
// lazily: the batch path keeps only the run's totals (dtot: Σ contributions' change, dcnt: count
// change, per batch)
hipError_t launch_delta_sums(const uint32_t *dslot, const uint8_t *heap, uint64_t n, uint8_t *obs, int32_t *ocnt,
                             int16_t *oinb, hipStream_t st);
// The compaction: the delta run's current fingerprints (contrib + the base's at brank), ops and
// base slots, the merge lists, and the merge of the delta run into the base run (keys, fps, block
// sums, search samples; mcnt as launch_merge_run's counts).  cfps / cops: nd * 32 / nd bytes.
hipError_t launch_compact(int key_kind, int kl, const uint8_t *bkeys, const uint8_t *bfps, uint64_t nb,
                          const uint8_t *dkeys, const uint32_t *dslot, const uint8_t *heap, uint64_t nd, Scratch &s,
                          uint8_t *cfps, uint8_t *cops, uint8_t *okeys, uint8_t *ofps, uint8_t *obs, uint64_t nbk, uint64_t *mcnt, uint64_t *osmp,
                          uint64_t *osmp2, hipStream_t st);
hipError_t launch_agg_merge(const uint64_t *base_agg, const uint64_t *delta_agg, const uint64_t *dlo,
                            const uint64_t *dhi, CntPrefix cp, uint64_t *out, hipStream_t st);
hipError_t launch_rank_merge(const uint32_t *rank_b, const uint32_t *rank_d, CntPrefix cp, uint64_t m,
                             uint64_t *out, hipStream_t st);

// protocol round: segment bounds -> base-run rank ranges (rank: 2 searched ranks per segment),
// and the keys at given ranks (kl a multiple of 4)
hipError_t launch_resolve_bounds(const uint32_t *rank, const uint8_t *skind, const uint8_t *ekind, uint64_t r,
                                 uint64_t n, uint64_t *lo, uint64_t *hi, hipStream_t st);
hipError_t launch_gather_keys(const uint8_t *keys, uint32_t kl, const uint64_t *sel, uint64_t m, uint8_t *out,
                              hipStream_t st);
// The delta merge alone (the small-batch path, small_batch.hpp): batch rows skeys [0, m) with the
// lists and counts (mcnt) its front wrote, merged into the delta run (keys + slots) -- the last
// step of launch_delta_apply.
hipError_t launch_delta_merge(int kk, int kl, const uint8_t *dkeys, const uint32_t *dslot, uint64_t nd,
                              const uint8_t *skeys, uint64_t m, const uint32_t *upos, const uint32_t *usrc,
                              const uint32_t *rlist, const uint64_t *mcnt, uint8_t *okeys, uint32_t *oslot,
                              uint64_t nbk, uint64_t *osmp, uint64_t *osmp2, const uint8_t *heap, uint64_t heap_base,
                              hipStream_t st);
// A batch with repeated keys reduced to the last row of each key, in input order (the staged
// batch's rule, rh_store_stage): keep[i] = 1 unless input row i's sorted successor (pos: each input
// row's sorted row, skeys: the stable key sort) has the same key; keep[m] = 0 (for the scan).
// Then dst = the exclusive scan of keep over m + 1 entries (dst[m] = rows kept), and each column
// compacted with launch_compact_rows.
hipError_t launch_compact_rows(const uint8_t *src, uint32_t row_bytes, const uint32_t *keep, const uint32_t *dst,
                               uint64_t m, uint8_t *out, hipStream_t st);
hipError_t launch_exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, Scratch &s, hipStream_t st);
// the delta run's DeltaRecs as the host tier's run-copy columns (k_tier_run); cnt has n + 1 entries
// (bsums: the 256-entry blocks' contribution sums too, nullable)
hipError_t launch_tier_run(const uint32_t *slot, const uint8_t *heap, uint64_t n, uint8_t *contrib, uint32_t *cnt,
                           uint8_t *flags, uint32_t *brank, hipStream_t st, uint8_t *bsums = nullptr);
// and select's index over it: entry 64 k's live keys at or below it (k_tier_gsamp)
hipError_t launch_tier_gsamp(const uint32_t *brank, const uint32_t *cntp, const uint8_t *flags, uint64_t n,
                             uint64_t *gsamp, hipStream_t st);
// All the run's columns at once for a short run (n <= RUNCOL_SMALL), one launch of one workgroup
// (k_run_columns_small): what launch_tier_run, two launch_reduce, launch_prefix, the count scan and
// launch_tier_gsamp form in eight launches
struct RunCols {
    uint8_t *contrib;
    uint32_t *cnt;
    uint8_t *flags;
    uint32_t *brank;
    uint8_t *pre, *bsums, *ssums, *spre, *bpre;  // row prefix (n + 1), block / super-block sums and prefixes
    uint32_t *cntp;                              // the count deltas' exclusive prefix (n + 1)
    uint64_t *gsamp;
};
constexpr uint64_t RUNCOL_SMALL = 4095;
hipError_t launch_run_columns_small(const uint32_t *slot, const uint8_t *heap, uint64_t n, const RunCols &o,
                                    hipStream_t st);
// pre-size the scratch slots a compaction of up to `plan` delta rows and a batch of `batch` rows use
// base_rows: the largest base a compaction writes (its merge tiles' bounds)
hipError_t reserve_merge_scratch(Scratch &s, uint64_t plan, uint64_t batch, uint64_t base_rows = 0);
hipError_t launch_exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, Scratch &s, hipStream_t st);

// nullptr if the store does not support this key type
StoreKeyOps *store_key_ops(int key_kind, int key_len);

}  // namespace rh
