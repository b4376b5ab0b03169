// snapshot_kernels.hpp -- device decode of an RCNL v1 snapshot's entries (snapshot_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "store_kernels.hpp"

namespace rh {

// Byte layout of one bincode (fixint, LE) entry (K, Entry<Timestamp, V>) of
// PersistedState.entries (lww-register/src/persistence.rs:32,62-70):
//   [key_pre: u64 len][key_len]  phys u64 | logical u32 | node u64  variant u32  [val_pre][val_len]
// variant 0 = State::Present (value follows), 1 = State::Tombstone (entry ends).
struct SnapFmt {
    uint64_t base = 16;  // file offset of entry 0: 8 B header + the Vec's u64 length
    uint64_t len = 0;    // bytes in the blob
    uint32_t key_pre = 0, key_len = 0, val_pre = 0, val_len = 0;
    uint32_t lt = 0, lp = 0;  // entry length: tombstone, present
    uint32_t g = 0;           // gcd(lt, lp): every entry starts at base + k * g
    uint32_t phases = 0;      // lp / g: candidate first-entry positions per segment
    uint64_t seg = 0;         // segment bytes (a multiple of g)
};

struct SnapResult {
    uint64_t parsed = 0;       // entries on the true chain before it ends (>= n for a good file)
    uint64_t tombstones = 0;
    uint64_t entries_end = 0;  // file offset just past entry n-1
};

// Where every segment's entries start (snapshot_locate's device tables).  words: [0] end of
// entry n-1, [1] listing inconsistency, [2] tombstones, [3] entries on the chain.
struct SnapTables {
    uint32_t *start = nullptr;   // per segment: first entry position (candidate index) or BAD
    uint64_t *basev = nullptr;   // per segment: index of its first entry
    uint32_t *segq = nullptr;    // per 256-entry block b: segment of entry min(256 b, n) - 1
    unsigned long long *words = nullptr;
    uint64_t nseg = 0;
    // the transfer-function tree between snapshot_walk and snapshot_place (level 0 = segments)
    uint32_t F = 0;
    std::vector<uint64_t> sizes;
    std::vector<uint32_t *> ex, lstart;
    std::vector<void *> cnt;
    std::vector<uint64_t *> lbase;
};
// walk (segments' transfer functions) + the tree's up-sweep: needs the file length, not the
// entry count; snapshot_place then (same stream) pushes the true positions down
hipError_t snapshot_walk(const SnapFmt &f, const uint8_t *blob, Scratch &s, hipStream_t st, SnapTables *t);
hipError_t snapshot_place(const SnapFmt &f, uint64_t n, bool with_segq, Scratch &s, hipStream_t st, SnapTables *t,
                          uint32_t *flag = nullptr);  // *flag zeroed on st
hipError_t snapshot_locate(const SnapFmt &f, const uint8_t *blob, uint64_t n, bool with_segq, Scratch &s,
                           hipStream_t st, SnapTables *t, uint32_t *flag = nullptr);  // both
// words[2] += Σ part[0 .. groups)
hipError_t snapshot_sum_tombstones(const uint32_t *part, uint64_t groups, unsigned long long *words, hipStream_t st);

// The fused reload pass (snap_lift.hpp): block b of 256 entries stages its segments, lists its
// entries, lifts them straight from the staged file bytes (dated, projection or both), writes
// the fingerprints and block sums, the keys and search samples into one or two stores, and flags
// an out-of-order key.
struct SnapLift {
    const uint8_t *blob = nullptr;
    SnapFmt f;
    uint64_t n = 0, nseg = 0;
    const uint32_t *start = nullptr, *segq = nullptr;
    const uint64_t *basev = nullptr;
    uint32_t nsmax = 0;                        // most segments one block's entries (+ predecessor) span
    uint8_t *keys = nullptr, *keys2 = nullptr;  // key rows of the two stores (keys2 may be null)
    uint8_t *fps = nullptr, *bsums = nullptr;   // the dated (or the only) store
    uint8_t *fps2 = nullptr, *bsums2 = nullptr; // the projection store of a dual reload
    unsigned long long *words = nullptr;
    uint32_t *tomb_part = nullptr;              // per block
    uint32_t *unsorted = nullptr;               // set to 1 if a key is not above its predecessor
    uint64_t *smp = nullptr, *smp2 = nullptr;   // the stores' search samples (SMP_STRIDE, SMP2_STRIDE)
    uint64_t *smp_2 = nullptr, *smp2_2 = nullptr;
};
// the fused pass's candidate-word stride: entries start every g bytes, so only every (g / 4)-th
// word can hold a State variant; a power of two dividing g / 4, at most 2
inline int snap_lift_stride(const SnapFmt &f) { return (f.g / 4) % 2 == 0 ? 2 : 1; }
// LDS of one fused-pass workgroup (mode: 0 dated, 1 projection, 2 both); 0: the pass does not
// apply to the format
uint64_t snap_lift_lds_bytes(const SnapFmt &f, uint32_t *nsmax);
// the schema-specialised launch (rsos_hip_abi.hip dispatches over schemas.def)
hipError_t launch_snap_lift_schema(int kk, int kl, int vk, int vl, int mode, const SnapLift &a, uint64_t lds,
                                   hipStream_t st, bool *supported);

// Locate and decode entries [0, n) of the device blob into SoA columns (keys key_len B,
// phys u64, logical u32, node u64, tags u8 = variant, values val_len B; tombstone values are
// zero-filled).  Synchronises `st`.  *corrupt = 1 if fewer than n entries parse.
hipError_t snapshot_decode(const SnapFmt &f, const uint8_t *blob, uint64_t n, uint8_t *keys, uint64_t *phys,
                           uint32_t *logical, uint64_t *node, uint8_t *tags, uint8_t *values, Scratch &s,
                           hipStream_t st, SnapResult *res, int *corrupt);

}  // namespace rh
