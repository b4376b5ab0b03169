// snapshot_kernels.hpp -- device decode of an RCNL v1 snapshot's entries (snapshot_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// Locate and decode entries [0, n) of the device blob into SoA columns (keys key_len B,
// phys u64, logical u32, node u64, tags u8 = variant, values val_len B; tombstone values are
// zero-filled).  Synchronises `st`.  *corrupt = 1 if fewer than n entries parse.
hipError_t snapshot_decode(const SnapFmt &f, const uint8_t *blob, uint64_t n, uint8_t *keys, uint64_t *phys,
                           uint32_t *logical, uint64_t *node, uint8_t *tags, uint8_t *values, Scratch &s,
                           hipStream_t st, SnapResult *res, int *corrupt);

}  // namespace rh
