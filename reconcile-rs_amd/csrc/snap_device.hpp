// snap_device.hpp -- device helpers shared by the snapshot locate kernels (snapshot_kernels.hip)
// and the fused locate + lift kernel (snap_lift.hpp): staging a run of the file in LDS and
// reading entry lengths from it.  The entry layout is SnapFmt's (snapshot_kernels.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "snapshot_kernels.hpp"

namespace rh {
namespace snap {

constexpr uint32_t BAD = 0xffffffffu;

// A run of the blob staged in LDS: bytes [a, a + 4 * words) (a 16-aligned), zero past the end.
struct Img {
    const uint32_t *w;
    uint64_t a;
    __device__ __forceinline__ uint32_t ld32(uint64_t p) const { return w[(p - a) >> 2]; }
    __device__ __forceinline__ uint64_t ld64(uint64_t p) const {
        return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32);
    }
};

// the 16 bytes at q, zero past `len`
__device__ __forceinline__ uint4 load16(const uint8_t *blob, uint64_t len, uint64_t q) {
    if (q + 16 <= len) return *reinterpret_cast<const uint4 *>(blob + q);
    uint32_t t[4];
#pragma unroll
    for (int d = 0; d < 4; d++) {
        uint32_t x = 0;
        for (int k = 0; k < 4; k++) {
            const uint64_t o = q + 4 * d + k;
            if (o < len) x |= (uint32_t)blob[o] << (8 * k);
        }
        t[d] = x;
    }
    return make_uint4(t[0], t[1], t[2], t[3]);
}

// stage blob bytes [a, b) (a 16-aligned) into lds; bytes at or past `len` read as 0.  Each lane
// issues up to STAGE_U 16-byte loads before its first LDS store, so a workgroup keeps several
// KiB in flight instead of one load per round trip.
constexpr int STAGE_U = 8;
__device__ __forceinline__ void stage(const uint8_t *blob, uint64_t len, uint64_t a, uint64_t b, uint32_t *lds) {
    const uint64_t step = 16ull * blockDim.x;
    for (uint64_t q0 = a + 16ull * threadIdx.x; q0 < b; q0 += step * STAGE_U) {
        uint4 v[STAGE_U];
#pragma unroll
        for (int u = 0; u < STAGE_U; u++) {
            const uint64_t q = q0 + step * u;
            if (q < b) v[u] = load16(blob, len, q);
        }
#pragma unroll
        for (int u = 0; u < STAGE_U; u++) {
            const uint64_t q = q0 + step * u;
            if (q < b) *reinterpret_cast<uint4 *>(lds + ((q - a) >> 2)) = v[u];
        }
    }
}

// length of the entry starting at p, or 0 if no valid entry starts there.  The image must
// cover p + lp or the end of the file.
__device__ __forceinline__ uint32_t entry_len(const Img &m, const SnapFmt &f, uint64_t p) {
    if (p + f.lt > f.len) return 0;
    // the variant and both Vec lengths in one LDS round trip (the value's length word is read
    // even for a tombstone: it lies inside the staged run, and only a present entry checks it)
    const uint32_t v = m.ld32(p + f.key_pre + f.key_len + 20);
    const uint64_t kl = f.key_pre ? m.ld64(p) : f.key_len;
    const uint64_t vl = f.val_pre ? m.ld64(p + f.lt) : f.val_len;
    if (kl != f.key_len) return 0;
    if (v == 1) return f.lt;
    if (v != 0 || p + f.lp > f.len || vl != f.val_len) return 0;
    return f.lp;
}

__device__ __forceinline__ uint64_t seg_start(const SnapFmt &f, uint64_t s) { return f.base + s * f.seg; }

// lane-strided walk over cnt rows of W dwords: fn(j, row, dword) with j = row * W + dword; the
// (row, dword) pair is advanced incrementally -- one division per lane, not one per dword
template <class Fn>
__device__ __forceinline__ void for_dwords(uint32_t cnt, uint32_t W, Fn fn) {
    if (W == 0) return;
    uint32_t e = threadIdx.x / W, q = threadIdx.x - e * W;
    const uint32_t de = blockDim.x / W, dq = blockDim.x - de * W;
    for (uint32_t j = threadIdx.x; j < cnt * W; j += blockDim.x) {
        fn(j, e, q);
        q += dq;
        e += de;
        if (q >= W) {
            q -= W;
            e++;
        }
    }
}

}  // namespace snap
}  // namespace rh
