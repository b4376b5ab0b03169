// fp_device.hpp -- 256-bit fingerprint words on the device (the Fingerprint group,
// rsos/src/fingerprint.rs:145-173: add with carry, subtract with borrow, mod 2^256), shared by the
// store kernels (store_kernels.hip) and the per-schema small-batch kernel (small_batch.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rh {

__device__ __forceinline__ void fp_load(const uint8_t *p, uint32_t f[8]) {
    const uint4 a = reinterpret_cast<const uint4 *>(p)[0], b = reinterpret_cast<const uint4 *>(p)[1];
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void fp_store(uint8_t *p, const uint32_t f[8]) {
    reinterpret_cast<uint4 *>(p)[0] = make_uint4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<uint4 *>(p)[1] = make_uint4(f[4], f[5], f[6], f[7]);
}
__device__ __forceinline__ void fp_add(const uint32_t a[8], const uint32_t b[8], uint32_t o[8]) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)a[i] + b[i] + c;
        o[i] = (uint32_t)t;
        c = t >> 32;
    }
}
__device__ __forceinline__ void fp_sub(const uint32_t a[8], const uint32_t b[8], uint32_t o[8]) {
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t t = (uint64_t)a[i] - b[i] - br;
        o[i] = (uint32_t)t;
        br = (t >> 63) & 1;  // borrow out
    }
}

__device__ __forceinline__ void words_of(const uint4 &v, uint32_t *w) {
    w[0] = v.x;
    w[1] = v.y;
    w[2] = v.z;
    w[3] = v.w;
}
__device__ __forceinline__ void words_of(const uint2 &v, uint32_t *w) {
    w[0] = v.x;
    w[1] = v.y;
}

}  // namespace rh
