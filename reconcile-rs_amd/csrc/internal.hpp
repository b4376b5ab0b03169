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
hipError_t launch_range_query(const uint8_t *fps, const uint8_t *bsums, const uint8_t *ssums, uint64_t n,
                              const uint64_t *lo, const uint64_t *hi, uint64_t r, uint64_t *out,
                              hipStream_t st, uint32_t stride = 32);
hipError_t launch_combine(const uint64_t *in, uint64_t parts, uint64_t r, uint64_t *out, hipStream_t st);

}  // namespace rh
