// pcie_copy.hip -- host <-> device copy rates of round-sized buffers (1-8 MiB) by page-locked
// allocation flags, and the rates of a kernel that writes / reads mapped host memory in whole lines: what a
// large protocol round's input / output copies could cost.
//   hipcc -O3 --offload-arch=gfx950 microbench/pcie_copy.hip -o /tmp/pcie_copy && /tmp/pcie_copy
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_write_lines(uint4 *dst, const uint4 *src, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t sizes[3] = {1u << 20, 3u << 20, 8u << 20};
    const unsigned flags[3] = {hipHostMallocDefault, hipHostMallocMapped | hipHostMallocNonCoherent,
                               hipHostMallocMapped | hipHostMallocCoherent};
    const char *names[3] = {"default", "mapped|noncoherent", "mapped|coherent"};
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    uint8_t *d;
    CK(hipMalloc(&d, 8u << 20));
    CK(hipMemset(d, 1, 8u << 20));
    for (int f = 0; f < 3; f++) {
        uint8_t *h;
        CK(hipHostMalloc(&h, 8u << 20, flags[f]));
        memset(h, 2, 8u << 20);
        for (int s = 0; s < 3; s++) {
            const size_t n = sizes[s];
            float best_d2h = 1e9, best_h2d = 1e9, best_k = 1e9;
            for (int rep = 0; rep < 20; rep++) {
                float ms;
                CK(hipEventRecord(a, st));
                CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, st));
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best_d2h) best_d2h = ms;
                CK(hipEventRecord(a, st));
                CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st));
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best_h2d) best_h2d = ms;
                if (f > 0) {
                    uint8_t *hd;
                    CK(hipHostGetDevicePointer((void **)&hd, h, 0));
                    CK(hipEventRecord(a, st));
                    hipLaunchKernelGGL(k_write_lines, dim3(1024), dim3(256), 0, st, (uint4 *)hd, (const uint4 *)d, n / 16);
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                    if (ms < best_k) best_k = ms;
                }
            }
            float best_r = 1e9;
            if (f > 0) {  // a kernel reading mapped host memory into device memory (the reverse)
                uint8_t *hd;
                CK(hipHostGetDevicePointer((void **)&hd, h, 0));
                for (int rep = 0; rep < 20; rep++) {
                    float ms;
                    CK(hipEventRecord(a, st));
                    hipLaunchKernelGGL(k_write_lines, dim3(1024), dim3(256), 0, st, (uint4 *)d, (const uint4 *)hd, n / 16);
                    CK(hipEventRecord(b, st));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                    if (ms < best_r) best_r = ms;
                }
            }
            printf("{\"alloc\": \"%s\", \"bytes\": %zu, \"d2h_us\": %.1f, \"d2h_GBs\": %.1f, \"h2d_us\": %.1f, \"h2d_GBs\": %.1f, "
                   "\"kernel_write_us\": %.1f, \"kernel_write_GBs\": %.1f, \"kernel_read_us\": %.1f, \"kernel_read_GBs\": %.1f}\n",
                   names[f], n, best_d2h * 1e3, n / (best_d2h * 1e6), best_h2d * 1e3, n / (best_h2d * 1e6),
                   f ? best_k * 1e3 : 0.0, f ? n / (best_k * 1e6) : 0.0, f ? best_r * 1e3 : 0.0,
                   f ? n / (best_r * 1e6) : 0.0);
        }
        CK(hipHostFree(h));
    }
    return 0;
}
