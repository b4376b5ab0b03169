// copy_rate.hip -- the HBM copy rate of the compaction's shape: n rows of a 16-byte key array and
// a 32-byte fingerprint array copied to two other arrays (what k_merge_run<16, 32> moves, with no
// merge logic), against hipMemcpyAsync of the same bytes.  Answers whether the compaction merge
// (2.2 ms per 110 M rows, 4.75 TB/s of read + write) is at the copy rate of this access shape.
//   hipcc -O3 --offload-arch=gfx950 microbench/copy_rate.hip -o microbench/copy_rate && ./microbench/copy_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

// each lane moves ROWS rows of (key, fp) per block of 256 rows, all loads issued before the stores
template <int ROWS>
__global__ __launch_bounds__(256) void k_copy_rows(const uint4 *__restrict__ k, const uint4 *__restrict__ f,
                                                   uint4 *__restrict__ ko, uint4 *__restrict__ fo, uint64_t n) {
    const uint64_t r0 = (uint64_t)blockIdx.x * 256 * ROWS + threadIdx.x;
    uint4 a[ROWS], b[ROWS], c[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; j++) {
        const uint64_t r = r0 + 256ull * j;
        if (r < n) { a[j] = k[r]; b[j] = f[2 * r]; c[j] = f[2 * r + 1]; }
    }
#pragma unroll
    for (int j = 0; j < ROWS; j++) {
        const uint64_t r = r0 + 256ull * j;
        if (r < n) { ko[r] = a[j]; fo[2 * r] = b[j]; fo[2 * r + 1] = c[j]; }
    }
}

// a 2,048-row tile per workgroup moved as 8 sequential blocks of 256 rows (one row per lane per
// block, the block's loads then its stores), as k_merge_run walks its tile; BAR: a workgroup
// barrier and an LDS round trip after each block (the merge's block sum)
template <bool BAR>
__global__ __launch_bounds__(256) void k_copy_seq8(const uint4 *__restrict__ k, const uint4 *__restrict__ f,
                                                   uint4 *__restrict__ ko, uint4 *__restrict__ fo, uint64_t n) {
    __shared__ uint32_t t[256];
    uint32_t acc = 0;
    for (int j = 0; j < 8; j++) {
        const uint64_t r = (uint64_t)blockIdx.x * 2048 + 256ull * j + threadIdx.x;
        if (r < n) {
            const uint4 a = k[r], b = f[2 * r], c = f[2 * r + 1];
            ko[r] = a; fo[2 * r] = b; fo[2 * r + 1] = c;
            acc += b.x;
        }
        if constexpr (BAR) {
            t[threadIdx.x] = acc;
            __syncthreads();
            acc += t[(threadIdx.x + 1) & 255];
            __syncthreads();
        }
    }
    if (acc == 0x12345678u) ko[0].x = acc;  // keeps the sums
}

template <class K>
static int run_k(const char *name, K kern, uint64_t rows_per_block, const uint4 *k, const uint4 *f, uint4 *ko, uint4 *fo,
                 uint64_t n, hipStream_t st) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t blocks = (n + rows_per_block - 1) / rows_per_block;
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(256), 0, st, k, f, ko, fo, n);
    CK(hipEventRecord(e0, st));
    const int reps = 10;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(256), 0, st, k, f, ko, fo, n);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / reps, bytes = 2.0 * 48.0 * (double)n;
    printf("{\"kernel\": \"%s\", \"rows\": %llu, \"ms\": %.3f, \"tb_s\": %.3f}\n", name, (unsigned long long)n, per,
           bytes / (per * 1e-3) / 1e12);
    return 0;
}

template <int ROWS>
static int run(const char *name, const uint4 *k, const uint4 *f, uint4 *ko, uint4 *fo, uint64_t n, hipStream_t st) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t blocks = (n + 256 * ROWS - 1) / (256 * ROWS);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k_copy_rows<ROWS>, dim3((uint32_t)blocks), dim3(256), 0, st, k, f, ko, fo, n);
    CK(hipEventRecord(e0, st));
    const int reps = 10;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_copy_rows<ROWS>, dim3((uint32_t)blocks), dim3(256), 0, st, k, f, ko, fo, n);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = ms / reps, bytes = 2.0 * 48.0 * (double)n;
    printf("{\"kernel\": \"%s\", \"rows\": %llu, \"ms\": %.3f, \"tb_s\": %.3f}\n", name, (unsigned long long)n, per,
           bytes / (per * 1e-3) / 1e12);
    return 0;
}

int main(int argc, char **argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 110000000ull;
    uint4 *k, *f, *ko, *fo;
    CK(hipMalloc(&k, n * 16));
    CK(hipMalloc(&f, n * 32));
    CK(hipMalloc(&ko, n * 16));
    CK(hipMalloc(&fo, n * 32));
    CK(hipMemset(k, 1, n * 16));
    CK(hipMemset(f, 2, n * 32));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    if (run<1>("rows1", k, f, ko, fo, n, st) || run<4>("rows4", k, f, ko, fo, n, st) ||
        run<8>("rows8", k, f, ko, fo, n, st) || run_k("seq8", k_copy_seq8<false>, 2048, k, f, ko, fo, n, st) ||
        run_k("seq8_barrier", k_copy_seq8<true>, 2048, k, f, ko, fo, n, st))
        return 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int w = 0; w < 2; w++) {
        CK(hipMemcpyAsync(ko, k, n * 16, hipMemcpyDeviceToDevice, st));
        CK(hipMemcpyAsync(fo, f, n * 32, hipMemcpyDeviceToDevice, st));
    }
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < 10; r++) {
        CK(hipMemcpyAsync(ko, k, n * 16, hipMemcpyDeviceToDevice, st));
        CK(hipMemcpyAsync(fo, f, n * 32, hipMemcpyDeviceToDevice, st));
    }
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"hipMemcpyAsync x2\", \"rows\": %llu, \"ms\": %.3f, \"tb_s\": %.3f}\n", (unsigned long long)n,
           ms / 10, 2.0 * 48.0 * (double)n / (ms / 10 * 1e-3) / 1e12);
    return 0;
}
