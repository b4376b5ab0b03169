// launch_latency -- the fixed cost of one small launch the host waits for, as the store's tiny
// rounds and questions pay it: hipLaunchKernel returns, the kernel stores a sequence word into
// mapped page-locked (coherent) memory after a system-scope fence, the host polls for it.
// Kernel arguments of 16 B and of ~2.4 KB (RoundTiny's size with its inline segments).
// Prints one JSON line: launch (call) and launch-to-seen times, mean and median over reps.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

struct Small {
    uint64_t *word;
    uint64_t seq;
};
struct Big {
    uint64_t pad[290];
    uint64_t *word;
    uint64_t seq;
};

__global__ void k_small(Small a) {
    __threadfence_system();
    if (threadIdx.x == 0) __hip_atomic_store(a.word, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_big(Big a) {
    __shared__ uint64_t s[64];
    if (threadIdx.x < 64) s[threadIdx.x] = a.pad[threadIdx.x * 4];
    __syncthreads();
    __threadfence_system();
    if (threadIdx.x == 0) __hip_atomic_store(a.word, a.seq + (s[1] & 0), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                           \
        }                                                                       \
    } while (0)

static int wait_word(volatile uint64_t *w, uint64_t seq) {
    const double t0 = now_us();
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != seq)
        if (now_us() - t0 > 1e6) return 1;  // a second: give up (the kernel did not run)
    return 0;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 2000;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint64_t *h = nullptr, *d = nullptr;
    CK(hipHostMalloc((void **)&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer((void **)&d, h, 0));
    *h = 0;
    uint64_t seq = 0;
    double res[2][2];
    for (int kind = 0; kind < 2; kind++) {
        std::vector<double> tl, tw;
        for (int i = 0; i < reps + 50; i++) {
            const double t0 = now_us();
            if (kind == 0) {
                Small a{d, ++seq};
                hipLaunchKernelGGL(k_small, dim3(1), dim3(512), 0, st, a);
            } else {
                Big a{};
                a.word = d, a.seq = ++seq;
                hipLaunchKernelGGL(k_big, dim3(1), dim3(512), 0, st, a);
            }
            const double t1 = now_us();
            if (wait_word(h, seq)) {
                fprintf(stderr, "kernel result word not seen\n");
                CK(hipStreamSynchronize(st));
                return 1;
            }
            const double t2 = now_us();
            if (i >= 50) tl.push_back(t1 - t0), tw.push_back(t2 - t0);
        }
        std::sort(tl.begin(), tl.end());
        std::sort(tw.begin(), tw.end());
        res[kind][0] = tl[tl.size() / 2];
        res[kind][1] = tw[tw.size() / 2];
    }
    CK(hipStreamSynchronize(st));
    printf("{\"reps\": %d, \"small_args_launch_us\": %.2f, \"small_args_seen_us\": %.2f, \"big_args_launch_us\": %.2f, "
           "\"big_args_seen_us\": %.2f}\n",
           reps, res[0][0], res[0][1], res[1][0], res[1][1]);
    CK(hipHostFree(h));
    CK(hipStreamDestroy(st));
    return 0;
}
