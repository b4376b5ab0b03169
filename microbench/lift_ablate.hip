// lift_ablate.hip -- time the 16 B / 64 B dated lift kernel against two ablations on the same
// 10 M records: MEM (all loads + stores, hash replaced by an XOR fold) and ALU (hash of words
// synthesised from the row index, no record loads).  Standalone diagnostic, not shipped.
#include "../reconcile-rs_amd/csrc/lift_kernels.hpp"
#include <cstdio>
#include <vector>

using namespace rh;

namespace rh {
// ---- persistent, software-pipelined form (whole record in registers) ----------------------
//
// The hash is VALU-bound (~3.8 issue cycles per instruction on gfx950, ~2,750 cycles per
// wave-compression), so the kernel's job is to keep the VALU busy: each workgroup owns a
// contiguous run of 256-row blocks and, while it hashes block b, the loads of block b+1 are
// already in flight into registers.  One-record-per-lane launches instead stall every wave
// of a CU on its loads at the same moment (all waves of a dispatch start together).
template <class L, int KK, int KL, int RK, bool TAGS>
struct RecRegs {
    static constexpr int KWN = L::KEY_ENC / 4 > 0 ? L::KEY_ENC / 4 : 1;
    uint32_t kw[KWN];
    uint32_t sw[5];
    uint32_t vw[L::VW > 0 ? L::VW : 1];
    bool tomb;

    __device__ __forceinline__ void load(const DevCols &c, uint64_t i) {
        load_key<KK, KL>(c.keys, i, kw);
        if constexpr (RK == REC_DATED) load_stamp(c, i, sw);
        if constexpr (L::VW > 0) ldw<L::VW, L::ROW_ALIGN>(c.values + i * (uint64_t)L::VAL_ROW, vw);
        tomb = TAGS ? (c.tags[i] != 0) : false;
    }
};

// lift of a record held in registers, as layout L2 (DATED or PROJECTION view of the same record)
template <class L2, int KK, int RK2, class R>
__device__ __forceinline__ void lift_regs(const R &r, uint32_t h[8]) {
    if (RK2 != REC_PLAIN && r.tomb) {
        uint32_t w[L2::LEN_TOMB / 4];
        build_prefix<L2, KK, RK2>(r.kw, r.sw, true, w);
        hash_words<L2::LEN_TOMB>(w, h);
    } else {
        uint32_t w[L2::LEN / 4];
        build_prefix<L2, KK, RK2>(r.kw, r.sw, false, w);
#pragma unroll
        for (int j = 0; j < L2::VW; j++) w[L2::PW + j] = r.vw[j];
        hash_words<L2::LEN>(w, h);
    }
}

template <int KK, int KL, int VK, int VL, int RK, bool TAGS, bool DUAL>
__device__ __forceinline__ void lift_pipe_body(const DevCols &c, uint64_t n, uint8_t *fps, uint8_t *bsums,
                                               uint8_t *fps2, uint8_t *bsums2, uint64_t nblk, uint64_t per) {
    using L = Layout<KK, KL, VK, VL, RK>;
    using LP = Layout<KK, KL, VK, VL, REC_PROJECTION>;
    static_assert(L::SMALL, "register-resident records only");
    __shared__ SumTile tile;
    const uint64_t b0 = (uint64_t)blockIdx.x * per;
    const uint64_t b1 = b0 + per < nblk ? b0 + per : nblk;
    RecRegs<L, KK, KL, RK, TAGS> cur, nxt;
    {
        const uint64_t i = b0 * LIFT_THREADS + threadIdx.x;
        if (b0 < b1 && i < n) cur.load(c, i);
    }
    for (uint64_t b = b0; b < b1; b++) {
        const uint64_t i = b * LIFT_THREADS + threadIdx.x;
        const uint64_t inext = i + LIFT_THREADS;
        if (b + 1 < b1 && inext < n) nxt.load(c, inext);  // in flight while `cur` is hashed
        uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        uint32_t h2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (i < n) {
            lift_regs<L, KK, RK>(cur, h);
            store_fp(fps, i, h);
            if constexpr (DUAL) {
                lift_regs<LP, KK, REC_PROJECTION>(cur, h2);
                store_fp(fps2, i, h2);
            }
        }
        if (bsums) {
            uint32_t f[8];
            block_sum_fps256(h, tile, f);
            if (threadIdx.x == 0) store_sum(bsums, b, f);
        }
        if constexpr (DUAL) {
            if (bsums2) {
                uint32_t f[8];
                block_sum_fps256(h2, tile, f);
                if (threadIdx.x == 0) store_sum(bsums2, b, f);
            }
        }
        cur = nxt;
    }
}

// occupancy target: 6 waves per SIMD (<= 80 VGPRs) -- two records' words live per lane
template <int KK, int KL, int VK, int VL, int RK, bool TAGS, bool DUAL>
__global__ __launch_bounds__(LIFT_THREADS) __attribute__((amdgpu_waves_per_eu(6, 8)))
void k_lift_pipe(DevCols c, uint64_t n, uint8_t *fps, uint8_t *bsums, uint8_t *fps2, uint8_t *bsums2,
                 uint64_t nblk, uint64_t per) {
    lift_pipe_body<KK, KL, VK, VL, RK, TAGS, DUAL>(c, n, fps, bsums, fps2, bsums2, nblk, per);
}

// workgroups of a kernel resident at once on the current device (cached per instantiation)
template <class K>
__host__ uint64_t resident_grid(K kernel) {
    static int per_cu = 0, cus = 0;
    if (!per_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, LIFT_THREADS, 0) != hipSuccess || per_cu <= 0)
            per_cu = 4;
    }
    return (uint64_t)per_cu * (uint64_t)cus;
}

}  // namespace rh

constexpr int KK = KEY_BYTES, KL = 16, VK = VAL_BYTES, VL = 64, RK = REC_DATED;
using L = Layout<KK, KL, VK, VL, RK>;

template <int MODE>
__global__ __launch_bounds__(256) void k_abl(DevCols c, uint64_t n, uint8_t *fps, uint8_t *bsums) {
    __shared__ SumTile tile;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (i < n) {
        uint32_t kw[L::KEY_ENC / 4], sw[5], pw[L::PW], w[L::LEN / 4];
        if (MODE == 2) {
#pragma unroll
            for (int j = 0; j < L::LEN / 4; j++) w[j] = (uint32_t)i * (j + 1);
            hash_words<L::LEN>(w, h);
        } else {
            load_key<KK, KL>(c.keys, i, kw);
            load_stamp(c, i, sw);
            build_prefix<L, KK, RK>(kw, sw, false, pw);
            const uint8_t *vrow = c.values + i * (uint64_t)VL;
            if (MODE == 1) {
#pragma unroll
                for (int j = 0; j < L::PW; j++) w[j] = pw[j];
                ldw<L::VW, 16>(vrow, w + L::PW);
#pragma unroll
                for (int j = 0; j < L::LEN / 4; j++) h[j & 7] ^= w[j];
            } else {
                hash_present<L>(pw, vrow, h);
            }
        }
        store_fp(fps, i, h);
    }
    uint32_t f[8];
    block_sum_fps256(h, tile, f);
    if (threadIdx.x == 0) store_sum(bsums, blockIdx.x, f);
}

template <int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8)))
void k_pipe(DevCols c, uint64_t n, uint8_t *fps, uint8_t *bsums, uint64_t nblk, uint64_t per) {
    lift_pipe_body<KK, KL, VK, VL, RK, false, false>(c, n, fps, bsums, nullptr, nullptr, nblk, per);
}
template <int W>
float time_pipe(DevCols c, uint64_t n, uint8_t *fps, uint8_t *bs, int mult) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    uint64_t nblk = (n + 255) / 256;
    int per_cu = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pipe<W>, 256, 0);
    uint64_t g = (uint64_t)per_cu * 256 * mult;
    if (g > nblk) g = nblk;
    uint64_t per = (nblk + g - 1) / g;
    g = (nblk + per - 1) / per;
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k_pipe<W>, dim3(g), dim3(256), 0, 0, c, n, fps, bs, nblk, per);
    hipEventRecord(e0);
    for (int r = 0; r < 20; r++) hipLaunchKernelGGL(k_pipe<W>, dim3(g), dim3(256), 0, 0, c, n, fps, bs, nblk, per);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("pipe W=%d per_cu=%d mult=%d grid=%lu per=%lu: %.1f us\n", W, per_cu, mult, (unsigned long)g, (unsigned long)per, ms / 20 * 1e3);
    return ms / 20;
}

__global__ void fill(uint8_t *p, uint64_t bytes) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < bytes / 4; i += (uint64_t)gridDim.x * blockDim.x)
        reinterpret_cast<uint32_t *>(p)[i] = (uint32_t)(i * 2654435761u) ^ 0x9e3779b9u;
}

template <int MODE>
float timeit(DevCols c, uint64_t n, uint8_t *fps, uint8_t *bs) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    dim3 g((n + 255) / 256);
    for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k_abl<MODE>, g, dim3(256), 0, 0, c, n, fps, bs);
    hipEventRecord(e0);
    for (int r = 0; r < 20; r++) hipLaunchKernelGGL(k_abl<MODE>, g, dim3(256), 0, 0, c, n, fps, bs);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms / 20;
}

int main() {
    const uint64_t n = 10000000;
    uint8_t *keys, *vals, *fps, *bs; uint64_t *phys, *node; uint32_t *lg;
    hipMalloc(&keys, n * 16); hipMalloc(&vals, n * 64); hipMalloc(&phys, n * 8); hipMalloc(&node, n * 8);
    hipMalloc(&lg, n * 4); hipMalloc(&fps, n * 32); hipMalloc(&bs, (n / 256 + 1) * 32);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, keys, n * 16);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, vals, n * 64);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t *)phys, n * 8);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t *)node, n * 8);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint8_t *)lg, n * 4);
    DevCols c{keys, phys, lg, node, nullptr, vals};
    for (int rep = 0; rep < 2; rep++) {
        time_pipe<4>(c, n, fps, bs, 1); time_pipe<5>(c, n, fps, bs, 1); time_pipe<6>(c, n, fps, bs, 1);
        time_pipe<8>(c, n, fps, bs, 1); time_pipe<4>(c, n, fps, bs, 2); time_pipe<5>(c, n, fps, bs, 2);
        float full = timeit<0>(c, n, fps, bs), mem = timeit<1>(c, n, fps, bs), alu = timeit<2>(c, n, fps, bs);
        printf("full %.1f us  mem-only %.1f us (%.2f TB/s of 132 B/rec)  alu-only %.1f us\n", full * 1e3, mem * 1e3,
               n * 132.0 / (mem / 1e3) / 1e12, alu * 1e3);
    }
    return 0;
}
