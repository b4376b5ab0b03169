// valu_rate.hip -- measures the gfx950 issue rate of the integer VALU instructions the BLAKE3
// compression is made of (v_xor_b32, v_add_u32, v_add3_u32, v_alignbit_b32), and the
// in-kernel clock (s_memtime / s_memrealtime at 100 MHz).  Standalone: hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters, uint64_t *clk) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t b = blockIdx.x | 1;
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) {
        if (OP == 0) {
            REP8(asm volatile("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (OP == 1) {
            REP8(asm volatile("v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (OP == 2) {
            REP8(asm volatile("v_add3_u32 %0, %0, %8, %8\n v_add3_u32 %1, %1, %8, %8\n v_add3_u32 %2, %2, %8, %8\n v_add3_u32 %3, %3, %8, %8\n v_add3_u32 %4, %4, %8, %8\n v_add3_u32 %5, %5, %8, %8\n v_add3_u32 %6, %6, %8, %8\n v_add3_u32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (OP == 3) {
            REP8(asm volatile("v_alignbit_b32 %0, %0, %0, 7\n v_alignbit_b32 %1, %1, %1, 7\n v_alignbit_b32 %2, %2, %2, 7\n v_alignbit_b32 %3, %3, %3, 7\n v_alignbit_b32 %4, %4, %4, 7\n v_alignbit_b32 %5, %5, %5, 7\n v_alignbit_b32 %6, %6, %6, 7\n v_alignbit_b32 %7, %7, %7, 7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));)
        } else if (OP == 4) {
            REP8(asm volatile("v_pk_add_f32 %0, %0, %8\n v_pk_add_f32 %2, %2, %8\n v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %6, %6, %8\n v_pk_add_f32 %0, %0, %8\n v_pk_add_f32 %2, %2, %8\n v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %6, %6, %8" : "+v"(*(uint64_t*)&a0), "+v"(a1), "+v"(*(uint64_t*)&a2), "+v"(a3), "+v"(*(uint64_t*)&a4), "+v"(a5), "+v"(*(uint64_t*)&a6), "+v"(a7) : "v"((uint64_t)b));)
        } else if (OP == 5) {
            REP8(asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (OP == 6) {
            REP8(asm volatile("v_perm_b32 %0, %0, %0, %8\n v_perm_b32 %1, %1, %1, %8\n v_perm_b32 %2, %2, %2, %8\n v_perm_b32 %3, %3, %3, %8\n v_perm_b32 %4, %4, %4, %8\n v_perm_b32 %5, %5, %5, %8\n v_perm_b32 %6, %6, %6, %8\n v_perm_b32 %7, %7, %7, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (OP == 7) {
            REP8(asm volatile("v_xad_u32 %0, %0, %8, %8\n v_xad_u32 %1, %1, %8, %8\n v_xad_u32 %2, %2, %8, %8\n v_xad_u32 %3, %3, %8, %8\n v_xad_u32 %4, %4, %8, %8\n v_xad_u32 %5, %5, %8, %8\n v_xad_u32 %6, %6, %8, %8\n v_xad_u32 %7, %7, %8, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if (OP == 8) {
            // mixed VOP2 (e32) add + VOP3 alignbit
            REP8(asm volatile("v_add_u32 %0, %0, %8\n v_alignbit_b32 %1, %1, %1, 7\n v_add_u32 %2, %2, %8\n v_alignbit_b32 %3, %3, %3, 7\n v_xor_b32 %4, %4, %8\n v_alignbit_b32 %5, %5, %5, 9\n v_xor_b32 %6, %6, %8\n v_alignbit_b32 %7, %7, %7, 9" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int OP>
void run(const char *name, int blocks, int iters, uint32_t *out, uint64_t *clk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, 4, clk);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    uint64_t h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    double waveinstr = 5.0 * blocks * 4 /*waves*/ * (double)iters * 64;
    double per_simd_per_s = waveinstr / (ms / 1e3) / 1024.0;
    double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    printf("%-16s %8.3f ms  %.3f Gwave-instr/s/SIMD  clock %.2f GHz  => %.2f cycles/wave-instr  (%.1f T lane-ops/s)\n",
           name, ms, per_simd_per_s / 1e9, ghz, ghz * 1e9 / per_simd_per_s, waveinstr * 64 / (ms / 1e3) / 1e12);
}

int main() {
    uint32_t *out; uint64_t *clk;
    int blocks = 256 * 8;  // 8 workgroups of 4 waves per CU = 8 waves/SIMD
    hipMalloc(&out, blocks * 256 * 4); hipMalloc(&clk, blocks * 16);
    int iters = 2000;
    run<0>("v_xor_b32", blocks, iters, out, clk);
    run<1>("v_add_u32", blocks, iters, out, clk);
    run<2>("v_add3_u32", blocks, iters, out, clk);
    run<3>("v_alignbit_b32", blocks, iters, out, clk);
    run<4>("v_pk_add_f32", blocks, iters, out, clk);
    run<5>("v_fma_f32", blocks, iters, out, clk);
    run<6>("v_perm_b32", blocks, iters, out, clk);
    run<7>("v_xad_u32", blocks, iters, out, clk);
    run<8>("mix_vop2_vop3", blocks, iters, out, clk);
    for (int b : {256 * 2, 256 * 4}) { printf("blocks=%d\n", b); run<0>("v_xor_b32", b, iters, out, clk); run<3>("v_alignbit_b32", b, iters, out, clk); }
    return 0;
}
