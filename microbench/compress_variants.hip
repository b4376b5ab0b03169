// compress_variants.hip -- cycles per BLAKE3 compression on gfx950 for different instruction
// selections of the G function (compute only, data synthesised per lane).
//   V0: v_add3_u32 + v_alignbit_b32 (what hipcc emits for the natural code)
//   V1: 2 x v_add_u32 + v_alignbit_b32
//   V2: 2 x v_add_u32 + shift/shift/or rotations (only "simple" VOP2 ops)
//   V3: v_add3_u32 + shift/shift/or rotations
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int V> __device__ __forceinline__ uint32_t rot(uint32_t x, int n) {
    if (V == 0 || V == 1) return __builtin_amdgcn_alignbit(x, x, n);
    uint32_t a, b, r;
    asm("v_lshrrev_b32 %0, %1, %2" : "=v"(a) : "i"(n), "v"(x));
    asm("v_lshlrev_b32 %0, %1, %2" : "=v"(b) : "i"(32 - n), "v"(x));
    asm("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
template <int V> __device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
    if (V == 0 || V == 3) return a + b + c;
    uint32_t t, r;
    asm("v_add_u32 %0, %1, %2" : "=v"(t) : "v"(a), "v"(b));
    asm("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(t), "v"(c));
    return r;
}
#define G(a, b, c, d, mx, my) a = add3<V>(a, b, mx); d = rot<V>(d ^ a, 16); c = c + d; b = rot<V>(b ^ c, 12); \
    a = add3<V>(a, b, my); d = rot<V>(d ^ a, 8); c = c + d; b = rot<V>(b ^ c, 7);
template <int V> __device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16], uint32_t ctr) {
    uint32_t v0 = cv[0], v1 = cv[1], v2 = cv[2], v3 = cv[3], v4 = cv[4], v5 = cv[5], v6 = cv[6], v7 = cv[7];
    uint32_t v8 = 0x6A09E667u, v9 = 0xBB67AE85u, v10 = 0x3C6EF372u, v11 = 0xA54FF53Au, v12 = ctr, v13 = 0, v14 = 64, v15 = 0;
#define R(s0,s1,s2,s3,s4,s5,s6,s7,s8,s9,s10,s11,s12,s13,s14,s15) G(v0,v4,v8,v12,m[s0],m[s1]) G(v1,v5,v9,v13,m[s2],m[s3]) \
    G(v2,v6,v10,v14,m[s4],m[s5]) G(v3,v7,v11,v15,m[s6],m[s7]) G(v0,v5,v10,v15,m[s8],m[s9]) G(v1,v6,v11,v12,m[s10],m[s11]) \
    G(v2,v7,v8,v13,m[s12],m[s13]) G(v3,v4,v9,v14,m[s14],m[s15])
    R(0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15) R(2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8) R(3,4,10,12,13,2,7,14,6,5,9,0,11,15,8,1)
    R(10,7,12,9,14,3,13,15,4,0,11,2,5,8,1,6) R(12,13,9,11,15,10,14,8,7,2,5,3,0,1,6,4) R(9,14,11,5,8,12,15,1,13,3,0,10,2,6,4,7)
    R(11,15,5,0,1,9,8,6,14,10,2,12,3,4,7,13)
    cv[0] = v0 ^ v8; cv[1] = v1 ^ v9; cv[2] = v2 ^ v10; cv[3] = v3 ^ v11; cv[4] = v4 ^ v12; cv[5] = v5 ^ v13; cv[6] = v6 ^ v14; cv[7] = v7 ^ v15;
}
template <int V> __global__ __launch_bounds__(256) void k(uint32_t *out, int iters, uint64_t *clk) {
    uint32_t cv[8], m[16];
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    for (int j = 0; j < 8; j++) cv[j] = t * (j + 3);
    for (int j = 0; j < 16; j++) m[j] = t ^ (j * 0x9e3779b9u);
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; i++) { compress<V>(cv, m, i); m[i & 15] ^= cv[0]; }
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[t] = cv[0] ^ cv[1] ^ cv[2] ^ cv[3] ^ cv[4] ^ cv[5] ^ cv[6] ^ cv[7];
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
template <int V> void run(int blocks, uint32_t *out, uint64_t *clk) {
    const int iters = 200;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, 2, clk);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    uint64_t h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    double comps = 5.0 * blocks * 256 * iters;
    double waves_per_simd = blocks * 4.0 / 1024.0;
    double cyc_per_comp_wave = (ms / 1e3) * ghz * 1e9 / (5.0 * iters * waves_per_simd);
    printf("V%d blocks %5d: %7.3f ms clock %.2f GHz  %.2f G compress/s  => %.0f SIMD-cycles per wave-compression\n", V, blocks,
           ms, ghz, comps / (ms / 1e3) / 1e9, cyc_per_comp_wave);
}
int main() {
    uint32_t *out; uint64_t *clk; hipMalloc(&out, 4096 * 256 * 4); hipMalloc(&clk, 4096 * 16);
    for (int b : {2048, 1024}) { run<0>(b, out, clk); run<1>(b, out, clk); run<2>(b, out, clk); run<3>(b, out, clk); }
    return 0;
}
