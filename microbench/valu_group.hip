#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_group1(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_xor_b32 v41, v41, v48\nv_alignbit_b32 v42, v42, v42, 7\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_xor_b32 v45, v45, v48\nv_alignbit_b32 v46, v46, v46, 7\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void k_group2(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void k_group4(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void k_group8(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void k_group16(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void k_group32(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void k_g4_12(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}
__global__ __launch_bounds__(256) void k_g8_24(uint32_t *out, int iters, uint64_t *clk) {
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("v_mov_b32 v48, %0\n" "v_mov_b32 v40, %0\n" "v_mov_b32 v41, %0\n" "v_mov_b32 v42, %0\n" "v_mov_b32 v43, %0\n" "v_mov_b32 v44, %0\n" "v_mov_b32 v45, %0\n" "v_mov_b32 v46, %0\n" "v_mov_b32 v47, %0\n" :: "v"(threadIdx.x) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  for (int i = 0; i < iters; i++) {
    asm volatile("v_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_alignbit_b32 v40, v40, v40, 7\nv_alignbit_b32 v41, v41, v41, 7\nv_alignbit_b32 v42, v42, v42, 7\nv_alignbit_b32 v43, v43, v43, 7\nv_alignbit_b32 v44, v44, v44, 7\nv_alignbit_b32 v45, v45, v45, 7\nv_alignbit_b32 v46, v46, v46, 7\nv_alignbit_b32 v47, v47, v47, 7\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48\nv_xor_b32 v40, v40, v48\nv_xor_b32 v41, v41, v48\nv_xor_b32 v42, v42, v48\nv_xor_b32 v43, v43, v48\nv_xor_b32 v44, v44, v48\nv_xor_b32 v45, v45, v48\nv_xor_b32 v46, v46, v48\nv_xor_b32 v47, v47, v48" ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48");
  }
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

typedef void (*KF)(uint32_t *, int, uint64_t *);
void run(const char *name, KF f, int blocks, int iters, uint32_t *out, uint64_t *clk) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 4, clk);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    uint64_t h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    double wi = 5.0 * blocks * 4 * (double)iters * 64;
    double per_simd = wi / (ms / 1e3) / 1024.0;
    double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    printf("%-18s blocks %5d  %7.3f ms clock %.2f GHz => %.2f cycles/wave-instr\n", name, blocks, ms, ghz, ghz * 1e9 / per_simd);
}

int main() {
    uint32_t *out; uint64_t *clk; int maxb = 2048;
    hipMalloc(&out, maxb * 256 * 4); hipMalloc(&clk, maxb * 16);
    run("group1", k_group1, 2048, 1000, out, clk);
    run("group1", k_group1, 512, 1000, out, clk);
    run("group2", k_group2, 2048, 1000, out, clk);
    run("group2", k_group2, 512, 1000, out, clk);
    run("group4", k_group4, 2048, 1000, out, clk);
    run("group4", k_group4, 512, 1000, out, clk);
    run("group8", k_group8, 2048, 1000, out, clk);
    run("group8", k_group8, 512, 1000, out, clk);
    run("group16", k_group16, 2048, 1000, out, clk);
    run("group16", k_group16, 512, 1000, out, clk);
    run("group32", k_group32, 2048, 1000, out, clk);
    run("group32", k_group32, 512, 1000, out, clk);
    run("g4_12", k_g4_12, 2048, 1000, out, clk);
    run("g4_12", k_g4_12, 512, 1000, out, clk);
    run("g8_24", k_g8_24, 2048, 1000, out, clk);
    run("g8_24", k_g8_24, 512, 1000, out, clk);
    return 0;
}