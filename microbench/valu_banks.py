"""Generates valu_banks.hip: which 3-source VALU forms issue at the full wave64 rate on gfx950.

Round-1 measurements (profiles/r01_micro_valu_*.log): plain 2-operand ops issue every ~2.2
cycles, every 3-operand form (v_alignbit_b32, v_add3_u32, v_bitop3_b32, v_lshl_or_b32) every
~4.2, and a stream with one 3-operand op in 16 already runs at ~3.8.  Two hypotheses (VERDICT r01,
item 7):
  (a) VGPR bank conflicts: the register file reads one operand per bank per cycle (bank =
      register index mod 4), and those tests read two operands from one bank (alignbit(x, x, n)
      reads x twice; add3 x, x, v48, v48 reads v48 twice);
  (b) the slow rate is a per-SIMD mode that a single 3-operand op from any wave switches on.
Each kernel below issues 64 independent instructions per iteration over 8 accumulators
(v40-v47) with sources in v48-v63; 8 waves per SIMD.  Usage:
  python3 microbench/valu_banks.py > microbench/valu_banks.hip
  hipcc -O3 --offload-arch=gfx950 microbench/valu_banks.hip -o microbench/valu_banks
"""

ACC = [40 + i for i in range(8)]


def src(bank, k=0):
    """a source register in v48..v63 with the given bank (index mod 4)"""
    return 48 + 4 * k + bank


def body(gen):
    lines = []
    for rep in range(8):
        for i, d in enumerate(ACC):
            lines.append(gen(i, d, rep))
    return lines


def alternate(g1, g2):
    return lambda i, d, rep: (g1 if (i + rep) % 2 == 0 else g2)(i, d, rep)


X = lambda i, d, rep: f"v_xor_b32 v{d}, v{d}, v{src((d + 1) % 4)}"  # noqa: E731 (fast reference)

KERNELS = {
    # 2-operand references
    "xor_distinct": X,
    "xor_samebank": lambda i, d, rep: f"v_xor_b32 v{d}, v{d}, v{src(d % 4)}",
    "add_self": lambda i, d, rep: f"v_add_u32 v{d}, v{d}, v{d}",
    # 3-source forms, operand banks distinct / shared / one register read twice
    "add3_distinct": lambda i, d, rep: f"v_add3_u32 v{d}, v{d}, v{src((d + 1) % 4)}, v{src((d + 2) % 4, 1)}",
    "add3_samebank": lambda i, d, rep: f"v_add3_u32 v{d}, v{d}, v{src(d % 4)}, v{src(d % 4, 1)}",
    "add3_twice": lambda i, d, rep: f"v_add3_u32 v{d}, v{d}, v{src((d + 1) % 4)}, v{src((d + 1) % 4)}",
    "add3_const": lambda i, d, rep: f"v_add3_u32 v{d}, v{d}, v{src((d + 1) % 4)}, 7",
    "bitop3_distinct": lambda i, d, rep: f"v_bitop3_b32 v{d}, v{d}, v{src((d + 1) % 4)}, v{src((d + 2) % 4, 1)} bitop3:0x96",
    "alignbit_self": lambda i, d, rep: f"v_alignbit_b32 v{d}, v{d}, v{d}, 7",
    "alignbit_distinct": lambda i, d, rep: f"v_alignbit_b32 v{d}, v{d}, v{src((d + 1) % 4)}, 7",
    "alignbit_vshift": lambda i, d, rep: f"v_alignbit_b32 v{d}, v{d}, v{src((d + 1) % 4)}, v{src((d + 2) % 4, 1)}",
    "lshl_or_distinct": lambda i, d, rep: f"v_lshl_or_b32 v{d}, v{d}, 7, v{src((d + 1) % 4)}",
    "xad_distinct": lambda i, d, rep: f"v_xad_u32 v{d}, v{d}, v{src((d + 1) % 4)}, v{src((d + 2) % 4, 1)}",
    "lshlrev_e64_self": lambda i, d, rep: f"v_lshlrev_b32_e64 v{d}, 7, v{d}",
    # mixes: 1:1 interleaved, and the same counts clustered (32 slow then 32 fast per iteration)
    "mix_add3d_xor": alternate(lambda i, d, rep: f"v_add3_u32 v{d}, v{d}, v{src((d + 1) % 4)}, v{src((d + 2) % 4, 1)}", X),
    "mix_align_xor": alternate(lambda i, d, rep: f"v_alignbit_b32 v{d}, v{d}, v{d}, 7", X),
}


def clustered(i, d, rep):
    return f"v_alignbit_b32 v{d}, v{d}, v{d}, 7" if rep < 4 else X(i, d, rep)


KERNELS["cluster_align_xor"] = clustered

CLOBBER = ", ".join(f'"v{r}"' for r in range(40, 64))

HEAD = r'''#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef void (*KF)(uint32_t *, int, uint64_t *);
'''


def kernel(name, lines, split=None):
    init = "".join(f'"v_mov_b32 v{r}, %0\\n"' for r in range(40, 64))
    asm = "\\n".join(lines)
    if split is None:
        loop = f'asm volatile("{asm}" ::: {CLOBBER});'
    else:  # odd waves run the second stream
        asm2 = "\\n".join(split)
        loop = (f'if ((threadIdx.x >> 6) & 1) asm volatile("{asm2}" ::: {CLOBBER});\n'
                f'    else asm volatile("{asm}" ::: {CLOBBER});')
    return f'''__global__ __launch_bounds__(256) void k_{name}(uint32_t *out, int iters, uint64_t *clk) {{
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile({init} :: "v"(threadIdx.x * 2654435761u + 12345u) : {CLOBBER});
  for (int i = 0; i < iters; i++) {{
    {loop}
  }}
  uint32_t r; asm volatile("v_mov_b32 %0, v40" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) {{ clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }}
}}
'''


MAIN = r'''
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
    printf("%-20s %7.3f ms clock %.2f GHz => %.2f cycles/wave-instr\n", name, ms, ghz, ghz * 1e9 / per_simd);
}
int main() {
    uint32_t *out; uint64_t *clk; int blocks = 2048;
    hipMalloc(&out, blocks * 256 * 4); hipMalloc(&clk, blocks * 16);
    // warm the clocks
    for (int k = 0; k < 20; k++) run("warm", k_xor_distinct, blocks, 1000, out, clk);
'''


def main():
    out = [HEAD]
    names = []
    for name, gen in KERNELS.items():
        out.append(kernel(name, body(gen)))
        names.append(name)
    # waves of one SIMD running different streams: even waves fast xor, odd waves alignbit
    out.append(kernel("split_xor_align", body(X), body(lambda i, d, rep: f"v_alignbit_b32 v{d}, v{d}, v{d}, 7")))
    names.append("split_xor_align")
    out.append(MAIN)
    for n in names:
        out.append(f'    run("{n}", k_{n}, blocks, 1000, out, clk);\n')
    out.append("    return 0;\n}\n")
    print("".join(out))


if __name__ == "__main__":
    main()
