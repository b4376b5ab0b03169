"""Generates valu_g.hip: candidate rotation instructions and whole BLAKE3 G-function encodings on gfx950.

Follows valu_banks.py (profiles/r02_micro_valu_banks.log).  Part 1: the issue rate of every
instruction that could rotate a 32-bit word.  Part 2: eight independent G chains per wave (the
a, b, c, d columns of a BLAKE3 round; messages in v80-v87), one G = the 8-step
add / xor / rotate sequence, in several encodings:
  cur     v_add3 + v_xor + v_alignbit (12 instructions; today's k_lift)
  split   a + m first (independent of b), then + b: 2 x v_add_u32 instead of v_add3 (14)
  simple  every rotate as shift, shift, or (22, no 3-operand op)
  bitop   rotations as two shifts + the OR merged into the NEXT xor by v_bitop3 (a ^ (x | y))
Reported per wave-instruction and per G.
  python3 microbench/valu_g.py > microbench/valu_g.hip && hipcc -O3 --offload-arch=gfx950 ...
"""

ACC = [40 + i for i in range(8)]


def rep8(gen):
    return [gen(i, d, rep) for rep in range(8) for i, d in enumerate(ACC)]


ROT = {
    "alignbyte_self": lambda i, d, r: f"v_alignbyte_b32 v{d}, v{d}, v{d}, 2",
    "perm_sgpr": lambda i, d, r: f"v_perm_b32 v{d}, v{d}, v{d}, s20",
    "pack_f16_opsel": lambda i, d, r: f"v_pack_b32_f16 v{d}, v{d}, v{d} op_sel:[1,0,0]",
    "bfi": lambda i, d, r: f"v_bfi_b32 v{d}, v{48 + (d + 1) % 4}, v{d}, v{52 + (d + 2) % 4}",
    "lshl_add": lambda i, d, r: f"v_lshl_add_u32 v{d}, v{d}, 7, v{48 + (d + 1) % 4}",
    "pk_lshlrev_b16": lambda i, d, r: f"v_pk_lshlrev_b16 v{d}, 3, v{d}",
    "lshrrev_e32": lambda i, d, r: f"v_lshrrev_b32 v{d}, 7, v{d}",
    "lshrrev_vgpr_amt": lambda i, d, r: f"v_lshrrev_b32 v{d}, v{60 + d % 4}, v{d}",
    "or_e32": lambda i, d, r: f"v_or_b32 v{d}, v{d}, v{48 + (d + 1) % 4}",
    "bitop3_xor_or": lambda i, d, r: f"v_bitop3_b32 v{d}, v{d}, v{48 + (d + 1) % 4}, v{52 + (d + 2) % 4} bitop3:0x1e",
    "add_co_ci": lambda i, d, r: f"v_add_co_u32 v{d}, vcc, v{d}, v{48 + (d + 1) % 4}",
    "mov_dpp_rowror": lambda i, d, r: f"v_mov_b32_dpp v{d}, v{d} row_ror:4 row_mask:0xf bank_mask:0xf",
}


# ---- G encodings: chain j uses state regs a = v(100+4j) .. d = v(103+4j); message m0/m1 in v80+j ----
def g_cur(j):
    a, b, c, d = (40 + 4 * j + k for k in range(4))
    m0, m1 = 72 + j, 80 + j
    return [f"v_add3_u32 v{a}, v{a}, v{b}, v{m0}", f"v_xor_b32 v{d}, v{d}, v{a}", f"v_alignbit_b32 v{d}, v{d}, v{d}, 16",
            f"v_add_u32 v{c}, v{c}, v{d}", f"v_xor_b32 v{b}, v{b}, v{c}", f"v_alignbit_b32 v{b}, v{b}, v{b}, 12",
            f"v_add3_u32 v{a}, v{a}, v{b}, v{m1}", f"v_xor_b32 v{d}, v{d}, v{a}", f"v_alignbit_b32 v{d}, v{d}, v{d}, 8",
            f"v_add_u32 v{c}, v{c}, v{d}", f"v_xor_b32 v{b}, v{b}, v{c}", f"v_alignbit_b32 v{b}, v{b}, v{b}, 7"]


def g_split(j):
    a, b, c, d = (40 + 4 * j + k for k in range(4))
    m0, m1 = 72 + j, 80 + j
    return [f"v_add_u32 v{a}, v{a}, v{m0}", f"v_add_u32 v{a}, v{a}, v{b}", f"v_xor_b32 v{d}, v{d}, v{a}",
            f"v_alignbit_b32 v{d}, v{d}, v{d}, 16", f"v_add_u32 v{c}, v{c}, v{d}", f"v_xor_b32 v{b}, v{b}, v{c}",
            f"v_alignbit_b32 v{b}, v{b}, v{b}, 12", f"v_add_u32 v{a}, v{a}, v{m1}", f"v_add_u32 v{a}, v{a}, v{b}",
            f"v_xor_b32 v{d}, v{d}, v{a}", f"v_alignbit_b32 v{d}, v{d}, v{d}, 8", f"v_add_u32 v{c}, v{c}, v{d}",
            f"v_xor_b32 v{b}, v{b}, v{c}", f"v_alignbit_b32 v{b}, v{b}, v{b}, 7"]


def rot_simple(x, n, t):
    return [f"v_lshlrev_b32 v{t}, {32 - n}, v{x}", f"v_lshrrev_b32 v{x}, {n}, v{x}", f"v_or_b32 v{x}, v{x}, v{t}"]


def g_simple(j):
    a, b, c, d = (40 + 4 * j + k for k in range(4))
    m0, m1, t = 72 + j, 80 + j, 88 + j
    return ([f"v_add_u32 v{a}, v{a}, v{m0}", f"v_add_u32 v{a}, v{a}, v{b}", f"v_xor_b32 v{d}, v{d}, v{a}"] +
            rot_simple(d, 16, t) + [f"v_add_u32 v{c}, v{c}, v{d}", f"v_xor_b32 v{b}, v{b}, v{c}"] + rot_simple(b, 12, t) +
            [f"v_add_u32 v{a}, v{a}, v{m1}", f"v_add_u32 v{a}, v{a}, v{b}", f"v_xor_b32 v{d}, v{d}, v{a}"] +
            rot_simple(d, 8, t) + [f"v_add_u32 v{c}, v{c}, v{d}", f"v_xor_b32 v{b}, v{b}, v{c}"] + rot_simple(b, 7, t))


def g_alt(j):  # alternate the chains' step types so consecutive instructions of one wave differ in class
    return g_cur(j)


def interleave(chains):
    out = []
    for k in range(max(len(c) for c in chains)):
        for c in chains:
            if k < len(c):
                out.append(c[k])
    return out


G_KINDS = {"cur": g_cur, "split": g_split, "simple": g_simple}

REGS = list(range(40, 96))

HEAD = r'''#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef void (*KF)(uint32_t *, int, uint64_t *);
'''


def kernel(name, lines, regs=range(40, 64)):
    CLOB = ", ".join(f'"v{r}"' for r in regs) + ', "s20", "vcc"'
    init = "".join(f'"v_mov_b32 v{r}, %0\\n"' for r in regs)
    init += '"s_mov_b32 s20, 0x1000302\\n"'
    asm = "\\n".join(lines)
    return f'''__global__ __launch_bounds__(256) void k_{name}(uint32_t *out, int iters, uint64_t *clk) {{
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  asm volatile({init} :: "v"(threadIdx.x * 2654435761u + 12345u) : {CLOB});
  for (int i = 0; i < iters; i++) {{
    asm volatile("{asm}" ::: {CLOB});
  }}
  uint32_t r; asm volatile("v_xor_b32 %0, v40, v41" : "=v"(r));
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if (threadIdx.x == 0) {{ clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }}
}}
'''


MAIN = r'''
void run(const char *name, KF f, int blocks, int iters, int per_iter, int gs, uint32_t *out, uint64_t *clk) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, 4, clk);
    hipEventRecord(e0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, out, iters, clk);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    uint64_t h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    double wi = 5.0 * blocks * 4 * (double)iters * per_iter;
    double per_simd = wi / (ms / 1e3) / 1024.0;
    double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    double cpi = ghz * 1e9 / per_simd;
    printf("%-20s %7.3f ms clock %.2f GHz => %.2f cycles/wave-instr", name, ms, ghz, cpi);
    if (gs) printf("  %.1f cycles/G (per wave)", cpi * per_iter / gs);
    printf("\n");
}
int main() {
    uint32_t *out; uint64_t *clk; int blocks = 2048;
    hipMalloc(&out, blocks * 256 * 4); hipMalloc(&clk, blocks * 16);
    for (int k = 0; k < 20; k++) run("warm", k_lshrrev_e32, blocks, 1000, 64, 0, out, clk);
'''


def main():
    out = [HEAD]
    runs = []
    for name, gen in ROT.items():
        out.append(kernel(name, rep8(gen)))
        runs.append((name, 64, 0, 1000))
    for name, g in G_KINDS.items():
        for nch in (4, 8):
            lines = interleave([g(j) for j in range(nch)])
            kname = f"g_{name}_{nch}"
            out.append(kernel(kname, lines, REGS))
            runs.append((kname, len(lines), nch, 300))
    out.append(MAIN)
    for n, per, gs, it in runs:
        out.append(f'    run("{n}", k_{n}, blocks, {it}, {per}, {gs}, out, clk);\n')
    out.append("    return 0;\n}\n")
    print("".join(out))


if __name__ == "__main__":
    main()
