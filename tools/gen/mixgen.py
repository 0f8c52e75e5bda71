"""Generates tools/valu_mix.hip: SIMD cycles per instruction for short repeating VALU op patterns on gfx950.
Each pattern is applied round-robin to 8 independent chains (v40..v47), repeated into a 1024-instruction body,
8 waves per SIMD.  Used to find which op mixes lose issue slots (design exploration)."""
OPS = {
    "alb": ("v_alignbit_b32 {d}, {d}, {d}, 27", 4),
    "xor": ("v_xor_b32 {d}, {d}, v49", 2),
    "bop": ("v_bitop3_b32 {d}, {d}, v49, v50 bitop3:0x96", 2),
    "add": ("v_add_u32 {d}, {d}, v49", 2),
    "ad3": ("v_add3_u32 {d}, {d}, v49, v50", 4),
    "shr": ("v_lshrrev_b32 {d}, 3, {d}", 2),
    "xad": ("v_xad_u32 {d}, {d}, v49, v50", 4),
    "bfi": ("v_bfi_b32 {d}, {d}, v49, v50", 4),
    "xs2": ("v_xor_b32 {d}, v51, v49", 2),   # reads no chain register
    "nop": ("s_nop 0", 0),
    "nop1": ("s_nop 1", 0),
    "sal": ("s_add_u32 s60, s60, 1", 0),
}
# "op" = next chain (independent of the previous instruction); "op@" = same chain as the previous instruction
PATTERNS = [
    ["alb", "xor@", "nop"], ["alb", "xor", "nop"], ["alb", "nop", "xor", "nop"],
    ["alb", "xor", "bop", "add", "nop"], ["ad3", "nop", "xor", "nop"],
    ["alb", "xor", "bop", "add", "ad3", "xor", "alb", "bop"],
    ["alb", "nop", "xor", "bop", "add", "ad3", "nop", "xor", "alb", "nop", "bop"],
    ["xor", "bop", "nop"], ["alb", "nop"],
]
OLD2 = [
    ["alb", "xor@"], ["alb", "xor"], ["alb", "xor@", "xor@"], ["alb", "bop@"], ["ad3", "bop@"], ["ad3", "xor@"],
    ["alb", "ad3@"], ["alb", "ad3@", "ad3@"], ["xor", "alb@"], ["bop", "ad3@"], ["alb", "xor@", "alb", "xor@"],
    ["alb", "xor@", "bop@", "add@"], ["alb", "xor@", "bop", "add@"],
    ["alb", "xor@", "bop@", "add@", "ad3@", "xor@", "alb@", "bop@"],
]
OLD_PATTERNS = [
    ["xor"], ["bop"], ["alb"], ["ad3"],
    ["alb", "xor"], ["alb", "bop"], ["alb", "add"], ["ad3", "xor"], ["ad3", "bop"], ["ad3", "add"],
    ["alb", "ad3"], ["alb", "xor", "xor"], ["alb", "alb", "xor", "xor"], ["alb", "xor", "bop", "add"],
    ["alb", "ad3", "xor", "xor"], ["xor", "bop"], ["xor", "add"], ["bop", "add"], ["xor", "bop", "add"],
    ["alb", "xor", "bop", "add", "ad3", "xor", "alb", "bop"],
    ["alb", "alb", "alb", "alb", "xor", "xor", "xor", "xor"],
    ["alb", "shr"], ["xad", "xor"], ["bfi", "xor"], ["alb", "xs2"],
]
N = 1024


def body(pat):
    lines = []
    chain = -1
    for i in range(N):
        op = pat[i % len(pat)]
        if op.endswith("@"):
            op = op[:-1]
        else:
            chain = (chain + 1) % 8
        if op in ("nop", "nop1", "sal"):
            lines.append(OPS[op][0])
            continue
        lines.append(OPS[op][0].format(d="v%d" % (40 + chain)))
    return "\\n".join(lines)


def main(path):
    out = ['#include <hip/hip_runtime.h>', '#include <stdio.h>', '#include <stdlib.h>',
           '#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s\\n", hipGetErrorString(e)); exit(1);} } while (0)']
    for k, pat in enumerate(PATTERNS):
        out.append('__global__ __launch_bounds__(256) void k%d(unsigned long long* clk, unsigned iters) {' % k)
        out.append('  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();')
        out.append('  asm volatile("v_mov_b32 v49, 3\\n v_mov_b32 v50, 5\\n v_mov_b32 v51, 7" ::: "v49", "v50", "v51");')
        out.append('  for (unsigned it = 0; it < iters; it++) asm volatile("%s" ::: "v40","v41","v42","v43","v44","v45","v46","v47","s60");' % body(pat))
        out.append('  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();')
        out.append('  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }')
        out.append('}')
    out.append('typedef void (*K)(unsigned long long*, unsigned);')
    out.append('static const K KS[] = {%s};' % ", ".join("k%d" % k for k in range(len(PATTERNS))))
    out.append('static const char* NAMES[] = {%s};' % ", ".join('"%s"' % "+".join(p) for p in PATTERNS))
    nv = lambda p: sum(1 for o in p if OPS[o.rstrip("@")][1])
    out.append('static const double ADDITIVE[] = {%s};' % ", ".join("%.3f" % (sum(OPS[o.rstrip("@")][1] for o in p) / nv(p)) for p in PATTERNS))
    out.append('static const double VFRAC[] = {%s};' % ", ".join("%.4f" % (nv(p) / len(p)) for p in PATTERNS))
    out.append('''int main() {
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  setvbuf(stdout, NULL, _IONBF, 0);
  const int cus = p.multiProcessorCount, blocks = cus * 8; const unsigned iters = 100;
  unsigned long long* d; CHK(hipMalloc(&d, (size_t)blocks * 16));
  unsigned long long* h = (unsigned long long*)malloc((size_t)blocks * 16);
  printf("{\\"results\\": [\\n");
  for (int k = 0; k < (int)(sizeof(KS) / sizeof(KS[0])); k++) {
    hipLaunchKernelGGL(KS[k], dim3(blocks), dim3(256), 0, 0, d, 4u); CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0, 0)); hipLaunchKernelGGL(KS[k], dim3(blocks), dim3(256), 0, 0, d, iters);
    CHK(hipEventRecord(e1, 0)); CHK(hipEventSynchronize(e1)); float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipMemcpy(h, d, (size_t)blocks * 16, hipMemcpyDeviceToHost));
    double cyc = 0, rt = 0; for (int i = 0; i < blocks; i++) { cyc += h[2 * i]; rt += h[2 * i + 1]; }
    const double clk = cyc / (rt / 100e6);
    const double insts = (double)blocks * 4 * iters * 1024 * VFRAC[k];
    printf("%s  {\\"pattern\\": \\"%s\\", \\"additive\\": %.3f, \\"measured\\": %.3f, \\"clock_mhz\\": %.0f}", k ? ",\\n" : "", NAMES[k], ADDITIVE[k], ms * 1e-3 * clk * cus * 4 / insts, clk / 1e6);
  }
  printf("]}\\n"); return 0; }''')
    open(path, "w").write("\n".join(out) + "\n")


if __name__ == "__main__":
    import sys
    main(sys.argv[1] if len(sys.argv) > 1 else "tools/valu_mix.hip")
