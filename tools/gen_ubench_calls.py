"""Generate tools/ubench_calls.hip: cost of per-coefficient XOR routines on gfx950.

Variant C: 16 x 15 v_xor on fixed accumulators (no indexing, no jumps).
Variant A: same, but each group runs under s_set_gpr_idx_on (SRC0|DST) with
           the accumulator block selected by an SGPR index.
Variant B: A + the group is a called routine (s_swappc / s_setpc).
All variants must produce identical XOR totals."""
import random

random.seed(1)
ACC0, PL0 = 64, 192
ROUTINES = []
for r in range(16):
    terms = [(random.randrange(8), random.randrange(30)) for _ in range(15)]
    ROUTINES.append(terms)

def xor_lines(terms, base_acc):
    return [f"v_xor_b32 v{base_acc + b}, v{base_acc + b}, v{PL0 + p}" for b, p in terms]

clob = ", ".join(f'"v{i}"' for i in range(ACC0, PL0 + 32)) + ', "s40","s41","s42","s43","s44","s45","s46","s47","m0"'

def kernel(name, mode):
    body = []
    body.append("s_mov_b32 s46, %[iters]")
    for i in range(ACC0, ACC0 + 128):
        body.append(f"v_mov_b32 v{i}, 0")
    for p in range(32):
        body.append(f"v_add_u32 v{PL0 + p}, {p * 7 + 1}, %[tid]")
    body.append("s_getpc_b64 s[44:45]")
    body.append(".Lbase_%s:" % name)
    body.append(".Lloop_%s:" % name)
    for j in range(16):
        r = j  # routine j for accumulator block j
        if mode == "C":
            body += xor_lines(ROUTINES[r], ACC0 + 8 * j)
        else:
            body.append(f"s_mov_b32 s47, {8 * j}")
            body.append("s_set_gpr_idx_on s47, gpr_idx(SRC0,DST)")
            if mode == "A":
                body += xor_lines(ROUTINES[r], ACC0)
            else:
                body.append(f"s_add_u32 s42, s44, .Lr{r}_{name}-.Lbase_{name}")
                body.append("s_addc_u32 s43, s45, 0")
                body.append("s_swappc_b64 s[40:41], s[42:43]")
            body.append("s_set_gpr_idx_off")
    body.append("s_sub_u32 s46, s46, 1")
    body.append("s_cmp_lg_u32 s46, 0")
    body.append(f"s_cbranch_scc1 .Lloop_{name}")
    if mode == "B":
        body.append(f"s_branch .Lend_{name}")
        for r in range(16):
            body.append(f".Lr{r}_{name}:")
            body += xor_lines(ROUTINES[r], ACC0)
            body.append("s_setpc_b64 s[40:41]")
        body.append(f".Lend_{name}:")
    # fold accumulators into %[res]
    body.append("v_mov_b32 %[res], 0")
    for i in range(ACC0, ACC0 + 128):
        body.append(f"v_xor_b32 %[res], %[res], v{i}")
    asm = "\\n\\t".join(body)
    return f'''
extern "C" __global__ void __launch_bounds__(256) {name}(unsigned* out, int iters) {{
    unsigned tid = threadIdx.x, res;
    asm volatile("{asm}" : [res] "=&v"(res) : [iters] "s"(iters), [tid] "v"(tid) : {clob}, "scc", "memory");
    out[blockIdx.x * blockDim.x + threadIdx.x] = res;
}}
'''

src = ['#include <hip/hip_runtime.h>', '#include <stdio.h>']
for n, m in (("kC", "C"), ("kA", "A"), ("kB", "B")):
    src.append(kernel(n, m))
src.append(r'''
typedef void (*kf)(unsigned*, int);
int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned* out; hipMalloc(&out, 64 << 20);
    unsigned* h = (unsigned*)malloc(64 << 20);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const char* names[3] = {"C_inline", "A_gpr_idx", "B_call"};
    kf ks[3] = {kC, kA, kB};
    unsigned ref0 = 0, ref1 = 0;
    printf("{");
    for (int w = 1; w <= 2; ++w) {
      for (int v = 0; v < 3; ++v) {
        int blocks = ncu * w, iters = 2048;
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, out, 16);
        hipEventRecord(a);
        hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, out, iters);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        hipMemcpy(h, out, blocks * 256 * 4, hipMemcpyDeviceToHost);
        unsigned x = 0; for (int i = 0; i < blocks * 256; ++i) x ^= h[i] * (i + 1);
        // cycles per call per wave at 2.37 GHz: waves per SIMD = w
        double calls = (double)iters * 16;
        double ns_per_call_per_simd = ms * 1e6 / calls / w;
        printf("%s\"%s@%dw\": {\"ms\": %.3f, \"cyc_per_call_per_simd\": %.1f, \"check\": %u}", (w == 1 && v == 0) ? "" : ", ",
               names[v], w, ms, ns_per_call_per_simd * 2.37, x);
      }
    }
    printf("}\n");
    return 0;
}
''')
open("tools/ubench_calls.hip", "w").write("\n".join(src))
print("ok")
