"""Generate tools/ubench_icache.hip: throughput of straight-line XOR blocks
(15 v_xor_b32 each, 60 B of code) versus the loop body size, to find where
instruction-cache misses start to cost on gfx950 (diagnostic)."""
import random

random.seed(2)
ACC0, PL0 = 64, 192
clob = ", ".join(f'"v{i}"' for i in range(ACC0, PL0 + 32)) + ', "s46"'
SIZES = [64, 256, 512, 1024, 1536, 2048]


def kernel(nb):
    body = ["s_mov_b32 s46, %[iters]"]
    body += [f"v_mov_b32 v{i}, 0" for i in range(ACC0, ACC0 + 128)]
    body += [f"v_add_u32 v{PL0 + p}, {p * 7 + 1}, %[tid]" for p in range(32)]
    body.append(f".Lloop{nb}:")
    for blk in range(nb):
        j = blk % 16
        for _ in range(15):
            b, p = random.randrange(8), random.randrange(30)
            body.append(f"v_xor_b32 v{ACC0 + 8 * j + b}, v{ACC0 + 8 * j + b}, v{PL0 + p}")
    body += ["s_sub_u32 s46, s46, 1", "s_cmp_lg_u32 s46, 0", f"s_cbranch_scc1 .Lloop{nb}"]
    body.append("v_mov_b32 %[res], 0")
    body += [f"v_xor_b32 %[res], %[res], v{i}" for i in range(ACC0, ACC0 + 128)]
    asm = "\\n\\t".join(body)
    return f'''
extern "C" __global__ void __launch_bounds__(256) k{nb}(unsigned* out, int iters) {{
    unsigned tid = threadIdx.x, res;
    asm volatile("{asm}" : [res] "=&v"(res) : [iters] "s"(iters), [tid] "v"(tid) : {clob}, "scc", "memory");
    out[blockIdx.x * blockDim.x + threadIdx.x] = res;
}}
'''


src = ["#include <hip/hip_runtime.h>", "#include <stdio.h>"]
src += [kernel(n) for n in SIZES]
src.append("typedef void (*kf)(unsigned*, int);")
src.append("int main() { int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);")
src.append("unsigned* out; hipMalloc(&out, 64 << 20); hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);")
src.append("kf ks[] = {" + ", ".join(f"k{n}" for n in SIZES) + "}; int nbs[] = {" + ", ".join(map(str, SIZES)) + "};")
src.append(r'''printf("{"); int first = 1;
for (int w = 1; w <= 3; ++w) for (int v = 0; v < (int)(sizeof(nbs)/sizeof(nbs[0])); ++v) {
  int iters = 65536 / nbs[v], blocks = ncu * w;
  hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, out, 2);
  hipEventRecord(a); hipLaunchKernelGGL(ks[v], dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b);
  double cyc = ms * 1e6 * 2.37 / ((double)iters * nbs[v]) / w;
  printf("%s\"blocks%d_code%dKB@%dw\": %.1f", first ? "" : ", ", nbs[v], nbs[v] * 60 / 1024, w, cyc); first = 0; }
printf("}\n"); return 0; }''')
open("tools/ubench_icache.hip", "w").write("\n".join(src))
print("ok")
