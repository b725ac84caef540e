// ubench_dep.hip -- dependent-issue latency of plain VALU on gfx950 (diagnostic).
// C independent v_xor / v_bitop3 chains per wave (C = 1, 2, 4, 8), 1 / 2 / 4 waves
// per SIMD (256 threads per workgroup = one wave per SIMD, W workgroups per CU):
// wave-instructions per SIMD per ns for each.  A dependency-bound stream issues
// one op per L cycles per chain; the rate tells L.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_dep tools/ubench_dep.hip && tools/ubench_dep
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 2048
#define XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(s1));
#define BOP(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(s1), "v"(s2));

// 64 ops per iteration over C chains (round robin: chain distance C)
#define R1(OP) OP(a0)
#define R2(OP) OP(a0) OP(a1)
#define R4(OP) OP(a0) OP(a1) OP(a2) OP(a3)
#define R8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)
#define X8(R, OP) R(OP) R(OP) R(OP) R(OP) R(OP) R(OP) R(OP) R(OP)

#define KERNEL(NAME, R, REP, OP)                                                              \
    __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed) {              \
        uint32_t s1 = seed ^ threadIdx.x, s2 = seed * 3 + threadIdx.x;                       \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,       \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                      \
        for (int i = 0; i < N_ITER; ++i) {                                                   \
            REP                                                                              \
        }                                                                                    \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;  \
    }

KERNEL(k_xor_c1, R1, X8(R1, XOR) X8(R1, XOR) X8(R1, XOR) X8(R1, XOR) X8(R1, XOR) X8(R1, XOR) X8(R1, XOR) X8(R1, XOR), XOR)
KERNEL(k_xor_c2, R2, X8(R2, XOR) X8(R2, XOR) X8(R2, XOR) X8(R2, XOR), XOR)
KERNEL(k_xor_c4, R4, X8(R4, XOR) X8(R4, XOR), XOR)
KERNEL(k_xor_c8, R8, X8(R8, XOR), XOR)
KERNEL(k_bop_c1, R1, X8(R1, BOP) X8(R1, BOP) X8(R1, BOP) X8(R1, BOP) X8(R1, BOP) X8(R1, BOP) X8(R1, BOP) X8(R1, BOP), BOP)
KERNEL(k_bop_c2, R2, X8(R2, BOP) X8(R2, BOP) X8(R2, BOP) X8(R2, BOP), BOP)
KERNEL(k_bop_c4, R4, X8(R4, BOP) X8(R4, BOP), BOP)
KERNEL(k_bop_c8, R8, X8(R8, BOP), BOP)

typedef void (*Kern)(uint32_t*, uint32_t);

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    if (hipMalloc(&out, (size_t)cus * 8 * 256 * 4) != hipSuccess) return 1;
    struct { const char* name; Kern k; } ks[] = {
        {"xor_c1", k_xor_c1}, {"xor_c2", k_xor_c2}, {"xor_c4", k_xor_c4}, {"xor_c8", k_xor_c8},
        {"bitop3_c1", k_bop_c1}, {"bitop3_c2", k_bop_c2}, {"bitop3_c4", k_bop_c4}, {"bitop3_c8", k_bop_c8}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d, \"ops_per_wave\": %d, \"results\": {", cus, 64 * N_ITER);
    bool first = true;
    for (auto& k : ks) {
        for (int w : {1, 2, 4}) {
            const int blocks = cus * w;
            hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 7u);
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, out, 7u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double waves = 5.0 * blocks * 4, instr = waves * 64.0 * N_ITER;
            const double per_simd_ns = instr / (cus * 4.0) / (ms * 1e6);
            printf("%s\"%s_w%d\": %.4f", first ? "" : ", ", k.name, w, per_simd_ns);
            first = false;
        }
    }
    printf("}, \"unit\": \"wave64 VALU instructions per SIMD per ns\"}\n");
    return 0;
}
