// ubench.hip -- VALU / LDS issue-rate microbenchmarks on gfx950 (diagnostic).
// hipcc --offload-arch=gfx950 -O3 -o tools/ubench tools/ubench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N_ITER 4096

// 8 independent chains x 8 instructions per iteration = 64 VALU per iter.
#define BODY8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

#define PERM(x) asm volatile("v_perm_b32 %0, %1, %2, %3" : "+v"(x) : "v"(s1), "v"(s2), "v"(x));
#define BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(s1), "v"(s2));
#define XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(s1));
#define AND(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(s1));
#define LSHR(x) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x));
#define ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(s1), "v"(s2));
#define BFI(x) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x) : "v"(s1), "v"(s2));
#define CNDMASK(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(s1));
#define PERMS(x) asm volatile("v_perm_b32 %0, %1, %2, %3" : "+v"(x) : "s"(u1), "v"(s2), "v"(x));
#define PKADD(x) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(s1));

#define KERNEL(NAME, OP)                                                                 \
    __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed, uint32_t u1) { \
        uint32_t s1 = seed ^ threadIdx.x, s2 = seed * 3 + threadIdx.x;                   \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,   \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                  \
        for (int i = 0; i < N_ITER; ++i) {                                               \
            BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) \
        }                                                                                \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
    }

KERNEL(k_perm, PERM)
KERNEL(k_bitop3, BITOP3)
KERNEL(k_xor, XOR)
KERNEL(k_and, AND)
KERNEL(k_lshr, LSHR)
KERNEL(k_andor, ANDOR)
KERNEL(k_bfi, BFI)
KERNEL(k_perms, PERMS)
KERNEL(k_pkadd, PKADD)

// 64-bit shifts (register pairs): would let the transpose network shift two
// dwords per instruction
#define LSHL64(x) asm volatile("v_lshlrev_b64 %0, 4, %0" : "+v"(x));
#define LSHR64(x) asm volatile("v_lshrrev_b64 %0, 2, %0" : "+v"(x));
#define KERNEL64(NAME, OP)                                                               \
    __global__ void __launch_bounds__(256) NAME(uint32_t* out, uint32_t seed, uint32_t u1) { \
        uint64_t a0 = threadIdx.x * 0x100000001ull + seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3,  \
                 a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                       \
        for (int i = 0; i < N_ITER; ++i) {                                               \
            BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) BODY8(OP) \
        }                                                                                \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    }
KERNEL64(k_lshl64, LSHL64)
KERNEL64(k_lshr64, LSHR64)

// mixed: the encode inner-loop ratio, 2 perm : 1 bitop3
#define MIX(x) PERM(x) PERM(x) BITOP3(x)
__global__ void __launch_bounds__(256) k_mix(uint32_t* out, uint32_t seed, uint32_t u1) {
    uint32_t s1 = seed ^ threadIdx.x, s2 = seed * 3 + threadIdx.x;
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7;
    for (int i = 0; i < N_ITER; ++i) {
        BODY8(MIX) BODY8(MIX) BODY8(MIX) BODY8(MIX) BODY8(MIX) BODY8(MIX) BODY8(MIX) BODY8(MIX)
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

// LDS broadcast read: every lane reads the same 16 bytes (the table pattern)
__global__ void __launch_bounds__(256) k_lds_bcast(uint32_t* out, uint32_t seed, uint32_t u1) {
    __shared__ uint4 tab[512];
    for (int i = threadIdx.x; i < 512; i += 256) tab[i] = make_uint4(i, i + seed, i * 3, i ^ seed);
    __syncthreads();
    uint32_t acc = 0;
    uint32_t idx = (seed & 7);
    for (int i = 0; i < N_ITER * 8; ++i) {
        uint4 v;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(idx * 16u) : "memory");
        acc ^= v.x ^ v.w;
        idx = (idx + 1) & 511;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void k_clock(uint64_t* o, int spin) {
    uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = threadIdx.x;
    for (int i = 0; i < spin; ++i) asm volatile("v_xor_b32 %0, %0, 1" : "+v"(x));
    uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { o[0] = t1 - t0; o[1] = r1 - r0; o[2] = x; }
}

typedef void (*kfn)(uint32_t*, uint32_t, uint32_t);

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    hipMalloc(&out, 64 << 20);
    uint64_t* clk;
    hipMalloc(&clk, 64);
    struct { const char* name; kfn f; int per_iter; } ks[] = {
        {"v_perm_b32", k_perm, 64}, {"v_bitop3_b32", k_bitop3, 64}, {"v_xor_b32", k_xor, 64},
        {"v_and_b32", k_and, 64}, {"v_lshrrev_b32", k_lshr, 64}, {"v_and_or_b32", k_andor, 64},
        {"v_bfi_b32", k_bfi, 64}, {"v_perm_b32(sgpr)", k_perms, 64}, {"v_pk_add_u16", k_pkadd, 64},
        {"mix 2perm:1bitop3", k_mix, 192}, {"v_lshlrev_b64", k_lshl64, 64}, {"v_lshrrev_b64", k_lshr64, 64},
    };
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // clock estimate
    hipLaunchKernelGGL(k_clock, dim3(ncu * 8), dim3(256), 0, 0, clk, 1 << 20);
    hipDeviceSynchronize();
    uint64_t hc[3];
    hipMemcpy(hc, clk, 24, hipMemcpyDeviceToHost);
    printf("{\"cus\": %d, \"clock_ghz_est\": %.3f", ncu, (double)hc[0] / (double)hc[1] * 0.1);
    for (int waves_per_simd : {2, 4, 8}) {
        int blocks = ncu * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
        for (auto& k : ks) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 7u, 5u);
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 7u, 5u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            double wave_instr = (double)blocks * 4 * N_ITER * 8 * k.per_iter;
            double per_simd_per_ns = wave_instr / (ncu * 4) / (ms * 1e6);
            printf(", \"%s@%dw\": {\"ms\": %.3f, \"wave_instr_per_simd_per_ns\": %.3f}", k.name,
                   waves_per_simd, ms, per_simd_per_ns);
        }
        {
            hipLaunchKernelGGL(k_lds_bcast, dim3(blocks), dim3(256), 0, 0, out, 7u, 5u);
            hipEventRecord(a);
            hipLaunchKernelGGL(k_lds_bcast, dim3(blocks), dim3(256), 0, 0, out, 7u, 5u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            double reads = (double)blocks * 4 * N_ITER * 8;
            printf(", \"ds_read_b128_bcast_dep@%dw\": {\"ms\": %.3f, \"reads_per_cu_per_ns\": %.3f}",
                   waves_per_simd, ms, reads / ncu / (ms * 1e6));
        }
    }
    printf("}\n");
    return 0;
}
