// qf_bs.h -- bit-sliced Cauchy encode kernels (generated gfx950 assembly).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qf {

struct BsCache {
    static const int kMax = 16;
    hipModule_t mod[kMax] = {};
    hipFunction_t fn[kMax] = {};
};

// Is there a specialised kernel for the Cauchy matrix of (k, r)?
bool bs_available(uint32_t k, uint32_t r);
// Encode G generations (rows of L bytes, L % 16 == 0, L >= 64; strides and
// generation strides < 2^32, 16-byte aligned).
hipError_t bs_launch(BsCache& cache, int num_cus, hipStream_t st, uint32_t k, uint32_t r,
                     const uint8_t* src, uint8_t* dst, uint64_t sgs, uint64_t dgs, uint64_t srs,
                     uint64_t drs, uint32_t L, uint32_t G);
void bs_unload(BsCache& cache);

}  // namespace qf
