// qf_wiedemann.hip -- the GF(2^8) decoder's strategy for k > 256:
// Decoder::wiedemann_algorithm (decoder.rs:794-975), which Decoder::new
// selects above 256 (decoder.rs:659-665), on the device.
//
// The k accepted rows are k - e systematic rows and e repair rows J with
// explicit coefficients A_J (e x k).  Eliminating the systematic rows leaves
// the e x e block M = A_J[:, E] on the erased sources E (M is singular iff
// the whole k x k system is), so the Krylov machinery runs on M:
//   k_w8_sequence  one workgroup: gathers M, the Krylov sequence
//                  a_t = u . M^t u for t < 2e with the reference's init
//                  vectors u_i = (i + b + 1) % 255 (decoder.rs:805-807,
//                  934-941), Berlekamp-Massey (decoder.rs:946-975) and the
//                  minimal polynomial f = the REVERSED connection polynomial
//                  (the reference uses the connection polynomial itself, so
//                  its singularity test poly[0] == 0 never fires: fix (a) in
//                  oracle/qf_oracle_wiedemann.c);
//   k_w8_horner    W = f_0^-1 sum_{i>=1} f_i M^(i-1), Horner, one launch per
//                  degree (decoder.rs:856-884 sums explicit powers instead);
//   k_w8_verify    M W == I.  The reference does not check; a projection whose
//                  sequence misses a factor of M's minimal polynomial gives a
//                  wrong W, so the host tries the next init vector b;
//   k_w8_dmat      D = W [A_J on the received sources | I on the repair slots]:
//                  the e x k recovery matrix over the accepted slots;
//   k_w8_apply     recovered rows = D . rows (decoder.rs:886-887), split over
//                  slot chunks and combined with 32-bit atomic XOR.
// Systematic rows take part with their payloads (the F4 fix, as on the
// Gauss-Jordan path).  Products in the small kernels use log/exp tables
// built in LDS; the payload pass uses the context's split tables (v_perm).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "gf256_tables.h"
#include "qf_fec.h"
#include "qf_internal.h"

#define QF_CHECK_HIP(expr)                         \
    do {                                           \
        hipError_t _e = (expr);                    \
        if (_e != hipSuccess) return QF_EDEVICE;   \
    } while (0)

namespace qf {
namespace {

constexpr uint32_t kTries = 8;            // init vectors b = 0..7
constexpr uint32_t kSeqThreads = 1024;
constexpr uint32_t kRepairBit = 0x80000000u;

__device__ __forceinline__ uint32_t gf_mul_slow(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & 0x100) a ^= 0x11D;
    }
    return r;
}

// exp[0..509] (exp[i + 255] = exp[i]), log[1..255]; threads < 255 each build one entry.
__device__ void build_tables(uint8_t* ex, uint8_t* lg) {
    const uint32_t i = threadIdx.x;
    if (i < 255) {
        uint32_t x = 1, base = 2, n = i;
        while (n) {
            if (n & 1) x = gf_mul_slow(x, base);
            base = gf_mul_slow(base, base);
            n >>= 1;
        }
        ex[i] = (uint8_t)x;
        ex[i + 255] = (uint8_t)x;
        lg[x] = (uint8_t)i;
    }
    if (i == 0) {
        lg[0] = 0;
        ex[510] = ex[511] = 0;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t gmul(const uint8_t* ex, const uint8_t* lg, uint32_t a, uint32_t b) {
    return (a && b) ? ex[(uint32_t)lg[a] + lg[b]] : 0u;
}

__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v ^= __shfl_xor(v, o, 64);
    return v;
}

// XOR of v over the block (all threads get it); red: one word per wave.
__device__ uint32_t block_xor(uint32_t v, uint32_t* red) {
    v = wave_xor(v);
    const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    uint32_t s = 0;
    for (uint32_t q = 0; q < nw; ++q) s ^= red[q];
    return s;
}

struct SeqArgs {
    const uint8_t* A;     // e x kp: repair coefficient rows
    const uint16_t* E;    // e erased sources, ascending
    uint8_t* M;           // e x ep (out)
    uint8_t* P;           // e x ep (out): identity, the Horner start (f_L = 1)
    uint8_t* poly;        // f_0..f_L (out)
    int32_t* info;        // [0] L, [1] 0 ok / 1 zero sequence / 2 singular
    uint32_t e, ep, kp, b;
    uint32_t m_lds;       // M also staged in LDS (e * e bytes after the vectors)
};

__global__ void __launch_bounds__(kSeqThreads) k_w8_sequence(SeqArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t e = a.e, n = 2 * e, tid = threadIdx.x, nt = blockDim.x;
    uint8_t* ex = lds;
    uint8_t* lg = ex + 512;
    uint32_t* red = reinterpret_cast<uint32_t*>(lg + 256);   // 16 words
    uint8_t* u = lg + 256 + 64;
    uint8_t* v = u + e;
    uint8_t* w = v + e;
    uint8_t* seq = w + e;
    uint8_t* C = seq + n;
    uint8_t* B = C + n + 1;
    uint8_t* T = B + n + 1;
    uint8_t* Ml = T + n + 1;
    build_tables(ex, lg);
    // M[i][j] = A[i][E[j]]; P = I
    for (uint32_t q = tid; q < e * e; q += nt) {
        const uint32_t i = q / e, j = q - i * e;
        const uint8_t mij = a.A[(size_t)i * a.kp + a.E[j]];
        a.M[(size_t)i * a.ep + j] = mij;
        a.P[(size_t)i * a.ep + j] = i == j ? 1 : 0;
        if (a.m_lds) Ml[q] = mij;
    }
    for (uint32_t i = tid; i < e; i += nt) {
        u[i] = (uint8_t)((i + a.b + 1) % 255);
        v[i] = u[i];
    }
    for (uint32_t i = tid; i <= n; i += nt) {
        C[i] = i == 0;
        B[i] = i == 0;
    }
    __threadfence_block();
    __syncthreads();
    // a_t = u . M^t u
    for (uint32_t t = 0; t < n; ++t) {
        uint32_t d = 0;
        for (uint32_t i = tid; i < e; i += nt) d ^= gmul(ex, lg, u[i], v[i]);
        d = block_xor(d, red);
        if (tid == 0) seq[t] = (uint8_t)d;
        for (uint32_t i = tid; i < e; i += nt) {
            const uint8_t* m = a.m_lds ? Ml + (size_t)i * e : a.M + (size_t)i * a.ep;
            uint32_t acc = 0;
            for (uint32_t j = 0; j < e; ++j) acc ^= gmul(ex, lg, m[j], v[j]);
            w[i] = (uint8_t)acc;
        }
        __syncthreads();
        for (uint32_t i = tid; i < e; i += nt) v[i] = w[i];
        __syncthreads();
    }
    // Berlekamp-Massey: s[i] = sum_{j=1..L} C[j] s[i-j]
    uint32_t L = 0, m = 1, bd = 1;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t d = 0;
        for (uint32_t j = 1 + tid; j <= L; j += nt) d ^= gmul(ex, lg, C[j], seq[i - j]);
        d = block_xor(d, red) ^ seq[i];
        if (d == 0) {
            ++m;
            continue;
        }
        const uint32_t coef = ex[(uint32_t)lg[d] + 255u - lg[bd]];   // d / bd
        const bool grow = 2 * L <= i;
        if (grow)
            for (uint32_t j = tid; j <= n; j += nt) T[j] = C[j];
        __syncthreads();
        for (uint32_t j = tid; j + m <= n; j += nt) C[j + m] ^= (uint8_t)gmul(ex, lg, coef, B[j]);
        __syncthreads();
        if (grow) {
            for (uint32_t j = tid; j <= n; j += nt) B[j] = T[j];
            __syncthreads();
            L = i + 1 - L;
            bd = d;
            m = 1;
        } else {
            ++m;
        }
    }
    // f_i = C[L - i]
    for (uint32_t i = tid; i <= L; i += nt) a.poly[i] = C[L - i];
    if (tid == 0) {
        a.info[0] = (int32_t)L;
        a.info[1] = L == 0 ? 1 : (C[L] == 0 ? 2 : 0);
    }
}

// mode 0: Pout = Pin M ^ fi I;  mode 1: Pout = scale Pin.  Block = row i.
struct HornerArgs {
    const uint8_t* Pin;
    uint8_t* Pout;
    const uint8_t* M;
    uint32_t e, ep, fi, scale, mode;
};

__global__ void __launch_bounds__(256) k_w8_horner(HornerArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* ex = lds;
    uint8_t* lg = ex + 512;
    uint8_t* row = lg + 256;
    build_tables(ex, lg);
    const uint32_t i = blockIdx.x, e = a.e;
    for (uint32_t l = threadIdx.x; l < e; l += blockDim.x) row[l] = a.Pin[(size_t)i * a.ep + l];
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < e; j += blockDim.x) {
        uint32_t acc;
        if (a.mode == 0) {
            acc = i == j ? a.fi : 0u;
            for (uint32_t l = 0; l < e; ++l) acc ^= gmul(ex, lg, row[l], a.M[(size_t)l * a.ep + j]);
        } else {
            acc = gmul(ex, lg, a.scale, row[j]);
        }
        a.Pout[(size_t)i * a.ep + j] = (uint8_t)acc;
    }
}

// info[2] |= 1 where (M W)[i][j] != [i == j].  Block = row i.
__global__ void __launch_bounds__(256) k_w8_verify(const uint8_t* M, const uint8_t* W, uint32_t e, uint32_t ep,
                                                   int32_t* info) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* ex = lds;
    uint8_t* lg = ex + 512;
    uint8_t* row = lg + 256;
    build_tables(ex, lg);
    const uint32_t i = blockIdx.x;
    for (uint32_t l = threadIdx.x; l < e; l += blockDim.x) row[l] = M[(size_t)i * ep + l];
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < e; j += blockDim.x) {
        uint32_t acc = 0;
        for (uint32_t l = 0; l < e; ++l) acc ^= gmul(ex, lg, row[l], W[(size_t)l * ep + j]);
        if (acc != (i == j ? 1u : 0u)) atomicOr(&info[2], 1);
    }
}

// D[t][q] over the k accepted slots: slot q is repair ordinal p (slot[q] =
// kRepairBit | p) -> W[t][p]; systematic source s -> sum_p W[t][p] A[p][s].
__global__ void __launch_bounds__(256) k_w8_dmat(const uint8_t* W, const uint8_t* A, const uint32_t* slot,
                                                 uint8_t* D, uint32_t e, uint32_t ep, uint32_t k, uint32_t kp) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* ex = lds;
    uint8_t* lg = ex + 512;
    uint8_t* row = lg + 256;
    build_tables(ex, lg);
    const uint32_t t = blockIdx.x;
    for (uint32_t p = threadIdx.x; p < e; p += blockDim.x) row[p] = W[(size_t)t * ep + p];
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < k; q += blockDim.x) {
        const uint32_t s = slot[q];
        uint32_t acc;
        if (s & kRepairBit) {
            acc = row[s & 0xFFFFu];
        } else {
            acc = 0;
            for (uint32_t p = 0; p < e; ++p) acc ^= gmul(ex, lg, row[p], A[(size_t)p * kp + s]);
        }
        D[(size_t)t * kp + q] = (uint8_t)acc;
    }
}

__device__ __forceinline__ uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

struct ApplyArgs {
    const uint8_t* rows;   // k slots, stride apart (16-B aligned, zero padded)
    const uint8_t* D;      // e x kp
    const uint32_t* tab;   // 256 split-table records of 8 dwords
    uint8_t* out;          // e rows, stride apart (zeroed)
    uint64_t stride;
    uint32_t e, k, kp, Lu;
};

constexpr uint32_t kApplyOut = 4;      // outputs per block
constexpr uint32_t kApplySlots = 64;   // slots per block (16 per wave)

// grid (ceil(Lu / 64), ceil(e / 4), ceil(k / 64)); lane = 16-byte unit,
// wave w takes slots z*64 + w + 4m.  Wave partials meet in LDS, then one
// atomic XOR per dword per output.
__global__ void __launch_bounds__(256) k_w8_apply(ApplyArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[256 * 8];
    __shared__ uint4 part[4][kApplyOut][64];
    for (uint32_t q = threadIdx.x; q < 256 * 8; q += blockDim.x) tab[q] = a.tab[q];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t u = blockIdx.x * 64 + lane, t0 = blockIdx.y * kApplyOut;
    uint4 acc[kApplyOut];
#pragma unroll
    for (uint32_t o = 0; o < kApplyOut; ++o) acc[o] = make_uint4(0, 0, 0, 0);
    if (u < a.Lu) {
        for (uint32_t mm = 0; mm < kApplySlots / 4; ++mm) {
            const uint32_t q = blockIdx.z * kApplySlots + wave + 4 * mm;
            if (q >= a.k) break;
            const uint4 x = *reinterpret_cast<const uint4*>(a.rows + (uint64_t)q * a.stride + (uint64_t)u * 16);
            const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (uint32_t o = 0; o < kApplyOut; ++o) {
                const uint32_t t = t0 + o;
                if (t >= a.e) break;
                const uint32_t c = a.D[(size_t)t * a.kp + q];
                if (c == 0) continue;
                const uint32_t* r = tab + 8 * c;
                uint32_t y[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const uint32_t s0 = xs[d] & 0x07070707u, s1 = (xs[d] >> 3) & 0x07070707u,
                                   s2 = (xs[d] >> 6) & 0x03030303u;
                    y[d] = vperm(r[1], r[0], s0) ^ vperm(r[3], r[2], s1) ^ vperm(r[4], r[4], s2);
                }
                acc[o].x ^= y[0];
                acc[o].y ^= y[1];
                acc[o].z ^= y[2];
                acc[o].w ^= y[3];
            }
        }
    }
#pragma unroll
    for (uint32_t o = 0; o < kApplyOut; ++o) part[wave][o][lane] = acc[o];
    __syncthreads();
    // wave w combines output w
    const uint32_t o = wave, t = t0 + o;
    if (t < a.e && u < a.Lu) {
        uint4 s = part[0][o][lane];
        for (uint32_t w = 1; w < 4; ++w) {
            const uint4 p = part[w][o][lane];
            s.x ^= p.x;
            s.y ^= p.y;
            s.z ^= p.z;
            s.w ^= p.w;
        }
        uint32_t* dst = reinterpret_cast<uint32_t*>(a.out + (uint64_t)t * a.stride + (uint64_t)u * 16);
        if (s.x) atomicXor(dst + 0, s.x);
        if (s.y) atomicXor(dst + 1, s.y);
        if (s.z) atomicXor(dst + 2, s.z);
        if (s.w) atomicXor(dst + 3, s.w);
    }
}

static inline uint32_t r16(uint32_t x) { return (x + 15) & ~15u; }

}  // namespace

int wiedemann_decode(qf_ctx* ctx, uint32_t k, uint32_t e, const uint8_t* A_ek, const uint16_t* E,
                     const uint32_t* slot, const uint8_t* d_rows, uint64_t stride, uint32_t L, uint8_t* d_rec,
                     uint32_t* tries_out) {
    if (tries_out) *tries_out = 0;
    if (!ctx || e == 0 || e > k || k > QF_DECODER_MAX_K || (stride & 15) || L > stride) return QF_EINVAL;
    std::unique_lock<std::mutex> lk;
    if (int s = ctx_lock(ctx, lk)) return s;
    hipStream_t st = ctx_stream(ctx);
    const uint32_t ep = r16(e), kp = r16(k);
    // workspace: A, E, slot, M, P0, P1, D, poly, info
    const size_t oA = 0, oE = oA + (size_t)e * kp, oS = oE + r16(2 * e), oM = oS + r16(4 * k);
    const size_t oP0 = oM + (size_t)e * ep, oP1 = oP0 + (size_t)e * ep, oD = oP1 + (size_t)e * ep;
    const size_t oPoly = oD + (size_t)e * kp, oInfo = oPoly + r16(2 * e + 2), total = oInfo + 16;
    uint8_t* w = nullptr;
    if (int s = ctx_work(ctx, total, &w)) return s;
    std::vector<uint8_t> hA((size_t)e * kp, 0);
    for (uint32_t p = 0; p < e; ++p) memcpy(&hA[(size_t)p * kp], A_ek + (size_t)p * k, k);
    QF_CHECK_HIP(hipMemcpyAsync(w + oA, hA.data(), hA.size(), hipMemcpyHostToDevice, st));
    QF_CHECK_HIP(hipMemcpyAsync(w + oE, E, (size_t)e * 2, hipMemcpyHostToDevice, st));
    QF_CHECK_HIP(hipMemcpyAsync(w + oS, slot, (size_t)k * 4, hipMemcpyHostToDevice, st));
    int32_t* info = reinterpret_cast<int32_t*>(w + oInfo);
    size_t seq_lds = 512 + 256 + 64 + 3 * (size_t)e + 2 * (size_t)e + 3 * (2 * (size_t)e + 1);
    const uint32_t m_lds = seq_lds + (size_t)e * e <= 128 * 1024;   // M in LDS up to e = 330
    if (m_lds) seq_lds += (size_t)e * e;
    const size_t row_lds = 512 + 256 + ep;
    if (seq_lds > 64 * 1024) {
        static std::once_flag once;
        hipError_t err = hipSuccess;
        std::call_once(once, [&] {
            err = hipFuncSetAttribute(reinterpret_cast<const void*>(k_w8_sequence),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        });
        QF_CHECK_HIP(err);
    }
    const auto& f = gf();
    uint8_t* W = nullptr;
    for (uint32_t b = 0; b < kTries; ++b) {
        if (tries_out) *tries_out = b + 1;
        SeqArgs sa{w + oA, reinterpret_cast<const uint16_t*>(w + oE), w + oM, w + oP0, w + oPoly, info, e, ep, kp, b,
                   m_lds};
        hipLaunchKernelGGL(k_w8_sequence, dim3(1), dim3(kSeqThreads), seq_lds, st, sa);
        QF_CHECK_HIP(hipGetLastError());
        int32_t hinfo[2] = {0, 0};
        QF_CHECK_HIP(hipMemcpyAsync(hinfo, info, 8, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipStreamSynchronize(st));
        if (hinfo[1] == 2) return QF_ERANK;    // x | f: M is singular
        if (hinfo[1] == 1) continue;           // zero sequence: no information
        const uint32_t Ld = (uint32_t)hinfo[0];
        std::vector<uint8_t> poly(Ld + 1);
        QF_CHECK_HIP(hipMemcpyAsync(poly.data(), w + oPoly, Ld + 1, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipStreamSynchronize(st));
        uint8_t f0inv = 0;
        if (!f.inv(poly[0], &f0inv)) return QF_ERANK;
        // Horner from P = I (f_L = 1): P <- P M ^ f_i I for i = L-1..1, then W = f_0^-1 P
        uint8_t* Pin = w + oP0;
        uint8_t* Pout = w + oP1;
        for (uint32_t i = Ld - 1; i >= 1; --i) {
            HornerArgs h{Pin, Pout, w + oM, e, ep, poly[i], 0, 0};
            hipLaunchKernelGGL(k_w8_horner, dim3(e), dim3(256), row_lds, st, h);
            QF_CHECK_HIP(hipGetLastError());
            std::swap(Pin, Pout);
        }
        HornerArgs h{Pin, Pout, w + oM, e, ep, 0, f0inv, 1};
        hipLaunchKernelGGL(k_w8_horner, dim3(e), dim3(256), row_lds, st, h);
        QF_CHECK_HIP(hipGetLastError());
        W = Pout;
        QF_CHECK_HIP(hipMemsetAsync(info + 2, 0, 4, st));
        hipLaunchKernelGGL(k_w8_verify, dim3(e), dim3(256), row_lds, st, w + oM, W, e, ep, info);
        QF_CHECK_HIP(hipGetLastError());
        int32_t bad = 0;
        QF_CHECK_HIP(hipMemcpyAsync(&bad, info + 2, 4, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipStreamSynchronize(st));
        if (!bad) break;
        W = nullptr;
    }
    if (!W) return QF_ERANK;
    hipLaunchKernelGGL(k_w8_dmat, dim3(e), dim3(256), row_lds, st, W, w + oA, reinterpret_cast<const uint32_t*>(w + oS),
                       w + oD, e, ep, k, kp);
    QF_CHECK_HIP(hipGetLastError());
    QF_CHECK_HIP(hipMemsetAsync(d_rec, 0, (size_t)e * stride, st));
    const uint32_t Lu = (L + 15) / 16;
    if (Lu) {
        ApplyArgs ap{d_rows, w + oD, ctx_tab256(ctx), d_rec, stride, e, k, kp, Lu};
        dim3 grid((Lu + 63) / 64, (e + kApplyOut - 1) / kApplyOut, (k + kApplySlots - 1) / kApplySlots);
        hipLaunchKernelGGL(k_w8_apply, grid, dim3(256), 0, st, ap);
        QF_CHECK_HIP(hipGetLastError());
    }
    return QF_OK;
}

}  // namespace qf
