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
//   k_w8_rows      row combinations with wave-uniform coefficients (split-table
//                  v_perm products), three uses:
//                  W = f_0^-1 sum_{i>=1} f_i M^(i-1) by Horner, one launch per
//                  degree (decoder.rs:856-884 sums explicit powers instead);
//                  the check M W == I (the reference does not check: a
//                  projection whose sequence misses a factor of M's minimal
//                  polynomial gives a wrong W, so the host tries the next init
//                  vector b, and after kTries of them inverts M exactly on the
//                  host -- a failed projection is not a rank verdict); and
//                  G = W A_J;
//   k_w8_apply     recovered rows = D . rows (decoder.rs:886-887) with
//                  D[t][q] = W[t][p] on repair slot q (ordinal p) and G[t][s]
//                  on the systematic slot of source s, split over slot chunks
//                  and combined with 32-bit atomic XOR.
// Systematic rows take part with their payloads (the F4 fix, as on the
// Gauss-Jordan path).  The sequence kernel multiplies in the log domain
// (tables built in LDS, M kept as logs); the others use the context's split
// tables (v_perm).
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <random>
#include <vector>

#include "gf256_tables.h"
#include "qf_fec.h"
#include "qf_internal.h"


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
    uint16_t* LMg;        // e x ep logs of M (global, when they do not fit LDS)
    uint8_t* poly;        // f_0..f_L (out)
    int32_t* info;        // [0] L, [1] 0 ok / 1 zero sequence / 2 singular
    uint32_t e, ep, kp, b;
    uint32_t seed;        // 0: the reference's init vector b; else a random projection (init_u)
    uint32_t lm_lds;      // logs of M in LDS (2 e^2 bytes after the vectors)
    // baby-step / giant-step Krylov (s > 1): a_{i s + j} = w_i . v_j with
    // v_j = M^j u (j < s) and w_i = (M^T)^(s i) u, so 2e / s + s dependent
    // matrix-vector steps instead of 2e
    uint32_t s;           // 1: plain
    uint8_t* MT;          // e x ep (out, phase 0): M^T, squared by the host into MsT
    const uint8_t* MsT;   // e x ep: (M^T)^s
    uint16_t* LMs;        // e x ep logs of MsT (global)
    uint8_t* V;           // s x ep: the baby-step vectors (global)
    uint32_t gather_only; // phase 0: write M, P and MT, then stop
};

constexpr uint32_t kLogZero = 0x200;     // log of 0: every sum with it indexes a zero
constexpr uint32_t kEx2 = 1040;          // exp over [0, 510), zero above
constexpr uint32_t kRed2Bytes = 4096;
constexpr uint32_t kBsgsMinE = 64;
constexpr uint32_t kPsMinE = 16, kPsMaxE = 1024;

// Entry i of the projection / start vector u: the reference's
// u_i = (i + b + 1) mod 255 (decoder.rs:805-807, 934-941) for seed 0, else a
// byte of a splitmix-style hash of (seed, i) -- a projection no sender can
// predict (QF_OPT_WIEDEMANN_PROJ).
__device__ __forceinline__ uint8_t init_u(const SeqArgs& a, uint32_t i) {
    if (a.seed == 0) return (uint8_t)((i + a.b + 1) % 255);
    uint64_t z = ((uint64_t)a.seed << 32 | i) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint8_t)((z ^ (z >> 31)) >> 24);
}

// Log-domain tables: ex2[lg[a] + lg[b]] = a * b for all a, b (lg[0] = kLogZero).
__device__ void build_log_tables(uint8_t* ex2, uint16_t* lg) {
    for (uint32_t i = threadIdx.x; i < kEx2; i += blockDim.x) {
        uint32_t x = 0;
        if (i < 510) {
            uint32_t base = 2, n = i % 255;
            x = 1;
            while (n) {
                if (n & 1) x = gf_mul_slow(x, base);
                base = gf_mul_slow(base, base);
                n >>= 1;
            }
            if (i < 255) lg[x] = (uint16_t)i;
        }
        ex2[i] = (uint8_t)x;
    }
    if (threadIdx.x == 0) lg[0] = kLogZero;
    __syncthreads();
}

__global__ void __launch_bounds__(kSeqThreads) k_w8_sequence(SeqArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t e = a.e, n = 2 * e, tid = threadIdx.x, nt = blockDim.x;
    uint8_t* ex2 = lds;
    uint16_t* lg = reinterpret_cast<uint16_t*>(lds + kEx2);            // 256
    uint32_t* red = reinterpret_cast<uint32_t*>(lds + kEx2 + 512);     // 16 words
    uint32_t* red2 = red + 16;                                         // 1,024 words: giant-step partials
    uint16_t* lu = reinterpret_cast<uint16_t*>(lds + kEx2 + 512 + 64 + kRed2Bytes);
    uint16_t* lv = lu + e;
    uint16_t* LMl = lv + e;                                            // e * e when lm_lds
    uint8_t* v = reinterpret_cast<uint8_t*>(a.lm_lds ? LMl + (size_t)e * e : LMl);
    uint8_t* w = v + e;
    uint8_t* seq = w + e;
    uint8_t* C = seq + n;
    uint8_t* B = C + n + 1;
    uint8_t* T = B + n + 1;
    build_log_tables(ex2, lg);
    uint16_t* LM = a.lm_lds ? LMl : a.LMg;
    const uint32_t lmp = a.lm_lds ? e : a.ep;
    // M[i][j] = A[i][E[j]], its logs; P = I
    for (uint32_t q = tid; q < e * e; q += nt) {
        const uint32_t i = q / e, j = q - i * e;
        const uint8_t mij = a.A[(size_t)i * a.kp + a.E[j]];
        a.M[(size_t)i * a.ep + j] = mij;
        a.P[(size_t)i * a.ep + j] = i == j ? 1 : 0;
        LM[(size_t)i * lmp + j] = lg[mij];
        if (a.gather_only) a.MT[(size_t)j * a.ep + i] = mij;
        else if (a.s > 1) a.LMs[(size_t)i * a.ep + j] = lg[a.MsT[(size_t)i * a.ep + j]];
    }
    if (a.gather_only) return;
    for (uint32_t i = tid; i < e; i += nt) {
        const uint8_t ui = init_u(a, i);
        lu[i] = lg[ui];
        v[i] = ui;
    }
    for (uint32_t i = tid; i <= n; i += nt) {
        C[i] = i == 0;
        B[i] = i == 0;
    }
    __threadfence_block();
    __syncthreads();
    // y = X x for an e x e matrix X given as logs (pitch xp), x in LDS as
    // bytes.  Row i takes S threads (a power of two <= 64, S = nt / e rounded
    // down), combined by shuffles inside the wave.
    uint32_t S = 1;
    while (S * 2 <= 64 && S * 2 * e <= nt) S *= 2;
    const uint32_t rows_per_pass = nt / S;
    auto matvec = [&](const uint16_t* X, uint32_t xp, uint8_t* x) {
        for (uint32_t i = tid; i < e; i += nt) lv[i] = lg[x[i]];
        __syncthreads();
        for (uint32_t i0 = 0; i0 < e; i0 += rows_per_pass) {
            const uint32_t i = i0 + tid / S, s0 = tid % S;
            uint32_t acc = 0;
            if (i < e) {
                const uint16_t* m = X + (size_t)i * xp;
                uint32_t j = s0;
                for (; j + 3 * S < e; j += 4 * S)
                    acc ^= ex2[m[j] + lv[j]] ^ ex2[m[j + S] + lv[j + S]] ^ ex2[m[j + 2 * S] + lv[j + 2 * S]] ^
                           ex2[m[j + 3 * S] + lv[j + 3 * S]];
                for (; j < e; j += S) acc ^= ex2[m[j] + lv[j]];
            }
            for (uint32_t o = 1; o < S; o <<= 1) acc ^= __shfl_xor(acc, o, 64);
            if (i < e && s0 == 0) w[i] = (uint8_t)acc;
        }
        __syncthreads();
        for (uint32_t i = tid; i < e; i += nt) x[i] = w[i];
        __syncthreads();
    };
    if (a.s <= 1) {
        // a_t = u . M^t u, one step per t
        for (uint32_t t = 0; t < n; ++t) {
            uint32_t d = 0;
            for (uint32_t i = tid; i < e; i += nt) d ^= ex2[lu[i] + lg[v[i]]];
            d = block_xor(d, red);
            if (tid == 0) seq[t] = (uint8_t)d;
            matvec(LM, lmp, v);
        }
    } else {
        // baby steps: V[j] = M^j u (v starts as u)
        for (uint32_t j = 0; j < a.s; ++j) {
            for (uint32_t i = tid; i < e; i += nt) a.V[(size_t)j * a.ep + i] = v[i];
            if (j + 1 < a.s) matvec(LM, lmp, v);
        }
        // giant steps: x = (M^T)^(s i) u; a_{i s + j} = x . V[j]; thread
        // (j = tid % s, stripe tid / s) sums a stripe, threads j < s fold
        for (uint32_t i = tid; i < e; i += nt) v[i] = init_u(a, i);
        __threadfence_block();
        __syncthreads();
        const uint32_t sp = a.s, nst = nt / sp;
        for (uint32_t gi = 0; gi * sp < n; ++gi) {
            for (uint32_t i = tid; i < e; i += nt) lv[i] = lg[v[i]];
            __syncthreads();
            const uint32_t j = tid % sp, st = tid / sp;
            uint32_t d = 0;
            if (st < nst)
                for (uint32_t q = st; q < e; q += nst) d ^= ex2[lv[q] + lg[a.V[(size_t)j * a.ep + q]]];
            // fold the stripes of each j: lanes tid, tid + sp, ... of a wave by shuffles, waves in LDS
            for (uint32_t o = sp; o < 64; o <<= 1) d ^= __shfl_xor(d, o, 64);
            __syncthreads();
            if ((tid & 63) < sp) red2[(tid >> 6) * sp + (tid & 63)] = d;
            __syncthreads();
            if (tid < sp && gi * sp + tid < n) {
                uint32_t sum = 0;
                for (uint32_t wv = 0; wv < nt / 64; ++wv) sum ^= red2[wv * sp + tid];
                seq[gi * sp + tid] = (uint8_t)sum;
            }
            if ((gi + 1) * sp < n) matvec(a.LMs, a.ep, v);
        }
    }
    // Berlekamp-Massey on wave 0 alone (the other waves end here, so its
    // barriers wait for nobody): s[i] = sum_{j=1..L} C[j] s[i-j]
    if (tid >= 64) return;
    const uint32_t nw = 64;
    uint32_t L = 0, m = 1, bd = 1;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t d = 0;
        for (uint32_t j = 1 + tid; j <= L; j += nw) d ^= ex2[lg[C[j]] + lg[seq[i - j]]];
        d = wave_xor(d) ^ seq[i];
        if (d == 0) {
            ++m;
            continue;
        }
        const uint32_t coef = ex2[(uint32_t)lg[d] + 255u - lg[bd]];   // d / bd
        const uint32_t lc = lg[coef];
        const bool grow = 2 * L <= i;
        if (grow)
            for (uint32_t j = tid; j <= n; j += nw) T[j] = C[j];
        __syncthreads();
        for (uint32_t j = tid; j + m <= n; j += nw) C[j + m] ^= ex2[lc + lg[B[j]]];
        __syncthreads();
        if (grow) {
            for (uint32_t j = tid; j <= n; j += nw) B[j] = T[j];
            __syncthreads();
            L = i + 1 - L;
            bd = d;
            m = 1;
        } else {
            ++m;
        }
    }
    // f_i = C[L - i]
    for (uint32_t i = tid; i <= L; i += nw) a.poly[i] = C[L - i];
    if (tid == 0) {
        a.info[0] = (int32_t)L;
        a.info[1] = L == 0 ? 1 : (C[L] == 0 ? 2 : 0);
    }
}

__device__ __forceinline__ uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// c * x for the four bytes of x, c's split-table record r (gf256_tables.h).
__device__ __forceinline__ uint32_t mul4(const uint32_t* r, uint32_t x) {
    return vperm(r[1], r[0], x & 0x07070707u) ^ vperm(r[3], r[2], (x >> 3) & 0x07070707u) ^
           vperm(r[4], r[4], (x >> 6) & 0x03030303u);
}

// Row combinations out[i][:] = sum_l coef[i][l] * in[l][:] over n input rows
// of `words` dwords: the Horner step (P M, plus diag on the diagonal), the
// check (M W == I) and G = W A_J.  Block (i, word chunk of 64); lane = dword,
// wave q takes l = q, q + 4, ...; the coefficient is wave-uniform (row i of
// coef staged in LDS), the product the split-table v_perm.
struct RowsArgs {
    const uint8_t* coef;
    const uint8_t* in;
    uint8_t* out;
    const uint32_t* tab;
    uint64_t coef_pitch, in_pitch, out_pitch;
    uint32_t n, words;
    uint32_t diag;     // out[i][i] ^= diag
    uint32_t scale;    // != 0: out = scale * in[i] (no combination)
    int32_t* check;    // != null: compare with the identity instead of storing
};

__global__ void __launch_bounds__(256) k_w8_rows(RowsArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[256 * 8];
    __shared__ uint32_t part[4][64];
    extern __shared__ __attribute__((aligned(16))) uint8_t crow[];
    const uint32_t i = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t wd = blockIdx.y * 64 + lane;
    for (uint32_t q = threadIdx.x; q < 256 * 8; q += blockDim.x) tab[q] = a.tab[q];
    if (!a.scale)
        for (uint32_t l = threadIdx.x; l < a.n; l += blockDim.x) crow[l] = a.coef[(uint64_t)i * a.coef_pitch + l];
    __syncthreads();
    uint32_t acc = 0;
    if (wd < a.words) {
        if (a.scale) {
            if (wave == 0) acc = mul4(tab + 8 * a.scale, *reinterpret_cast<const uint32_t*>(a.in + (uint64_t)i * a.in_pitch + 4 * wd));
        } else {
            const uint8_t* col = a.in + 4 * (uint64_t)wd;
            uint32_t l = wave;
            for (; l + 12 < a.n; l += 16) {   // four rows in flight per wave
                const uint32_t x0 = *reinterpret_cast<const uint32_t*>(col + (uint64_t)l * a.in_pitch);
                const uint32_t x1 = *reinterpret_cast<const uint32_t*>(col + (uint64_t)(l + 4) * a.in_pitch);
                const uint32_t x2 = *reinterpret_cast<const uint32_t*>(col + (uint64_t)(l + 8) * a.in_pitch);
                const uint32_t x3 = *reinterpret_cast<const uint32_t*>(col + (uint64_t)(l + 12) * a.in_pitch);
                acc ^= mul4(tab + 8 * crow[l], x0) ^ mul4(tab + 8 * crow[l + 4], x1) ^
                       mul4(tab + 8 * crow[l + 8], x2) ^ mul4(tab + 8 * crow[l + 12], x3);
            }
            for (; l < a.n; l += 4)
                acc ^= mul4(tab + 8 * crow[l], *reinterpret_cast<const uint32_t*>(col + (uint64_t)l * a.in_pitch));
        }
    }
    part[wave][lane] = acc;
    __syncthreads();
    if (wave != 0 || wd >= a.words) return;
    uint32_t v = part[0][lane] ^ part[1][lane] ^ part[2][lane] ^ part[3][lane];
    if (wd == (i >> 2)) v ^= a.diag << (8 * (i & 3));
    if (a.check) {
        const uint32_t want = wd == (i >> 2) ? 1u << (8 * (i & 3)) : 0u;
        // bytes past n in the last word are padding: compare the real ones
        const uint32_t nb = a.n - 4 * wd < 4 ? a.n - 4 * wd : 4;
        const uint32_t mask = nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1);
        if ((v ^ want) & mask) atomicOr(a.check, 1);
        return;
    }
    *reinterpret_cast<uint32_t*>(a.out + (uint64_t)i * a.out_pitch + 4 * wd) = v;
}

struct ApplyArgs {
    const uint8_t* rows;   // k slots, stride apart (16-B aligned, zero padded)
    const uint8_t* G;      // e x kp: G[t][s] = sum_p W[t][p] A_J[p][s]
    const uint8_t* W;      // e x ep
    const uint32_t* slot;  // k: source index, or kRepairBit | repair ordinal
    const uint32_t* tab;   // 256 split-table records of 8 dwords
    uint8_t* out;          // e rows, stride apart (zeroed)
    uint64_t stride;
    uint32_t e, k, kp, ep, Lu;
};

constexpr uint32_t kApplyOut = 4;      // outputs per block
constexpr uint32_t kApplySlots = 64;   // slots per block (16 per wave)

// recovered[t] = sum over slots q of D[t][q] rows[q], D[t][q] = W[t][p] for
// repair slot q (ordinal p), G[t][s] for systematic slot q (source s).
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
            const uint32_t sq = a.slot[q];
            const uint4 x = *reinterpret_cast<const uint4*>(a.rows + (uint64_t)q * a.stride + (uint64_t)u * 16);
#pragma unroll
            for (uint32_t o = 0; o < kApplyOut; ++o) {
                const uint32_t t = t0 + o;
                if (t >= a.e) break;
                const uint32_t c = (sq & kRepairBit) ? a.W[(size_t)t * a.ep + (sq & 0xFFFFu)]
                                                     : a.G[(size_t)t * a.kp + sq];
                if (c == 0) continue;
                const uint32_t* r = tab + 8 * c;
                acc[o].x ^= mul4(r, x.x);
                acc[o].y ^= mul4(r, x.y);
                acc[o].z ^= mul4(r, x.z);
                acc[o].w ^= mul4(r, x.w);
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

// dst ^= c * src over n bytes (n % 16 == 0): nibble tables, 16 lookups per pshufb
__attribute__((target("ssse3"))) static void row_axpy(uint8_t* dst, const uint8_t* src, uint8_t c, size_t n) {
    const Gf256& f = gf();
    alignas(16) uint8_t lo[16], hi[16];
    for (int v = 0; v < 16; ++v) {
        lo[v] = f.mul(c, (uint8_t)v);
        hi[v] = f.mul(c, (uint8_t)(v << 4));
    }
    const __m128i tl = _mm_load_si128(reinterpret_cast<const __m128i*>(lo));
    const __m128i th = _mm_load_si128(reinterpret_cast<const __m128i*>(hi));
    const __m128i m = _mm_set1_epi8(0x0f);
    for (size_t i = 0; i < n; i += 16) {
        const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i p = _mm_xor_si128(_mm_shuffle_epi8(tl, _mm_and_si128(x, m)),
                                        _mm_shuffle_epi8(th, _mm_and_si128(_mm_srli_epi16(x, 4), m)));
        __m128i* d = reinterpret_cast<__m128i*>(dst + i);
        _mm_storeu_si128(d, _mm_xor_si128(_mm_loadu_si128(d), p));
    }
}

// A nonzero 32-bit seed per random projection: splitmix64 over a per-process
// secret (std::random_device at first use) and a counter, so the projections
// of a k > 256 decode cannot be predicted from the packets it receives.
static uint32_t projection_seed() {
    static const uint64_t key = [] {
        std::random_device rd;
        return ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    }();
    static std::atomic<uint64_t> ctr{0};
    uint64_t z = key + 0x9E3779B97F4A7C15ull * (ctr.fetch_add(1, std::memory_order_relaxed) + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    const uint32_t v = (uint32_t)((z ^ (z >> 31)) >> 16);
    return v ? v : 1;
}

// The exact fallback when no init vector verifies (every projection missed a
// factor of M's minimal polynomial -- possible for a nonsingular M, so it is
// not a rank verdict): Gauss-Jordan on [M | I] on the host, W = M^-1 with row
// stride ep.  Returns false iff M is singular.  O(e^3 / 16) pshufb steps.
static bool exact_inverse(const uint8_t* A_ek, uint32_t k, const uint16_t* E, uint32_t e, uint32_t ep,
                          std::vector<uint8_t>& W) {
    const Gf256& f = gf();
    const size_t w2 = 2 * (size_t)ep;
    std::vector<uint8_t> T((size_t)e * w2, 0);
    for (uint32_t i = 0; i < e; ++i) {
        for (uint32_t j = 0; j < e; ++j) T[(size_t)i * w2 + j] = A_ek[(size_t)i * k + E[j]];
        T[(size_t)i * w2 + ep + i] = 1;
    }
    for (uint32_t c = 0; c < e; ++c) {
        uint32_t p = c;
        while (p < e && T[(size_t)p * w2 + c] == 0) ++p;
        if (p == e) return false;
        if (p != c) std::swap_ranges(&T[(size_t)p * w2], &T[(size_t)p * w2] + w2, &T[(size_t)c * w2]);
        uint8_t* rc = &T[(size_t)c * w2];
        uint8_t iv = 0;
        f.inv(rc[c], &iv);
        if (iv != 1) {
            for (size_t j = 0; j < w2; ++j) rc[j] = f.mul(iv, rc[j]);
        }
        for (uint32_t i = 0; i < e; ++i) {
            const uint8_t a = T[(size_t)i * w2 + c];
            if (i != c && a) row_axpy(&T[(size_t)i * w2], rc, a, w2);
        }
    }
    W.assign((size_t)e * ep, 0);
    for (uint32_t i = 0; i < e; ++i) memcpy(&W[(size_t)i * ep], &T[(size_t)i * w2 + ep], e);
    return true;
}

// hipFuncSetAttribute for the sequence kernel's 160 KB of LDS, once per
// device (the attribute is per device; a failure is remembered and returned)
static hipError_t seq_lds_attribute() {
    static std::mutex mu;
    static hipError_t state[64];
    static bool set[64] = {};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(mu);
    if (!set[dev]) {
        state[dev] = hipFuncSetAttribute(reinterpret_cast<const void*>(k_w8_sequence),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        set[dev] = true;
    }
    return state[dev];
}

hipError_t launch_rows(const RowsArgs& a, uint32_t rows, hipStream_t st) {
    const size_t lds = a.scale ? 0 : (size_t)a.n;
    hipLaunchKernelGGL(k_w8_rows, dim3(rows, (a.words + 63) / 64), dim3(256), lds, st, a);
    return hipGetLastError();
}

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
    const uint32_t* tab = ctx_tab256(ctx);
    // workspace: A, E, slot, M, P0, P1, G, poly, info
    const size_t oA = 0, oE = oA + (size_t)e * kp, oS = oE + r16(2 * e), oM = oS + r16(4 * k);
    const size_t oP0 = oM + (size_t)e * ep, oP1 = oP0 + (size_t)e * ep, oG = oP1 + (size_t)e * ep;
    const size_t oPoly = oG + (size_t)e * kp, oInfo = oPoly + r16(2 * e + 2), oLM = oInfo + 16;
    // baby-step / giant-step Krylov from e = 64 (below, the squarings cost
    // more than the steps they save): s = 2^ceil(log2 sqrt(2e)) <= 64
    uint32_t sb = 1;
    if (e >= kBsgsMinE)
        while (sb < 64 && (uint64_t)sb * sb < 2ull * e) sb *= 2;
    const size_t oMT = oLM + 2 * (size_t)e * ep, oX0 = oMT + (size_t)e * ep, oX1 = oX0 + (size_t)e * ep;
    const size_t oLMs = oX1 + (size_t)e * ep, oV = oLMs + 2 * (size_t)e * ep;
    const size_t bsgs_end = sb > 1 ? oV + r16(sb * ep) : oMT;
    // Paterson-Stockmeyer for W (degree L <= e): powers M^0..M^(s-1) plus a
    // product slot, M^s, and the block coefficients
    uint32_t ps_max = 0;
    if (e >= kPsMinE && e <= kPsMaxE)
        while ((uint64_t)ps_max * ps_max < e) ++ps_max;
    const size_t mat = (size_t)e * ep;
    const size_t oPw = bsgs_end, oMs = oPw + (ps_max + 1) * mat, oPc = oMs + mat;
    const size_t total = ps_max ? oPc + r16(e * (ps_max + 1)) : bsgs_end;
    uint8_t* w = nullptr;
    if (int s = ctx_work(ctx, total, &w)) return s;
    std::vector<uint8_t> hA((size_t)e * kp, 0);
    for (uint32_t p = 0; p < e; ++p) memcpy(&hA[(size_t)p * kp], A_ek + (size_t)p * k, k);
    QF_CHECK_HIP(hipMemcpyAsync(w + oA, hA.data(), hA.size(), hipMemcpyHostToDevice, st));
    QF_CHECK_HIP(hipMemcpyAsync(w + oE, E, (size_t)e * 2, hipMemcpyHostToDevice, st));
    QF_CHECK_HIP(hipMemcpyAsync(w + oS, slot, (size_t)k * 4, hipMemcpyHostToDevice, st));
    int32_t* info = reinterpret_cast<int32_t*>(w + oInfo);
    size_t seq_lds = kEx2 + 512 + 64 + kRed2Bytes + 4 * (size_t)e + 2 * (size_t)e + 2 * (size_t)e + 3 * (2 * (size_t)e + 1);
    const uint32_t lm_lds = seq_lds + 2 * (size_t)e * e <= 144 * 1024;   // logs of M in LDS up to e = 262
    if (lm_lds) seq_lds += 2 * (size_t)e * e;
    if (seq_lds > 64 * 1024) QF_CHECK_HIP(seq_lds_attribute());
    // about 8 threads per row of M for the Krylov products (1 wave at e <= 8)
    const uint32_t seq_threads = std::min<uint32_t>(kSeqThreads, (8 * e + 63) / 64 * 64);
    const auto& f = gf();
    uint8_t* W = nullptr;
    const uint32_t ew = (e + 3) / 4;
    SeqArgs sa{w + oA, reinterpret_cast<const uint16_t*>(w + oE), w + oM, w + oP0,
               reinterpret_cast<uint16_t*>(w + oLM), w + oPoly, info, e, ep, kp, 0, 0, lm_lds};
    sa.s = sb;
    if (sb > 1) {
        // M^T (gather pass), then (M^T)^s by squaring: out[i] = sum_l X[i][l] X[l]
        sa.MT = w + oMT;
        sa.gather_only = 1;
        hipLaunchKernelGGL(k_w8_sequence, dim3(1), dim3(seq_threads), seq_lds, st, sa);
        QF_CHECK_HIP(hipGetLastError());
        uint8_t* X = w + oMT;
        uint8_t* bufs[2] = {w + oX0, w + oX1};
        for (uint32_t p = 1, q = 0; p < sb; p *= 2, q ^= 1) {
            RowsArgs sq{X, X, bufs[q], tab, ep, ep, ep, e, ew, 0, 0, nullptr};
            QF_CHECK_HIP(launch_rows(sq, e, st));
            X = bufs[q];
        }
        sa.gather_only = 0;
        sa.MsT = X;
        sa.LMs = reinterpret_cast<uint16_t*>(w + oLMs);
        sa.V = w + oV;
    }
    const bool random_proj = ctx_opt(ctx, QF_OPT_WIEDEMANN_PROJ) != 0;
    for (uint32_t b = 0; b < kTries; ++b) {
        if (tries_out) *tries_out = b + 1;
        sa.b = b;
        sa.seed = random_proj && b > 0 ? projection_seed() : 0;
        hipLaunchKernelGGL(k_w8_sequence, dim3(1), dim3(seq_threads), seq_lds, st, sa);
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
        uint8_t* Pin = w + oP0;
        uint8_t* Pout = w + oP1;
        std::vector<uint8_t> pc;
        if (ps_max && Ld >= kPsMinE) {
            // P = sum_{m < L} f_(m+1) M^m = sum_q (M^s)^q B_q, B_q = sum_{j < s} f_(qs+j+1) M^j, by
            // Horner in M^s: s + 2 L / s matrix launches instead of L
            uint32_t sp = 1;
            while (sp * sp < Ld) ++sp;
            const uint32_t Q = (Ld + sp - 1) / sp;
            uint8_t* Pw = w + oPw;
            QF_CHECK_HIP(hipMemcpyAsync(Pw, w + oP0, mat, hipMemcpyDeviceToDevice, st));   // M^0 = I
            QF_CHECK_HIP(hipMemcpyAsync(Pw + mat, w + oM, mat, hipMemcpyDeviceToDevice, st));
            for (uint32_t j = 2; j <= sp; ++j) {   // M^j = M^(j-1) M; j = sp lands in Ms
                RowsArgs pw{Pw + (j - 1) * mat, w + oM, j < sp ? Pw + j * mat : w + oMs, tab, ep, ep, ep, e, ew, 0, 0,
                            nullptr};
                QF_CHECK_HIP(launch_rows(pw, e, st));
            }
            if (sp == 1) QF_CHECK_HIP(hipMemcpyAsync(w + oMs, w + oM, mat, hipMemcpyDeviceToDevice, st));
            // coefficient rows: q -> f_(qs+j+1) for j < s, then 1 for the product slot
            pc.assign((size_t)Q * (sp + 1), 0);
            for (uint32_t q = 0; q < Q; ++q) {
                for (uint32_t j = 0; j < sp && q * sp + j < Ld; ++j) pc[(size_t)q * (sp + 1) + j] = poly[q * sp + j + 1];
                pc[(size_t)q * (sp + 1) + sp] = q + 1 < Q ? 1 : 0;
            }
            QF_CHECK_HIP(hipMemcpyAsync(w + oPc, pc.data(), pc.size(), hipMemcpyHostToDevice, st));
            // flattened matrices: one output row of e*ep bytes = sum of the s + 1 slots
            const uint32_t mw = (uint32_t)(mat / 4);
            for (uint32_t q = Q; q-- > 0;) {
                if (q + 1 < Q) {   // product slot = P M^s
                    RowsArgs pr{Pin, w + oMs, Pw + (size_t)sp * mat, tab, ep, ep, ep, e, ew, 0, 0, nullptr};
                    QF_CHECK_HIP(launch_rows(pr, e, st));
                }
                RowsArgs bq{w + oPc + (size_t)q * (sp + 1), Pw, Pout, tab, 0, mat, 0, sp + 1, mw, 0, 0, nullptr};
                QF_CHECK_HIP(launch_rows(bq, 1, st));
                std::swap(Pin, Pout);
            }
        } else {
            // Horner from P = I (f_L = 1): P <- P M ^ f_i I for i = L-1..1
            for (uint32_t i = Ld - 1; i >= 1; --i) {
                RowsArgs h{Pin, w + oM, Pout, tab, ep, ep, ep, e, ew, poly[i], 0, nullptr};
                QF_CHECK_HIP(launch_rows(h, e, st));
                std::swap(Pin, Pout);
            }
        }
        // W = f_0^-1 P
        RowsArgs sc{nullptr, Pin, Pout, tab, 0, ep, ep, e, ew, 0, f0inv, nullptr};
        QF_CHECK_HIP(launch_rows(sc, e, st));
        W = Pout;
        QF_CHECK_HIP(hipMemsetAsync(info + 2, 0, 4, st));
        RowsArgs vf{w + oM, W, nullptr, tab, ep, ep, 0, e, ew, 0, 0, info + 2};
        QF_CHECK_HIP(launch_rows(vf, e, st));
        int32_t bad = 0;
        QF_CHECK_HIP(hipMemcpyAsync(&bad, info + 2, 4, hipMemcpyDeviceToHost, st));
        QF_CHECK_HIP(hipStreamSynchronize(st));
        if (!bad) break;
        W = nullptr;
    }
    std::vector<uint8_t> hW;
    if (!W) {
        // no projection verified: exact elimination decides (tries = kTries + 1)
        if (tries_out) *tries_out = kTries + 1;
        if (!exact_inverse(A_ek, k, E, e, ep, hW)) return QF_ERANK;
        W = w + oP1;
        QF_CHECK_HIP(hipMemcpyAsync(W, hW.data(), hW.size(), hipMemcpyHostToDevice, st));
        QF_CHECK_HIP(hipStreamSynchronize(st));   // (hW is pageable and local)
    }
    // G = W A_J (e x k), then the payload pass
    RowsArgs g{W, w + oA, w + oG, tab, ep, kp, kp, e, (k + 3) / 4, 0, 0, nullptr};
    QF_CHECK_HIP(launch_rows(g, e, st));
    QF_CHECK_HIP(hipMemsetAsync(d_rec, 0, (size_t)e * stride, st));
    const uint32_t Lu = (L + 15) / 16;
    if (Lu) {
        ApplyArgs ap{d_rows, w + oG, W, reinterpret_cast<const uint32_t*>(w + oS), tab, d_rec, stride, e, k, kp, ep, Lu};
        dim3 grid((Lu + 63) / 64, (e + kApplyOut - 1) / kApplyOut, (k + kApplySlots - 1) / kApplySlots);
        hipLaunchKernelGGL(k_w8_apply, grid, dim3(256), 0, st, ap);
        QF_CHECK_HIP(hipGetLastError());
    }
    return QF_OK;
}

}  // namespace qf
