// qf_gf16_fft.hip -- GF(2^16) Cauchy encode for k = 2^a by the additive FFT
// (Extreme mode's windows, k = 1,024 .. 4,096 in
// adaptive.rs:131, and every other power-of-two k without a bit-sliced kernel).
//
// Encoder16 (decoder.rs:10-88) forms repair j as sum_i C[j][i] x_i with
// C[j][i] = gf16_inv(i ^ (k + j)) (decoder.rs:77-80): k r products per symbol
// column, 1,048,576 for a 1,024-source window with 1,024 repairs.  For
// k = 2^a the source points V = {0 .. k-1} are a GF(2)-subspace of GF(2^16)
// and the repair points k + j (first + r <= k) lie on its coset k + V, so (the
// algebra of lch_fft.py, which does the same for GF(2^8)):
//     p_j = kappa f(k + j),  kappa = Delta / P_V(k),
// f the degree < k polynomial interpolating the sources over V.  f comes from
// an inverse Lin-Chung-Han transform over V (a layers of k/2 butterflies), is
// folded onto the R-point coset k + V_b (R = 2^b >= first + r) with the
// factors prod_{q in [b, a), bit q of i} xhat(q, k) and kappa, and evaluated
// there by a forward transform (b layers of R/2 butterflies): about
// (a k / 2 + k + b R / 2) products per column, 11,264 instead of 1,048,576
// for k = r = 1,024.
//
// Every constant derives from W_q(2^m), W_q the subspace polynomial of
// {0 .. 2^q - 1} (GF(2)-linear in t):
//     W_0(t) = t,  W_{q+1}(t) = W_q(t) (W_q(t) + W_q(2^q)),
//     xhat(q, t) = W_q(t) / W_q(2^q),  Delta = prod_{q<a} W_q(2^q),  P_V(k) = W_a(k),
// a 16 x 16 table the host builds with ~250 products and passes by value;
// k_fft16_consts turns it into the log-form butterfly constants.  The numpy
// restatement in tests/test_gf16_fft_cpu.py runs the same schedule against the
// oracle.
//
// Layout (k_fft16): one 1,024-thread workgroup per CU, persistent over the
// (generation, strip of S symbol columns) items.  The k x S strip sits in LDS
// as logs beside a 128 KiB Zech table, so a butterfly is two LDS lookups and a
// log sum; two layers per pass (radix 4) on column pairs, one barrier per
// pass.  The same kernel computes the decode's syndromes (syn) and its solve
// x_E = C[J,E]^-1 s (solve), both through this transform.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "qf_fec.h"
#include "qf_internal.h"

namespace {

constexpr uint32_t kNoLog16 = 0xFFFF;   // log of 0 (no product)
constexpr uint32_t kOrd16 = 65535;
constexpr uint32_t kFftThreads = 1024;
constexpr uint32_t kFftLdsSymbols = 8192;    // 16 KiB strips beside the 128 KiB Zech table
constexpr uint32_t kFftLdsConsts = 8192;     // and 16 KiB of butterfly constants (k <= 2,048)
constexpr uint32_t kFftMinK = 16;

#define QF_HIP(x) QF_CHECK_HIP(x)

struct Fft16Table {
    uint16_t W[16][16];   // W[q][m] = W_q(2^m), q <= a
    uint16_t xk[16];      // xhat(q, k), q < a
    uint16_t kappa;
};

struct Fft16ConstArgs {
    Fft16Table t;
    uint16_t* out;        // [k - 1 inverse][k fold][R - 1 forward], logs (normal: field elements)
    const uint16_t* glog;
    const uint16_t* gexp;
    uint32_t k, a, R, b;
    uint32_t normal;      // 1: the elements themselves (k_fft16_bs), 0: their logs (k_fft16)
};

struct Fft16Args {
    const uint8_t* src;
    uint64_t sgs, srs;
    uint8_t* rep;
    uint64_t rgs, rrs;
    const uint16_t* cst;  // k_fft16_consts output
    const uint16_t* glog;
    const uint16_t* gexp;
    const uint16_t* zech;   // Z[d] = log(1 + alpha^d), 65,536 entries
    uint32_t k, a, R, b, r, first, rot, nsym, S, lgS, strips;
    // decode syndromes (syn != 0; qf_gf16.hip k_dec16_bsmaps): src = the
    // received rows, source i at slot smap[g k + i] (0xFFFF: erased, reads
    // zero); output row rpos[g r + t] (0xFFFF: none) = coset value t XOR the
    // accepted row of repair k + t (slot rslot[g r + t]); skip[g]: not ours
    const uint16_t* smap;
    const uint16_t* rpos;
    const uint16_t* rslot;
    const uint32_t* skip;
    uint32_t syn;
    // decode solve (solve != 0): src = the syndrome rows s_a (a < e_g), placed
    // times D_a = Qx_a / Px_a at source position j_a = J_a - k; output row b
    // (b < e_g) = D_b' out[E_b], D_b' = Qy_b / Py_b (logs in lprod, the closed
    // form of k_dec16_cauchy_prod); skipped: status != 0, e_g == 0, solve_fb[g]
    const uint32_t* st_e;    // e_g at st_e[g * st_stride]
    uint32_t st_stride;
    const int32_t* status;
    const uint16_t* J;
    const uint16_t* E;
    const uint32_t* lprod;   // [g][4 em]: log Qx, log Px, log Qy, log Py
    uint64_t em;
    const uint32_t* solve_fb;
    uint32_t solve;
    uint32_t r4;             // k_fft16_bs: two layers per LDS pass (QF_OPT_GF16_FFT_BS 3), else one
};

__device__ __forceinline__ uint32_t wq_at(const Fft16Table& t, uint32_t q, uint32_t x) {
    uint32_t v = 0;
    for (uint32_t m = 0; x; ++m, x >>= 1)
        if (x & 1) v ^= t.W[q][m];
    return v;
}

__device__ __forceinline__ uint32_t lg_of(const uint16_t* glog, uint32_t v) { return v ? glog[v] : kNoLog16; }

__device__ __forceinline__ uint32_t lg_mul(uint32_t la, uint32_t lb) {
    if (la == kNoLog16 || lb == kNoLog16) return kNoLog16;
    const uint32_t s = la + lb;
    return s >= kOrd16 ? s - kOrd16 : s;
}

// log xhat(q, x) = log W_q(x) - log W_q(2^q)
__device__ __forceinline__ uint32_t lg_xhat(const Fft16ConstArgs& a, uint32_t q, uint32_t x) {
    const uint32_t lw = lg_of(a.glog, wq_at(a.t, q, x));
    if (lw == kNoLog16) return kNoLog16;
    const uint32_t ld = a.glog[a.t.W[q][q]];
    return lw >= ld ? lw - ld : lw + kOrd16 - ld;
}

__global__ void __launch_bounds__(256) k_fft16_consts(Fft16ConstArgs a) {
    const uint32_t n_inv = a.k - 1, n_all = n_inv + a.k + a.R - 1;
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n_all; e += gridDim.x * blockDim.x) {
        uint32_t v;
        if (e < n_inv) {             // inverse layer q: k >> (q + 1) blocks at k - (k >> q)
            uint32_t q = 0;
            while (e >= a.k - (a.k >> (q + 1))) ++q;
            const uint32_t blk = e - (a.k - (a.k >> q));
            v = lg_xhat(a, q, blk << (q + 1));
        } else if (e < n_inv + a.k) {   // fold x kappa of source i
            const uint32_t i = e - n_inv;
            v = a.glog[a.t.kappa];
            for (uint32_t q = a.b; q < a.a; ++q)
                if (i >> q & 1) v = lg_mul(v, a.glog[a.t.xk[q]]);
        } else {                     // forward layer q: R >> (q + 1) blocks at R - (R >> q)
            const uint32_t f = e - n_inv - a.k;
            uint32_t q = 0;
            while (f >= a.R - (a.R >> (q + 1))) ++q;
            const uint32_t blk = f - (a.R - (a.R >> q));
            v = lg_xhat(a, q, a.k ^ (blk << (q + 1)));
        }
        a.out[e] = (uint16_t)(a.normal ? (v == kNoLog16 ? 0u : (uint32_t)a.gexp[v]) : v);
    }
}

// bytes b0 b1 b2 b3 of two big-endian symbols <-> (b0 b1) | (b2 b3) << 16
__device__ __forceinline__ uint32_t bswap_sym2(uint32_t w) { return __builtin_amdgcn_perm(w, w, 0x02030001u); }

// log-domain arithmetic (kNoLog16 = log 0): products add logs, sums go
// through the Zech table Z[d] = log(1 + alpha^d) (Z[0] = log 0), in LDS
__device__ __forceinline__ uint32_t lmul(uint32_t a, uint32_t b) {
    uint32_t s = a + b;
    s = s >= kOrd16 ? s - kOrd16 : s;
    return (a == kNoLog16 || b == kNoLog16) ? kNoLog16 : s;
}

__device__ __forceinline__ uint32_t ladd(const uint16_t* Z, uint32_t a, uint32_t b) {
    // alpha^a + alpha^b = alpha^a (1 + alpha^(b - a)); both indices stay < 65,536
    uint32_t d = b + kOrd16 - a;
    d = d >= kOrd16 ? d - kOrd16 : d;
    const uint32_t z = Z[d];
    uint32_t s = a + z;
    s = s >= kOrd16 ? s - kOrd16 : s;
    s = z == kNoLog16 ? kNoLog16 : s;
    s = a == kNoLog16 ? b : s;
    return b == kNoLog16 ? a : s;
}

// two logs per dword (column pairs); both Zech lookups issued together
__device__ __forceinline__ uint32_t ladd2(const uint16_t* Z, uint32_t a, uint32_t b) {
    const uint32_t a0 = a & 0xFFFF, a1 = a >> 16, b0 = b & 0xFFFF, b1 = b >> 16;
    uint32_t d0 = b0 + kOrd16 - a0, d1 = b1 + kOrd16 - a1;
    d0 = d0 >= kOrd16 ? d0 - kOrd16 : d0;
    d1 = d1 >= kOrd16 ? d1 - kOrd16 : d1;
    const uint32_t z0 = Z[d0], z1 = Z[d1];
    auto fin = [](uint32_t x, uint32_t y, uint32_t z) {
        uint32_t t = x + z;
        t = t >= kOrd16 ? t - kOrd16 : t;
        t = z == kNoLog16 ? kNoLog16 : t;
        t = x == kNoLog16 ? y : t;
        return y == kNoLog16 ? x : t;
    };
    return fin(a0, b0, z0) | (fin(a1, b1, z1) << 16);
}

__device__ __forceinline__ uint32_t lmul2(uint32_t s, uint32_t y) {
    return lmul(s, y & 0xFFFF) | (lmul(s, y >> 16) << 16);
}

// inverse butterfly y_j += y_i; y_i += s y_j / forward d_i += s d_j; d_j += d_i
__device__ __forceinline__ void ibfly(const uint16_t* Z, uint32_t& yi, uint32_t& yj, uint32_t s) {
    yj = ladd2(Z, yj, yi);
    yi = ladd2(Z, yi, lmul2(s, yj));
}

__device__ __forceinline__ void fbfly(const uint16_t* Z, uint32_t& di, uint32_t& dj, uint32_t s) {
    di = ladd2(Z, di, lmul2(s, dj));
    dj = ladd2(Z, dj, di);
}

// Four independent log sums a[u] += b[u] with the four Zech lookups issued
// together (one LDS round trip instead of four)
__device__ __forceinline__ uint32_t zidx(uint32_t a, uint32_t b) {
    const uint32_t d = b + kOrd16 - a;
    return d >= kOrd16 ? d - kOrd16 : d;
}

__device__ __forceinline__ uint32_t zfin(uint32_t a, uint32_t b, uint32_t z) {
    uint32_t s = a + z;
    s = s >= kOrd16 ? s - kOrd16 : s;
    s = z == kNoLog16 ? kNoLog16 : s;
    s = a == kNoLog16 ? b : s;
    return b == kNoLog16 ? a : s;
}

__device__ __forceinline__ void ladd_x4(const uint16_t* Z, uint32_t (&a)[4], const uint32_t (&b)[4]) {
    uint32_t z[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) z[u] = Z[zidx(a[u], b[u])];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = zfin(a[u], b[u], z[u]);
}

// Two butterflies on column pairs in lockstep: (p, q) with constant sp and
// (r, t) with constant sr.  Inverse: q += p; p += s q.  Forward: p += s q; q += p.
__device__ __forceinline__ void ibfly_x2(const uint16_t* Z, uint32_t& p, uint32_t& q, uint32_t sp, uint32_t& r,
                                         uint32_t& t, uint32_t sr) {
    uint32_t x[4] = {q & 0xFFFF, q >> 16, t & 0xFFFF, t >> 16};
    const uint32_t y[4] = {p & 0xFFFF, p >> 16, r & 0xFFFF, r >> 16};
    ladd_x4(Z, x, y);
    uint32_t w[4] = {y[0], y[1], y[2], y[3]};
    const uint32_t m[4] = {lmul(sp, x[0]), lmul(sp, x[1]), lmul(sr, x[2]), lmul(sr, x[3])};
    ladd_x4(Z, w, m);
    p = w[0] | (w[1] << 16);
    r = w[2] | (w[3] << 16);
    q = x[0] | (x[1] << 16);
    t = x[2] | (x[3] << 16);
}

__device__ __forceinline__ void fbfly_x2(const uint16_t* Z, uint32_t& p, uint32_t& q, uint32_t sp, uint32_t& r,
                                         uint32_t& t, uint32_t sr) {
    uint32_t w[4] = {p & 0xFFFF, p >> 16, r & 0xFFFF, r >> 16};
    const uint32_t qv[4] = {q & 0xFFFF, q >> 16, t & 0xFFFF, t >> 16};
    const uint32_t m[4] = {lmul(sp, qv[0]), lmul(sp, qv[1]), lmul(sr, qv[2]), lmul(sr, qv[3])};
    ladd_x4(Z, w, m);
    uint32_t x[4] = {qv[0], qv[1], qv[2], qv[3]};
    ladd_x4(Z, x, w);
    p = w[0] | (w[1] << 16);
    r = w[2] | (w[3] << 16);
    q = x[0] | (x[1] << 16);
    t = x[2] | (x[3] << 16);
}

// One workgroup per CU (the Zech table fills 128 KiB of LDS, the strip the
// other 32 KiB), persistent over the (generation, strip) items.  The strip is
// held as logs: a butterfly is two Zech lookups and a log sum, and only the
// strip's load and store touch the global log / exp tables.
// LC: the constants of every layer in LDS (k <= 2,048), else read from global
// memory; a template so that every access has a known address space (a
// pointer that may be either compiles to flat loads, and those make the
// compiler wait for all LDS and global traffic after each Zech lookup)
template <bool LC>
__global__ void __launch_bounds__(kFftThreads) k_fft16(Fft16Args A, uint32_t G) {
    __shared__ uint16_t sz[65536];
    __shared__ uint16_t buf[kFftLdsSymbols];
    __shared__ uint16_t scst[kFftLdsConsts];
    const uint32_t S = A.S, lgS = A.lgS, k = A.k, tid = threadIdx.x;
    const uint16_t* __restrict__ glog = A.glog;
    const uint16_t* __restrict__ gexp = A.gexp;
    {
        const uint4* gz = reinterpret_cast<const uint4*>(A.zech);
        uint4* lz = reinterpret_cast<uint4*>(sz);
        for (uint32_t w = tid; w < 65536 / 8; w += kFftThreads) lz[w] = gz[w];
    }
    // the butterfly constants of every layer, once per workgroup, when they fit
    const uint32_t n_cst = 2 * k + A.R - 2;
    if (LC)
        for (uint32_t e = tid; e < n_cst; e += kFftThreads) scst[e] = A.cst[e];
    const uint16_t* cst = LC ? scst : A.cst;
    const uint16_t* cinv = cst;
    const uint16_t* cfk = cst + (k - 1);
    const uint16_t* cfwd = cfk + k;
    const uint64_t items = (uint64_t)G * A.strips;
    for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const uint64_t g = it / A.strips;
        const uint32_t c0 = (uint32_t)(it - g * A.strips) << lgS;
        const uint32_t ncol = min(S, A.nsym - c0);
        __syncthreads();   // the table (first item) / the previous item's stores
        if (A.syn && A.skip[g]) continue;   // uniform over the block
        const uint8_t* gsrc = A.src + g * A.sgs;
        const uint16_t* smap = A.syn ? A.smap + g * k : nullptr;
        uint32_t e_g = 0;
        const uint16_t *gJ = nullptr, *gE = nullptr;
        const uint32_t* lp = nullptr;
        if (A.solve) {
            if (A.status[g] != 0 || A.solve_fb[g] != 0) continue;
            e_g = A.st_e[g * A.st_stride];
            if (e_g == 0) continue;
            gJ = A.J + g * A.em;
            gE = A.E + g * A.em;
            lp = A.lprod + g * 4 * A.em;
            // every source position starts at zero; the e_g scaled syndromes go to theirs
            for (uint32_t p = tid; p < (k << lgS); p += kFftThreads) buf[p] = (uint16_t)kNoLog16;
            __syncthreads();
            for (uint32_t p = tid; p < (e_g << lgS); p += kFftThreads) {
                const uint32_t a = p >> lgS, c = p & (S - 1);
                if (c >= ncol) continue;
                const uint8_t* row = gsrc + (uint64_t)a * A.srs + 2ull * (c0 + c);
                uint32_t da = lp[a] + kOrd16 - lp[A.em + a];
                da = da >= kOrd16 ? da - kOrd16 : da;
                buf[(((uint32_t)gJ[a] - k) << lgS) + c] =
                    (uint16_t)lmul(da, glog[((uint32_t)row[0] << 8) | row[1]]);
            }
        }
        // strip in, as logs: window position i reads ring slot (rot + i) mod k
        // (decode: slot smap[i], none = zero); big-endian symbols, two per
        // dword (S >= 2 column pairs; the rows are 16-byte aligned)
        if (!A.solve) {
            const uint32_t lgP = lgS - 1;
            for (uint32_t p = tid; p < (k << lgP); p += kFftThreads) {
                const uint32_t i = p >> lgP, c = (p & ((S >> 1) - 1)) << 1;
                const uint32_t slot = smap ? smap[i] : ((A.rot + i) & (k - 1));
                const uint8_t* row = gsrc + (uint64_t)slot * A.srs + 2ull * (c0 + c);
                uint32_t v = 0;
                if (smap && slot == 0xFFFFu)
                    v = 0;
                else if (c + 1 < ncol)
                    v = bswap_sym2(*reinterpret_cast<const uint32_t*>(row));
                else if (c < ncol)
                    v = ((uint32_t)row[0] << 8) | row[1];
                reinterpret_cast<uint32_t*>(buf)[p] = (uint32_t)glog[v & 0xFFFF] | ((uint32_t)glog[v >> 16] << 16);
            }
        }
        __syncthreads();
        // inverse transform over V (y_j += y_i; y_i += s y_j), two layers per
        // pass (radix 4: four rows, three constants, one barrier) on column
        // pairs (one dword of two logs per LDS access)
        uint32_t* b32 = reinterpret_cast<uint32_t*>(buf);
        const uint32_t lgP = lgS - 1, P = S >> 1;
        // (radix 2 throughout when a radix-4 pass would leave threads idle: G = 1)
        const bool r4 = ((k >> 2) << lgP) >= kFftThreads;
        uint32_t q = 0;
        for (; r4 && q + 1 < A.a; q += 2) {
            const uint32_t h = 1u << q;
            const uint16_t* c0 = cinv + (k - (k >> q));
            const uint16_t* c1 = cinv + (k - (k >> (q + 1)));
            for (uint32_t p = tid; p < ((k >> 2) << lgP); p += kFftThreads) {
                const uint32_t cp = p & (P - 1), qi = p >> lgP, B = qi >> q;
                uint32_t* w = b32 + ((((B << (q + 2)) + (qi & (h - 1))) << lgP) + cp);
                const uint32_t st = h << lgP;
                uint32_t y0 = w[0], y1 = w[st], y2 = w[2 * st], y3 = w[3 * st];
                ibfly_x2(sz, y0, y1, c0[2 * B], y2, y3, c0[2 * B + 1]);
                const uint32_t s1 = c1[B];
                ibfly_x2(sz, y0, y2, s1, y1, y3, s1);
                w[0] = y0;
                w[st] = y1;
                w[2 * st] = y2;
                w[3 * st] = y3;
            }
            __syncthreads();
        }
        for (; q < A.a; ++q) {   // the rest (an odd layer count: the last layer alone)
            const uint32_t h = 1u << q;
            const uint16_t* c0 = cinv + (k - (k >> q));
            for (uint32_t p = tid; p < ((k >> 1) << lgP); p += kFftThreads) {
                const uint32_t cp = p & (P - 1), bi = p >> lgP, blk = bi >> q;
                uint32_t* w = b32 + ((((blk << (q + 1)) | (bi & (h - 1))) << lgP) + cp);
                const uint32_t st = h << lgP;
                uint32_t y0 = w[0], y1 = w[st];
                ibfly(sz, y0, y1, c0[blk]);
                w[0] = y0;
                w[st] = y1;
            }
            __syncthreads();
        }
        // fold onto the R-point coset, times kappa (in place: row t < R is
        // written only by the thread that reads every row i = t mod R)
        for (uint32_t p = tid; p < (A.R << lgP); p += kFftThreads) {
            const uint32_t t = p >> lgP, cp = p & (P - 1);
            uint32_t acc = kNoLog16 | (kNoLog16 << 16);
            for (uint32_t i = t; i < k; i += A.R) acc = ladd2(sz, acc, lmul2(cfk[i], b32[(i << lgP) + cp]));
            b32[p] = acc;
        }
        __syncthreads();
        // forward transform over k + V_b (d_i += s d_j; d_j += d_i), layers
        // b-1 .. 0, two per pass as above
        int qq = (int)A.b - 1;
        for (; ((A.R >> 2) << lgP) >= kFftThreads && qq >= 1; qq -= 2) {
            const uint32_t ql = (uint32_t)qq - 1, h = 1u << ql;
            const uint16_t* c0 = cfwd + (A.R - (A.R >> ql));
            const uint16_t* c1 = cfwd + (A.R - (A.R >> (ql + 1)));
            for (uint32_t p = tid; p < ((A.R >> 2) << lgP); p += kFftThreads) {
                const uint32_t cp = p & (P - 1), qi = p >> lgP, B = qi >> ql;
                uint32_t* w = b32 + ((((B << (ql + 2)) + (qi & (h - 1))) << lgP) + cp);
                const uint32_t st = h << lgP;
                uint32_t d0 = w[0], d1 = w[st], d2 = w[2 * st], d3 = w[3 * st];
                const uint32_t s1 = c1[B];
                fbfly_x2(sz, d0, d2, s1, d1, d3, s1);
                fbfly_x2(sz, d0, d1, c0[2 * B], d2, d3, c0[2 * B + 1]);
                w[0] = d0;
                w[st] = d1;
                w[2 * st] = d2;
                w[3 * st] = d3;
            }
            __syncthreads();
        }
        for (; qq >= 0; --qq) {   // the rest, one layer per pass
            const uint32_t ql = (uint32_t)qq, h = 1u << ql;
            const uint16_t* c0 = cfwd + (A.R - (A.R >> ql));
            for (uint32_t p = tid; p < ((A.R >> 1) << lgP); p += kFftThreads) {
                const uint32_t cp = p & (P - 1), bi = p >> lgP, blk = bi >> ql;
                uint32_t* w = b32 + ((((blk << (ql + 1)) | (bi & (h - 1))) << lgP) + cp);
                const uint32_t st = h << lgP;
                uint32_t d0 = w[0], d1 = w[st];
                fbfly(sz, d0, d1, c0[blk]);
                w[0] = d0;
                w[st] = d1;
            }
            __syncthreads();
        }
        if (A.solve) {   // recovered row b = D_b' out[E_b]
            for (uint32_t p = tid; p < (e_g << lgS); p += kFftThreads) {
                const uint32_t bb = p >> lgS, c = p & (S - 1);
                if (c >= ncol) continue;
                uint32_t db = lp[2 * A.em + bb] + kOrd16 - lp[3 * A.em + bb];
                db = db >= kOrd16 ? db - kOrd16 : db;
                const uint32_t l = lmul(db, buf[((uint32_t)gE[bb] << lgS) + c]);
                const uint32_t v = l == kNoLog16 ? 0u : (uint32_t)gexp[l];
                uint8_t* o = A.rep + g * A.rgs + (uint64_t)bb * A.rrs + 2ull * (c0 + c);
                o[0] = (uint8_t)(v >> 8);
                o[1] = (uint8_t)v;
            }
            continue;
        }
        // repairs first .. first + r - 1 = coset points t = first + jj (decode:
        // the syndrome of the accepted repair k + jj, its received row XORed in)
        const uint16_t* rpos = A.syn ? A.rpos + g * A.r : nullptr;
        const uint16_t* rslot = A.syn ? A.rslot + g * A.r : nullptr;
        {
            const uint32_t lgP = lgS - 1;
            for (uint32_t p = tid; p < (A.r << lgP); p += kFftThreads) {
                const uint32_t jj = p >> lgP, c = (p & ((S >> 1) - 1)) << 1;
                if (c >= ncol) continue;
                const uint32_t lv = reinterpret_cast<const uint32_t*>(buf)[(((A.first + jj) << lgS) + c) >> 1];
                const uint32_t l0 = lv & 0xFFFF, l1 = lv >> 16;
                uint32_t v = (l0 == kNoLog16 ? 0u : (uint32_t)gexp[l0]) | ((l1 == kNoLog16 ? 0u : (uint32_t)gexp[l1]) << 16);
                uint64_t orow = jj;
                const uint8_t* base = nullptr;
                if (rpos) {
                    orow = rpos[jj];
                    if (orow == 0xFFFFu) continue;
                    base = gsrc + (uint64_t)rslot[jj] * A.srs + 2ull * (c0 + c);
                }
                uint8_t* o = A.rep + g * A.rgs + orow * A.rrs + 2ull * (c0 + c);
                if (c + 1 < ncol) {
                    if (base) v ^= bswap_sym2(*reinterpret_cast<const uint32_t*>(base));
                    *reinterpret_cast<uint32_t*>(o) = bswap_sym2(v);
                } else {
                    if (base) v ^= ((uint32_t)base[0] << 8) | base[1];
                    o[0] = (uint8_t)(v >> 8);
                    o[1] = (uint8_t)v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Bit-sliced transform (k_fft16_bs, k <= 2,048): the same schedule on field
// elements in normal form, 32 symbol columns per lane as 16 bit planes (plane
// p = bit p of the 32 symbols), so a butterfly is plane XORs and one
// multiplication by its constant -- no table lookups and no dependent LDS
// round trips.  s x by Horner over the bits of s, x alpha = the planes
// shifted up with plane 15 folded into planes 0, 1, 3 and 12 (0x1100B):
// 16 x 16 masked XORs (v_bitop3) plus 45 for the shifts, ~10 VALU per symbol
// and butterfly; where the wave's butterflies share their block's constant
// (layer q >= 6 and each transform's top layer) a scalar branch per bit of s
// leaves only the set bits' XORs.  The strip lives in LDS plane-major ([16][k cg] dwords, cg
// column groups of 32 symbols), one butterfly per thread per layer.
// ---------------------------------------------------------------------------
constexpr uint32_t kBsThreads = 512;          // k <= 1,024: k / 2 x cg butterflies per layer
constexpr uint32_t kBsRows = 1024;            // strip rows (k cg) of the 512-thread kernel
constexpr uint32_t kBsConsts = 3072;          // its butterfly constants (2 k + R - 2 <= 3 k)
constexpr uint32_t kBsMaxK = 2048;            // k = 2,048: 1,024 threads, 128 KiB strip

__device__ __forceinline__ void bs_mulx(uint32_t (&x)[16]) {
    const uint32_t t = x[15];
#pragma unroll
    for (int p = 15; p > 0; --p) x[p] = x[p - 1];
    x[0] = t;
    x[1] ^= t;
    x[3] ^= t;
    x[12] ^= t;
}

// y ^= s x: Horner over the bits of s (s per lane), acc = acc alpha ^ (x & m_j)
// with m_j = bit j of s spread over the dword, one v_bitop3 per plane
__device__ __forceinline__ void bs_muladd(uint32_t (&y)[16], const uint32_t (&x)[16], uint32_t s) {
    uint32_t acc[16];
    {
        const uint32_t m = 0u - (s >> 15);
#pragma unroll
        for (int p = 0; p < 16; ++p) acc[p] = x[p] & m;
    }
#pragma unroll
    for (int j = 14; j >= 0; --j) {
        bs_mulx(acc);
        const uint32_t m = 0u - ((s >> j) & 1u);
#pragma unroll
        for (int p = 0; p < 16; ++p) acc[p] = __builtin_amdgcn_bitop3_b32(acc[p], x[p], m, 0x78);   // acc ^ (x & m)
    }
#pragma unroll
    for (int p = 0; p < 16; ++p) y[p] ^= acc[p];
}

// y ^= s x with s uniform over the wave: a scalar branch per bit of s, so only
// the set bits' 16 XORs issue (45 + 16 popcount(s) VALU against 317)
__device__ __forceinline__ void bs_muladd_uni(uint32_t (&y)[16], const uint32_t (&x)[16], uint32_t s) {
    s = __builtin_amdgcn_readfirstlane(s);
    uint32_t acc[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) acc[p] = 0;
#pragma unroll
    for (int j = 15; j >= 0; --j) {
        bs_mulx(acc);
        if (__builtin_expect((s >> j) & 1u, 0)) {
#pragma unroll
            for (int p = 0; p < 16; ++p) acc[p] ^= x[p];
        }
    }
#pragma unroll
    for (int p = 0; p < 16; ++p) y[p] ^= acc[p];
}

// uni: every active lane of the wave multiplies by the same s (one block)
__device__ __forceinline__ void bs_muladd(uint32_t (&y)[16], const uint32_t (&x)[16], uint32_t s, bool uni) {
    if (uni)
        bs_muladd_uni(y, x, s);
    else
        bs_muladd(y, x, s);
}

// 16 dwords of one row's 32 big-endian symbols <-> 16 planes.  Dword d holds
// symbols 2d (low half) and 2d + 1 (high half) after a byte swap; a 16 x 16
// bit transpose of both halves at once gives plane p: bit i = symbol 2i,
// bit 16 + i = symbol 2i + 1.  The transpose is its own inverse.
template <int W, uint32_t M>
__device__ __forceinline__ void bs_transpose_stage(uint32_t (&d)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        if (i & W) continue;
        const uint32_t t = ((d[i] >> W) ^ d[i + W]) & M;
        d[i + W] ^= t;
        d[i] ^= t << W;
    }
}

__device__ __forceinline__ void bs_transpose(uint32_t (&d)[16]) {
    bs_transpose_stage<8, 0x00FF00FFu>(d);
    bs_transpose_stage<4, 0x0F0F0F0Fu>(d);
    bs_transpose_stage<2, 0x33333333u>(d);
    bs_transpose_stage<1, 0x55555555u>(d);
}

__device__ __forceinline__ uint32_t bs_swap16x2(uint32_t w) { return __builtin_amdgcn_perm(w, w, 0x02030001u); }

// 2 n bytes (n <= 32 symbols) of a row -> planes; dword loads (rows are 4-byte aligned)
__device__ __forceinline__ void bs_load_row(const uint8_t* row, uint32_t n, uint32_t (&d)[16]) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        uint32_t v = 0;
        if (2u * q + 1 < n)
            v = *reinterpret_cast<const uint32_t*>(row + 4 * q);
        else if (2u * q < n)
            v = (uint32_t)row[4 * q] | ((uint32_t)row[4 * q + 1] << 8);
        d[q] = bs_swap16x2(v);
    }
    bs_transpose(d);
}

// planes -> 2 n bytes of a row (xr: XOR the received row's bytes in, decode syndromes)
__device__ __forceinline__ void bs_store_row(uint8_t* row, uint32_t n, uint32_t (&d)[16], const uint8_t* xr) {
    bs_transpose(d);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        uint32_t v = bs_swap16x2(d[q]);
        if (2u * q + 1 < n) {
            if (xr) v ^= *reinterpret_cast<const uint32_t*>(xr + 4 * q);
            *reinterpret_cast<uint32_t*>(row + 4 * q) = v;
        } else if (2u * q < n) {
            if (xr) v ^= (uint32_t)xr[4 * q] | ((uint32_t)xr[4 * q + 1] << 8);
            row[4 * q] = (uint8_t)v;
            row[4 * q + 1] = (uint8_t)(v >> 8);
        }
    }
}

template <int N>
__device__ __forceinline__ void bs_lds_load(const uint32_t* pl, uint32_t row, uint32_t (&y)[16]) {
#pragma unroll
    for (int p = 0; p < 16; ++p) y[p] = pl[p * N + row];
}

template <int N>
__device__ __forceinline__ void bs_lds_store(uint32_t* pl, uint32_t row, const uint32_t (&y)[16]) {
#pragma unroll
    for (int p = 0; p < 16; ++p) pl[p * N + row] = y[p];
}

// MODE 0 encode, 1 decode syndromes, 2 decode solve (as k_fft16).  BIG: k =
// 2,048 (1,024 threads, one column group); else k <= 1,024, 512 threads,
// cg = A.S column groups (k cg <= 1,024).  A.cst: the constants as elements.
template <int MODE, bool BIG>
__global__ void __launch_bounds__(BIG ? 1024 : kBsThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) k_fft16_bs(Fft16Args A, uint32_t G) {
    constexpr int NT = BIG ? 1024 : (int)kBsThreads;
    constexpr int N = BIG ? (int)kBsMaxK : (int)kBsRows;   // plane stride (rows)
    constexpr int NC = BIG ? 2 * (int)kBsMaxK + (int)kBsMaxK : (int)kBsConsts;
    __shared__ uint32_t pl[16 * N];
    __shared__ uint16_t scst[NC];
    const uint32_t k = A.k, cg = A.S, tid = threadIdx.x;
    const uint32_t lgk = A.a, hk = k >> 1;
    const uint32_t n_cst = 2 * k + A.R - 2;
    for (uint32_t e = tid; e < n_cst; e += NT) scst[e] = A.cst[e];
    const uint16_t* cinv = scst;
    const uint16_t* cfk = scst + (k - 1);
    const uint16_t* cfwd = cfk + k;
    const uint32_t rows = k * cg;   // strip rows: column group c, row i at c k + i
    // this thread's butterfly slot: column group bc, pair index bp
    const uint32_t bc = tid >> (lgk - 1), bp = tid & (hk - 1);
    const bool bact = bc < cg;
    // radix-4 slot: column group qc, quad index qu (k / 4 per group)
    const uint32_t qc = tid >> (lgk - 2), qu = tid & ((k >> 2) - 1);
    const bool qact = qc < cg;
    const uint64_t items = (uint64_t)G * A.strips;
    for (uint64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const uint64_t g = it / A.strips;
        const uint32_t col0 = (uint32_t)(it - g * A.strips) * 32u * cg;   // first symbol column
        __syncthreads();   // constants (first item) / the previous item's output reads
        if (MODE == 1 && A.skip[g]) continue;   // uniform over the block
        const uint8_t* gsrc = A.src + g * A.sgs;
        uint32_t e_g = 0;
        const uint16_t *gJ = nullptr, *gE = nullptr;
        const uint32_t* lp = nullptr;
        if (MODE == 2) {
            if (A.status[g] != 0 || A.solve_fb[g] != 0) continue;
            e_g = A.st_e[g * A.st_stride];
            if (e_g == 0) continue;
            gJ = A.J + g * A.em;
            gE = A.E + g * A.em;
            lp = A.lprod + g * 4 * A.em;
            for (uint32_t w = tid; w < 16 * (uint32_t)N; w += NT) pl[w] = 0;
            __syncthreads();
            // source position J_a - k gets D_a s_a, D_a = Qx_a / Px_a
            for (uint32_t q = tid; q < e_g * cg; q += NT) {
                const uint32_t a = q / cg, c = q - a * cg;
                const uint32_t cc = col0 + 32u * c;
                if (cc >= A.nsym) continue;
                uint32_t y[16], z[16];
                bs_load_row(gsrc + (uint64_t)a * A.srs + 2ull * cc, min(32u, A.nsym - cc), y);
                uint32_t da = lp[a] + kOrd16 - lp[A.em + a];
                da = da >= kOrd16 ? da - kOrd16 : da;
#pragma unroll
                for (int p = 0; p < 16; ++p) z[p] = 0;
                bs_muladd(z, y, A.gexp[da]);
                bs_lds_store<N>(pl, c * k + ((uint32_t)gJ[a] - k), z);
            }
        } else {
            // strip in: window position i reads ring slot (rot + i) mod k
            // (decode: slot smap[i], none = zero)
            const uint16_t* smap = MODE == 1 ? A.smap + g * k : nullptr;
            for (uint32_t q = tid; q < rows; q += NT) {
                const uint32_t c = q >> lgk, i = q & (k - 1);
                const uint32_t cc = col0 + 32u * c;
                uint32_t y[16];
                const uint32_t slot = MODE == 1 ? smap[i] : ((A.rot + i) & (k - 1));
                if (cc >= A.nsym || (MODE == 1 && slot == 0xFFFFu)) {
#pragma unroll
                    for (int p = 0; p < 16; ++p) y[p] = 0;
                } else {
                    bs_load_row(gsrc + (uint64_t)slot * A.srs + 2ull * cc, min(32u, A.nsym - cc), y);
                }
                bs_lds_store<N>(pl, q, y);
            }
        }
        __syncthreads();
        // inverse transform over V: y_j += y_i; y_i += s y_j, layer q's
        // pairs (i, i + 2^q) in blocks of 2^(q+1), constant per block.  r4:
        // layers q and q + 1 in one LDS pass, a thread's four rows i0 + {0, h,
        // 2h, 3h} (h = 2^q) in registers
        uint32_t q = 0;
        for (; !BIG && A.r4 && q + 1 < lgk; q += 2) {   // (k = 2,048: the 128-VGPR budget of 1,024 threads)
            if (qact) {
                const uint32_t h = 1u << q, B = qu >> q;
                const uint32_t i0 = qc * k + (B << (q + 2)) + (qu & (h - 1));
                const uint16_t* c0 = cinv + (k - (k >> q));
                const uint16_t* c1 = cinv + (k - (k >> (q + 1)));
                uint32_t y0[16], y1[16], y2[16], y3[16];
                bs_lds_load<N>(pl, i0, y0);
                bs_lds_load<N>(pl, i0 + h, y1);
                bs_lds_load<N>(pl, i0 + 2 * h, y2);
                bs_lds_load<N>(pl, i0 + 3 * h, y3);
#pragma unroll
                for (int p = 0; p < 16; ++p) {
                    y1[p] ^= y0[p];
                    y3[p] ^= y2[p];
                }
                const bool uni = q >= 6 || q + 2 == lgk;   // a wave's quads in one block
                bs_muladd(y0, y1, c0[2 * B], uni);
                bs_muladd(y2, y3, c0[2 * B + 1], uni);
                const uint32_t s1 = c1[B];
                // (rows stored as soon as they are final: the register budget)
#pragma unroll
                for (int p = 0; p < 16; ++p) y2[p] ^= y0[p];
                bs_muladd(y0, y2, s1, uni);
                bs_lds_store<N>(pl, i0, y0);
                bs_lds_store<N>(pl, i0 + 2 * h, y2);
#pragma unroll
                for (int p = 0; p < 16; ++p) y3[p] ^= y1[p];
                bs_muladd(y1, y3, s1, uni);
                bs_lds_store<N>(pl, i0 + h, y1);
                bs_lds_store<N>(pl, i0 + 3 * h, y3);
            }
            __syncthreads();
        }
        for (; q < lgk; ++q) {
            if (bact) {
                const uint32_t h = 1u << q, blk = bp >> q;
                const uint32_t i = bc * k + ((blk << (q + 1)) | (bp & (h - 1)));
                uint32_t yi[16], yj[16];
                bs_lds_load<N>(pl, i, yi);
                bs_lds_load<N>(pl, i + h, yj);
#pragma unroll
                for (int p = 0; p < 16; ++p) yj[p] ^= yi[p];
                bs_muladd(yi, yj, cinv[(k - (k >> q)) + blk], q >= 6 || q + 1 == lgk);
                bs_lds_store<N>(pl, i, yi);
                bs_lds_store<N>(pl, i + h, yj);
            }
            __syncthreads();
        }
        // fold onto the R-point coset, times kappa: every row times its
        // factor, then row t < R = the sum of rows t mod R
        for (uint32_t q = tid; q < rows; q += NT) {
            const uint32_t i = q & (k - 1);
            uint32_t y[16], z[16];
            bs_lds_load<N>(pl, q, y);
#pragma unroll
            for (int p = 0; p < 16; ++p) z[p] = 0;
            bs_muladd(z, y, cfk[i]);
            bs_lds_store<N>(pl, q, z);
        }
        __syncthreads();
        if (A.R < k) {
            for (uint32_t q = tid; q < A.R * cg; q += NT) {
                const uint32_t c = q / A.R, t = q - c * A.R;
                uint32_t y[16], z[16];
                bs_lds_load<N>(pl, c * k + t, y);
                for (uint32_t i = t + A.R; i < k; i += A.R) {
                    bs_lds_load<N>(pl, c * k + i, z);
#pragma unroll
                    for (int p = 0; p < 16; ++p) y[p] ^= z[p];
                }
                bs_lds_store<N>(pl, c * k + t, y);
            }
            __syncthreads();
        }
        // forward transform over k + V_b: d_i += s d_j; d_j += d_i, layers
        // b-1 .. 0 (r4: layers ql + 1 and ql in one pass)
        int qq = (int)A.b - 1;
        for (; !BIG && A.r4 && qq >= 1; qq -= 2) {
            const uint32_t ql = (uint32_t)qq - 1, h = 1u << ql;
            if (qact && qu < (A.R >> 2)) {
                const uint32_t B = qu >> ql;
                const uint32_t i0 = qc * k + (B << (ql + 2)) + (qu & (h - 1));
                const uint16_t* c0 = cfwd + (A.R - (A.R >> ql));
                const uint16_t* c1 = cfwd + (A.R - (A.R >> (ql + 1)));
                uint32_t d0[16], d1[16], d2[16], d3[16];
                bs_lds_load<N>(pl, i0, d0);
                bs_lds_load<N>(pl, i0 + h, d1);
                bs_lds_load<N>(pl, i0 + 2 * h, d2);
                bs_lds_load<N>(pl, i0 + 3 * h, d3);
                const uint32_t s1 = c1[B];
                const bool uni = ql >= 6 || ql + 2 == A.b;
                bs_muladd(d0, d2, s1, uni);
                bs_muladd(d1, d3, s1, uni);
#pragma unroll
                for (int p = 0; p < 16; ++p) {
                    d2[p] ^= d0[p];
                    d3[p] ^= d1[p];
                }
                bs_muladd(d0, d1, c0[2 * B], uni);
#pragma unroll
                for (int p = 0; p < 16; ++p) d1[p] ^= d0[p];
                bs_lds_store<N>(pl, i0, d0);
                bs_lds_store<N>(pl, i0 + h, d1);
                bs_muladd(d2, d3, c0[2 * B + 1], uni);
#pragma unroll
                for (int p = 0; p < 16; ++p) d3[p] ^= d2[p];
                bs_lds_store<N>(pl, i0 + 2 * h, d2);
                bs_lds_store<N>(pl, i0 + 3 * h, d3);
            }
            __syncthreads();
        }
        for (; qq >= 0; --qq) {
            const uint32_t ql = (uint32_t)qq, h = 1u << ql;
            if (bact && bp < (A.R >> 1)) {
                const uint32_t blk = bp >> ql;
                const uint32_t i = bc * k + ((blk << (ql + 1)) | (bp & (h - 1)));
                uint32_t di[16], dj[16];
                bs_lds_load<N>(pl, i, di);
                bs_lds_load<N>(pl, i + h, dj);
                bs_muladd(di, dj, cfwd[(A.R - (A.R >> ql)) + blk], ql >= 6 || ql + 1 == A.b);
#pragma unroll
                for (int p = 0; p < 16; ++p) dj[p] ^= di[p];
                bs_lds_store<N>(pl, i, di);
                bs_lds_store<N>(pl, i + h, dj);
            }
            __syncthreads();
        }
        if (MODE == 2) {   // recovered row b = D_b' out[E_b], D_b' = Qy_b / Py_b
            for (uint32_t q = tid; q < e_g * cg; q += NT) {
                const uint32_t bb = q / cg, c = q - bb * cg;
                const uint32_t cc = col0 + 32u * c;
                if (cc >= A.nsym) continue;
                uint32_t y[16], z[16];
                bs_lds_load<N>(pl, c * k + (uint32_t)gE[bb], y);
                uint32_t db = lp[2 * A.em + bb] + kOrd16 - lp[3 * A.em + bb];
                db = db >= kOrd16 ? db - kOrd16 : db;
#pragma unroll
                for (int p = 0; p < 16; ++p) z[p] = 0;
                bs_muladd(z, y, A.gexp[db]);
                bs_store_row(A.rep + g * A.rgs + (uint64_t)bb * A.rrs + 2ull * cc, min(32u, A.nsym - cc), z, nullptr);
            }
            continue;
        }
        // repairs first .. first + r - 1 = coset points first + jj (decode:
        // the syndrome of the accepted repair k + jj, its received row XORed in)
        const uint16_t* rpos = MODE == 1 ? A.rpos + g * A.r : nullptr;
        const uint16_t* rslot = MODE == 1 ? A.rslot + g * A.r : nullptr;
        for (uint32_t q = tid; q < A.r * cg; q += NT) {
            const uint32_t jj = q / cg, c = q - jj * cg;
            const uint32_t cc = col0 + 32u * c;
            if (cc >= A.nsym) continue;
            uint64_t orow = jj;
            const uint8_t* xr = nullptr;
            if (MODE == 1) {
                orow = rpos[jj];
                if (orow == 0xFFFFu) continue;
                xr = gsrc + (uint64_t)rslot[jj] * A.srs + 2ull * cc;
            }
            uint32_t y[16];
            bs_lds_load<N>(pl, c * k + A.first + jj, y);
            bs_store_row(A.rep + g * A.rgs + orow * A.rrs + 2ull * cc, min(32u, A.nsym - cc), y, xr);
        }
    }
}

uint32_t hmul16(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        b >>= 1;
        a <<= 1;
        if (a & 0x10000) a ^= 0x1100B;
    }
    return r;
}

uint32_t hinv16(uint32_t a) {   // a^65534, a != 0
    uint32_t r = 1, x = a;
    for (uint32_t p = 0xFFFE; p; p >>= 1) {
        if (p & 1) r = hmul16(r, x);
        x = hmul16(x, x);
    }
    return r;
}

}  // namespace

namespace qf {

bool gf16_fft_has(uint32_t k, uint32_t r, uint32_t first) {
    return k >= kFftMinK && k <= kFftLdsSymbols / 2 && (k & (k - 1)) == 0 && r >= 1 && first + r <= k;
}

bool gf16_fft_pays(uint32_t k, uint32_t nout, uint32_t npoints) {
    // products per symbol column: nout k direct (k_matvec16, ~4 T/s) against
    // a k / 2 + k + b R / 2 here (~0.45 T/s, tools/bench_gf16.py r03ae/af):
    // the FFT where it does ~9x fewer
    uint32_t a = 0, R = 1, b = 0;
    while ((1u << a) < k) ++a;
    while (R < npoints) {
        R <<= 1;
        ++b;
    }
    const uint64_t fft = (uint64_t)a * k / 2 + k + (uint64_t)b * R / 2;
    return (uint64_t)nout * k > 9 * fft;
}

namespace {

int fft16_launch(qf_ctx* ctx, hipStream_t st, Fft16Args A, uint32_t G, uint32_t L, uint8_t* work, const char* name) {
    const uint32_t k = A.k, r = A.r, first = A.first;
    uint32_t a = 0, R = 1, b = 0;
    while ((1u << a) < k) ++a;
    while (R < first + r) {
        R <<= 1;
        ++b;
    }
    // the table W_q(2^m), q = 0 .. a
    Fft16ConstArgs ca{};
    for (uint32_t m = 0; m < 16; ++m) ca.t.W[0][m] = (uint16_t)(1u << m);
    for (uint32_t q = 0; q < a; ++q)
        for (uint32_t m = 0; m < 16; ++m)
            ca.t.W[q + 1][m] = (uint16_t)hmul16(ca.t.W[q][m], ca.t.W[q][m] ^ ca.t.W[q][q]);
    auto w_at = [&](uint32_t q, uint32_t x) {
        uint32_t v = 0;
        for (uint32_t m = 0; x; ++m, x >>= 1)
            if (x & 1) v ^= ca.t.W[q][m];
        return v;
    };
    uint32_t delta = 1;
    for (uint32_t q = 0; q < a; ++q) {
        delta = hmul16(delta, ca.t.W[q][q]);
        ca.t.xk[q] = (uint16_t)hmul16(w_at(q, k), hinv16(ca.t.W[q][q]));
    }
    ca.t.kappa = (uint16_t)hmul16(delta, hinv16(w_at(a, k)));
    uint16_t* cst = reinterpret_cast<uint16_t*>(work);
    // the bit-sliced kernel (k <= 2,048) unless QF_OPT_GF16_FFT_BS = 0
    // the bit-plane kernel (k <= 2,048): an item (generation, 32 symbol
    // columns) runs its whole transform in one workgroup, so it pays once
    // the items fill a quarter of the CUs (one Extreme window at L = 1,200
    // is 19 items: the log kernel's narrower strips spread it wider)
    const int64_t bs_opt = qf::ctx_opt(ctx, QF_OPT_GF16_FFT_BS);
    const uint64_t bs_items = (uint64_t)G * ((L / 2 + 31) / 32);
    const bool bs = k <= kBsMaxK && (bs_opt >= 2 || (bs_opt == 1 && bs_items >= (uint64_t)qf::ctx_num_cus(ctx) / 4));
    A.r4 = bs_opt == 3 ? 1u : 0u;
    ca.out = cst;
    ca.glog = A.glog;
    ca.gexp = A.gexp;
    ca.k = k;
    ca.a = a;
    ca.R = R;
    ca.b = b;
    ca.normal = bs ? 1u : 0u;
    const uint32_t n_c = 2 * k + R - 2;
    hipLaunchKernelGGL(k_fft16_consts, dim3(std::min<uint32_t>((n_c + 255) / 256, 1024)), dim3(256), 0, st, ca);
    QF_HIP(hipGetLastError());
    const uint32_t nsym = L / 2;
    if (bs) {
        // item = (generation, cg column groups of 32 symbols); cg narrowed
        // until the items cover the workgroup slots (two per CU for k <= 1,024)
        const bool big = k > kBsRows;
        const uint32_t slots = (uint32_t)qf::ctx_num_cus(ctx) * (big ? 1u : 2u);
        const uint32_t groups = (nsym + 31) / 32;
        uint32_t cg = big ? 1u : kBsRows / k;
        while (cg > 1 && cg / 2 >= groups) cg >>= 1;
        while (cg > 1 && (uint64_t)G * ((groups + cg - 1) / cg) < slots) cg >>= 1;
        A.cst = cst;
        A.a = a;
        A.R = R;
        A.b = b;
        A.nsym = nsym;
        A.S = cg;
        A.strips = (groups + cg - 1) / cg;
        const uint64_t items = (uint64_t)G * A.strips;
        const dim3 grid((uint32_t)std::min<uint64_t>(items, slots));
        const int mode = A.solve ? 2 : A.syn ? 1 : 0;
        hipEvent_t ev = qf::ctx_prof_begin(ctx, st);
        auto launch = [&](auto kern, uint32_t nt) { hipLaunchKernelGGL(kern, grid, dim3(nt), 0, st, A, G); };
        if (big)
            mode == 0 ? launch(k_fft16_bs<0, true>, 1024) : mode == 1 ? launch(k_fft16_bs<1, true>, 1024)
                                                           : launch(k_fft16_bs<2, true>, 1024);
        else
            mode == 0 ? launch(k_fft16_bs<0, false>, kBsThreads) : mode == 1 ? launch(k_fft16_bs<1, false>, kBsThreads)
                                                                  : launch(k_fft16_bs<2, false>, kBsThreads);
        QF_HIP(hipGetLastError());
        qf::ctx_prof_end(ctx, st, ev, name);
        return QF_OK;
    }
    // strip width: the 32 KiB LDS strip, narrowed until the items cover the CUs
    uint32_t S = kFftLdsSymbols / k, lgS = 0;
    while ((1u << (lgS + 1)) <= S) ++lgS;
    S = 1u << lgS;
    const uint32_t cus = (uint32_t)qf::ctx_num_cus(ctx);
    while (S > 2 && (uint64_t)G * ((nsym + S - 1) / S) < cus) {
        S >>= 1;
        --lgS;
    }
    while (S > 2 && S / 2 >= nsym) {   // no strip wider than the row (S >= 2: column pairs)
        S >>= 1;
        --lgS;
    }
    A.cst = cst;
    A.a = a;
    A.R = R;
    A.b = b;
    A.nsym = nsym;
    A.S = S;
    A.lgS = lgS;
    A.strips = (nsym + S - 1) / S;
    const uint64_t items = (uint64_t)G * A.strips;
    hipEvent_t ev = qf::ctx_prof_begin(ctx, st);
    const dim3 grid((uint32_t)std::min<uint64_t>(items, cus));
    if (n_c <= kFftLdsConsts)
        hipLaunchKernelGGL(k_fft16<true>, grid, dim3(kFftThreads), 0, st, A, G);
    else
        hipLaunchKernelGGL(k_fft16<false>, grid, dim3(kFftThreads), 0, st, A, G);
    QF_HIP(hipGetLastError());
    qf::ctx_prof_end(ctx, st, ev, name);
    return QF_OK;
}

}  // namespace

int gf16_fft_encode(qf_ctx* ctx, hipStream_t st, uint32_t k, uint32_t r, uint32_t first, uint32_t rot, uint32_t L,
                    uint32_t G, const uint8_t* src, uint64_t sgs, uint64_t srs, uint8_t* rep, uint64_t rgs,
                    uint64_t rrs, const uint16_t* glog, const uint16_t* gexp, uint8_t* work) {
    if (!gf16_fft_has(k, r, first) || (L & 1)) return kGf16BsNone;
    Fft16Args A{};
    A.src = src;
    A.sgs = sgs;
    A.srs = srs;
    A.rep = rep;
    A.rgs = rgs;
    A.rrs = rrs;
    A.glog = glog;
    A.gexp = gexp;
    A.k = k;
    A.r = r;
    A.first = first;
    A.rot = rot;
    const int zs = qf::ctx_gf16_zech(ctx, &A.zech);
    if (zs) return zs;
    return fft16_launch(ctx, st, A, G, L, work, "k_fft16_encode");
}

int gf16_fft_syndromes(qf_ctx* ctx, hipStream_t st, uint32_t k, uint32_t r, uint32_t L, uint32_t G,
                       const uint8_t* rows, uint64_t rgs, uint64_t rs, const uint16_t* smap, const uint16_t* rpos,
                       const uint16_t* rslot, const uint32_t* skip, uint8_t* synd, uint64_t synd_gs, uint64_t synd_rs,
                       const uint16_t* glog, const uint16_t* gexp, uint8_t* work) {
    if (!gf16_fft_has(k, r, 0) || (L & 1)) return kGf16BsNone;
    Fft16Args A{};
    A.src = rows;
    A.sgs = rgs;
    A.srs = rs;
    A.rep = synd;
    A.rgs = synd_gs;
    A.rrs = synd_rs;
    A.glog = glog;
    A.gexp = gexp;
    A.k = k;
    A.r = r;
    A.smap = smap;
    A.rpos = rpos;
    A.rslot = rslot;
    A.skip = skip;
    A.syn = 1;
    const int zs = qf::ctx_gf16_zech(ctx, &A.zech);
    if (zs) return zs;
    return fft16_launch(ctx, st, A, G, L, work, "k_fft16_syndromes");
}

int gf16_fft_solve(qf_ctx* ctx, hipStream_t st, uint32_t k, uint32_t L, uint32_t G, const uint8_t* synd,
                   uint64_t synd_gs, uint64_t synd_rs, uint8_t* rec, uint64_t rec_gs, uint64_t rec_rs,
                   const uint32_t* st_e, uint32_t st_stride, const int32_t* status, const uint16_t* J,
                   const uint16_t* E, const uint32_t* lprod, uint64_t em, const uint32_t* solve_fb,
                   const uint16_t* glog, const uint16_t* gexp, uint8_t* work) {
    if (!gf16_fft_has(k, k, 0) || (L & 1)) return kGf16BsNone;
    Fft16Args A{};
    A.src = synd;
    A.sgs = synd_gs;
    A.srs = synd_rs;
    A.rep = rec;
    A.rgs = rec_gs;
    A.rrs = rec_rs;
    A.glog = glog;
    A.gexp = gexp;
    A.k = k;
    A.r = k;   // outputs at every point of the coset (E_b < k)
    A.st_e = st_e;
    A.st_stride = st_stride;
    A.status = status;
    A.J = J;
    A.E = E;
    A.lprod = lprod;
    A.em = em;
    A.solve_fb = solve_fb;
    A.solve = 1;
    const int zs = qf::ctx_gf16_zech(ctx, &A.zech);
    if (zs) return zs;
    return fft16_launch(ctx, st, A, G, L, work, "k_fft16_solve");
}

}  // namespace qf
