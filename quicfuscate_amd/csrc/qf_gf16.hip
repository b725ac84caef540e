// qf_gf16.hip -- the GF(2^16) "Extreme mode" codec on the device
// (SURVEY 8(f) rank 3): Encoder16 / Decoder16 of decoder.rs:10-88 and
// 536-656 over gf_tables.rs:331-380, batched like the GF(2^8) path.
//
// Field: GF(2^16) mod 0x1100B (primitive; generator 2), multiplication as
// gf16_mul intends it (gf_tables.rs:333-353).  Symbols are
// big-endian u16 pairs of payload bytes (decoder.rs:42-54); L must be even.
//
// Multiplication by a coefficient c is exp[log c + log x] with the exp
// table in LDS (128 KB, one period) and the log table read from global
// memory (L2-resident, 128 KB).  log x of a payload symbol is computed once
// per row and reused for every coefficient applied to it.
//
//   k_encode16          repairs of G generations, up to 8 repairs per pass
//   k_decode16_prepare  acceptance exactly as Decoder16::add_packet
//                       (decoder.rs:563-592: the first k rows, systematic
//                       column id % k, no duplicate filtering), Gauss-Jordan
//                       inverse of the erased-column block (e <= 64) in LDS,
//                       per-slot recovery coefficients W = C[J,E]^-1 [I | C[J,S]]
//   k_combine16         recovered rows = W x received rows
// Deviation from Decoder16 (as for GF(2^8)): systematic rows carry
// their payloads, so the recovered bytes are the original bytes; decoding
// happens whenever k rows are present (Decoder16 only tries after a repair
// row, decoder.rs:592, so a generation whose k-th row is systematic never
// decodes there).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "qf_fec.h"
#include "qf_internal.h"

namespace {

#define QF_DEV __device__ __forceinline__

constexpr uint32_t kOrder = 65535;  // multiplicative group order
constexpr uint32_t kNoLog = 0xFFFF; // log of 0 (no product)
constexpr uint32_t kEMax = 64;      // erasures per generation the decode handles
constexpr int kR16 = 8;             // outputs per pass (encode and combine)
constexpr int kThreads16 = 1024;
constexpr uint32_t kLogifyBlocks = 4;  // output blocks of 8 from which inputs go to log form first
constexpr uint64_t kLogifyUnits = 1u << 18;  // or input units (16 B) from which they do (large batches)

// ---- host arithmetic ------------------------------------------------------
uint16_t h_mul(uint16_t a, uint16_t b) {
    uint32_t aa = a, res = 0;
    while (b) {
        if (b & 1) res ^= aa;
        b >>= 1;
        aa <<= 1;
        if (aa & 0x10000u) aa ^= 0x1100Bu;
    }
    return (uint16_t)res;
}

bool h_inv(uint16_t a, uint16_t* out) {
    if (!a) return false;
    uint16_t r = 1, x = a;
    for (uint32_t p = 0x10000u - 2; p; p >>= 1) {
        if (p & 1) r = h_mul(r, x);
        x = h_mul(x, x);
    }
    *out = r;
    return true;
}

// ---- device helpers ---------------------------------------------------------
// 16 payload bytes -> 8 big-endian symbols, as 4 dwords of two symbols each
// (bytes b0 b1 b2 b3 -> b1 | b0 << 8 | b3 << 16 | b2 << 24)
QF_DEV uint32_t bswap16x2(uint32_t w) { return __builtin_amdgcn_perm(w, w, 0x02030001u); }

QF_DEV uint4 load16_partial(const uint8_t* p, uint32_t nb) {
    if (nb >= 16) return *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t b = 0; b < nb; ++b) w[b >> 2] |= (uint32_t)p[b] << (8 * (b & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

QF_DEV void store16_partial(uint8_t* p, const uint32_t (&w)[4], uint32_t nb) {
    if (nb >= 16) {
        *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
        return;
    }
    for (uint32_t b = 0; b < nb; ++b) p[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
}

// Branch-free products: operands are byte offsets 2*log into the LDS exp
// table, a zero operand is kZeroOff (far beyond any sum of two logs).  The
// sum of two offsets is reduced mod 2*65535 by min(t, t - 2*65535) (the
// subtraction wraps for t below the period) and clamped to 2*65535, the
// offset of the table's extra zero entry: 3 VALU ops and one LDS read.
constexpr uint32_t kZeroOff = 0x40000000u;
constexpr uint32_t kPeriodOff = 2 * kOrder;

QF_DEV uint32_t log_off(uint32_t lg) { return lg == kNoLog ? kZeroOff : 2 * lg; }

// log offsets of the 8 symbols of a unit
QF_DEV void symbol_logs(const uint4& raw, const uint16_t* __restrict__ glog, uint32_t (&lx)[8]) {
    const uint32_t w[4] = {bswap16x2(raw.x), bswap16x2(raw.y), bswap16x2(raw.z), bswap16x2(raw.w)};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        // glog[0] = kNoLog: gather unconditionally, select (no branch)
        const uint32_t lg = glog[(w[q >> 1] >> (16 * (q & 1))) & 0xFFFF];
        lx[q] = lg == kNoLog ? kZeroOff : 2u * lg;
    }
}

QF_DEV uint32_t prod_lds(const char* base, uint32_t lx, uint32_t lc) {
    const uint32_t t = lx + lc;
    return *reinterpret_cast<const uint16_t*>(base + min(min(t, t - kPeriodOff), kPeriodOff));
}

// acc ^= c * x for 8 symbols held as 4 dwords of (symbol 2d | symbol 2d+1 << 16),
// lc = log_off(log c)
QF_DEV void mul_acc(uint32_t (&acc)[4], uint32_t lc, const uint32_t (&lx)[8], const uint16_t* sexp) {
    const char* base = reinterpret_cast<const char*>(sexp);
    uint32_t p[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) p[q] = prod_lds(base, lx[q], lc);
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[d] ^= p[2 * d] | (p[2 * d + 1] << 16);
}

// packed symbols <-> 16 payload bytes (big-endian symbols)
QF_DEV void pack_symbols(const uint32_t (&acc)[4], uint32_t (&w)[4]) {
#pragma unroll
    for (int d = 0; d < 4; ++d) w[d] = bswap16x2(acc[d]);
}

QF_DEV void load_exp_lds(uint16_t* sexp, const uint16_t* gexp) {
    const uint4* g = reinterpret_cast<const uint4*>(gexp);
    uint4* l = reinterpret_cast<uint4*>(sexp);
    for (uint32_t w = threadIdx.x; w < (kOrder + 1) / 8; w += blockDim.x) l[w] = g[w];
    __syncthreads();
    if (threadIdx.x == 0) sexp[kOrder] = 0;  // the zero product (offset kPeriodOff)
    __syncthreads();
}

// ---- generalized row combination -------------------------------------------
// out[b] = base[b] ^ sum_c M[b][c] * in[c] for the rows of one or many
// generations; lanes over (generation, block of 8 outputs, input chunk,
// 16-B unit), units fastest so a wave reads consecutive units of one row.
// Encode, the syndromes and the final solve are all this kernel.  With one
// input chunk the lane stores its rows; with several (few generations, long
// rows: an Extreme window) every chunk XORs its partial rows into a zeroed
// padded accumulator with 32-bit atomics and k_finish16 copies them out.
struct Mv16Args {
    const uint8_t* in;
    uint64_t igs, irs;
    const uint16_t* isel;   // row slot of input c: isel[g*isel_gs + c] (null: c)
    uint64_t isel_gs;
    const uint8_t* base;    // optional XOR base rows
    uint64_t bgs, brs;
    const uint16_t* bsel;   // row slot of base b (null: b)
    uint64_t bsel_gs;
    uint8_t* out;
    uint64_t ogs, ors;
    const uint16_t* m;      // logs, m[g*mgs + b*mrs + c] (kNoLog = 0)
    uint64_t mgs, mrs;
    const uint32_t* nout_g; // outputs of generation g (null: nout)
    const uint32_t* nin_g;  // inputs of generation g at nin_g[g * nin_gs] (null: nin)
    uint32_t nin_gs;
    const uint16_t* log;
    const uint16_t* exp;
    uint32_t* acc_ws;       // split: nsplit slabs [g][nout][Lu][4 dwords] of partial rows
    uint64_t slab;          // dwords per slab
    uint32_t nout, nin, L, Lu, nob, nsplit, kchunk;
    uint64_t total_units;
    uint32_t in_log;        // in holds the symbols' logs (k_logify16), not the symbols
    // device-shaped launch (decode: e_g is known only after acceptance):
    // k_shape16 sizes nob / nsplit / kchunk / total_units from the largest
    // nout_g and nin_g instead of nout and nin; null: the fields above
    struct Mv16Shape* shape;
    uint64_t G, want;
    uint32_t ns_cap;        // slabs acc_ws holds
};

struct Mv16Shape {
    uint32_t nob, nsplit, kchunk, pad;
    uint64_t total;
};

// Input chunks per lane-unit.  The grid holds `want` lanes at once (one
// 1,024-thread block per CU: the exp table fills the LDS), and every unit
// costs its chunk's rows, so a launch takes ceil(lanes * ns / want) rounds of
// ceil(nin / ns) rows.  The old rule (the smallest ns with lanes * ns >=
// want) could leave a second round a few % full: an Extreme window (9,600
// lanes, ns 28) ran two rounds of 37 rows where ns 27 runs one of 38.  A
// split launch adds k_finish16 (priced at 4 rows) and one slab of partial
// rows per chunk (1/8 row each).
__host__ __device__ uint32_t matvec_split(uint64_t lanes, uint32_t nin, uint64_t want) {
    const uint32_t max_ns = nin / 16 > 1 ? nin / 16 : 1;   // chunks of at least 16 rows
    uint32_t best = 1;
    uint64_t best_cost = ((lanes + want - 1) / want) * nin;
    for (uint32_t ns = 2; ns <= max_ns; ++ns) {
        const uint64_t cost = ((lanes * ns + want - 1) / want) * ((nin + ns - 1) / ns) + 4 + ns / 8;
        if (cost < best_cost) {
            best_cost = cost;
            best = ns;
        }
    }
    return best;
}

// one block: the launch shape from the largest nout_g / nin_g of the batch
__global__ void __launch_bounds__(1024) k_shape16(Mv16Args a) {
    __shared__ uint32_t red[2][16];
    uint32_t mo = 0, mi = 0;
    for (uint64_t g = threadIdx.x; g < a.G; g += blockDim.x) {
        mo = max(mo, a.nout_g ? min(a.nout_g[g], a.nout) : a.nout);
        mi = max(mi, a.nin_g ? min(a.nin_g[g * a.nin_gs], a.nin) : a.nin);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        mo = max(mo, (uint32_t)__shfl_xor((int)mo, o, 64));
        mi = max(mi, (uint32_t)__shfl_xor((int)mi, o, 64));
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = mo;
        red[1][threadIdx.x >> 6] = mi;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (uint32_t w = 1; w < blockDim.x / 64; ++w) {
        mo = max(mo, red[0][w]);
        mi = max(mi, red[1][w]);
    }
    mo = max(mo, red[0][0]);
    mi = max(mi, red[1][0]);
    Mv16Shape sh{};
    sh.nob = (mo + kR16 - 1) / kR16;
    const uint64_t lanes = a.G * sh.nob * a.Lu;
    uint32_t ns = lanes && mi && lanes < a.want ? matvec_split(lanes, mi, a.want) : 1;
    ns = min(ns, max(a.ns_cap, 1u));
    sh.nsplit = ns;
    sh.kchunk = mi ? (mi + ns - 1) / ns : 1;
    sh.total = mi ? lanes * ns : 0;
    *a.shape = sh;
}

// the 8 logs of a unit of a log row (k_logify16): kNoLog -> the zero offset
QF_DEV void unpack_logs(const uint4& raw, uint32_t (&lx)[8]) {
    const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const uint32_t lg = (w[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
        lx[q] = lg == kNoLog ? kZeroOff : 2u * lg;
    }
}

// Input rows -> log rows, once per matvec: symbol q of unit u of input c of
// generation g -> its log (kNoLog for 0) at out + ((g nin + c) Lu + u) 16 + 2q.
// An input feeds every block of 8 outputs, so k_matvec16 would otherwise
// gather the same logs once per block (128 times for an Extreme window).
// The log table sits in LDS (65,536 x 2 B = 128 KiB): the 8 random lookups
// per unit were global gathers (0.57 TB/s of rows for the k = 64 batch),
// from LDS they cost about what the row traffic does.
__global__ void __launch_bounds__(kThreads16) k_logify16(Mv16Args a, uint64_t G, uint16_t* out) {
    __shared__ __attribute__((aligned(16))) uint16_t slog[kOrder + 1];
    {
        const uint4* g = reinterpret_cast<const uint4*>(a.log);
        uint4* l = reinterpret_cast<uint4*>(slog);
        for (uint32_t w = threadIdx.x; w < (kOrder + 1) / 8; w += blockDim.x) l[w] = g[w];
        __syncthreads();
    }
    const uint64_t total = G * a.nin * a.Lu;
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total;
         f += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = f / a.Lu;
        const uint32_t u = (uint32_t)(f - t * a.Lu);
        const uint64_t g = t / a.nin;
        const uint32_t c = (uint32_t)(t - g * a.nin);
        const uint32_t nin = a.nin_g ? min(a.nin_g[g * a.nin_gs], a.nin) : a.nin;
        if (c >= nin) continue;   // never read
        const uint32_t nb = min(16u, a.L - 16 * u);
        const uint32_t slot = a.isel ? a.isel[g * a.isel_gs + c] : c;
        const uint4 raw = load16_partial(a.in + g * a.igs + (uint64_t)slot * a.irs + 16ull * u, nb);
        const uint32_t w[4] = {bswap16x2(raw.x), bswap16x2(raw.y), bswap16x2(raw.z), bswap16x2(raw.w)};
        uint32_t o[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = (uint32_t)slog[w[d] & 0xFFFF] | ((uint32_t)slog[w[d] >> 16] << 16);
        *reinterpret_cast<uint4*>(out + (f * 8)) = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

__global__ void __launch_bounds__(kThreads16) k_matvec16(Mv16Args a) {
    __shared__ uint16_t sexp[kOrder + 1];  // static: LDS offsets fold into the reads
    uint32_t nob = a.nob, nsplit = a.nsplit, kchunk = a.kchunk;
    uint64_t total = a.total_units;
    if (a.shape) {
        const Mv16Shape sh = *a.shape;
        nob = sh.nob;
        nsplit = sh.nsplit;
        kchunk = sh.kchunk;
        total = sh.total;
    }
    // a block without units leaves before the 128 KiB table copy (device-shaped
    // launches with nothing to do: the FFT paths' fallback matvecs)
    if ((uint64_t)blockIdx.x * blockDim.x >= total) return;
    load_exp_lds(sexp, a.exp);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total; f += stride) {
        uint64_t t = f / a.Lu;
        const uint32_t u = (uint32_t)(f - t * a.Lu);
        const uint32_t ks = (uint32_t)(t % nsplit);
        t /= nsplit;
        const uint64_t g = t / nob;
        const uint32_t b0 = (uint32_t)(t - g * nob) * kR16;
        const uint32_t nout = a.nout_g ? min(a.nout_g[g], a.nout) : a.nout;
        if (b0 >= nout) continue;
        const uint32_t no = min((uint32_t)kR16, nout - b0);
        const uint32_t nin = a.nin_g ? min(a.nin_g[g * a.nin_gs], a.nin) : a.nin;
        const uint32_t c0 = ks * kchunk, c1 = min(nin, c0 + kchunk);
        const uint32_t nb = min(16u, a.L - 16 * u);
        uint32_t acc[kR16][4];
#pragma unroll
        for (int bb = 0; bb < kR16; ++bb) {
            acc[bb][0] = acc[bb][1] = acc[bb][2] = acc[bb][3] = 0;
            if (a.base && ks == 0 && (uint32_t)bb < no) {
                const uint32_t slot = a.bsel ? a.bsel[g * a.bsel_gs + b0 + bb] : b0 + bb;
                const uint4 raw = load16_partial(a.base + g * a.bgs + (uint64_t)slot * a.brs + 16ull * u, nb);
                acc[bb][0] = bswap16x2(raw.x);
                acc[bb][1] = bswap16x2(raw.y);
                acc[bb][2] = bswap16x2(raw.z);
                acc[bb][3] = bswap16x2(raw.w);
            }
        }
        const uint8_t* ip = a.in + g * a.igs + 16ull * u;
        const uint16_t* isel = a.isel ? a.isel + g * a.isel_gs : nullptr;
        const uint16_t* m = a.m + g * a.mgs + (uint64_t)b0 * a.mrs;
        // software pipeline: row c + 2's bytes and row c + 1's log gathers
        // are in flight while row c's products are formed
        uint4 nxt = make_uint4(0, 0, 0, 0);
        uint32_t lxn[8], lcr[kR16];
        // coefficient logs of row c (outputs past `no` read a valid row and count as 0)
        auto coef_row = [&](uint32_t c, uint32_t (&out)[kR16]) {
#pragma unroll
            for (int bb = 0; bb < kR16; ++bb) out[bb] = m[(uint64_t)min((uint32_t)bb, no - 1) * a.mrs + c];
        };
        if (c0 < c1) {
            const uint4 raw0 = load16_partial(ip + (uint64_t)(isel ? isel[c0] : c0) * a.irs, nb);
            if (a.in_log) unpack_logs(raw0, lxn);
            else symbol_logs(raw0, a.log, lxn);
            coef_row(c0, lcr);
        }
        if (c0 + 1 < c1) nxt = load16_partial(ip + (uint64_t)(isel ? isel[c0 + 1] : c0 + 1) * a.irs, nb);
        for (uint32_t c = c0; c < c1; ++c) {
            uint32_t lx[8], lc[kR16];
#pragma unroll
            for (int q = 0; q < 8; ++q) lx[q] = lxn[q];
#pragma unroll
            for (int bb = 0; bb < kR16; ++bb) lc[bb] = (uint32_t)bb < no ? log_off(lcr[bb]) : kZeroOff;
            if (c + 1 < c1) {
                // next row's log gathers and coefficients in flight during this row
                if (a.in_log) unpack_logs(nxt, lxn);
                else symbol_logs(nxt, a.log, lxn);
                coef_row(c + 1, lcr);
                if (c + 2 < c1) nxt = load16_partial(ip + (uint64_t)(isel ? isel[c + 2] : c + 2) * a.irs, nb);
            }
#pragma unroll
            for (int bb = 0; bb < kR16; ++bb) mul_acc(acc[bb], lc[bb], lx, sexp);
        }
        if (nsplit == 1) {
            uint8_t* op = a.out + g * a.ogs + 16ull * u;
#pragma unroll
            for (int bb = 0; bb < kR16; ++bb) {
                if ((uint32_t)bb >= no) break;
                uint32_t w[4];
                pack_symbols(acc[bb], w);
                store16_partial(op + (uint64_t)(b0 + bb) * a.ors, w, nb);
            }
        } else {
            // chunk ks's partial rows go to slab ks (plain stores; k_finish16 XORs the slabs)
            uint32_t* wp = a.acc_ws + ks * a.slab + ((g * a.nout + b0) * a.Lu + u) * 4;
#pragma unroll
            for (int bb = 0; bb < kR16; ++bb) {
                if ((uint32_t)bb >= no) break;
                uint32_t w[4];
                pack_symbols(acc[bb], w);
                *reinterpret_cast<uint4*>(wp + (uint64_t)bb * a.Lu * 4) = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
    }
}

// XOR of the split slabs -> output rows (exactly L bytes per row)
__global__ void __launch_bounds__(256) k_finish16(Mv16Args a) {
    const uint32_t nsplit = a.shape ? a.shape->nsplit : a.nsplit;
    if (nsplit <= 1) return;   // a device-shaped launch that did not split wrote the rows itself
    const uint64_t total = a.G * a.nout * a.Lu;
    for (uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total; f += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = f / a.Lu;
        const uint32_t u = (uint32_t)(f - t * a.Lu);
        const uint64_t g = t / a.nout;
        const uint32_t b = (uint32_t)(t - g * a.nout);
        const uint32_t nout = a.nout_g ? min(a.nout_g[g], a.nout) : a.nout;
        if (b >= nout) continue;
        uint32_t w[4] = {0, 0, 0, 0};
        for (uint32_t ks = 0; ks < nsplit; ++ks) {
            const uint4 v = reinterpret_cast<const uint4*>(a.acc_ws + ks * a.slab)[f];
            w[0] ^= v.x;
            w[1] ^= v.y;
            w[2] ^= v.z;
            w[3] ^= v.w;
        }
        store16_partial(a.out + g * a.ogs + (uint64_t)b * a.ors + 16ull * u, w, min(16u, a.L - 16 * u));
    }
}

// Logs of the Cauchy rows first..first+r-1 over a ring of k source slots
// whose window position i sits in slot (rot + i) % k:
//   m[q][slot] = log inv(i ^ (k + first + q)) = -log(i ^ y)   (decoder.rs:77-80)
// be_out (optional): each row's coefficient block in window order, big-endian
// u16 (decoder.rs:62-66).
__global__ void __launch_bounds__(256) k_cauchy16_logs(uint16_t* m, uint32_t k, uint32_t r, uint32_t first, uint32_t rot,
                                                       const uint16_t* glog, const uint16_t* gexp, uint8_t* be_out) {
    const uint64_t total = (uint64_t)k * r;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t q = (uint32_t)(t / k), slot = (uint32_t)(t % k);
        const uint32_t i = slot >= rot ? slot - rot : slot + k - rot;
        const uint32_t l = glog[i ^ ((k + first + q) & 0xFFFF)];  // i ^ y != 0: i < k <= y
        const uint32_t nl = l ? kOrder - l : 0;
        m[t] = (uint16_t)nl;
        if (be_out) {
            const uint32_t c = gexp[nl];
            be_out[((uint64_t)q * k + i) * 2] = (uint8_t)(c >> 8);
            be_out[((uint64_t)q * k + i) * 2 + 1] = (uint8_t)c;
        }
    }
}

// ---- decode -----------------------------------------------------------------
QF_DEV uint32_t dmul(uint32_t a, uint32_t b, const uint16_t* glog, const uint16_t* gexp) {
    if (!a || !b) return 0;
    return gexp[(uint32_t)glog[a] + glog[b]];
}

QF_DEV uint32_t dinv(uint32_t a, const uint16_t* glog, const uint16_t* gexp) {
    return gexp[kOrder - glog[a]];  // a != 0
}

QF_DEV uint32_t lmod(int64_t x) {
    int64_t m = x % (int64_t)kOrder;
    return (uint32_t)(m < 0 ? m + kOrder : m);
}

// Per-generation decode state in the workspace (the large-erasure path).
struct Dec16State {
    uint32_t e, nin;                // erasures, systematic rows among the first k
};

struct Dec16Args {
    const uint16_t* row_index;
    const uint32_t* n_rows;
    const uint16_t* row_coeffs;  // [g][max_rows][k] or null (Cauchy rows)
    const uint16_t* log;
    const uint16_t* exp;
    uint16_t* wl;                // small path: [g][e_max][k] logs of W
    uint32_t* n_out;
    uint16_t* rec_index;         // [g][e_max]
    int32_t* status;
    uint32_t k, r, e_max, max_rows;
};

// coefficient of source column i in the repair row at slot s (index idx)
QF_DEV uint32_t coef(const uint16_t* row_coeffs, uint64_t g, uint32_t max_rows, uint32_t k, uint32_t s,
                     uint32_t idx, uint32_t i, const uint16_t* glog, const uint16_t* gexp) {
    if (row_coeffs) return row_coeffs[(g * max_rows + s) * k + i];
    return dinv(i ^ idx, glog, gexp);  // decoder.rs:77-80: (i as u16) ^ ((k + j) as u16); i < k <= idx
}

// Small path (e_max <= 64): one block per generation; acceptance, Gauss-
// Jordan inverse of C[J,E] in LDS, W = C[J,E]^-1 [I | C[J,S]] over the first
// k slots, so that the recovered rows are one k_matvec16 over the rows.
__global__ void __launch_bounds__(256) k_decode16_prepare(Dec16Args a) {
    __shared__ uint16_t aug[kEMax][2 * kEMax];
    __shared__ __align__(4) uint8_t present[4096];
    __shared__ uint16_t J[kEMax], Jslot[kEMax], E[kEMax];
    __shared__ int32_t s_status;
    __shared__ uint32_t s_e, s_piv;
    const uint64_t g = blockIdx.x;
    const uint32_t tid = threadIdx.x, k = a.k;
    const uint32_t n = a.n_rows ? min(a.n_rows[g], a.max_rows) : a.max_rows;
    const uint16_t* ridx = a.row_index + g * a.max_rows;
    for (uint32_t i = tid; i < k; i += blockDim.x) present[i] = 0;
    if (tid == 0) s_status = n < k ? QF_ENOTREADY : QF_OK;
    __syncthreads();
    // the first k rows (decoder.rs:563-566); systematic column id % k: the
    // batch row index < k is that column.  A duplicated column makes the
    // system singular (Decoder16 does not filter duplicates).
    if (s_status == QF_OK) {
        for (uint32_t s = tid; s < k; s += blockDim.x) {
            const uint32_t idx = ridx[s];
            if (idx < k &&
                (atomicAdd(reinterpret_cast<uint32_t*>(&present[idx & ~3u]), 1u << (8 * (idx & 3))) &
                 (0xFFu << (8 * (idx & 3)))))
                s_status = QF_ERANK;
        }
    }
    __syncthreads();
    if (s_status == QF_OK && tid == 0) {
        uint32_t e = 0, nj = 0;
        for (uint32_t i = 0; i < k; ++i)
            if (!present[i]) {
                if (e < kEMax) E[e] = (uint16_t)i;
                ++e;
            }
        for (uint32_t s = 0; s < k && nj < kEMax; ++s)
            if (ridx[s] >= k) {
                J[nj] = ridx[s];
                Jslot[nj] = (uint16_t)s;
                ++nj;
            }
        if (e > a.e_max) s_status = QF_ERANGE;
        s_e = e;
    }
    __syncthreads();
    const uint32_t e = s_e;
    if (s_status == QF_OK) {
        // [C[J,E] | I] in LDS, Gauss-Jordan with a pivot search (decoder.rs:598-640)
        for (uint32_t t = tid; t < e * 2 * e; t += blockDim.x) {
            const uint32_t b = t / (2 * e), c = t % (2 * e);
            aug[b][c] = c < e ? (uint16_t)coef(a.row_coeffs, g, a.max_rows, k, Jslot[b], J[b], E[c], a.log, a.exp)
                              : (uint16_t)(c - e == b);
        }
        __syncthreads();
        for (uint32_t c = 0; c < e; ++c) {
            if (tid == 0) {
                uint32_t p = c;
                while (p < e && aug[p][c] == 0) ++p;
                s_piv = p;
                if (p == e) s_status = QF_ERANK;
            }
            __syncthreads();
            if (s_status != QF_OK) break;
            const uint32_t p = s_piv;
            if (p != c) {
                for (uint32_t t = tid; t < 2 * e; t += blockDim.x) {
                    const uint16_t v = aug[c][t];
                    aug[c][t] = aug[p][t];
                    aug[p][t] = v;
                }
                __syncthreads();
            }
            const uint32_t iv = dinv(aug[c][c], a.log, a.exp);
            __syncthreads();
            for (uint32_t t = tid; t < 2 * e; t += blockDim.x) aug[c][t] = (uint16_t)dmul(aug[c][t], iv, a.log, a.exp);
            __syncthreads();
            for (uint32_t t = tid; t < e * 2 * e; t += blockDim.x) {
                const uint32_t b = t / (2 * e), cc = t % (2 * e);
                if (b == c || cc == c) continue;
                const uint32_t f = aug[b][c];
                if (f) aug[b][cc] ^= (uint16_t)dmul(f, aug[c][cc], a.log, a.exp);
            }
            __syncthreads();
            for (uint32_t b = tid; b < e; b += blockDim.x)
                if (b != c) aug[b][c] = 0;
            __syncthreads();
        }
    }
    __syncthreads();
    const bool ok = s_status == QF_OK;
    // W[b][slot] over the first k slots: repair slot Jslot[a'] -> D[b][a'];
    // systematic slot of source i -> sum_a' D[b][a'] C[J[a'], i]
    uint16_t* wl = a.wl + g * a.e_max * k;
    for (uint32_t t = tid; t < a.e_max * k; t += blockDim.x) {
        const uint32_t b = t / k, s = t % k;
        uint32_t w = 0;
        if (ok && b < e) {
            const uint32_t idx = ridx[s];
            if (idx >= k) {
                uint32_t ap = 0;
                while (Jslot[ap] != s) ++ap;
                w = aug[b][e + ap];
            } else {
                for (uint32_t ap = 0; ap < e; ++ap)
                    w ^= dmul(aug[b][e + ap], coef(a.row_coeffs, g, a.max_rows, k, Jslot[ap], J[ap], idx, a.log, a.exp),
                              a.log, a.exp);
            }
        }
        wl[t] = (uint16_t)(w ? a.log[w] : kNoLog);
    }
    for (uint32_t b = tid; b < a.e_max; b += blockDim.x)
        a.rec_index[g * a.e_max + b] = (ok && b < e) ? E[b] : 0;
    if (tid == 0) {
        a.status[g] = s_status;
        a.n_out[g] = ok ? e : 0;
    }
}

// Large path (e_max > 64, Extreme windows): chunks of generations, one grid
// z-slice per generation, everything in the workspace (per-generation
// strides below).  Lists of the accepted rows:
struct BigWs {
    Dec16State* st;
    uint16_t* J;      // repair row index, by repair order a
    uint16_t* Jslot;  // its slot
    uint16_t* E;      // erased source columns, ascending
    uint16_t* Sslot;  // systematic slots (sources present), by slot order
    uint16_t* Scol;   // their source columns
    uint16_t* mlog;   // [e_max][k] logs of C[J_a][Scol c]
    uint16_t* dlog;   // [e_max][e_max] logs of C[J,E]^-1
    uint16_t* aug;    // [e_max][2 e_max] general Gauss-Jordan
    uint32_t* mark;   // [e_max] step + 1 at which the row became a pivot
    uint32_t* pivrow; // [e_max] pivot row of column c
    uint32_t* lprod;  // [4][e_max] Cauchy log products
    uint8_t* synd;    // [e_max][Lp] syndrome rows
};

struct BigArgs {
    BigWs w;
    const uint16_t* row_index;   // [g][max_rows]
    uint32_t n_rows;             // max_rows
    const uint32_t* n_rows_dev;  // [g] (or null)
    const uint16_t* row_coeffs;  // [g][max_rows][k] or null
    const uint16_t* log;
    const uint16_t* exp;
    uint32_t* n_out;             // [g]
    uint16_t* rec_index;         // [g][e_max]
    int32_t* status;             // [g]
    uint32_t k, e_max;
    uint64_t Lp;                 // syndrome row bytes
};

// the arguments of generation g of the chunk (pointers offset by its strides)
QF_DEV BigArgs view(const BigArgs& A, uint32_t g) {
    BigArgs a = A;
    const uint64_t em = A.e_max, k = A.k;
    a.w.st = A.w.st + g;
    a.w.J = A.w.J + g * em;
    a.w.Jslot = A.w.Jslot + g * em;
    a.w.E = A.w.E + g * em;
    a.w.Sslot = A.w.Sslot + g * k;
    a.w.Scol = A.w.Scol + g * k;
    a.w.mlog = A.w.mlog + g * em * k;
    a.w.dlog = A.w.dlog + g * em * em;
    a.w.aug = A.w.aug ? A.w.aug + g * em * 2 * em : nullptr;
    a.w.mark = A.w.mark + g * em;
    a.w.pivrow = A.w.pivrow + g * em;
    a.w.lprod = A.w.lprod + g * 4 * em;
    a.w.synd = A.w.synd + g * em * A.Lp;
    a.row_index = A.row_index + (uint64_t)g * A.n_rows;
    a.n_rows_dev = A.n_rows_dev ? A.n_rows_dev + g : nullptr;
    a.row_coeffs = A.row_coeffs ? A.row_coeffs + (uint64_t)g * A.n_rows * k : nullptr;
    a.n_out = A.n_out + g;
    a.rec_index = A.rec_index + g * em;
    a.status = A.status + g;
    return a;
}

QF_DEV void big_fail(const BigArgs& a, int32_t s) {
    *a.status = s;
    *a.n_out = 0;
}

// exclusive prefix sum of one count per thread over the block (power of two)
QF_DEV uint32_t block_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
    const uint32_t tid = threadIdx.x, n = blockDim.x;
    sh[tid] = v;
    __syncthreads();
    for (uint32_t d = 1; d < n; d <<= 1) {
        const uint32_t x = tid >= d ? sh[tid - d] : 0;
        __syncthreads();
        sh[tid] += x;
        __syncthreads();
    }
    const uint32_t incl = sh[tid];
    *total = sh[n - 1];
    __syncthreads();
    return incl - v;
}

// acceptance (decoder.rs:563-578) and the row lists; one block per
// generation of a power of two >= k / 4 threads (64..1024), thread t owns
// slots / columns [4t, 4t + 4) (k <= 4096), lists compacted in order with
// block scans
__global__ void __launch_bounds__(1024) k_dec16_accept(BigArgs A) {
    const BigArgs a = view(A, blockIdx.z);
    __shared__ __align__(4) uint8_t present[4096];
    __shared__ uint32_t scan[1024];
    __shared__ int32_t s_status;
    const uint32_t tid = threadIdx.x, k = a.k;
    const uint32_t n = a.n_rows_dev ? min(*a.n_rows_dev, a.n_rows) : a.n_rows;
    for (uint32_t i = tid; i < k; i += blockDim.x) present[i] = 0;
    if (tid == 0) s_status = n < k ? QF_ENOTREADY : QF_OK;
    __syncthreads();
    uint32_t idx[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t sl = 4 * tid + q;
        idx[q] = (s_status == QF_OK && sl < k) ? a.row_index[sl] : 0xFFFFFFFFu;
        if (idx[q] < k &&
            (atomicAdd(reinterpret_cast<uint32_t*>(&present[idx[q] & ~3u]), 1u << (8 * (idx[q] & 3))) &
             (0xFFu << (8 * (idx[q] & 3)))))
            s_status = QF_ERANK;
    }
    __syncthreads();
    for (uint32_t b = tid; b < a.e_max; b += blockDim.x) a.rec_index[b] = 0;
    if (s_status != QF_OK) {
        if (tid == 0) {
            a.w.st->e = a.w.st->nin = 0;
            big_fail(a, s_status);
        }
        return;
    }
    // erased columns, ascending
    uint32_t ce = 0, cj = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        ce += (4 * tid + q < k && !present[4 * tid + q]);
        cj += (idx[q] != 0xFFFFFFFFu && idx[q] >= k);
    }
    uint32_t e, nj;
    uint32_t oe = block_scan(ce, scan, &e);
    uint32_t oj = block_scan(cj, scan, &nj);
    uint32_t os = 4 * tid - oj;  // systematic slots before this thread's
    if (e > a.e_max) {
        if (tid == 0) {
            a.w.st->e = a.w.st->nin = 0;
            big_fail(a, QF_ERANGE);
        }
        return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = 4 * tid + q;
        if (i < k && !present[i]) {
            a.w.E[oe] = (uint16_t)i;
            a.rec_index[oe] = (uint16_t)i;
            ++oe;
        }
        if (idx[q] == 0xFFFFFFFFu) continue;
        if (idx[q] >= k) {
            a.w.J[oj] = (uint16_t)idx[q];
            a.w.Jslot[oj] = (uint16_t)i;
            ++oj;
        } else {
            a.w.Sslot[os] = (uint16_t)i;
            a.w.Scol[os] = (uint16_t)idx[q];
            ++os;
        }
    }
    if (tid == 0) {
        a.w.st->e = e;
        a.w.st->nin = k - nj;
        *a.status = QF_OK;
        *a.n_out = e;
    }
}

// Maps of the bit-sliced syndrome kernel (qf_gf16_bs.hip), one block per
// generation of the chunk: smap[i] = slot of received source i (0xFFFF: not
// received), rpos[j] / rslot[j] = position in J and slot of the accepted
// repair k + j.  skip = the kernel leaves the generation alone: failed,
// nothing erased, or a repair it has no Cauchy row for (index >= k + r, or
// the same repair twice); nout_fb = e for the last kind, which the general
// syndrome matvec then computes.
__global__ void __launch_bounds__(64) k_dec16_bsmaps(BigArgs A, uint32_t r, uint16_t* smap, uint16_t* rpos,
                                                     uint16_t* rslot, uint32_t* skip, uint32_t* nout_fb,
                                                     uint32_t* solve_fb) {
    const uint32_t g = blockIdx.z, tid = threadIdx.x;
    const BigArgs a = view(A, g);
    const uint32_t k = a.k;
    __shared__ uint32_t seen[2048];   // repairs k + j seen (j < 65,536)
    __shared__ uint32_t s_bad, s_far;
    uint16_t* sm = smap + (uint64_t)g * k;
    uint16_t* rp = rpos + (uint64_t)g * r;
    uint16_t* rsl = rslot + (uint64_t)g * r;
    const bool ok = *a.status == QF_OK;
    const uint32_t e = ok ? a.w.st->e : 0, nin = ok ? a.w.st->nin : 0;
    for (uint32_t i = tid; i < k; i += 64) sm[i] = 0xFFFF;
    for (uint32_t j = tid; j < r; j += 64) {
        rp[j] = 0xFFFF;
        rsl[j] = 0;
    }
    for (uint32_t w = tid; w < 2048; w += 64) seen[w] = 0;
    if (tid == 0) s_bad = s_far = 0;
    __syncthreads();
    for (uint32_t c = tid; c < nin; c += 64) sm[a.w.Scol[c]] = a.w.Sslot[c];   // columns distinct (else ERANK)
    for (uint32_t q = tid; q < e; q += 64) {
        const uint32_t j = (uint32_t)a.w.J[q] - k;
        if (j >= k) s_far = 1;   // past the FFT solve's coset (index >= 2k)
        if (j < r && !(atomicOr(&seen[j >> 5], 1u << (j & 31)) & (1u << (j & 31)))) {
            rp[j] = (uint16_t)q;
            rsl[j] = a.w.Jslot[q];
        } else {
            s_bad = 1;   // no Cauchy row of the kernel, or the same repair twice
        }
    }
    __syncthreads();
    if (tid == 0) {
        skip[g] = (!ok || e == 0 || s_bad) ? 1u : 0u;
        nout_fb[g] = (ok && s_bad) ? e : 0u;
        if (solve_fb) solve_fb[g] = (ok && s_far) ? e : 0u;
    }
}

// mlog[a][c] = log C[J_a][Scol c] (syndromes: rows_J ^ C[J,S] x_S); with
// nout_fb only for the generations the bit-sliced / FFT kernels leave to the matvec
__global__ void __launch_bounds__(256) k_dec16_synmat(BigArgs A, const uint32_t* nout_fb) {
    if (nout_fb && nout_fb[blockIdx.z] == 0) return;
    const BigArgs a = view(A, blockIdx.z);
    const uint32_t e = a.w.st->e, ns = a.w.st->nin, k = a.k;
    const uint64_t total = (uint64_t)e * ns;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(t / ns), c = (uint32_t)(t % ns);
        const uint32_t v = coef(a.row_coeffs, 0, 0, k, a.w.Jslot[r], a.w.J[r], a.w.Scol[c], a.log, a.exp);
        a.w.mlog[(uint64_t)r * k + c] = (uint16_t)(v ? a.log[v] : kNoLog);
    }
}

// Cauchy inverse in closed form: with x_a = J_a, y_b = E_b (C_ab = 1/(x_a ^ y_b)),
//   (C^-1)_ba = Qx_a Qy_b / ((x_a ^ y_b) Px_a Py_b),
//   Qx_a = prod_c (x_a ^ y_c), Qy_b = prod_c (x_c ^ y_b),
//   Px_a = prod_{c != a} (x_a ^ x_c), Py_b = prod_{c != b} (y_b ^ y_c).
// One block per row / column value, logs summed across the block.  A
// repeated repair row (x_a = x_c) is singular: QF_ERANK.
__global__ void __launch_bounds__(256) k_dec16_cauchy_prod(BigArgs A) {
    const BigArgs a = view(A, blockIdx.z);
    __shared__ uint64_t sq[256], sp[256];
    __shared__ uint32_t s_zero;
    const uint32_t e = a.w.st->e;
    const uint32_t t = blockIdx.x;
    if (t >= 2 * e) return;
    const bool row = t < e;
    const uint32_t q = row ? t : t - e;
    const uint32_t v = row ? a.w.J[q] : a.w.E[q];
    const uint16_t* other = row ? a.w.E : a.w.J;  // Q partners
    const uint16_t* same = row ? a.w.J : a.w.E;   // P partners
    if (threadIdx.x == 0) s_zero = 0;
    uint64_t lq = 0, lp = 0;
    bool zero = false;
    for (uint32_t c = threadIdx.x; c < e; c += blockDim.x) {
        lq += a.log[v ^ other[c]];
        if (c != q) {
            const uint32_t d = v ^ same[c];
            zero |= d == 0;
            lp += d ? a.log[d] : 0;
        }
    }
    sq[threadIdx.x] = lq;
    sp[threadIdx.x] = lp;
    __syncthreads();
    if (zero) s_zero = 1;
    for (uint32_t d = blockDim.x / 2; d; d >>= 1) {   // blockDim: power of two, 64..256
        if (threadIdx.x < d) {
            sq[threadIdx.x] += sq[threadIdx.x + d];
            sp[threadIdx.x] += sp[threadIdx.x + d];
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    if (s_zero) {
        big_fail(a, QF_ERANK);
        return;
    }
    a.w.lprod[(row ? 0 : 2) * a.e_max + q] = (uint32_t)(sq[0] % kOrder);
    a.w.lprod[(row ? 1 : 3) * a.e_max + q] = (uint32_t)(sp[0] % kOrder);
}

// (with solve_fb: only for the generations the FFT solve leaves to the matvec)
__global__ void __launch_bounds__(256) k_dec16_cauchy_inv(BigArgs A, const uint32_t* solve_fb) {
    if (solve_fb && solve_fb[blockIdx.z] == 0) return;
    const BigArgs a = view(A, blockIdx.z);
    const uint32_t e = a.w.st->e;
    if (*a.status != QF_OK) return;
    const uint64_t total = (uint64_t)e * e;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t b = (uint32_t)(t / e), r = (uint32_t)(t % e);
        const int64_t l = (int64_t)a.w.lprod[r] + a.w.lprod[2 * a.e_max + b] - a.log[a.w.J[r] ^ a.w.E[b]] -
                          a.w.lprod[a.e_max + r] - a.w.lprod[3 * a.e_max + b];
        a.w.dlog[(uint64_t)b * a.e_max + r] = (uint16_t)lmod(l);
    }
}

// The same closed form for e_max <= 64 in one block per generation: thread t
// < 2e forms the log products of row (J) or column (E) value t with a serial
// loop, then the block writes the e^2 logs of the inverse (one launch of gc
// blocks instead of 2 e_max gc product blocks and a separate inverse grid).
__global__ void __launch_bounds__(128) k_dec16_cauchy_small(BigArgs A, const uint32_t* solve_fb) {
    const BigArgs a = view(A, blockIdx.z);
    __shared__ uint32_t s_zero;
    const uint32_t tid = threadIdx.x;
    if (*a.status != QF_OK) return;   // uniform (accept wrote it)
    const uint32_t e = a.w.st->e;
    if (tid == 0) s_zero = 0;
    __syncthreads();
    if (tid < 2 * e) {
        const bool row = tid < e;
        const uint32_t q = row ? tid : tid - e;
        const uint32_t v = row ? a.w.J[q] : a.w.E[q];
        const uint16_t* other = row ? a.w.E : a.w.J;
        const uint16_t* same = row ? a.w.J : a.w.E;
        uint64_t lq = 0, lp = 0;
        bool zero = false;
        for (uint32_t c = 0; c < e; ++c) {
            lq += a.log[v ^ other[c]];
            const uint32_t d = v ^ same[c];
            zero |= (c != q && d == 0);
            lp += (c != q && d) ? a.log[d] : 0;
        }
        if (zero) s_zero = 1;
        a.w.lprod[(row ? 0 : 2) * a.e_max + q] = (uint32_t)(lq % kOrder);
        a.w.lprod[(row ? 1 : 3) * a.e_max + q] = (uint32_t)(lp % kOrder);
    }
    __syncthreads();
    if (s_zero) {
        if (tid == 0) big_fail(a, QF_ERANK);
        return;
    }
    if (solve_fb && solve_fb[blockIdx.z] == 0) return;   // the FFT solve needs only lprod
    for (uint32_t t = tid; t < e * e; t += blockDim.x) {
        const uint32_t b = t / e, r = t % e;
        const int64_t l = (int64_t)a.w.lprod[r] + a.w.lprod[2 * a.e_max + b] - a.log[a.w.J[r] ^ a.w.E[b]] -
                          a.w.lprod[a.e_max + r] - a.w.lprod[3 * a.e_max + b];
        a.w.dlog[(uint64_t)b * a.e_max + r] = (uint16_t)lmod(l);
    }
}

// General rows: Gauss-Jordan on [C[J,E] | I] in the workspace, one launch per
// column.  Rows are not swapped: a column's pivot is the first row not yet
// used as a pivot with a nonzero entry there (the same pivot as the swap-based
// search of decoder.rs:600-606 up to row order), eliminated from all other rows
// in the columns to its right only (finished columns are never read again).
__global__ void __launch_bounds__(256) k_dec16_gj_init(BigArgs A) {
    const BigArgs a = view(A, blockIdx.z);
    const uint32_t e = a.w.st->e;
    const uint64_t total = (uint64_t)e * 2 * e;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = (uint32_t)(t / (2 * e)), c = (uint32_t)(t % (2 * e));
        a.w.aug[(uint64_t)r * 2 * a.e_max + c] =
            c < e ? (uint16_t)coef(a.row_coeffs, 0, 0, a.k, a.w.Jslot[r], a.w.J[r], a.w.E[c], a.log, a.exp)
                  : (uint16_t)(c - e == r);
        if (c == 0) a.w.mark[r] = 0;
    }
}

__global__ void __launch_bounds__(1024) k_dec16_gj_pivot(BigArgs A, uint32_t c) {
    const BigArgs a = view(A, blockIdx.z);
    const uint32_t e = a.w.st->e;
    if (c >= e || *a.status != QF_OK) return;
    __shared__ uint32_t s_p;
    if (threadIdx.x == 0) s_p = e;
    __syncthreads();
    const uint64_t ld = 2 * a.e_max;
    for (uint32_t p = threadIdx.x; p < e; p += blockDim.x)
        if (a.w.mark[p] == 0 && a.w.aug[p * ld + c] != 0) atomicMin(&s_p, p);
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (s_p == e) {
        big_fail(a, QF_ERANK);
        return;
    }
    a.w.mark[s_p] = c + 1;
    a.w.pivrow[c] = s_p;
}

// rows in blockIdx.y, columns (c, 2e) in x
__global__ void __launch_bounds__(256) k_dec16_gj_step(BigArgs A, uint32_t c) {
    const BigArgs a = view(A, blockIdx.z);
    const uint32_t e = a.w.st->e;
    const uint32_t r = blockIdx.y;
    if (c >= e || r >= e || *a.status != QF_OK) return;
    const uint32_t p = a.w.pivrow[c];
    const uint64_t ld = 2 * a.e_max;
    if (r == p) return;
    const uint32_t f = a.w.aug[r * ld + c];
    if (!f) return;
    const uint32_t lf = lmod((int64_t)a.log[f] - a.log[a.w.aug[(uint64_t)p * ld + c]]);
    for (uint32_t cc = c + 1 + blockIdx.x * blockDim.x + threadIdx.x; cc < 2 * e; cc += gridDim.x * blockDim.x) {
        const uint32_t v = a.w.aug[(uint64_t)p * ld + cc];
        if (v) {
            uint32_t t = a.log[v] + lf;
            t = t >= kOrder ? t - kOrder : t;
            a.w.aug[(uint64_t)r * ld + cc] ^= a.exp[t];
        }
    }
}

// dlog[c][a] = log(aug[piv c][e + a] / aug[piv c][c])
__global__ void __launch_bounds__(256) k_dec16_gj_final(BigArgs A) {
    const BigArgs a = view(A, blockIdx.z);
    const uint32_t e = a.w.st->e;
    if (*a.status != QF_OK) return;
    const uint64_t ld = 2 * a.e_max;
    const uint64_t total = (uint64_t)e * e;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t c = (uint32_t)(t / e), r = (uint32_t)(t % e);
        const uint32_t p = a.w.pivrow[c];
        const uint32_t v = a.w.aug[p * ld + e + r];
        a.w.dlog[(uint64_t)c * a.e_max + r] =
            (uint16_t)(v ? lmod((int64_t)a.log[v] - a.log[a.w.aug[p * ld + c]]) : kNoLog);
    }
}


int grid16(qf_ctx* ctx, uint64_t units) {
    const uint64_t want = (units + kThreads16 - 1) / kThreads16;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)qf::ctx_num_cus(ctx)));
}

#define QF_HIP(x) QF_CHECK_HIP(x)

}  // namespace

extern "C" {

uint16_t qf_gf16_mul(uint16_t a, uint16_t b) { return h_mul(a, b); }

int qf_gf16_inv(uint16_t a, uint16_t* out) {
    if (!out) return QF_EINVAL;
    return h_inv(a, out) ? QF_OK : QF_ERANGE;
}

int qf_cauchy16_coeffs(uint32_t k, uint32_t r, uint16_t* out_rxk) {
    if (!out_rxk || k == 0) return QF_EINVAL;
    for (uint32_t j = 0; j < r; ++j) {
        const uint16_t y = (uint16_t)(k + j);
        for (uint32_t i = 0; i < k; ++i)
            if (!h_inv((uint16_t)((uint16_t)i ^ y), &out_rxk[(size_t)j * k + i])) return QF_ERANGE;
    }
    return QF_OK;
}

namespace {

std::vector<uint16_t> host_log16() {
    std::vector<uint16_t> lg(65536, (uint16_t)kNoLog);
    uint32_t x = 1;
    for (uint32_t i = 0; i < kOrder; ++i) {
        lg[x] = (uint16_t)i;
        x <<= 1;
        if (x & 0x10000u) x ^= 0x1100Bu;
    }
    return lg;
}

// lanes for 4 waves per SIMD: fewer lanes than this split the inputs
uint64_t matvec_lanes_wanted(qf_ctx* ctx) { return (uint64_t)qf::ctx_num_cus(ctx) * 4 * 4 * 64; }

constexpr size_t kShapeBytes = 256;   // Mv16Shape at the end of the split workspace

// bytes of split slabs (+ the shape record) launch_matvec wants for G
// generations (0: no split)
size_t matvec_acc_bytes(qf_ctx* ctx, uint64_t G, uint32_t nout, uint32_t nin, uint32_t L) {
    const uint64_t lanes = G * ((nout + kR16 - 1) / kR16) * ((L + 15) / 16);
    if (lanes >= matvec_lanes_wanted(ctx) || nin < 64) return 0;
    const uint32_t ns = matvec_split(lanes, nin, matvec_lanes_wanted(ctx));
    return ns > 1 ? (size_t)ns * G * nout * (((size_t)L + 15) / 16 * 16) + kShapeBytes : 0;
}

// acc: acc_bytes of workspace for split slabs (matvec_acc_bytes; null: never
// split).  With per-generation sizes on the device (nout_g / nin_g, the
// decode) and a split workspace, k_shape16 sizes the launch from the largest
// e_g instead of e_max: a window decode with e = 512 of e_max = 1,024 ran
// three quarters of its lanes idle at the e_max shape.
int launch_matvec(qf_ctx* ctx, hipStream_t st, Mv16Args& a, uint64_t G, const char* name, uint8_t* acc = nullptr,
                  size_t acc_bytes = 0, bool logify_ok = true) {
    if (!a.nin_gs) a.nin_gs = 1;
    a.Lu = (a.L + 15) / 16;
    a.nob = (a.nout + kR16 - 1) / kR16;
    const uint64_t lanes = G * a.nob * a.Lu;
    if (!lanes || !a.nin) return QF_OK;
    // enough lanes for 4 waves per SIMD, input chunks of at least 16 rows
    const uint64_t want = matvec_lanes_wanted(ctx);
    const uint64_t slab = G * a.nout * a.Lu * 4;   // dwords
    const uint64_t ns_cap = acc && acc_bytes > kShapeBytes ? (acc_bytes - kShapeBytes) / (4 * slab) : 0;
    uint32_t ns = acc && lanes < want ? matvec_split(lanes, a.nin, want) : 1;
    ns = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(ns, ns_cap));
    // QF_OPT_GF16_DYN 0: size split launches from e_max on the host
    const bool dyn = acc && ns_cap >= 1 && (a.nout_g || a.nin_g) && qf::ctx_opt(ctx, QF_OPT_GF16_DYN);
    a.shape = dyn ? reinterpret_cast<Mv16Shape*>(acc + acc_bytes - kShapeBytes) : nullptr;
    a.G = G;
    a.want = want;
    a.ns_cap = (uint32_t)std::min<uint64_t>(ns_cap, 1024);
    a.nsplit = ns;
    a.kchunk = (a.nin + ns - 1) / ns;
    a.acc_ws = reinterpret_cast<uint32_t*>(acc);
    a.slab = slab;
    a.total_units = lanes * ns;
    // inputs feeding >= kLogifyBlocks blocks of outputs, or a batch of at
    // least kLogifyUnits input units, go to log form once: k_logify16 looks
    // the logs up in LDS, the matvec would gather them from global memory
    // (QF_GF16_LOGIFY=0: gather in the matvec; QF_GF16_LOGIFY_MIN_BLOCKS
    // overrides kLogifyBlocks)
    a.in_log = 0;
    {
        const uint32_t min_blocks = (uint32_t)qf::ctx_opt(ctx, QF_OPT_GF16_LOGIFY_MIN_BLOCKS);
        const uint64_t n = G * a.nin * a.Lu;
        if (logify_ok && qf::ctx_opt(ctx, QF_OPT_GF16_LOGIFY) && (a.nob >= min_blocks || n >= kLogifyUnits)) {
            uint8_t* lr = nullptr;
            int s = qf::ctx_gf16_logrows(ctx, n * 16, &lr);
            if (s) return s;
            hipEvent_t ev0 = qf::ctx_prof_begin(ctx, st);
            hipLaunchKernelGGL(k_logify16, dim3(grid16(ctx, n)), dim3(kThreads16), 0, st, a, G,
                               reinterpret_cast<uint16_t*>(lr));
            QF_HIP(hipGetLastError());
            qf::ctx_prof_end(ctx, st, ev0, "k_logify16");
            a.in = lr;
            a.igs = (uint64_t)a.nin * a.Lu * 16;
            a.irs = (uint64_t)a.Lu * 16;
            a.isel = nullptr;
            a.isel_gs = 0;
            a.in_log = 1;
        }
    }
    hipEvent_t ev = qf::ctx_prof_begin(ctx, st);
    if (dyn) hipLaunchKernelGGL(k_shape16, dim3(1), dim3(1024), 0, st, a);
    const int grid = dyn ? qf::ctx_num_cus(ctx) : grid16(ctx, a.total_units);
    hipLaunchKernelGGL(k_matvec16, dim3(grid), dim3(kThreads16), 0, st, a);
    QF_HIP(hipGetLastError());
    if (ns > 1 || dyn) {
        const uint64_t n = G * a.nout * a.Lu;
        hipLaunchKernelGGL(k_finish16, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, st, a);
        QF_HIP(hipGetLastError());
    }
    qf::ctx_prof_end(ctx, st, ev, name);
    return QF_OK;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

}  // extern "C"

namespace qf {

int encode16_window(qf_ctx* ctx, const qf_encode_shape* sh, uint32_t G, const uint8_t* src, uint8_t* rep,
                    const uint16_t* coeff_rxk, uint32_t first, uint32_t rot, uint8_t* coeff_be_dev) {
    if (!ctx || !sh) return QF_EINVAL;
    const uint32_t k = sh->k, r = sh->r, L = sh->L;
    if (k == 0 || k > 65535 || (L & 1) || sh->flags) return QF_EINVAL;
    if (G == 0 || r == 0 || L == 0) return QF_OK;
    if (!src || !rep || (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(rep) & 15) ||
        (sh->src_row_stride & 15) || (sh->src_gen_stride & 15) || (sh->rep_row_stride & 15) ||
        (sh->rep_gen_stride & 15))
        return QF_EINVAL;
    if (!coeff_rxk && (uint64_t)k + first + r > 65536) return QF_ERANGE;  // gf16_inv(0) in the Cauchy rows
    if (rot >= k || (coeff_rxk && (first || rot || coeff_be_dev))) return QF_EINVAL;
    std::unique_lock<std::mutex> lk;
    int s = qf::ctx_lock(ctx, lk);
    if (s) return s;
    hipStream_t st = qf::ctx_stream(ctx);
    // the reference's fixed Cauchy rows over an unrotated window: the
    // bit-sliced kernel of (k, r) if one is generated (qf_gf16_bs.hip)
    if (!coeff_rxk && !first && !rot && !coeff_be_dev && qf::ctx_opt(ctx, QF_OPT_GF16_BITSLICED)) {
        // the bit-sliced kernel reads a partial last unit (L % 16 != 0) as a
        // whole 16 B: up to 15 bytes past L.  Only the batch's last row can
        // end its buffer, so the last generation takes the general path below
        const uint32_t Gb = L % 16 ? G - 1 : G;
        s = Gb ? qf::gf16_bs_encode(ctx, st, k, r, L, Gb, src, sh->src_gen_stride, sh->src_row_stride, rep,
                                    sh->rep_gen_stride, sh->rep_row_stride)
               : (qf::gf16_bs_has(k, r) ? QF_OK : qf::kGf16BsNone);
        if (s != qf::kGf16BsNone) {
            if (s != QF_OK || Gb == G) return s;
            src += (size_t)Gb * sh->src_gen_stride;
            rep += (size_t)Gb * sh->rep_gen_stride;
            G = 1;
        }
    }
    const uint16_t *glog, *gexp;
    s = qf::ctx_gf16_tables(ctx, &glog, &gexp);
    if (s) return s;
    // power-of-two windows: the additive FFT (qf_gf16_fft.hip), O(k log k)
    // products per column instead of k r
    const int64_t fft_opt = qf::ctx_opt(ctx, QF_OPT_GF16_FFT);
    if (!coeff_rxk && fft_opt && qf::gf16_fft_has(k, r, first) &&
        (fft_opt == 2 || qf::gf16_fft_pays(k, r, first + r))) {
        const size_t fb = align256(2 * (3ull * k)), mb = coeff_be_dev ? align256((size_t)r * k * 2) : 0;
        uint8_t* w;
        s = qf::ctx_work(ctx, fb + mb, &w);
        if (s) return s;
        if (coeff_be_dev) {   // the repairs' coefficient blocks (framing)
            const uint64_t n = (uint64_t)r * k;
            hipLaunchKernelGGL(k_cauchy16_logs, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256),
                               0, st, reinterpret_cast<uint16_t*>(w + fb), k, r, first, rot, glog, gexp, coeff_be_dev);
            QF_HIP(hipGetLastError());
        }
        s = qf::gf16_fft_encode(ctx, st, k, r, first, rot, L, G, src, sh->src_gen_stride, sh->src_row_stride, rep,
                                sh->rep_gen_stride, sh->rep_row_stride, glog, gexp, w);
        if (s != qf::kGf16BsNone) return s;
    }
    const size_t cb = align256((size_t)r * k * 2), ab = matvec_acc_bytes(ctx, G, r, k, L);
    uint8_t* w;
    s = qf::ctx_work(ctx, cb + ab, &w);
    if (s) return s;
    if (coeff_rxk) {
        // coefficient logs (host tables: the same field); the upload reads
        // host memory, so the call finishes before returning
        static const std::vector<uint16_t> lg = host_log16();
        std::vector<uint16_t> c((size_t)r * k);
        for (size_t q = 0; q < c.size(); ++q) c[q] = lg[coeff_rxk[q]];
        QF_HIP(hipMemcpyAsync(w, c.data(), c.size() * 2, hipMemcpyHostToDevice, st));
        QF_HIP(hipStreamSynchronize(st));
    } else {
        const uint64_t n = (uint64_t)r * k;
        hipLaunchKernelGGL(k_cauchy16_logs, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                           reinterpret_cast<uint16_t*>(w), k, r, first, rot, glog, gexp, coeff_be_dev);
        QF_HIP(hipGetLastError());
    }
    Mv16Args a{};
    a.in = src;
    a.igs = sh->src_gen_stride;
    a.irs = sh->src_row_stride;
    a.out = rep;
    a.ogs = sh->rep_gen_stride;
    a.ors = sh->rep_row_stride;
    a.m = reinterpret_cast<const uint16_t*>(w);
    a.mrs = k;
    a.log = glog;
    a.exp = gexp;
    a.nout = r;
    a.nin = k;
    a.L = L;
    return launch_matvec(ctx, st, a, G, "k_encode16", ab ? w + cb : nullptr, ab);
}

}  // namespace qf

extern "C" {

int qf_encode16_batch(qf_ctx* ctx, const qf_encode_shape* sh, uint32_t G, const uint8_t* src, uint8_t* rep,
                      const uint16_t* coeff_rxk) {
    return qf::encode16_window(ctx, sh, G, src, rep, coeff_rxk, 0, 0, nullptr);
}

int qf_decode16_batch(qf_ctx* ctx, const qf_decode_shape* sh, uint32_t G, const uint8_t* rows,
                      const uint16_t* row_index, const uint32_t* n_rows, const uint16_t* row_coeffs, uint8_t* rec,
                      uint16_t* rec_index, uint32_t* n_rec, int32_t* status) {
    if (!ctx || !sh) return QF_EINVAL;
    const uint32_t k = sh->k, r = sh->r, L = sh->L, max_rows = sh->max_rows;
    const uint32_t e_max = std::min(k, r);
    // r sizes the recovered rows (e <= min(k, r)); r = 0 leaves nothing to solve with
    if (k == 0 || r == 0 || k > 4096 || (L & 1) || max_rows == 0 || max_rows > 65536) return QF_EINVAL;
    if (G == 0) return QF_OK;
    if (!rows || !row_index || !n_rec || !status || !rec || !rec_index) return QF_EINVAL;
    if ((reinterpret_cast<uintptr_t>(rows) & 15) || (sh->row_stride & 15) || (sh->rows_gen_stride & 15) ||
        (reinterpret_cast<uintptr_t>(rec) & 15) || (sh->rec_row_stride & 15) || (sh->rec_gen_stride & 15))
        return QF_EINVAL;
    std::unique_lock<std::mutex> lk;
    int s = qf::ctx_lock(ctx, lk);
    if (s) return s;
    const uint16_t *glog, *gexp;
    s = qf::ctx_gf16_tables(ctx, &glog, &gexp);
    if (s) return s;
    hipStream_t st = qf::ctx_stream(ctx);
    const uint32_t ew = std::max<uint32_t>(e_max, 1);
    uint8_t* w;
    // QF_GF16_LDS_GJ=1: the all-generations-at-once Gauss-Jordan in LDS
    // (W = C[J,E]^-1 [I | C[J,S]] over every slot) for e_max <= 64; default:
    // the syndrome path below for every shape
    if (e_max <= kEMax && qf::ctx_opt(ctx, QF_OPT_GF16_LDS_GJ)) {
        // small path: every generation at once
        const size_t wb = align256((size_t)G * ew * k * 2), ab = matvec_acc_bytes(ctx, G, e_max, k, L);
        s = qf::ctx_work(ctx, wb + ab, &w);
        if (s) return s;
        Dec16Args d{};
        d.row_index = row_index;
        d.n_rows = n_rows;
        d.row_coeffs = row_coeffs;
        d.log = glog;
        d.exp = gexp;
        d.wl = reinterpret_cast<uint16_t*>(w);
        d.n_out = n_rec;
        d.rec_index = rec_index;
        d.status = status;
        d.k = k;
        d.r = r;
        d.e_max = ew;
        d.max_rows = max_rows;
        hipEvent_t ev = qf::ctx_prof_begin(ctx, st);
        hipLaunchKernelGGL(k_decode16_prepare, dim3(G), dim3(256), 0, st, d);
        QF_HIP(hipGetLastError());
        qf::ctx_prof_end(ctx, st, ev, "k_decode16_prepare");
        Mv16Args c{};
        c.in = rows;
        c.igs = sh->rows_gen_stride;
        c.irs = sh->row_stride;
        c.out = rec;
        c.ogs = sh->rec_gen_stride;
        c.ors = sh->rec_row_stride;
        c.m = d.wl;
        c.mgs = (uint64_t)ew * k;
        c.mrs = k;
        c.nout_g = n_rec;
        c.log = glog;
        c.exp = gexp;
        c.nout = e_max;
        c.nin = k;
        c.L = L;
        return launch_matvec(ctx, st, c, G, "k_combine16", ab ? w + wb : nullptr, ab);
    }
    // syndrome path: chunks of generations (grid z = generation), syndromes
    // s = p_J ^ C[J,S] x_S, then x_E = C[J,E]^-1 s with the inverse in closed
    // form (Cauchy rows) or by Gauss-Jordan in the workspace
    const size_t Lp = ((size_t)L + 15) / 16 * 16;
    const uint64_t em = e_max;
    // Cauchy rows of a (k, r) with a generated bit-sliced kernel: syndromes
    // from qf_gf16bs_syn_* (maps 13..17, zero row), the general matvec only
    // for the generations it skips
    // (L % 16 != 0: the bit-sliced syndrome kernel reads whole 16-B units, up
    // to 15 bytes past the last row; the other syndrome paths read bytewise)
    const bool bs = !row_coeffs && r <= 64 && L % 16 == 0 && qf::ctx_opt(ctx, QF_OPT_GF16_BITSLICED) &&
                    qf::gf16_bs_has(k, r);
    // power-of-two k without one: the additive-FFT syndromes (qf_gf16_fft.hip)
    // over the same maps, constants in workspace slab 20
    const int64_t fft_opt = qf::ctx_opt(ctx, QF_OPT_GF16_FFT);
    const bool fft = !bs && !row_coeffs && fft_opt && qf::gf16_fft_has(k, r, 0) &&
                     (fft_opt == 2 || qf::gf16_fft_pays(k, e_max, r));
    const bool maps = bs || fft;
    const size_t per_gen[19] = {sizeof(Dec16State), 2 * em, 2 * em, 2 * em, 2ull * k, 2ull * k, 2 * em * k, 2 * em * em,
                                row_coeffs ? 4 * em * em : 0, 4 * em, 4 * em, 16 * em, Lp * em,
                                maps ? 2ull * k : 0, maps ? 2ull * r : 0, maps ? 2ull * r : 0, maps ? 4u : 0u,
                                maps ? 4u : 0u, fft ? 4u : 0u};
    size_t gen_bytes = 0;
    for (int q = 0; q < 19; ++q) gen_bytes += per_gen[q];
    // chunk: <= 65535 generations (grid z) and about 1 GiB of workspace
    const uint32_t chunk = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)G, 65535ull,
                                                                             (1ull << 30) / gen_bytes}));
    size_t off[22], tot = 0;
    for (int q = 0; q < 19; ++q) {
        off[q] = tot;
        tot += align256(std::max<size_t>(per_gen[q] * chunk, 1));
    }
    const size_t acc_bytes = std::max(matvec_acc_bytes(ctx, chunk, e_max, k, L),
                                      matvec_acc_bytes(ctx, chunk, e_max, e_max, L));
    off[19] = tot;
    tot += align256(std::max<size_t>(acc_bytes, 1));
    const size_t zero_bytes = bs ? align256(64 * ((((size_t)L + 15) / 16 + 3) / 4) + 64) : 0;
    off[20] = tot;
    tot += zero_bytes;
    off[21] = tot;
    tot += fft ? align256(2 * (3ull * k)) : 0;
    s = qf::ctx_work(ctx, tot, &w);
    if (s) return s;
    if (bs) QF_HIP(hipMemsetAsync(w + off[20], 0, zero_bytes, st));
    BigArgs b{};
    b.w.st = reinterpret_cast<Dec16State*>(w + off[0]);
    b.w.J = reinterpret_cast<uint16_t*>(w + off[1]);
    b.w.Jslot = reinterpret_cast<uint16_t*>(w + off[2]);
    b.w.E = reinterpret_cast<uint16_t*>(w + off[3]);
    b.w.Sslot = reinterpret_cast<uint16_t*>(w + off[4]);
    b.w.Scol = reinterpret_cast<uint16_t*>(w + off[5]);
    b.w.mlog = reinterpret_cast<uint16_t*>(w + off[6]);
    b.w.dlog = reinterpret_cast<uint16_t*>(w + off[7]);
    b.w.aug = row_coeffs ? reinterpret_cast<uint16_t*>(w + off[8]) : nullptr;
    b.w.mark = reinterpret_cast<uint32_t*>(w + off[9]);
    b.w.pivrow = reinterpret_cast<uint32_t*>(w + off[10]);
    b.w.lprod = reinterpret_cast<uint32_t*>(w + off[11]);
    b.w.synd = w + off[12];
    b.log = glog;
    b.exp = gexp;
    b.k = k;
    b.e_max = e_max;
    b.n_rows = max_rows;
    b.Lp = Lp;
    uint8_t* acc = acc_bytes ? w + off[19] : nullptr;
    const int cus = qf::ctx_num_cus(ctx);
    const uint32_t mgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((em * k + 255) / 256, 8ull * cus / 1));
    const uint32_t dgrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((em * em + 255) / 256, 8ull * cus));
    for (uint32_t g0 = 0; g0 < G; g0 += chunk) {
        const uint32_t gc = std::min(chunk, G - g0);
        b.row_index = row_index + (size_t)g0 * max_rows;
        b.n_rows_dev = n_rows ? n_rows + g0 : nullptr;
        b.row_coeffs = row_coeffs ? row_coeffs + (size_t)g0 * max_rows * k : nullptr;
        b.n_out = n_rec + g0;
        b.rec_index = rec_index + (size_t)g0 * e_max;
        b.status = status + g0;
        hipEvent_t ev = qf::ctx_prof_begin(ctx, st);
        uint32_t acc_threads = 64;
        while (acc_threads * 4 < k) acc_threads <<= 1;
        hipLaunchKernelGGL(k_dec16_accept, dim3(1, 1, gc), dim3(acc_threads), 0, st, b);
        // the maps of the bit-sliced / FFT syndrome kernels; the matvec's
        // coefficient logs then only for the generations those skip
        uint16_t* smap = reinterpret_cast<uint16_t*>(w + off[13]);
        uint16_t* rpos = reinterpret_cast<uint16_t*>(w + off[14]);
        uint16_t* rslot = reinterpret_cast<uint16_t*>(w + off[15]);
        uint32_t* skip = reinterpret_cast<uint32_t*>(w + off[16]);
        uint32_t* nout_fb = maps ? reinterpret_cast<uint32_t*>(w + off[17]) : nullptr;
        uint32_t* solve_fb = fft ? reinterpret_cast<uint32_t*>(w + off[18]) : nullptr;
        if (maps)
            hipLaunchKernelGGL(k_dec16_bsmaps, dim3(1, 1, gc), dim3(64), 0, st, b, r, smap, rpos, rslot, skip, nout_fb,
                               solve_fb);
        hipLaunchKernelGGL(k_dec16_synmat, dim3(mgrid, 1, gc), dim3(256), 0, st, b, nout_fb);
        if (!row_coeffs) {
            if (e_max <= 64) {
                hipLaunchKernelGGL(k_dec16_cauchy_small, dim3(1, 1, gc), dim3(128), 0, st, b, solve_fb);
            } else {
                uint32_t prod_threads = 64;
                while (prod_threads < e_max && prod_threads < 256) prod_threads <<= 1;
                hipLaunchKernelGGL(k_dec16_cauchy_prod, dim3(2 * e_max, 1, gc), dim3(prod_threads), 0, st, b);
                hipLaunchKernelGGL(k_dec16_cauchy_inv, dim3(dgrid, 1, gc), dim3(256), 0, st, b, solve_fb);
            }
        } else {
            hipLaunchKernelGGL(k_dec16_gj_init,
                               dim3((uint32_t)std::min<uint64_t>((em * 2 * em + 255) / 256, 8ull * cus), 1, gc),
                               dim3(256), 0, st, b);
            // the erasure counts are on the device: launch for e_max columns,
            // the steps past a generation's e return at once
            for (uint32_t c = 0; c < e_max; ++c) {
                hipLaunchKernelGGL(k_dec16_gj_pivot, dim3(1, 1, gc), dim3(1024), 0, st, b, c);
                hipLaunchKernelGGL(k_dec16_gj_step, dim3((2 * e_max - c + 255) / 256, e_max, gc), dim3(256), 0, st,
                                   b, c);
            }
            hipLaunchKernelGGL(k_dec16_gj_final, dim3(dgrid, 1, gc), dim3(256), 0, st, b);
        }
        QF_HIP(hipGetLastError());
        qf::ctx_prof_end(ctx, st, ev, "k_dec16_prepare_large");
        // syndromes s_a = row(J_a) ^ C[J_a, S] x_S
        if (bs) {
            s = qf::gf16_bs_syndromes(ctx, st, k, r, L, gc, rows + (size_t)g0 * sh->rows_gen_stride,
                                      sh->rows_gen_stride, sh->row_stride, smap, k, rpos, rslot, skip, w + off[20],
                                      b.w.synd, em * Lp, Lp);
            if (s) return s;
        } else if (fft) {
            s = qf::gf16_fft_syndromes(ctx, st, k, r, L, gc, rows + (size_t)g0 * sh->rows_gen_stride,
                                       sh->rows_gen_stride, sh->row_stride, smap, rpos, rslot, skip, b.w.synd, em * Lp,
                                       Lp, glog, gexp, w + off[21]);
            if (s) return s;
        }
        Mv16Args sy{};
        sy.in = rows + (size_t)g0 * sh->rows_gen_stride;
        sy.igs = sh->rows_gen_stride;
        sy.irs = sh->row_stride;
        sy.isel = b.w.Sslot;
        sy.isel_gs = k;
        sy.base = sy.in;
        sy.bgs = sh->rows_gen_stride;
        sy.brs = sh->row_stride;
        sy.bsel = b.w.Jslot;
        sy.bsel_gs = e_max;
        sy.out = b.w.synd;
        sy.ogs = em * Lp;
        sy.ors = Lp;
        sy.m = b.w.mlog;
        sy.mgs = em * k;
        sy.mrs = k;
        // (bs: only the generations the bit-sliced kernel skipped, rows gathered
        // as symbols: no logify pass over the whole batch)
        sy.nout_g = maps ? nout_fb : n_rec + g0;
        sy.nin_g = &b.w.st->nin;
        sy.nin_gs = sizeof(Dec16State) / 4;
        sy.log = glog;
        sy.exp = gexp;
        sy.nout = e_max;
        sy.nin = k;
        sy.L = L;
        s = launch_matvec(ctx, st, sy, gc, maps ? "k_syndromes16_fallback" : "k_syndromes16", acc, acc_bytes, !maps);
        if (s) return s;
        // x_E = C[J,E]^-1 s
        Mv16Args so{};
        so.in = b.w.synd;
        so.igs = em * Lp;
        so.irs = Lp;
        so.out = rec + (size_t)g0 * sh->rec_gen_stride;
        so.ogs = sh->rec_gen_stride;
        so.ors = sh->rec_row_stride;
        so.m = b.w.dlog;
        so.mgs = em * em;
        so.mrs = e_max;
        // x_E = D_b (C^T (D_a s))_E by the FFT for the Cauchy generations
        // (qf_gf16_fft.hip); the matvec for those with a repair index >= 2k
        if (fft) {
            s = qf::gf16_fft_solve(ctx, st, k, L, gc, b.w.synd, em * Lp, Lp, rec + (size_t)g0 * sh->rec_gen_stride,
                                   sh->rec_gen_stride, sh->rec_row_stride, reinterpret_cast<const uint32_t*>(b.w.st),
                                   sizeof(Dec16State) / 4, status + g0, b.w.J, b.w.E, b.w.lprod, em, solve_fb, glog,
                                   gexp, w + off[21]);
            if (s) return s;
        }
        so.nout_g = fft ? solve_fb : n_rec + g0;
        so.nin_g = n_rec + g0;
        so.log = glog;
        so.exp = gexp;
        so.nout = e_max;
        so.nin = e_max;
        so.L = L;
        s = launch_matvec(ctx, st, so, gc, fft ? "k_combine16_fallback" : "k_combine16", acc, acc_bytes, !fft);
        if (s) return s;
    }
    return QF_OK;
}

}  // extern "C"
