// qf_gf16_bs.hip -- bit-sliced GF(2^16) Cauchy encode (SURVEY 8(f) rank 3,
// Extreme mode's field) for the (k, r) shapes gf16_codegen.py generates.
//
// Encoder16 (decoder.rs:10-88) multiplies every source symbol by the fixed
// Cauchy coefficient C[j][i] = gf16_inv(i ^ (k + j)) (decoder.rs:77-80).  The
// general kernel (qf_gf16.hip, k_matvec16) forms each product as
// exp[log c + log x] with the exp table in LDS: one random 16-bit LDS read
// per symbol product, bound by bank conflicts.  Here each product by a fixed
// c is compiled into XORs of bit planes (gf16_codegen.py): a lane transposes
// its 64 bytes of a row (4 units of 16 B, 32 symbols) into 16 planes, forms
// the 15 combinations of each group of 4 planes, and adds at most 4 of them
// into each output plane.  8 repairs per pass; the passes of one lane-chunk
// block run on one XCD at about the same time (block mapping in the
// generated kernel), so the later passes re-read the rows from L2.
//
// Lane layout: lane-chunk f = G x Q, g = f / Q, q = f % Q, Q = ceil(Lu / 4);
// the lane owns units q, q + Q, q + 2Q, q + 3Q (< Lu) of row i of generation g,
// so each 16-B load instruction covers consecutive units of a row.  The last
// unit of a row with L % 16 != 0 is read whole (16-B aligned rows: the bytes
// past L stay inside the same aligned 16 B) and stored bytewise.  That read
// can pass the end of the caller's buffer only on the batch's last row, so
// the host never gives this kernel the last generation of such a batch
// (qf_encode16_batch: general path for it) and never runs the syndrome
// kernel at L % 16 != 0 (qf_gf16.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "qf_fec.h"
#include "qf_internal.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct Gf16BsArgs {
    const uint8_t* src;        // encode: sources; syn: the received rows (arrival order)
    uint8_t* rep;              // encode: repairs; syn: the syndrome rows (in accepted-repair order)
    uint64_t sgs, srs, rgs, rrs;
    uint64_t total;   // lane-chunks: G * Q
    uint32_t L, Lu, Q, tail;   // tail: L % 16 (bytes of the last unit; 0 = whole)
    // syn only (per generation g, built by k_dec16_bsmaps in qf_gf16.hip)
    const uint16_t* smap;      // [g][smap_gs]: slot of source i (0xFFFF: not received)
    const uint16_t* rpos;      // [g][r]: position a of accepted repair k + j (0xFFFF: none)
    const uint16_t* rslot;     // [g][r]: its slot
    const uint32_t* skip;      // [g]: nonzero = not this kernel's generation
    const uint8_t* zero;       // >= 64 Q zero bytes (the row of a source not received)
    uint64_t smap_gs;
    uint32_t r;
};

struct Gf16BsLane {
    uint64_t g;
    const uint8_t* s;   // unit q of row 0 of the lane's generation
    uint8_t* d;
    const uint8_t* z;   // unit q of the zero row
    uint64_t hq;        // 16 Q: byte distance between the lane's units
    uint32_t off[4];    // load offset of unit h (h 16 Q, or 0 past the row)
    uint32_t valid;     // bit h: unit q + h Q < Lu
    uint32_t tailh;     // bit h: unit q + h Q is the partial last unit
};

__device__ __forceinline__ Gf16BsLane gf16bs_lane(const Gf16BsArgs& a, uint64_t f) {
    Gf16BsLane ln;
    const uint64_t g = f / a.Q;
    const uint32_t q = (uint32_t)(f - g * a.Q);
    ln.g = g;
    ln.s = a.src + g * a.sgs + 16ull * q;
    ln.d = a.rep + g * a.rgs + 16ull * q;
    ln.z = a.zero + 16ull * q;
    ln.hq = 16ull * a.Q;
    ln.valid = 0;
    ln.tailh = 0;
#pragma unroll
    for (uint32_t h = 0; h < 4; ++h) {
        const uint32_t u = q + h * a.Q;
        if (u < a.Lu) ln.valid |= 1u << h;
        ln.off[h] = u < a.Lu ? 16u * h * a.Q : 0u;
        if (a.tail && u == a.Lu - 1) ln.tailh |= 1u << h;
    }
    return ln;
}

// transpose masks in VGPRs (an SGPR operand halves the issue rate of 3-source
// VALU ops, DESIGN 3.2 "Operand classes")
__device__ __forceinline__ void gf16bs_masks(uint32_t (&tm)[4]) {
    asm volatile("v_mov_b32 %0, %1" : "=v"(tm[0]) : "s"(0x55555555u));
    asm volatile("v_mov_b32 %0, %1" : "=v"(tm[1]) : "s"(0x33333333u));
    asm volatile("v_mov_b32 %0, %1" : "=v"(tm[2]) : "s"(0x0F0F0F0Fu));
    asm volatile("v_mov_b32 %0, %1" : "=v"(tm[3]) : "s"(0x00FF00FFu));
}

// The bit-plane operations as v_bitop3 intrinsics: the compiler allocates
// registers, schedules and checks hazards, but does not split, merge or
// reassociate them (from plain C expressions it produced 40 % more
// instructions, and opaque inline asm made it pad them with s_nop).
__device__ __forceinline__ uint32_t bs_bfi(uint32_t m, uint32_t x, uint32_t y) {   // (x & m) | (y & ~m)
    return __builtin_amdgcn_bitop3_b32(m, x, y, 0xca);
}

// a ^ b ^ c (gfx950 has no v_xor3_b32: v_bitop3 0x96)
__device__ __forceinline__ uint32_t bs_xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t bs_xor(uint32_t a, uint32_t b) { return a ^ b; }

template <int S>
__device__ __forceinline__ uint32_t bs_shl(uint32_t a) {
    return a << S;
}

template <int S>
__device__ __forceinline__ uint32_t bs_shr(uint32_t a) {
    return a >> S;
}

// stage i of the involution swaps row bit i with column bit i
// (gf16_codegen.transpose16): per pair 2 shifts + 2 bit-selects (v_bitop3
// 0xca with the mask in a VGPR: full rate)
template <int I>
__device__ __forceinline__ void gf16bs_stage(uint32_t (&x)[16], uint32_t m) {
    constexpr int s = 1 << I;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if (r & s) continue;
        const uint32_t a = x[r], b = x[r + s];
        x[r] = bs_bfi(m, a, bs_shl<s>(b));
        x[r + s] = bs_bfi(m, bs_shr<s>(a), b);
    }
}

__device__ __forceinline__ void gf16bs_transpose(uint32_t (&x)[16], const uint32_t (&tm)[4]) {
    gf16bs_stage<0>(x, tm[0]);
    gf16bs_stage<1>(x, tm[1]);
    gf16bs_stage<2>(x, tm[2]);
    gf16bs_stage<3>(x, tm[3]);
}

__device__ __forceinline__ void gf16bs_load_row(const Gf16BsArgs& a, const Gf16BsLane& ln, uint32_t i,
                                                uint32_t (&x)[16]) {
    // no branch around the loads (exact vmcnt tracking): a unit past the row
    // (q + h Q >= Lu) reads unit q instead; its symbols are independent of the
    // others' and its outputs are never stored
    const uint8_t* p = ln.s + (uint64_t)i * a.srs;
#pragma unroll
    for (uint32_t h = 0; h < 4; ++h) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + ln.off[h]));
        x[4 * h] = v.x;
        x[4 * h + 1] = v.y;
        x[4 * h + 2] = v.z;
        x[4 * h + 3] = v.w;
    }
}

__device__ __forceinline__ void gf16bs_store_row(const Gf16BsArgs& a, const Gf16BsLane& ln, uint32_t j,
                                                 const uint32_t (&x)[16]) {
    uint8_t* p = ln.d + (uint64_t)j * a.rrs;
#pragma unroll
    for (uint32_t h = 0; h < 4; ++h) {
        if (!(ln.valid >> h & 1)) continue;
        uint8_t* q = p + h * ln.hq;
        if (ln.tailh >> h & 1) {
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b)
                if (b < a.tail) q[b] = (uint8_t)(x[4 * h + (b >> 2)] >> (8 * (b & 3)));
        } else {
            const u32x4 v = {x[4 * h], x[4 * h + 1], x[4 * h + 2], x[4 * h + 3]};
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(q));
        }
    }
}

// syn: source row at slot `slot` of the lane's generation, or the zero row
__device__ __forceinline__ void gf16bs_load_row_sel(const Gf16BsArgs& a, const Gf16BsLane& ln, uint32_t slot,
                                                    uint32_t (&x)[16]) {
    const uint8_t* p = slot == 0xFFFFu ? ln.z : ln.s + (uint64_t)slot * a.srs;
#pragma unroll
    for (uint32_t h = 0; h < 4; ++h) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + ln.off[h]));
        x[4 * h] = v.x;
        x[4 * h + 1] = v.y;
        x[4 * h + 2] = v.z;
        x[4 * h + 3] = v.w;
    }
}

// syn: C[j, S] x_S of repair j -> syndrome a = that ^ the accepted row of
// repair k + j (whole units: the syndrome rows are padded to 16 B)
__device__ __forceinline__ void gf16bs_store_syn(const Gf16BsArgs& a, const Gf16BsLane& ln, uint32_t j,
                                                 const uint32_t (&x)[16]) {
    const uint32_t pos = a.rpos[ln.g * a.r + j];
    if (pos == 0xFFFFu) return;
    const uint8_t* p = ln.s + (uint64_t)a.rslot[ln.g * a.r + j] * a.srs;
    uint8_t* o = ln.d + (uint64_t)pos * a.rrs;
#pragma unroll
    for (uint32_t h = 0; h < 4; ++h) {
        if (!(ln.valid >> h & 1)) continue;
        const u32x4 v = *reinterpret_cast<const u32x4*>(p + ln.off[h]);
        const u32x4 w = {x[4 * h] ^ v.x, x[4 * h + 1] ^ v.y, x[4 * h + 2] ^ v.z, x[4 * h + 3] ^ v.w};
        *reinterpret_cast<u32x4*>(o + ln.off[h]) = w;
    }
}

typedef void (*Gf16BsKernel)(Gf16BsArgs);

struct Gf16BsEntry {
    uint32_t k, r, passes;
    Gf16BsKernel fn;
    const char* name;
    Gf16BsKernel syn;
    const char* syn_name;
};

#include "qf_gf16_bs.inc"

}  // namespace

namespace qf {

// kGf16BsNone (> 0) when no generated kernel exists for (k, r): the caller
// takes the general path.
int gf16_bs_encode(qf_ctx* ctx, hipStream_t st, uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t* src,
                   uint64_t sgs, uint64_t srs, uint8_t* rep, uint64_t rgs, uint64_t rrs) {
    const Gf16BsEntry* e = nullptr;
    for (const auto& t : kGf16BsTable)
        if (t.k == k && t.r == r) e = &t;
    if (!e) return kGf16BsNone;
    Gf16BsArgs a{};
    a.src = src;
    a.rep = rep;
    a.sgs = sgs;
    a.srs = srs;
    a.rgs = rgs;
    a.rrs = rrs;
    a.L = L;
    a.Lu = (L + 15) / 16;
    a.Q = (a.Lu + 3) / 4;
    a.tail = L % 16;
    a.total = (uint64_t)G * a.Q;
    const uint64_t blocks = (a.total + 255) / 256;
    const uint64_t grid = (blocks + 7) / 8 * 8 * e->passes;
    if (grid > 0x7FFFFFFFull) return QF_ERANGE;
    hipEvent_t ev = ctx_prof_begin(ctx, st);
    hipLaunchKernelGGL(e->fn, dim3((uint32_t)grid), dim3(256), 0, st, a);
    QF_CHECK_HIP(hipGetLastError());
    ctx_prof_end(ctx, st, ev, e->name);
    return QF_OK;
}

bool gf16_bs_has(uint32_t k, uint32_t r) {
    for (const auto& t : kGf16BsTable)
        if (t.k == k && t.r == r) return true;
    return false;
}

int gf16_bs_syndromes(qf_ctx* ctx, hipStream_t st, uint32_t k, uint32_t r, uint32_t L, uint32_t G,
                      const uint8_t* rows, uint64_t rgs, uint64_t rs, const uint16_t* smap, uint64_t smap_gs,
                      const uint16_t* rpos, const uint16_t* rslot, const uint32_t* skip, const uint8_t* zero,
                      uint8_t* synd, uint64_t synd_gs, uint64_t synd_rs) {
    const Gf16BsEntry* e = nullptr;
    for (const auto& t : kGf16BsTable)
        if (t.k == k && t.r == r) e = &t;
    if (!e) return kGf16BsNone;
    Gf16BsArgs a{};
    a.src = rows;
    a.rep = synd;
    a.sgs = rgs;
    a.srs = rs;
    a.rgs = synd_gs;
    a.rrs = synd_rs;
    a.L = L;
    a.Lu = (L + 15) / 16;
    a.Q = (a.Lu + 3) / 4;
    a.tail = 0;   // syndrome rows are padded: whole units
    a.total = (uint64_t)G * a.Q;
    a.smap = smap;
    a.rpos = rpos;
    a.rslot = rslot;
    a.skip = skip;
    a.zero = zero;
    a.smap_gs = smap_gs;
    a.r = r;
    const uint64_t blocks = (a.total + 255) / 256;
    const uint64_t grid = (blocks + 7) / 8 * 8 * e->passes;
    if (grid > 0x7FFFFFFFull) return QF_ERANGE;
    hipEvent_t ev = ctx_prof_begin(ctx, st);
    hipLaunchKernelGGL(e->syn, dim3((uint32_t)grid), dim3(256), 0, st, a);
    QF_CHECK_HIP(hipGetLastError());
    ctx_prof_end(ctx, st, ev, e->syn_name);
    return QF_OK;
}

}  // namespace qf
