// gf256_tables.h -- GF(2^8) field tables and the split-index v_perm tables
// used by the MI355X kernels.  Host-side construction only; the kernels
// receive the tables through device memory / LDS.
//
// Field: polynomial 0x11D, generator 2, table semantics exactly as
// gf_tables.rs:384-408 (init_gf_tables) and gf_tables.rs:47-57 (gf_mul_table).
//
// v_perm split tables (the core of the encode/decode kernels):
// a byte x is split as x = x0 + 8*x1 + 64*x2 with x0, x1 in [0,8), x2 in [0,4).
// Because multiplication by a fixed c is GF(2)-linear,
//     c*x = T0[x0] ^ T1[x1] ^ T2[x2],
//     T0[v] = c*v, T1[v] = c*(v<<3), T2[v] = c*(v<<6).
// T0/T1 are 8-byte tables (two dwords: lo = entries 0..3, hi = 4..7) and T2 a
// 4-byte table (one dword).  v_perm_b32(hi, lo, sel) returns, for each byte
// of sel in 0..7, the byte sel of {hi:lo}, i.e. four table lookups per
// instruction.  A packed record per coefficient value is 8 dwords:
//     { T0lo, T0hi, T1lo, T1hi, T2, 0, 0, 0 }.
#pragma once
#include <stdint.h>

namespace qf {

struct Gf256 {
    uint8_t exp[512];
    uint8_t log[256];
    Gf256() {
        for (int i = 0; i < 512; ++i) exp[i] = 0;
        for (int i = 0; i < 256; ++i) log[i] = 0;
        uint32_t x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            exp[i + 255] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x >= 256) x ^= 0x11D;
        }
    }
    uint8_t mul(uint8_t a, uint8_t b) const {
        if (a == 0 || b == 0) return 0;
        return exp[(uint32_t)log[a] + (uint32_t)log[b]];
    }
    // returns false for a == 0 (the reference panics)
    bool inv(uint8_t a, uint8_t* out) const {
        if (a == 0) return false;
        *out = exp[255 - log[a]];
        return true;
    }
};

const Gf256& gf();

inline uint32_t pack4(uint8_t a, uint8_t b, uint8_t c, uint8_t d) {
    return (uint32_t)a | ((uint32_t)b << 8) | ((uint32_t)c << 16) | ((uint32_t)d << 24);
}

// 8-dword split-table record for coefficient c.
inline void perm_record(uint8_t c, uint32_t out[8]) {
    const Gf256& f = gf();
    uint8_t t0[8], t1[8], t2[4];
    for (int v = 0; v < 8; ++v) {
        t0[v] = f.mul(c, (uint8_t)v);
        t1[v] = f.mul(c, (uint8_t)(v << 3));
    }
    for (int v = 0; v < 4; ++v) t2[v] = f.mul(c, (uint8_t)(v << 6));
    out[0] = pack4(t0[0], t0[1], t0[2], t0[3]);
    out[1] = pack4(t0[4], t0[5], t0[6], t0[7]);
    out[2] = pack4(t1[0], t1[1], t1[2], t1[3]);
    out[3] = pack4(t1[4], t1[5], t1[6], t1[7]);
    out[4] = pack4(t2[0], t2[1], t2[2], t2[3]);
    out[5] = out[6] = out[7] = 0;
}

// Host emulation of v_perm_b32 for the byte selectors 0..7 the kernels use.
inline uint32_t perm_emul(uint32_t hi, uint32_t lo, uint32_t sel) {
    uint64_t pool = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int b = 0; b < 4; ++b) {
        uint32_t s = (sel >> (8 * b)) & 0xFF;
        uint32_t byte = (s < 8) ? (uint32_t)((pool >> (8 * s)) & 0xFF) : 0;
        r |= byte << (8 * b);
    }
    return r;
}

// Host emulation of one split-table multiply of four packed bytes.
inline uint32_t perm_mul4_emul(const uint32_t rec[8], uint32_t x) {
    uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
    return perm_emul(rec[1], rec[0], s0) ^ perm_emul(rec[3], rec[2], s1) ^
           perm_emul(rec[4], rec[4], s2);
}

}  // namespace qf
