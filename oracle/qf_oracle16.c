/*
 * qf_oracle16.c -- CPU restatement of QuicFuscate's GF(2^16) "Extreme" codec.
 *
 * TEST INFRASTRUCTURE ONLY (see qf_oracle.h).  Scalar, single-threaded, in the
 * reference's loop order:
 *   gf_tables.rs:333-353  gf16_mul: shift-and-add mod GF16_POLY = 0x1100B.  As
 *                         written the reduction test `a & 0x10000` is on a u16
 *                         and can never fire (it does not even compile, SURVEY
 *                         F2); restated with the reduction the code intends:
 *                         the bit shifted out of position 15 reduces by 0x1100B.
 *   gf_tables.rs:355-376  gf16_pow, gf16_inv = x^(2^16 - 2) (0 -> error, the
 *                         reference panics)
 *   decoder.rs:21-75      Encoder16::generate_repair_packet: big-endian u16
 *                         symbols (data[j] high byte, data[j+1] low byte) for
 *                         j + 1 < len; repair = XOR over the window of c_i * s_i
 *   decoder.rs:77-80      coefficients c_i = gf16_inv((i as u16) ^ ((k + j) as u16))
 *   decoder.rs:563-656    Decoder16: the first k rows are used (no duplicate
 *                         filtering), a systematic id maps to column id % k,
 *                         Gauss-Jordan with a pivot search from row i down and
 *                         a row swap; payloads carried for systematic rows too
 *                         (the F4 fix of the GF(2^8) decoder applies here
 *                         unchanged: decoder.rs:575-581 stores None for them).
 * Parity is pinned by the reference's own contract tests/fec.rs:52-82
 * (gf16_encode_decode) and by golden16.json (independent Python
 * restatement, tests/golden/gen_golden16.py).
 */
#include "qf_oracle.h"

#include <stdlib.h>
#include <string.h>

/* gf_tables.rs:333-353 (reduction as intended) */
uint16_t oracle_gf16_mul(uint16_t a, uint16_t b) {
    uint32_t aa = a, res = 0;
    while (b != 0) {
        if (b & 1) res ^= aa;
        b >>= 1;
        aa <<= 1;
        if (aa & 0x10000u) aa ^= 0x1100Bu;
    }
    return (uint16_t)res;
}

/* gf_tables.rs:355-376 */
int oracle_gf16_inv(uint16_t a, uint16_t *out) {
    if (a == 0) return ORACLE_ERANGE;
    uint16_t result = 1, x = a;
    uint32_t power = 0x10000u - 2;
    while (power > 0) {
        if (power & 1) result = oracle_gf16_mul(result, x);
        x = oracle_gf16_mul(x, x);
        power >>= 1;
    }
    *out = result;
    return ORACLE_OK;
}

/* decoder.rs:77-80: y = (k + j) as u16; c_i = gf16_inv((i as u16) ^ y) */
int oracle_cauchy16(uint32_t k, uint32_t r, uint16_t *out_rxk) {
    for (uint32_t j = 0; j < r; ++j) {
        const uint16_t y = (uint16_t)(k + j);
        for (uint32_t i = 0; i < k; ++i)
            if (oracle_gf16_inv((uint16_t)((uint16_t)i ^ y), &out_rxk[(size_t)j * k + i]) != ORACLE_OK)
                return ORACLE_ERANGE;
    }
    return ORACLE_OK;
}

static inline uint16_t sym(const uint8_t *p, uint32_t j) { return (uint16_t)(p[j] << 8 | p[j + 1]); }
static inline void put(uint8_t *p, uint32_t j, uint16_t v) {
    p[j] = (uint8_t)(v >> 8);
    p[j + 1] = (uint8_t)v;
}

/* decoder.rs:21-75 for repairs 0..r-1 of one window (coeff NULL = Cauchy) */
int oracle_encode16(uint32_t k, uint32_t r, uint32_t L, const uint8_t *src, size_t src_stride,
                    const uint16_t *coeff, uint8_t *rep, size_t rep_stride) {
    if (k == 0 || !src || !rep) return ORACLE_EINVAL;
    uint16_t *own = NULL;
    if (!coeff) {
        own = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)k * (r ? r : 1));
        if (!own) return ORACLE_EINVAL;
        if (oracle_cauchy16(k, r, own) != ORACLE_OK) {
            free(own);
            return ORACLE_ERANGE;
        }
        coeff = own;
    }
    for (uint32_t j = 0; j < r; ++j) {
        uint8_t *repair = rep + (size_t)j * rep_stride;
        memset(repair, 0, L); /* decoder.rs:33-34 */
        for (uint32_t i = 0; i < k; ++i) {
            const uint16_t c = coeff[(size_t)j * k + i];
            if (c == 0) continue; /* decoder.rs:38-40 */
            const uint8_t *s = src + (size_t)i * src_stride;
            for (uint32_t t = 0; t + 1 < L; t += 2)
                put(repair, t, (uint16_t)(oracle_gf16_mul(c, sym(s, t)) ^ sym(repair, t)));
        }
    }
    free(own);
    return ORACLE_OK;
}

/* decoder.rs:563-640 restated densely (payloads carried for every row).
 * Rows: the first k of n_rows in arrival order; row_index[s] < k = systematic
 * source, >= k = repair j = row_index[s] - k with coefficients row_coeffs[s]
 * (k u16) or the Cauchy row of j when row_coeffs is NULL.  out: k rows of L
 * bytes, row i = source i.  Statuses: ORACLE_ENOTREADY (< k rows),
 * ORACLE_ERANK (no pivot: singular, e.g. a duplicated row), ORACLE_ERANGE
 * (Cauchy coefficient undefined), ORACLE_EINVAL. */
int oracle_decode16(uint32_t k, uint32_t L, uint32_t n_rows, const uint16_t *row_index,
                    const uint8_t *rows, size_t row_stride, const uint16_t *row_coeffs,
                    uint8_t *out, size_t out_stride, uint8_t *received_mask) {
    if (k == 0 || (L & 1)) return ORACLE_EINVAL;
    if (n_rows < k) return ORACLE_ENOTREADY;
    uint16_t *m = (uint16_t *)calloc((size_t)k * k, sizeof(uint16_t));
    uint8_t *pay = (uint8_t *)malloc((size_t)k * (L ? L : 1));
    uint16_t *cr = (uint16_t *)malloc(sizeof(uint16_t) * k);
    int status = ORACLE_OK;
    if (!m || !pay || !cr) { status = ORACLE_EINVAL; goto done; }
    if (received_mask) memset(received_mask, 0, k);
    for (uint32_t q = 0; q < k; ++q) {
        const uint32_t idx = row_index[q];
        uint16_t *row = m + (size_t)q * k;
        if (idx < k) {
            row[idx] = 1; /* decoder.rs:573-578 */
            if (received_mask) received_mask[idx] = 1;
        } else if (row_coeffs) {
            memcpy(row, row_coeffs + (size_t)q * k, sizeof(uint16_t) * k);
        } else {
            const uint16_t y = (uint16_t)(k + (idx - k));
            for (uint32_t i = 0; i < k; ++i)
                if (oracle_gf16_inv((uint16_t)((uint16_t)i ^ y), &row[i]) != ORACLE_OK) {
                    status = ORACLE_ERANGE;
                    goto done;
                }
        }
        memcpy(pay + (size_t)q * L, rows + (size_t)q * row_stride, L);
    }
    for (uint32_t i = 0; i < k; ++i) { /* decoder.rs:598-640 */
        uint32_t p = i;
        while (p < k && m[(size_t)p * k + i] == 0) ++p;
        if (p == k) { status = ORACLE_ERANK; goto done; }
        if (p != i) {
            for (uint32_t c = 0; c < k; ++c) {
                uint16_t t = m[(size_t)i * k + c];
                m[(size_t)i * k + c] = m[(size_t)p * k + c];
                m[(size_t)p * k + c] = t;
            }
            for (uint32_t t = 0; t < L; ++t) {
                uint8_t v = pay[(size_t)i * L + t];
                pay[(size_t)i * L + t] = pay[(size_t)p * L + t];
                pay[(size_t)p * L + t] = v;
            }
        }
        uint16_t inv;
        oracle_gf16_inv(m[(size_t)i * k + i], &inv);
        for (uint32_t c = 0; c < k; ++c) m[(size_t)i * k + c] = oracle_gf16_mul(m[(size_t)i * k + c], inv);
        for (uint32_t t = 0; t + 1 < L; t += 2)
            put(pay + (size_t)i * L, t, oracle_gf16_mul(sym(pay + (size_t)i * L, t), inv));
        for (uint32_t rr = 0; rr < k; ++rr) {
            const uint16_t f = m[(size_t)rr * k + i];
            if (rr == i || f == 0) continue;
            for (uint32_t c = 0; c < k; ++c)
                m[(size_t)rr * k + c] ^= oracle_gf16_mul(f, m[(size_t)i * k + c]);
            for (uint32_t t = 0; t + 1 < L; t += 2)
                put(pay + (size_t)rr * L, t,
                    (uint16_t)(oracle_gf16_mul(f, sym(pay + (size_t)i * L, t)) ^ sym(pay + (size_t)rr * L, t)));
        }
    }
    for (uint32_t i = 0; i < k; ++i) memcpy(out + (size_t)i * out_stride, pay + (size_t)i * L, L);
done:
    free(m);
    free(pay);
    free(cr);
    return status;
}
