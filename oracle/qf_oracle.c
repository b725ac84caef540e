/*
 * qf_oracle.c -- CPU restatement of QuicFuscate src/fec (GF(2^8) RLNC).
 *
 * TEST INFRASTRUCTURE ONLY (see qf_oracle.h).  Scalar, single-threaded,
 * deliberately written in the reference's loop order so that it can also
 * serve as the "port" CPU baseline in bench.py.
 */
#include "qf_oracle.h"

#include <stdlib.h>
#include <string.h>

static uint8_t EXP_TABLE[512];
static uint8_t LOG_TABLE[256];
static int g_init = 0;

/* gf_tables.rs:384-408 */
void oracle_gf_init(void) {
    if (g_init) return;
    uint16_t x = 1;
    for (int i = 0; i < 255; ++i) {
        EXP_TABLE[i] = (uint8_t)x;
        EXP_TABLE[i + 255] = (uint8_t)x; /* wrap-around copy */
        LOG_TABLE[x] = (uint8_t)i;
        x <<= 1;
        if (x >= 256) x ^= 0x11D;
    }
    /* EXP[510], EXP[511] and LOG[0] stay 0 as in the reference. */
    g_init = 1;
}

void oracle_gf_tables(uint8_t *exp512, uint8_t *log256) {
    oracle_gf_init();
    memcpy(exp512, EXP_TABLE, 512);
    memcpy(log256, LOG_TABLE, 256);
}

/* gf_tables.rs:47-57 */
uint8_t oracle_gf_mul(uint8_t a, uint8_t b) {
    if (a == 0 || b == 0) return 0;
    return EXP_TABLE[(uint16_t)LOG_TABLE[a] + (uint16_t)LOG_TABLE[b]];
}

/* gf_tables.rs:59-74 */
uint8_t oracle_gf_mul_shift(uint8_t a, uint8_t b) {
    uint8_t res = 0;
    while (b != 0) {
        if (b & 1) res ^= a;
        uint8_t carry = a & 0x80;
        a = (uint8_t)(a << 1);
        if (carry) a ^= (uint8_t)0x11D;
        b >>= 1;
    }
    return res;
}

/* gf_tables.rs:127-141: clmul(a, b) then the xor-shift fold. */
uint8_t oracle_gf_mul_clmul_fold(uint8_t a, uint8_t b) {
    uint16_t prod = 0;
    for (int i = 0; i < 8; ++i)
        if (b & (1u << i)) prod ^= (uint16_t)((uint16_t)a << i);
    uint16_t t = prod ^ (prod >> 8);
    t ^= t >> 4;
    t ^= t >> 2;
    t ^= t >> 1;
    return (uint8_t)(t & 0xFF);
}

/* gf_tables.rs:304-309 */
int oracle_gf_inv(uint8_t a, uint8_t *out) {
    if (a == 0) return -1; /* reference: panic!("Inverse of 0 ...") */
    *out = EXP_TABLE[255 - LOG_TABLE[a]];
    return 0;
}

/* gf_tables.rs:255-274 (the `_ =>` table arm: the contract) */
void oracle_gf_mul_slice(const uint8_t *a, const uint8_t *b, uint8_t *out, size_t n) {
    for (size_t i = 0; i < n; ++i) out[i] = oracle_gf_mul(a[i], b[i]);
}

/* decoder.rs:280-298: y = (k + j) as u8; c_i = gf_inv((i as u8) ^ y) */
int oracle_cauchy_coeffs(uint32_t k, uint32_t r, uint8_t *out_rxk) {
    oracle_gf_init();
    for (uint32_t j = 0; j < r; ++j) {
        uint8_t y = (uint8_t)(k + j);
        for (uint32_t i = 0; i < k; ++i) {
            uint8_t c;
            if (oracle_gf_inv((uint8_t)((uint8_t)i ^ y), &c) != 0) return -1;
            out_rxk[(size_t)j * k + i] = c;
        }
    }
    return 0;
}

typedef uint8_t (*mul_fn)(uint8_t, uint8_t);

static int encode_window_impl(uint32_t k, uint32_t r, uint32_t L, const uint8_t *src,
                              size_t src_stride, const uint8_t *coeff, uint8_t *rep,
                              size_t rep_stride, mul_fn mul) {
    oracle_gf_init();
    if (k == 0 || src == NULL || rep == NULL) return ORACLE_EINVAL;
    uint8_t *own = NULL;
    if (coeff == NULL) {
        own = (uint8_t *)malloc((size_t)k * r);
        if (!own) return ORACLE_EINVAL;
        if (oracle_cauchy_coeffs(k, r, own) != 0) {
            free(own);
            return ORACLE_ERANGE;
        }
        coeff = own;
    }
    for (uint32_t j = 0; j < r; ++j) {
        uint8_t *repair = rep + (size_t)j * rep_stride;
        memset(repair, 0, L); /* decoder.rs:182-183 zeroes the block */
        /* decoder.rs:228-260: sequential arm, window order */
        for (uint32_t i = 0; i < k; ++i) {
            uint8_t c = coeff[(size_t)j * k + i];
            if (c == 0) continue;
            const uint8_t *s = src + (size_t)i * src_stride;
            for (uint32_t t = 0; t < L; ++t) repair[t] = (uint8_t)(mul(c, s[t]) ^ repair[t]);
        }
    }
    free(own);
    return ORACLE_OK;
}

int oracle_encode_window(uint32_t k, uint32_t r, uint32_t L, const uint8_t *src,
                         size_t src_stride, const uint8_t *coeff, uint8_t *rep,
                         size_t rep_stride) {
    return encode_window_impl(k, r, L, src, src_stride, coeff, rep, rep_stride,
                              oracle_gf_mul);
}

int oracle_encode_window_clmul_fold(uint32_t k, uint32_t r, uint32_t L, const uint8_t *src,
                                    size_t src_stride, const uint8_t *coeff, uint8_t *rep,
                                    size_t rep_stride) {
    return encode_window_impl(k, r, L, src, src_stride, coeff, rep, rep_stride,
                              oracle_gf_mul_clmul_fold);
}

/* ---- decoder ----------------------------------------------------------- */

typedef struct {
    uint8_t *coef;   /* k bytes */
    uint8_t *pay;    /* L bytes, or NULL (as-written systematic rows) */
} dense_row;

/* Row acceptance of decoder.rs:678-701.  Fills acc[] with accepted slots
 * (at most k) and returns how many; -1 for a bad row index. */
static int accept_rows(uint32_t k, uint32_t n_rows, const uint16_t *row_index,
                       uint32_t *acc, uint8_t *present) {
    uint32_t n = 0;
    memset(present, 0, k);
    for (uint32_t s = 0; s < n_rows && n < k; ++s) {
        uint32_t idx = row_index[s];
        if (idx < k) {
            if (present[idx]) continue; /* duplicate (decoder.rs:687-691) */
            present[idx] = 1;
        } else if (idx - k >= 256) {
            return -1;
        }
        acc[n++] = s;
    }
    return (int)n;
}

static int coeff_row(uint32_t k, uint32_t idx, const uint8_t *row_coeffs, uint32_t slot,
                     uint8_t *out) {
    if (idx < k) {
        memset(out, 0, k);
        out[idx] = 1; /* identity row, decoder.rs:685-686 */
        return 0;
    }
    if (row_coeffs) {
        memcpy(out, row_coeffs + (size_t)slot * k, k);
        return 0;
    }
    uint8_t y = (uint8_t)(k + (idx - k));
    for (uint32_t i = 0; i < k; ++i)
        if (oracle_gf_inv((uint8_t)((uint8_t)i ^ y), &out[i]) != 0) return -1;
    return 0;
}

/* decoder.rs:720-783 restated densely.  `as_written` keeps defect F4. */
static int gauss_jordan(uint32_t k, uint32_t L, dense_row *m, uint32_t nrows, int as_written) {
    uint32_t rank = 0;
    for (uint32_t i = 0; i < k; ++i) {
        uint32_t p = nrows;
        for (uint32_t r = i; r < nrows; ++r)
            if (m[r].coef[i] != 0) { p = r; break; }
        if (p == nrows) continue;
        if (p != i) { dense_row t = m[i]; m[i] = m[p]; m[p] = t; } /* swap_rows */
        uint8_t inv;
        oracle_gf_inv(m[i].coef[i], &inv);
        /* scale_row (decoder.rs:407-455) */
        for (uint32_t c = 0; c < k; ++c) m[i].coef[c] = oracle_gf_mul(m[i].coef[c], inv);
        if (m[i].pay)
            for (uint32_t t = 0; t < L; ++t) m[i].pay[t] = oracle_gf_mul(m[i].pay[t], inv);
        /* add_scaled_row for every other row (decoder.rs:457-517) */
        for (uint32_t r = 0; r < nrows; ++r) {
            if (r == i) continue;
            uint8_t f = m[r].coef[i];
            if (f == 0) continue;
            for (uint32_t c = 0; c < k; ++c)
                m[r].coef[c] ^= oracle_gf_mul(m[i].coef[c], f);
            int do_payload = as_written ? (m[i].pay && m[r].pay) : 1;
            if (do_payload && m[r].pay && m[i].pay)
                for (uint32_t t = 0; t < L; ++t)
                    m[r].pay[t] = (uint8_t)(oracle_gf_mul(f, m[i].pay[t]) ^ m[r].pay[t]);
        }
        if (++rank == k) break; /* early exit (decoder.rs:749-752) */
    }
    return rank == k ? ORACLE_OK : ORACLE_ERANK;
}

static int decode_impl(uint32_t k, uint32_t L, uint32_t n_rows, const uint16_t *row_index,
                       const uint8_t *rows, size_t row_stride, const uint8_t *row_coeffs,
                       uint8_t *out, size_t out_stride, uint8_t *received_mask,
                       int as_written) {
    oracle_gf_init();
    if (k == 0 || k > 256) return ORACLE_EINVAL;
    uint32_t *acc = (uint32_t *)malloc(sizeof(uint32_t) * k);
    uint8_t *present = (uint8_t *)malloc(k);
    uint8_t *store = (uint8_t *)calloc((size_t)k, (size_t)k + L);
    dense_row *m = (dense_row *)malloc(sizeof(dense_row) * k);
    int status = ORACLE_OK;
    if (!acc || !present || !store || !m) { status = ORACLE_EINVAL; goto done; }
    int n = accept_rows(k, n_rows, row_index, acc, present);
    if (n < 0) { status = ORACLE_EINVAL; goto done; }
    if ((uint32_t)n < k) { status = ORACLE_ENOTREADY; goto done; }
    for (uint32_t q = 0; q < k; ++q) {
        uint32_t s = acc[q];
        uint32_t idx = row_index[s];
        m[q].coef = store + (size_t)q * (k + L);
        if (coeff_row(k, idx, row_coeffs, s, m[q].coef) != 0) { status = ORACLE_ERANGE; goto done; }
        m[q].pay = m[q].coef + k;
        if (as_written && idx < k) m[q].pay = NULL; /* decoder.rs:692 */
        else memcpy(m[q].pay, rows + (size_t)s * row_stride, L);
    }
    status = gauss_jordan(k, L, m, k, as_written);
    if (status != ORACLE_OK) goto done;
    for (uint32_t i = 0; i < k; ++i) {
        uint8_t *dst = out + (size_t)i * out_stride;
        if (as_written) {
            /* decoder.rs:763-780: missing systematic i <- payload of row i */
            if (!present[i] && m[i].pay) memcpy(dst, m[i].pay, L);
            else if (present[i]) {
                for (uint32_t q = 0; q < k; ++q)
                    if (row_index[acc[q]] == i) { memcpy(dst, rows + (size_t)acc[q] * row_stride, L); break; }
            } else memset(dst, 0, L);
        } else {
            memcpy(dst, m[i].pay, L);
        }
        if (received_mask) received_mask[i] = present[i];
    }
done:
    free(acc);
    free(present);
    free(store);
    free(m);
    return status;
}

int oracle_decode_generation(uint32_t k, uint32_t L, uint32_t n_rows, const uint16_t *row_index,
                             const uint8_t *rows, size_t row_stride, const uint8_t *row_coeffs,
                             uint8_t *out, size_t out_stride, uint8_t *received_mask) {
    return decode_impl(k, L, n_rows, row_index, rows, row_stride, row_coeffs, out, out_stride,
                       received_mask, 0);
}

int oracle_decode_generation_as_written(uint32_t k, uint32_t L, uint32_t n_rows,
                                        const uint16_t *row_index, const uint8_t *rows,
                                        size_t row_stride, const uint8_t *row_coeffs,
                                        uint8_t *out, size_t out_stride) {
    return decode_impl(k, L, n_rows, row_index, rows, row_stride, row_coeffs, out, out_stride,
                       NULL, 1);
}

static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_fill_splitmix(uint8_t *buf, size_t n, uint64_t seed, uint64_t word_offset) {
    size_t t = 0;
    uint64_t w = word_offset;
    for (; t + 8 <= n; t += 8, ++w) {
        uint64_t v = splitmix64(seed + w);
        memcpy(buf + t, &v, 8); /* little-endian host */
    }
    if (t < n) {
        uint64_t v = splitmix64(seed + w);
        memcpy(buf + t, &v, n - t);
    }
}
