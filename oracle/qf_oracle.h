/*
 * qf_oracle.h -- CPU restatement of QuicFuscate's GF(2^8) RLNC FEC path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X
 * library (libqf_fec.so).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path never links,
 * calls or falls back to anything in oracle/.
 *
 * Parity pinning: the reference (Rust, src/fec) cannot be compiled in this
 * image (no rustc/cargo), so oracle/_ref does not exist.
 * The restatement is pinned by (a) the reference's own test contracts
 * (exhaustive gf_mul == gf_mul_table, recovery of the original bytes in
 * tests/fec.rs and src/fec/mod.rs, panic -> error for k+r > 256) and
 * (b) an independent pure-Python restatement whose outputs are committed
 * under tests/golden/ (tests/golden/gen_golden.py).
 *
 * Every function cites the reference lines it restates.
 */
#ifndef QF_ORACLE_H
#define QF_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* gf_tables.rs:384-408 init_gf_tables (poly 0x11D, generator 2). */
void oracle_gf_init(void);
/* Copies of the tables (EXP has 512 entries, LOG 256). */
void oracle_gf_tables(uint8_t *exp512, uint8_t *log256);
/* gf_tables.rs:47-57 gf_mul_table -- the semantic contract. */
uint8_t oracle_gf_mul(uint8_t a, uint8_t b);
/* gf_tables.rs:59-74 gf_mul_shift (shift-and-add, unused by the reference). */
uint8_t oracle_gf_mul_shift(uint8_t a, uint8_t b);
/* gf_tables.rs:127-141 gf_mul_bitsliced_sse2 as written: carry-less multiply
 * followed by the t^=t>>8..>>1 fold.  NOT a field multiply; kept
 * only to document the defect and to time the "as-written" CPU loop. */
uint8_t oracle_gf_mul_clmul_fold(uint8_t a, uint8_t b);
/* gf_tables.rs:304-309 gf_inv.  Returns 0 and writes *out, or -1 for a == 0
 * (the reference panics). */
int oracle_gf_inv(uint8_t a, uint8_t *out);
/* gf_tables.rs:255-274 gf_mul_slice (table semantics): out[i] = a[i]*b[i]. */
void oracle_gf_mul_slice(const uint8_t *a, const uint8_t *b, uint8_t *out, size_t n);

/* decoder.rs:280-298 generate_cauchy_coefficients for repairs 0..r-1:
 * out[j*k + i] = gf_inv((u8)i ^ (u8)(k + j)).  Returns 0, or -1 where the
 * reference would panic on gf_inv(0) (k + r > 256). */
int oracle_cauchy_coeffs(uint32_t k, uint32_t r, uint8_t *out_rxk);

/* decoder.rs:172-275 generate_repair_packet for j = 0..r-1 of one window:
 * rep[j*rep_stride + t] = XOR_{i<k} coeff[j*k+i] * src[i*src_stride + t],
 * t < L, in window order, zero coefficients skipped (decoder.rs:229-232).
 * coeff == NULL -> Cauchy coefficients.  Returns 0 or -1 (invalid shape). */
int oracle_encode_window(uint32_t k, uint32_t r, uint32_t L,
                         const uint8_t *src, size_t src_stride,
                         const uint8_t *coeff, uint8_t *rep, size_t rep_stride);

/* Same loop, but multiplying with the as-written CLMUL fold (F3).  Output is
 * NOT a valid repair; timing baseline only. */
int oracle_encode_window_clmul_fold(uint32_t k, uint32_t r, uint32_t L,
                                    const uint8_t *src, size_t src_stride,
                                    const uint8_t *coeff, uint8_t *rep,
                                    size_t rep_stride);

/* Status codes shared with include/qf_fec.h. */
#define ORACLE_OK 0
#define ORACLE_ENOTREADY (-3)
#define ORACLE_ERANK (-4)
#define ORACLE_EINVAL (-1)
#define ORACLE_ERANGE (-2)

/* One generation of decoder.rs:658-791 (Decoder::add_packet / try_decode /
 * gaussian_elimination / get_decoded_packets), with the F4 fix (systematic
 * rows carry their payloads, so the solved rows are the original bytes).
 *   row_index[s] < k   : systematic source row (the reference's id % k)
 *   row_index[s] >= k  : repair row j = row_index[s] - k
 *   row_coeffs         : k bytes per slot (only read for repair rows), or
 *                        NULL -> Cauchy coefficients of repair j
 * Rows are taken in arrival order; the first k accepted rows win and
 * duplicate systematic rows are ignored (decoder.rs:679-691).
 * On success out[i*out_stride .. +L] holds source row i for all i < k and
 * received_mask[i] = 1 for rows that arrived systematically.
 * Returns ORACLE_OK, ORACLE_ENOTREADY (< k rows), ORACLE_ERANK (singular),
 * ORACLE_ERANGE (Cauchy coefficient undefined) or ORACLE_EINVAL. */
int oracle_decode_generation(uint32_t k, uint32_t L, uint32_t n_rows,
                             const uint16_t *row_index, const uint8_t *rows,
                             size_t row_stride, const uint8_t *row_coeffs,
                             uint8_t *out, size_t out_stride,
                             uint8_t *received_mask);

/* decoder.rs:720-783 exactly as written (F4 defect kept): systematic rows
 * have no payload and add_scaled_row skips payload updates unless both rows
 * own payloads.  Used only by a test that documents the deviation. */
int oracle_decode_generation_as_written(uint32_t k, uint32_t L, uint32_t n_rows,
                                        const uint16_t *row_index,
                                        const uint8_t *rows, size_t row_stride,
                                        const uint8_t *row_coeffs,
                                        uint8_t *out, size_t out_stride);

/* decoder.rs:794-975 Decoder::wiedemann_algorithm, the strategy
 * Decoder::new selects for k > 256 (decoder.rs:659-665), with the two fixes
 * qf_oracle_wiedemann.c lists (minimal polynomial = reversed connection
 * polynomial; systematic payloads in B) and a checked solution: init vector
 * b = 0, 1, ... (decoder.rs:805-807) until A X == B, at most 8 tries.
 * Same arguments and statuses as oracle_decode_generation, any k <= 65535;
 * repair rows need row_coeffs unless the reference's u8 Cauchy rows are
 * defined (otherwise ORACLE_ERANGE, where the reference panics).  *tries
 * (nullable) = init vectors used. */
int oracle_wiedemann_decode(uint32_t k, uint32_t L, uint32_t n_rows, const uint16_t *row_index,
                            const uint8_t *rows, size_t row_stride, const uint8_t *row_coeffs,
                            uint8_t *out, size_t out_stride, uint8_t *received_mask,
                            uint32_t *tries);

/* ---- Packet framing (qf_oracle_wire.c, encoder.rs:18-152) --------------
 * One code per reference error string: */
#define ORACLE_FR_EMPTY (-10)             /* "Raw data is empty" (encoder.rs:25) */
#define ORACLE_FR_NO_COEFF_LEN (-11)      /* "Buffer too short for coefficient length" */
#define ORACLE_FR_COEFF_TRUNCATED (-12)   /* "Buffer too short for coefficients" */
#define ORACLE_FR_POOL_TOO_SMALL (-13)    /* "Buffer from pool is too small" (encoder.rs:55) */
#define ORACLE_FR_INVALID_LEN (-14)       /* "Invalid raw packet length" (encoder.rs:81) */
#define ORACLE_FR_BUFFER_TOO_SHORT (-15)  /* quiche::Error::BufferTooShort (encoder.rs:130) */
#define ORACLE_FR_PANIC (-16)             /* coefficient vector longer than a pool block */
int oracle_packet_to_raw(int is_systematic, int has_coeffs, const uint8_t *coeffs,
                         uint32_t coeff_len, int has_data, const uint8_t *data, uint32_t len,
                         uint8_t *buffer, size_t buffer_len, size_t *written);
int oracle_packet_from_raw(const uint8_t *raw, size_t raw_len, size_t block_size,
                           int *is_systematic, uint32_t *coeff_len, size_t *coeff_off,
                           size_t *payload_off, size_t *len);
int oracle_packet_from_block(uint8_t *block, size_t block_len, size_t len, int *is_systematic,
                             uint8_t *coeffs_out, uint32_t *coeff_len, size_t *payload_len);

/* Deterministic synthetic payload: byte t of the flat buffer is
 * byte (t & 7) of splitmix64(seed + (t >> 3)). */
void oracle_fill_splitmix(uint8_t *buf, size_t n, uint64_t seed, uint64_t word_offset);


/* cpu_variants.c: CPU comparison encoders for bench.py; G dense
 * generations, generations split over `threads` pthreads. */
int cpu_encode_table(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src,
                     uint8_t *rep, uint32_t threads);
int cpu_encode_avx2(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src,
                    uint8_t *rep, uint32_t threads);
int cpu_has_avx2(void);
int cpu_encode_gfni(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src,
                    uint8_t *rep, uint32_t threads);
int cpu_encode_clmul(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src,
                     uint8_t *rep, uint32_t threads);
int cpu_encode_clmul_dispatch(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src,
                              uint8_t *rep, uint32_t threads);
int cpu_has_gfni(void);
int cpu_has_pclmul(void);

/* ---- GF(2^16) Extreme mode (qf_oracle16.c) ----------------------------- */
uint16_t oracle_gf16_mul(uint16_t a, uint16_t b);
int oracle_gf16_inv(uint16_t a, uint16_t *out);
int oracle_cauchy16(uint32_t k, uint32_t r, uint16_t *out_rxk);
int oracle_encode16(uint32_t k, uint32_t r, uint32_t L, const uint8_t *src, size_t src_stride,
                    const uint16_t *coeff, uint8_t *rep, size_t rep_stride);
int oracle_decode16(uint32_t k, uint32_t L, uint32_t n_rows, const uint16_t *row_index,
                    const uint8_t *rows, size_t row_stride, const uint16_t *row_coeffs,
                    uint8_t *out, size_t out_stride, uint8_t *received_mask);

#ifdef __cplusplus
}
#endif
#endif
