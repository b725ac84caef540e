/*
 * qf_fec.h -- C ABI of the MI355X-native GF(2^8) RLNC FEC library
 *             (libqf_fec.so, hand-written HIP kernels for gfx950).
 *
 * This is the drop-in boundary for QuicFuscate's src/fec hot path.  Every
 * entry point names the reference interface it replaces (paths relative to
 * the reference repository, Christopher-Schulze/QuicFuscate @ 2025-07-18).
 * INTEGRATION.md shows the Rust FFI a maintainer would add on the reference
 * side.
 *
 * Conventions
 *  - All functions return int status: QF_OK (0) or a negative QF_E* code.
 *    Nothing panics or aborts; the reference's panics (gf_inv(0), k + r > 256)
 *    become QF_ERANGE.
 *  - Buffers are caller-owned.  The library never frees or zeroes caller
 *    memory.  "_dev" pointers are device (HBM) pointers; "_host" pointers are
 *    host memory (pinned for full PCIe rate).
 *  - Work is enqueued asynchronously on the context's stream; qf_sync()
 *    waits.  One context per host thread; distinct contexts are independent.
 *  - Arithmetic is GF(2^8) with polynomial 0x11D and generator 2, table
 *    semantics (gf_tables.rs:47-57, 384-408).
 */
#ifndef QF_FEC_H
#define QF_FEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QF_OK 0
#define QF_EINVAL (-1)     /* bad argument / shape                               */
#define QF_ERANGE (-2)     /* gf_inv(0): k + r > 256, Cauchy undefined (F5)      */
#define QF_ENOTREADY (-3)  /* window not full / fewer than k rows received       */
#define QF_ERANK (-4)      /* decode matrix singular                             */
#define QF_EDEVICE (-5)    /* HIP runtime error                                  */
#define QF_ENOMEM (-6)     /* allocation failed                                  */
#define QF_ETOOSMALL (-7)  /* output buffer too short (quiche BufferTooShort)    */

#define QF_ABI_VERSION 1
int qf_abi_version(void);
const char *qf_strerror(int status);
/* The cause of the calling thread's most recent QF_EDEVICE: the failing HIP
 * call's source file:line and error name, and, when a generated kernel's
 * launch checks refused the call, which check ("... (qf_bs.hip:339 launch
 * refused)").  Thread-local, like errno: kept until the next device failure on
 * this thread; "" if there was none.  No reference counterpart (the
 * reference's codec has no device). */
const char *qf_last_error(void);

/* ---------------------------------------------------------------------------
 * GF(2^8) scalar helpers (host).  These mirror the reference's public GF API
 * for callers and parity tests; the hot path never calls them.
 * ------------------------------------------------------------------------- */
/* replaces gf_tables.rs:392 init_gf_tables (idempotent) */
int qf_gf256_init(void);
/* replaces gf_tables.rs:283 gf_mul and :47 gf_mul_table (same result) */
uint8_t qf_gf256_mul(uint8_t a, uint8_t b);
/* replaces gf_tables.rs:327 gf_mul_add: a*b ^ c */
uint8_t qf_gf256_mul_add(uint8_t a, uint8_t b, uint8_t c);
/* replaces gf_tables.rs:304 gf_inv / :312 gf_inv_prefetch; QF_ERANGE for 0 */
int qf_gf256_inv(uint8_t a, uint8_t *out);
/* replaces decoder.rs:280-298 Encoder::generate_cauchy_coefficients for
 * repairs 0..r-1: out[j*k + i] = inv((u8)i ^ (u8)(k + j)).  QF_ERANGE where
 * the reference panics (k + r > 256). */
int qf_cauchy_coeffs(uint32_t k, uint32_t r, uint8_t *out_rxk);

/* ---------------------------------------------------------------------------
 * Context
 * ------------------------------------------------------------------------- */
typedef struct qf_ctx qf_ctx;
/* device: HIP device ordinal.  stream: hipStream_t to enqueue on (NULL = the
 * context creates its own non-blocking stream; QF_STREAM_NULL = the device's
 * null stream, ordered with other work on it, e.g. torch's default stream). */
#define QF_STREAM_NULL ((void *)1)
int qf_ctx_create(int device, void *stream, qf_ctx **out);
int qf_ctx_destroy(qf_ctx *ctx);
int qf_ctx_set_stream(qf_ctx *ctx, void *stream);
void *qf_ctx_stream(qf_ctx *ctx);
/* Split-phase decode.  The next qf_decode_batch on ctx enqueues its
 * acceptance pass (row indices only: first k rows win, slot map, LU/inverse
 * records -- the bookkeeping the reference's Decoder::add_packet does on
 * arrival, decoder.rs:678-701) at once, and makes its payload pass
 * (Decoder::try_decode / gaussian_elimination, decoder.rs:720-783) wait for
 * `event` (a hipEvent_t recorded on any stream, e.g. after the H2D copy of
 * the rows).  The setting is cleared when that qf_decode_batch returns;
 * NULL clears it.  No reference counterpart beyond the add_packet /
 * try_decode split. */
int qf_ctx_set_payload_wait(qf_ctx *ctx, void *event);
/* Split-phase decode on two streams.  The next qf_decode_batch on ctx keeps
 * its acceptance pass on the context's stream and enqueues its payload pass
 * on `stream` (a hipStream_t; QF_STREAM_NULL = the null stream) after it, so
 * a caller whose rows are produced on `stream` needs no cross-stream wait
 * before the payload and none after it: the call's work is complete when
 * `stream` reaches that point.  Combines with qf_ctx_set_payload_wait.  The
 * fused decode runs its payload kernel on `stream`; the other decode paths
 * finish on the context's stream and `stream` waits for them.  The context's
 * own stream also waits for the payload pass (an event, no host block), so a
 * later call on ctx -- the next decode rewriting the context's workspace,
 * qf_sync, qf_ctx_destroy -- is ordered after it.  Cleared when
 * that qf_decode_batch returns; NULL clears it.  qf_decode_batch_host and
 * qf_decode_batch_desc clear it and run on the context's stream. */
int qf_ctx_set_payload_stream(qf_ctx *ctx, void *stream);
int qf_sync(qf_ctx *ctx);

/* Kernel-path options of a context.  No reference counterpart: the
 * reference codec has no tuning knobs (core.rs:189-303 builds it with its
 * defaults), and the defaults here are the fastest measured paths.  They let
 * a host pin a kernel path per context (A/B, work-arounds); every call on the
 * context reads the context's values, and no call reads the environment.
 * qf_ctx_create sets each option to its default and then, once, to the
 * integer in the environment variable named in brackets when that is set
 * (tooling compatibility).  Values are clamped to the ranges given;
 * QF_EINVAL for an unknown option. */
enum {
    QF_OPT_FFT_KERNELS = 0,      /* 1: additive-FFT Cauchy kernels where generated; 0: one coefficient
                                    block per repair [QF_FFT_KERNELS; default 1] */
    QF_OPT_BITSLICED,            /* 0: no bit-sliced Cauchy kernels, v_perm paths only
                                    [QF_DISABLE_BS=1 sets 0; default 1] */
    QF_OPT_ENCODE_SMALL,         /* small-batch encode kernel: -1 auto, 0 never, 1 always [QF_ENCODE_SMALL] */
    QF_OPT_ENCODE_KSPLIT,        /* 1: row-split encode passes for <= 1 item per CU; 0 never [QF_ENCODE_KSPLIT] */
    QF_OPT_ENCODE_V,             /* 16-B units per lane of k_combine_uniform: 1 or 2 [QF_ENCODE_V] */
    QF_OPT_ENCODE_PD,            /* prefetch depth of k_combine_uniform, 1..3 [QF_ENCODE_PD; default 2] */
    QF_OPT_DECODE_PATH,          /* Cauchy decode: 0 fused lane-chunk, 1 syndromes + combine
                                    [QF_DECODE_SYN=1], 2 fused item layout [QF_DECODE_LEGACY=1] */
    QF_OPT_DECODE_KSPLIT,        /* 1: row-split fused decode for <= 1 item per CU; 0 never [QF_DECODE_KSPLIT] */
    QF_OPT_DECODE_SYNW,          /* 1: scalar-map syndrome passes at long rows (r > 16); 0 never
                                    [QF_DECODE_NO_SYNW=1 sets 0] */
    QF_OPT_DECODE_PD,            /* prefetch depth of k_combine_slots, 1..3 [QF_DECODE_PD; default 1] */
    QF_OPT_DECODE_CHUNK,         /* generations per chunk of the general decode, 0 = all [QF_DECODE_CHUNK] */
    QF_OPT_DECODE_OVERLAP,       /* 1: chunked general decode overlaps chunks on two streams [QF_DECODE_OVERLAP] */
    QF_OPT_COMBINE_BS,           /* 1: bit-sliced payload pass (qf_combine_bs) at long rows; 0 never [QF_COMBINE_BS] */
    QF_OPT_COMBINE_BS_MIN_Q,     /* its smallest row, in 32-B lane-chunks [QF_COMBINE_BS_MIN_Q; default 64] */
    QF_OPT_COMBINE_SPLIT,        /* 1: slot-split payload pass for <= 1 item per CU; 0 never [QF_COMBINE_SPLIT] */
    QF_OPT_PREPARE_GRID,         /* split-phase acceptance pass grid, 0 = one block per CU [QF_PREPARE_GRID] */
    QF_OPT_ENC_BLOCKS_PER_CU,    /* cap of the bit-sliced encode grid, 0 = none [QF_ENC_BLOCKS_PER_CU] */
    QF_OPT_DEC_BLOCKS_PER_CU,    /* cap of the fused decode grid, 0 = none [QF_DEC_BLOCKS_PER_CU] */
    QF_OPT_SEND_FUSED,           /* 1: one-launch per-packet send (k_send_window); 0 never [QF_SEND_FUSED] */
    QF_OPT_SEND_WINDOWS_MIN_TILES, /* send batches: tiles from which k_encode_windows is used [default 256] */
    QF_OPT_SEND_CHUNKS,          /* send batches: D2H chunks, 1..8 [QF_SEND_CHUNKS; default 1] */
    QF_OPT_SEND_PROFILE,         /* 1: phase timing of send batches on stderr at qf_ctx_destroy [QF_SEND_PROFILE] */
    QF_OPT_COPY_THREADS,         /* host copy-out workers of send/receive batches, -1 = auto.  Process-wide:
                                    the first batch call creates the pool [QF_COPY_THREADS] */
    QF_OPT_GF16_DYN,             /* 1: GF(2^16) decode launches shaped on the device; 0 from e_max [QF_GF16_DYN] */
    QF_OPT_GF16_LOGIFY,          /* 1: GF(2^16) inputs in log form for wide matvecs; 0 never [QF_GF16_LOGIFY] */
    QF_OPT_GF16_LOGIFY_MIN_BLOCKS, /* output blocks from which inputs are logified [QF_GF16_LOGIFY_MIN_BLOCKS] */
    QF_OPT_GF16_LDS_GJ,          /* 1: GF(2^16) Gauss-Jordan in LDS for e <= 64 [QF_GF16_LDS_GJ; default 0] */
    QF_OPT_GF16_BITSLICED,       /* 1: bit-sliced GF(2^16) Cauchy encode and decode syndromes where
                                    generated; 0 never [QF_GF16_BITSLICED; default 1] */
    QF_OPT_GF16_FFT,             /* additive-FFT GF(2^16) Cauchy encode / decode syndromes for
                                    k = 2^a in [16, 4096] (first + r <= k) without a bit-sliced kernel:
                                    1 where it needs ~9x fewer products than the matvec, 2 always,
                                    0 never [QF_GF16_FFT; default 1] */
    QF_OPT_WIEDEMANN_PROJ,       /* k > 256 decoder's projections: 1 = the reference's first init vector
                                    (decoder.rs:805-807, b = 0), then random vectors drawn per attempt
                                    from a per-process secret (a packet sender cannot craft a matrix
                                    that defeats them and forces the exact host fallback); 0 = the
                                    reference's init vectors b = 0..7 only [QF_WIEDEMANN_PROJ; default 1] */
    QF_OPT_GF16_FFT_BS,          /* the GF(2^16) additive FFT for k <= 2048 bit-sliced (field elements
                                    in 16 bit planes, no table lookups): 1 where a batch has items for
                                    a quarter of the CUs, 2 always, 3 always with two layers per LDS
                                    pass; 0 the log / Zech-table kernel for every k
                                    [QF_GF16_FFT_BS; default 1] */
    QF_OPT_PREPARE_LANES,        /* 1: the fused decode's acceptance pass runs one generation per lane
                                    (k_decode_prepare_lu_lanes); 0: one per wave [QF_PREPARE_LANES;
                                    default 1] */
    QF_OPT_ENCODE_MERGED,        /* 1: multi-pass work in ONE dispatch each: the encode passes of a
                                    code with more repairs than one kernel holds (C5 r > 22; a
                                    workgroup's waves run the passes on one item, so each source row
                                    is read from HBM once), and the decode's syndrome and payload
                                    passes (pass-major workgroup ranges); 0: one launch per pass
                                    [QF_ENCODE_MERGED; default 1] */
    QF_OPT_SYNW_SHARED,          /* 1: the additive-FFT syndrome passes of the C5 decode item-major in
                                    one dispatch, the passes' waves sharing the source rows' gather,
                                    transposes and chunk butterflies through LDS; 0: pass-major
                                    (each pass re-reads the sources) [QF_SYNW_SHARED; default 1] */
    QF_OPT_COMBINE_WIDE,         /* 1: a bit-sliced payload pass with 17-24 outputs (e_max) runs as one
                                    24-output pass reading two coefficient records per row; 0: two
                                    16-output passes (pass-major) [QF_COMBINE_WIDE; default 1] */
    QF_OPT_COMBINE_XCD,          /* 1: the pass-major payload pass item-major: the passes of one
                                    generation's lane-chunk run together on one XCD, so the later
                                    passes read the syndrome rows from its L2 instead of HBM; 0: pass
                                    p's workgroups after pass p - 1's [QF_COMBINE_XCD; default 0:
                                    where the last pass is short it runs ahead of the others and the
                                    reuse is lost, 5 % slower at e = 39 / 59, DESIGN 3.7] */
    QF_OPT_COMBINE_JUMP,         /* 1: the bit-sliced payload pass multiplies by a runtime coefficient c
                                    with a call into c's code block (8 destination-indexed 3-input
                                    XORs); 0: M0-indexed XORs, one index write per XOR
                                    [QF_COMBINE_JUMP; default 1] */
    QF_OPT_COMBINE_PM24,         /* 1: with QF_COMBINE_JUMP, a payload pass of 49-64 outputs (e_max) runs
                                    as 3 24-output passes in one launch instead of 4 16-output ones
                                    (the syndrome rows read and transposed once less);
                                    0: 16-output passes [QF_COMBINE_PM24; default 1] */
    QF_OPT_SLIDING_KERNELS,      /* 1: an encode batch whose generations overlap (generation stride
                                    below k row strides: sliding windows) runs the shape's sliding-window
                                    kernel where one is built (cached row loads; (48, 8) as the hybrid
                                    FFT pass); 0: the block kernels [QF_SLIDING_KERNELS; default 1] */
    QF_OPT_COUNT
};
int qf_ctx_set_option(qf_ctx *ctx, int option, int64_t value);
int qf_ctx_get_option(qf_ctx *ctx, int option, int64_t *value);

/* Kernel timing (no reference counterpart; benches/ replacement).  While on,
 * every kernel the context launches is bracketed by HIP events recorded on
 * the stream it runs on; totals accumulate per kernel name.  on != 0 clears
 * the totals and starts, on == 0 stops.  qf_ctx_profile_read synchronises
 * the pending events and returns the i-th kernel (first-launch order):
 * name (owned by ctx), number of launches, summed duration in ms;
 * QF_EINVAL once i >= number of kernels seen. */
int qf_ctx_profile(qf_ctx *ctx, int on);
int qf_ctx_profile_read(qf_ctx *ctx, uint32_t i, const char **name, uint32_t *launches,
                        double *total_ms);

/* ---------------------------------------------------------------------------
 * Element-wise slice multiply on the device.
 * replaces gf_tables.rs:255-274 gf_mul_slice (benches/gf_mul_slice_bench.rs)
 * out[i] = a[i] * b[i] for i < n (device pointers).
 * ------------------------------------------------------------------------- */
int qf_gf256_mul_slice_dev(qf_ctx *ctx, const uint8_t *a_dev, const uint8_t *b_dev,
                           uint8_t *out_dev, size_t n);

/* ---------------------------------------------------------------------------
 * Batched block encode (device resident).
 * replaces decoder.rs:172-275 Encoder::generate_repair_packet, for r repairs
 * of G independent generations in one launch:
 *   rep[g][j][t] = XOR_{i<k} C[j][i] * src[g][i][t]      (t < L, j < r)
 * Row i of generation g starts at src_dev + g*src_gen_stride + i*src_row_stride;
 * repair j at rep_dev + g*rep_gen_stride + j*rep_row_stride.  Exactly L bytes
 * per repair row are written (plus the zero tail with QF_ENCODE_ZERO_TAIL).  coeff_rxk (host, r*k bytes, row-major) or NULL
 * for the reference's Cauchy matrix (decoder.rs:280-298).
 * Sliding windows (adaptive.rs:519-562, one window per source packet) are the
 * special case src_gen_stride == src_row_stride.
 * Fast path: src/rep pointers and strides 16-byte aligned (any L).
 * ------------------------------------------------------------------------- */
/* qf_encode_shape.flags: the caller lets the library write zeros to bytes
 * [L, round_up(L, 128)) of every repair row when rep_row_stride covers them
 * (the reference's repair is a pool block that is zero beyond L,
 * decoder.rs:182/264 + optimize.rs:524).  With 128-B aligned repair rows this
 * lets the encode kernel store whole 128-B lines only.  When
 * L % 16 != 0 the kernel then also reads each source row's last 16-byte unit
 * whole (up to round_up(L, 16): inside the 16-byte row stride, and for the
 * buffer's last row within the same page); those extra bytes never reach the
 * output. */
#define QF_ENCODE_ZERO_TAIL 1u

typedef struct qf_encode_shape {
    uint32_t k;              /* generation (window) size, 1..255 */
    uint32_t r;              /* repairs per generation, k + r <= 256 for Cauchy */
    uint32_t L;              /* payload bytes per packet */
    uint32_t flags;          /* QF_ENCODE_* bits; 0: exactly L bytes per repair row */
    uint64_t src_row_stride;
    uint64_t src_gen_stride;
    uint64_t rep_row_stride;
    uint64_t rep_gen_stride;
} qf_encode_shape;

int qf_encode_batch(qf_ctx *ctx, const qf_encode_shape *shape, uint32_t G,
                    const uint8_t *src_dev, uint8_t *rep_dev, const uint8_t *coeff_rxk);

/* Same, host-resident src/rep (pinned memory recommended).  Chunks of
 * generations are streamed H2D -> encode -> D2H on several HIP streams with
 * device staging owned by the context.  Synchronous on return. */
int qf_encode_batch_host(qf_ctx *ctx, const qf_encode_shape *shape, uint32_t G,
                         const uint8_t *src_host, uint8_t *rep_host,
                         const uint8_t *coeff_rxk);

/* ---------------------------------------------------------------------------
 * Batched decode (device resident).
 * replaces decoder.rs:658-791 Decoder::{add_packet, try_decode,
 * gaussian_elimination, get_decoded_packets} for G independent generations:
 *  - rows: the received packets of generation g in arrival order,
 *    rows_dev + g*rows_gen_stride + slot*row_stride, slot < n_rows[g]
 *  - row_index_dev[g*max_rows + slot]: < k = systematic source index
 *    (the reference's id % k, decoder.rs:684); >= k = repair j = value - k
 *  - row_coeffs_dev: NULL (repair coefficients are the Cauchy row of j) or
 *    k coefficient bytes per slot at row_coeffs_dev + (g*max_rows + slot)*k
 *    (the packet's coefficient block, decoder.rs:694-696)
 *  - n_rows_dev: per-generation slot count, or NULL (= max_rows)
 * Acceptance follows decoder.rs:678-701: the first k rows win, duplicate
 * systematic rows are ignored.  For each generation the erased source rows
 * are recovered (ascending source index) into
 *   rec_dev + g*rec_gen_stride + m*rec_row_stride,  m < n_rec[g] <= min(k, r)
 * with rec_index_dev[g*min(k,r) + m] = source index of recovered row m and
 * status_dev[g] = QF_OK / QF_ENOTREADY / QF_ERANK / QF_ERANGE / QF_EINVAL.
 * Received systematic rows are not copied (they are already the payload).
 * Deviation from the reference: systematic rows carry their
 * payloads, so the recovered bytes are the original bytes.
 * ------------------------------------------------------------------------- */
typedef struct qf_decode_shape {
    uint32_t k;
    uint32_t r;              /* max repairs that may arrive (bounds n_rec) */
    uint32_t L;
    uint32_t max_rows;       /* slots per generation in row_index / rows   */
    uint64_t row_stride;
    uint64_t rows_gen_stride;
    uint64_t rec_row_stride;
    uint64_t rec_gen_stride;
} qf_decode_shape;

int qf_decode_batch(qf_ctx *ctx, const qf_decode_shape *shape, uint32_t G,
                    const uint8_t *rows_dev, const uint16_t *row_index_dev,
                    const uint32_t *n_rows_dev, const uint8_t *row_coeffs_dev,
                    uint8_t *rec_dev, uint16_t *rec_index_dev, uint32_t *n_rec_dev,
                    int32_t *status_dev);

/* Same, every buffer host-resident (pinned memory recommended): the receive
 * side starting from datagrams in host memory (core.rs:203-232).  Chunks of
 * about 64 MiB of rows are streamed H2D -> decode -> D2H on several HIP
 * streams; each chunk's acceptance pass starts once its indices have landed
 * and its payload pass once its rows have (qf_ctx_set_payload_wait).
 * Generation g's rows must lie in [g*rows_gen_stride, (g+1)*rows_gen_stride);
 * recovered rows must be dense per generation (rec_gen_stride ==
 * min(k, r) * rec_row_stride).  Bytes [0, L) of recovered rows
 * n_rec[g] .. min(k, r) - 1 of a generation are unspecified on return (the
 * device path leaves them untouched).  Synchronous on return. */
int qf_decode_batch_host(qf_ctx *ctx, const qf_decode_shape *shape, uint32_t G,
                         const uint8_t *rows_host, const uint16_t *row_index_host,
                         const uint32_t *n_rows_host, const uint8_t *row_coeffs_host,
                         uint8_t *rec_host, uint16_t *rec_index_host, uint32_t *n_rec_host,
                         int32_t *status_host);

/* ---------------------------------------------------------------------------
 * Heterogeneous batches (SURVEY 8(b) qf_gen_desc): one call over generations
 * whose (k, r, L) and placement differ per generation -- the ASW-RLNC-X mix
 * of window sizes (adaptive.rs:124-153, BASELINE config C5).  Generations
 * are grouped by shape inside the call; each group runs the batch kernels
 * above with per-generation offset tables (no payload is copied).
 * replaces per-generation Encoder::generate_repair_packet (decoder.rs:171-275)
 * / Decoder::add_packet + try_decode (decoder.rs:678-791) calls.
 * ------------------------------------------------------------------------- */
typedef struct qf_gen_desc {
    uint32_t k, r, L;        /* generation size, repairs (k + r <= 256), payload bytes */
    uint32_t flags;          /* QF_ENCODE_ZERO_TAIL: bytes [L, 16*ceil8(L/16)) of each repair row may be zeroed */
    uint64_t src_offset;     /* source row i at src_dev + src_offset + i * src_row_stride */
    uint64_t src_row_stride;
    uint64_t rep_offset;     /* repair row j at rep_dev + rep_offset + j * rep_row_stride */
    uint64_t rep_row_stride;
} qf_gen_desc;
/* Offsets and strides are multiples of 16; QF_ERANGE if any k + r > 256. */
int qf_encode_batch_desc(qf_ctx *ctx, const qf_gen_desc *gens_host, uint32_t G, const uint8_t *src_dev,
                         uint8_t *rep_dev);

typedef struct qf_dec_desc {
    uint32_t k, r, L;
    uint32_t n_rows;            /* received rows of this generation (<= 255), arrival order */
    uint64_t rows_offset;       /* received row s at rows_dev + rows_offset + s * row_stride */
    uint64_t row_stride;
    uint64_t row_index_offset;  /* its n_rows indices (< k source, k + j repair j) at row_index_dev + this (elements) */
    uint64_t rec_offset;        /* recovered row m at rec_dev + rec_offset + m * rec_row_stride */
    uint64_t rec_row_stride;
    uint64_t rec_index_offset;  /* min(k, r) u16 entries at rec_index_dev + this (elements) */
} qf_dec_desc;
/* Cauchy-coded generations (repair coefficients = the Cauchy row of the
 * repair index, decoder.rs:280-298).  n_rec_dev / status_dev: one entry per
 * descriptor, in descriptor order (status as qf_decode_batch). */
int qf_decode_batch_desc(qf_ctx *ctx, const qf_dec_desc *gens_host, uint32_t G, const uint8_t *rows_dev,
                         const uint16_t *row_index_dev, uint8_t *rec_dev, uint16_t *rec_index_dev,
                         uint32_t *n_rec_dev, int32_t *status_dev);

/* ---------------------------------------------------------------------------
 * Per-connection objects mirroring the reference's Rust API one call at a
 * time (what core.rs drives).  Payload state lives in HBM.
 * ------------------------------------------------------------------------- */
typedef struct qf_encoder qf_encoder;
/* replaces decoder.rs:156 Encoder::new(k, n); max_len bounds packet length */
int qf_encoder_new(qf_ctx *ctx, uint32_t k, uint32_t n, uint32_t max_len, qf_encoder **out);
int qf_encoder_free(qf_encoder *enc);
/* replaces decoder.rs:164 Encoder::add_source_packet (slides the window) */
int qf_encoder_add_source_packet(qf_encoder *enc, uint64_t id, const uint8_t *data,
                                 uint32_t len);
/* replaces decoder.rs:172 Encoder::generate_repair_packet(j).  QF_ENOTREADY
 * while the window holds fewer than k packets (the reference's None).
 * out_data receives len = window[0].len bytes, out_coeffs k bytes,
 * *out_id = last.id + 1 + j. */
int qf_encoder_generate_repair_packet(qf_encoder *enc, uint32_t repair_index,
                                      uint8_t *out_data, uint32_t out_cap,
                                      uint32_t *out_len, uint8_t *out_coeffs,
                                      uint64_t *out_id);
/* All repairs first..first+count-1 of the current window in one launch
 * (adaptive.rs:546-562 emit_repairs). out_data rows are out_stride apart. */
int qf_encoder_generate_repairs(qf_encoder *enc, uint32_t first, uint32_t count,
                                uint8_t *out_data, uint32_t out_stride, uint32_t *out_len,
                                uint8_t *out_coeffs, uint64_t *out_ids);
int qf_encoder_window_len(const qf_encoder *enc);

typedef struct qf_decoder qf_decoder;
/* Largest k of a GF(2^8) decoder: the largest window any mode uses
 * (Extreme, adaptive.rs:131-133).  k > 256 needs explicit coefficients on
 * every repair row (the reference's u8 Cauchy rows wrap there). */
#define QF_DECODER_MAX_K 4096
/* replaces decoder.rs:659 Decoder::new(k, pool): k <= 256 decodes by
 * Gauss-Jordan (or the Cauchy kernels), 256 < k <= QF_DECODER_MAX_K by the
 * Wiedemann strategy (decoder.rs:660-664, 794-975; qf_wiedemann.hip). */
int qf_decoder_new(qf_ctx *ctx, uint32_t k, uint32_t max_len, qf_decoder **out);
/* replaces decoder.rs:520-524 DecodingStrategy: 0 GaussianElimination,
 * 1 Wiedemann, as Decoder::new chose it; QF_EINVAL for NULL. */
#define QF_STRATEGY_GAUSSIAN 0
#define QF_STRATEGY_WIEDEMANN 1
int qf_decoder_strategy(const qf_decoder *dec);
/* Projections the last Wiedemann solve of this decoder tried (1..8; 9 = none
 * verified and exact elimination decided); 0 before any
 * Wiedemann solve and for k <= 256 decoders. */
int qf_decoder_solve_attempts(const qf_decoder *dec);
int qf_decoder_free(qf_decoder *dec);
/* replaces decoder.rs:678 Decoder::add_packet.  Returns 1 when the generation
 * is decoded, 0 when more packets are needed, QF_EINVAL for a repair packet
 * without coefficients ("Repair packet missing coefficients.").  A singular
 * matrix leaves the decoder undecoded, as in the reference. */
int qf_decoder_add_packet(qf_decoder *dec, uint64_t id, int is_systematic,
                          const uint8_t *data, uint32_t len, const uint8_t *coeffs,
                          uint32_t coeff_len);
/* replaces the decoder.rs:532 field is_decoded */
int qf_decoder_is_decoded(const qf_decoder *dec);
/* replaces decoder.rs:785 get_decoded_packets: drains the k source packets in
 * index order.  out_data holds k rows of out_stride bytes; out_len[i] and
 * out_ids[i] describe row i; *count = number of packets returned (k, or 0 if
 * not decoded or already drained). */
int qf_decoder_get_decoded_packets(qf_decoder *dec, uint8_t *out_data, uint32_t out_stride,
                                   uint32_t *out_len, uint64_t *out_ids, uint32_t *count);

/* ---------------------------------------------------------------------------
 * Adaptive FEC driver (adaptive.rs:44-631, mod.rs:56-79): loss estimator
 * (EMA + burst window + optional Kalman filter), PID-driven mode manager with
 * dwell time, hysteresis, emergency override and dynamic window, and the
 * per-connection sliding-window codec with a 32-packet cross-fade between
 * configurations.  The arithmetic is f32 exactly as the reference (no FP
 * contraction).  Time is in seconds on a monotonic clock; the *_at variants
 * take it explicitly (deterministic tests), the others read CLOCK_MONOTONIC.
 *
 * Codec: the GF(2^8) encoder/decoder objects above, and in Extreme mode the
 * GF(2^16) ones (decoder.rs:96-102; coefficient blocks of 2k bytes, so
 * coeff_stride >= 2k there).  A configuration the field cannot realise
 * (GF(2^8): k + r > 256, where the reference panics in gf_inv(0); GF(2^16):
 * k > 4096 or n > 65536) has no codec: on_send still emits the systematic
 * packet and returns QF_ERANGE.
 * ------------------------------------------------------------------------- */
#define QF_MODE_ZERO 0
#define QF_MODE_LIGHT 1
#define QF_MODE_NORMAL 2
#define QF_MODE_MEDIUM 3
#define QF_MODE_STRONG 4
#define QF_MODE_EXTREME 5
#define QF_CROSS_FADE_LEN 32   /* ModeManager::CROSS_FADE_LEN (adaptive.rs:114) */

typedef struct qf_fec_config {   /* FecConfig (adaptive.rs:338-349) */
    float lambda;                /* EMA smoothing factor */
    uint32_t burst_window;       /* burst-detection window (packets) */
    float hysteresis;
    float kp, ki, kd;            /* PidConfig */
    int32_t initial_mode;
    int32_t kalman_enabled;
    float kalman_q, kalman_r;
    uint32_t window_sizes[6];    /* initial window W0 per mode */
    uint32_t max_len;            /* payload capacity of the codec objects (bytes) */
} qf_fec_config;

/* FecConfig::default (adaptive.rs:435-452) + default_windows (352-362);
 * max_len = 1500. */
void qf_fec_config_default(qf_fec_config *cfg);
/* FecConfig::validate (adaptive.rs:455-471): QF_EINVAL on a bad field. */
int qf_fec_config_validate(const qf_fec_config *cfg);
/* ModeManager::params_for (adaptive.rs:149-153): k = window,
 * n = ceil(window * overhead_ratio(mode)) in f32. */
int qf_mode_params_for(int32_t mode, uint32_t window, uint32_t *k, uint32_t *n);
/* ModeManager::window_range (adaptive.rs:124-133). */
int qf_mode_window_range(int32_t mode, uint32_t *lo, uint32_t *hi);
/* ModeManager::overhead_ratio (adaptive.rs:135-147). */
float qf_mode_overhead_ratio(int32_t mode);

typedef struct qf_packet_desc {
    uint64_t id;
    uint32_t len;            /* payload bytes */
    uint32_t coeff_len;      /* coefficient bytes of a repair packet, else 0 */
    int32_t is_systematic;
    uint32_t reserved;
} qf_packet_desc;

typedef struct qf_adaptive qf_adaptive;
/* AdaptiveFec::new (adaptive.rs:473-508).  ctx may be NULL: controller only
 * (no codec objects; on_send emits the systematic packet, on_receive
 * recovers nothing) -- the mode logic then runs without a GPU. */
int qf_adaptive_new(qf_ctx *ctx, const qf_fec_config *cfg, qf_adaptive **out);
int qf_adaptive_new_at(qf_ctx *ctx, const qf_fec_config *cfg, double now_s, qf_adaptive **out);
int qf_adaptive_free(qf_adaptive *a);
/* current_mode / is_transitioning (adaptive.rs:510-517) and the rest of the
 * controller state (any pointer may be NULL). */
int qf_adaptive_state(const qf_adaptive *a, int32_t *mode, uint32_t *window, uint32_t *k,
                      uint32_t *n, int32_t *transitioning, uint32_t *transition_left,
                      float *estimated_loss);
/* Largest number of packets one on_send can emit (1 + repairs of the
 * current and the cross-fade configuration). */
uint32_t qf_adaptive_max_send_packets(const qf_adaptive *a);
/* Largest number of packets one on_receive can recover: the k of the
 * current decoder plus the k of the cross-fade decoder (both may complete
 * on the same packet, adaptive.rs:566-599).  A host sizes its reusable
 * receive buffers from it (INTEGRATION.md AdaptiveFec). */
uint32_t qf_adaptive_max_receive_packets(const qf_adaptive *a);
/* Smallest coeff_stride on_send accepts for the current and cross-fade
 * encoders: k bytes (GF(2^8)) or 2 k bytes (GF(2^16) Extreme windows). */
uint32_t qf_adaptive_max_coeff_bytes(const qf_adaptive *a);
/* AdaptiveFec::on_send (adaptive.rs:519-544) + emit_repairs (546-562): the
 * systematic packet, then the cross-fade configuration's repairs (while more
 * than CROSS_FADE_LEN/2 packets of the fade remain), then the current
 * configuration's repairs.  Packet i goes to out_data + i*out_stride (and
 * its coefficients to out_coeffs + i*coeff_stride); *n_out packets.
 * QF_ETOOSMALL if out_cap is too small (nothing is consumed then). */
int qf_adaptive_on_send(qf_adaptive *a, uint64_t id, const uint8_t *data, uint32_t len,
                        uint8_t *out_data, uint32_t out_stride, uint8_t *out_coeffs,
                        uint32_t coeff_stride, qf_packet_desc *out_desc, uint32_t out_cap,
                        uint32_t *n_out);
/* on_send for M connections at once (the server side of many QUIC
 * connections, core.rs:170-188 per packet): conns[m] sends packet (ids[m],
 * data[m], lens[m]).  The result is that of calling qf_adaptive_on_send for
 * m = 0..M-1 in order -- connection m's packets occupy out_data rows
 * [first_m, first_m + n_out[m]) with first_m = n_out[0] + ... + n_out[m-1],
 * and statuses[m] (nullable) gets that call's status -- but the steady-state
 * GF(2^8) connections of one context share one upload, one small-batch
 * encode launch per (k, n) class and one download.  A connection may appear
 * more than once (its packets are taken in order): a burst of one
 * connection's packets is one launch too, its overlapping windows read from
 * a staging copy of the ring's newest k - 1 rows and the burst (Normal mode,
 * 1,200-B packets: 18.5 us per packet alone, 1.2 us at 256 per call).  out_cap must cover the
 * sum of qf_adaptive_max_send_packets; out_stride / coeff_stride follow
 * qf_adaptive_on_send.  An argument error fails the whole call before any
 * state changes (QF_EINVAL / QF_ETOOSMALL); otherwise QF_OK. */
int qf_adaptive_on_send_batch(qf_adaptive *const *conns, uint32_t M, const uint64_t *ids,
                              const uint8_t *const *data, const uint32_t *lens, uint8_t *out_data,
                              uint32_t out_stride, uint8_t *out_coeffs, uint32_t coeff_stride,
                              qf_packet_desc *out_desc, uint32_t out_cap, uint32_t *n_out,
                              int32_t *statuses);
/* AdaptiveFec::on_receive (adaptive.rs:566-599): recovered packets (the
 * whole generation when a decoder completes, in source order: a received
 * systematic packet keeps its id, a reconstructed one gets id = i,
 * decoder.rs:688/771).  QF_EINVAL for a repair packet without coefficients. */
int qf_adaptive_on_receive(qf_adaptive *a, uint64_t id, int is_systematic, const uint8_t *data,
                           uint32_t len, const uint8_t *coeffs, uint32_t coeff_len,
                           uint8_t *out_data, uint32_t out_stride, qf_packet_desc *out_desc,
                           uint32_t out_cap, uint32_t *n_out);
/* on_receive for M connections at once: conns[m] receives packet m (ids,
 * is_systematic, data/lens, coeffs/coeff_lens: coeffs and coeff_lens may be
 * NULL when no packet carries coefficients).  The result is that of calling
 * qf_adaptive_on_receive for m = 0..M-1 in order -- connection m's recovered
 * packets occupy out_data rows [first_m, first_m + n_out[m]), first_m =
 * n_out[0] + ... + n_out[m-1], statuses[m] (nullable) gets that call's status
 * (e.g. QF_EINVAL for a repair without coefficients; such a packet is
 * dropped and the batch goes on) -- but the GF(2^8) decoders of one context
 * take their rows in one upload, and the generations that complete in the
 * call decode in one heterogeneous decode with one download.  out_cap must
 * cover the sum over connections of their decoders' k (the most one
 * on_receive can recover).  An argument error fails the whole call before any
 * state changes. */
int qf_adaptive_on_receive_batch(qf_adaptive *const *conns, uint32_t M, const uint64_t *ids,
                                 const int32_t *is_systematic, const uint8_t *const *data,
                                 const uint32_t *lens, const uint8_t *const *coeffs,
                                 const uint32_t *coeff_lens, uint8_t *out_data, uint32_t out_stride,
                                 qf_packet_desc *out_desc, uint32_t out_cap, uint32_t *n_out,
                                 int32_t *statuses);
/* AdaptiveFec::report_loss (adaptive.rs:602-630).  QF_EINVAL if lost > total
 * (the reference underflows). */
int qf_adaptive_report_loss(qf_adaptive *a, uint32_t lost, uint32_t total);
int qf_adaptive_report_loss_at(qf_adaptive *a, uint32_t lost, uint32_t total, double now_s);

/* ---------------------------------------------------------------------------
 * Wire framing, byte-compatible with encoder.rs:124-152 (to_raw) and
 * encoder.rs:18-68 (from_raw): [u8 sys(1/0)] [u16 BE coeff_len][coeffs] payload
 * (the coefficient header is present only when coeffs != NULL).
 * ------------------------------------------------------------------------- */
int qf_packet_to_raw(int is_systematic, const uint8_t *coeffs, uint32_t coeff_len,
                     const uint8_t *payload, uint32_t len, uint8_t *out, uint32_t out_cap,
                     uint32_t *out_len);
/* Parses a frame; pointers returned point into raw.  coeffs is NULL for
 * systematic frames. */
int qf_packet_from_raw(const uint8_t *raw, uint32_t raw_len, int *is_systematic,
                       const uint8_t **coeffs, uint32_t *coeff_len,
                       const uint8_t **payload, uint32_t *len);
/* replaces Packet::from_block (encoder.rs:72-121), the receive path of
 * core.rs:219-224: a frame of `len` valid bytes in a block of block_len bytes
 * is parsed in place; the coefficients are copied to coeffs_out (coeffs_cap
 * bytes) and the payload is moved to the front of the block (copy_within).
 * QF_EINVAL: len == 0 or len > block_len ("Invalid raw packet length");
 * QF_ETOOSMALL: coefficient length or coefficients truncated, or longer than
 * coeffs_cap / the block (where the reference would panic). */
int qf_packet_from_block(uint8_t *block, uint32_t block_len, uint32_t len, int *is_systematic,
                         uint8_t *coeffs_out, uint32_t coeffs_cap, uint32_t *coeff_len,
                         uint32_t *payload_len);

/* ---------------------------------------------------------------------------
 * Wire framing on the device (encoder.rs:18-152): the
 * step between UDP datagrams and the batch codec.
 * ------------------------------------------------------------------------- */
/* Frames of an encode batch, as Packet::to_raw writes them (encoder.rs:124-152):
 * generation g's k sources then its r repairs, frame f = g*(k+r) + i at
 * frames_dev + f*frame_stride:
 *   source i  0x01 | payload (L bytes)                                1 + L bytes
 *   repair j  0x00 | k as BE u16 | C[j][0..k) | payload (L bytes)     3 + k + L bytes
 * with C the reference's Cauchy rows (decoder.rs:280-298).  frame_len_dev
 * (may be NULL) receives each frame's length.  frame_stride % 16 == 0,
 * >= 3 + k + L; bytes of a frame past its length are not written. */
int qf_frame_batch_dev(qf_ctx *ctx, const qf_encode_shape *shape, uint32_t G, const uint8_t *src_dev,
                       const uint8_t *rep_dev, uint8_t *frames_dev, uint64_t frame_stride,
                       uint32_t *frame_len_dev);
/* Received frames -> qf_decode_batch input (Packet::from_raw, encoder.rs:18-68,
 * then Decoder::add_packet's column rule, decoder.rs:684).  Frame s of
 * generation g: frames_dev + (g*max_rows + s)*frame_stride, frame_len_dev[g*max_rows+s]
 * bytes, transport id ids_dev[g*max_rows+s]; n_frames_dev[g] frames (NULL: max_rows).
 * Valid frames are compacted in arrival order into rows_dev (payload zero
 * padded to L) with row_index_dev = id % k for a systematic frame, k + j for a
 * repair whose coefficient vector is Cauchy row j < r; n_rows_dev[g] = their
 * count.  frame_status_dev: QF_OK, QF_EINVAL (empty, payload > L),
 * QF_ETOOSMALL (coefficient length or coefficients truncated), QF_ERANGE
 * (coefficients are not a Cauchy row of this (k, r)).  max_rows <= 1024. */
int qf_parse_frames_dev(qf_ctx *ctx, uint32_t k, uint32_t r, uint32_t L, uint32_t G, uint32_t max_rows,
                        const uint8_t *frames_dev, uint64_t frame_stride, const uint32_t *frame_len_dev,
                        const uint64_t *ids_dev, const uint32_t *n_frames_dev, uint8_t *rows_dev,
                        uint64_t row_stride, uint64_t rows_gen_stride, uint16_t *row_index_dev,
                        uint32_t *n_rows_dev, int32_t *frame_status_dev);

/* ---------------------------------------------------------------------------
 * GF(2^16) "Extreme mode" codec.
 * replaces gf_tables.rs:331-380 (gf16_mul / gf16_pow / gf16_inv / gf16_mul_add)
 * and decoder.rs:10-88 (Encoder16), 536-656 (Decoder16).  Field mod 0x1100B
 * with the reduction gf16_mul intends (as written its u16 test of bit 16
 * never fires).  Payload symbols are big-endian u16 byte pairs
 * (decoder.rs:42-54); L must be even.
 * ------------------------------------------------------------------------- */
/* gf_tables.rs:333 gf16_mul (host helper) */
uint16_t qf_gf16_mul(uint16_t a, uint16_t b);
/* gf_tables.rs:370 gf16_inv; QF_ERANGE for 0 (the reference panics) */
int qf_gf16_inv(uint16_t a, uint16_t *out);
/* decoder.rs:77-80: out[j*k + i] = gf16_inv((u16)i ^ (u16)(k + j));
 * QF_ERANGE when k + r > 65536 (gf16_inv(0)). */
int qf_cauchy16_coeffs(uint32_t k, uint32_t r, uint16_t *out_rxk);
/* replaces decoder.rs:21-75 Encoder16::generate_repair_packet for r repairs
 * of G generations (layout as qf_encode_batch, shape->flags must be 0);
 * coeff_rxk: host u16 r x k matrix or NULL for the Cauchy rows. */
int qf_encode16_batch(qf_ctx *ctx, const qf_encode_shape *shape, uint32_t G, const uint8_t *src_dev,
                      uint8_t *rep_dev, const uint16_t *coeff_rxk);
/* replaces decoder.rs:563-656 Decoder16::{add_packet, try_decode,
 * get_decoded_packets} for G generations (layout as qf_decode_batch).
 * Acceptance as Decoder16: the first k rows, row index < k = systematic
 * column (the reference's id % k), no duplicate filtering (a duplicated
 * column is singular: QF_ERANK).  row_coeffs_dev: NULL (row index k + j
 * carries Cauchy row j) or k u16 per slot at (g*max_rows + slot)*k (the
 * packet's big-endian coefficient block, converted).  r sizes the output:
 * up to min(k, r) erasures per generation (QF_ERANGE status beyond).
 * min(k, r) <= 64: all generations at once (Gauss-Jordan in LDS); larger:
 * one generation at a time (closed-form Cauchy inverse, or Gauss-Jordan in
 * the workspace for explicit coefficients).  k <= 4096, r >= 1,
 * max_rows <= 65536 (QF_EINVAL beyond).  Recovered rows: erased sources
 * ascending, with rec_index / n_rec / status as qf_decode_batch. */
int qf_decode16_batch(qf_ctx *ctx, const qf_decode_shape *shape, uint32_t G, const uint8_t *rows_dev,
                      const uint16_t *row_index_dev, const uint32_t *n_rows_dev,
                      const uint16_t *row_coeffs_dev, uint8_t *rec_dev, uint16_t *rec_index_dev,
                      uint32_t *n_rec_dev, int32_t *status_dev);

/* GF(2^16) per-connection objects (the Extreme-mode codec of
 * EncoderVariant / DecoderVariant, decoder.rs:90-153).  k <= 4096 (Extreme
 * windows, adaptive.rs:131).  Coefficient blocks are 2k bytes, big-endian u16
 * (decoder.rs:62-66). */
typedef struct qf_encoder16 qf_encoder16;
/* replaces decoder.rs:17 Encoder16::new(k, n) */
int qf_encoder16_new(qf_ctx *ctx, uint32_t k, uint32_t n, uint32_t max_len, qf_encoder16 **out);
int qf_encoder16_free(qf_encoder16 *enc);
/* replaces decoder.rs:25 Encoder16::add_source_packet (slides the window) */
int qf_encoder16_add_source_packet(qf_encoder16 *enc, uint64_t id, const uint8_t *data, uint32_t len);
/* replaces decoder.rs:33 Encoder16::generate_repair_packet(j): QF_ENOTREADY
 * while the window is not full (None); len = window[0].len (an odd last
 * byte is 0, decoder.rs:44); out_coeffs 2k bytes; id = last.id + 1 + j. */
int qf_encoder16_generate_repair_packet(qf_encoder16 *enc, uint32_t repair_index, uint8_t *out_data,
                                        uint32_t out_cap, uint32_t *out_len, uint8_t *out_coeffs,
                                        uint64_t *out_id);
/* Repairs first..first+count-1 of the window in one launch; coefficient
 * blocks packed 2k bytes apart.  QF_ERANGE when k + first + count > 65536. */
int qf_encoder16_generate_repairs(qf_encoder16 *enc, uint32_t first, uint32_t count, uint8_t *out_data,
                                  uint32_t out_stride, uint32_t *out_len, uint8_t *out_coeffs,
                                  uint64_t *out_ids);
int qf_encoder16_window_len(const qf_encoder16 *enc);
typedef struct qf_decoder16 qf_decoder16;
/* replaces decoder.rs:545 Decoder16::new(k, pool) */
int qf_decoder16_new(qf_ctx *ctx, uint32_t k, uint32_t max_len, qf_decoder16 **out);
int qf_decoder16_free(qf_decoder16 *dec);
/* replaces decoder.rs:555 Decoder16::add_packet: the first k packets are the
 * system (no duplicate filtering); decoding runs when the k-th arrives
 * (whatever its kind).  1 = decoded, 0 = not (yet, or singular: stays so),
 * QF_EINVAL for a repair without coefficients ("missing coeffs"). */
int qf_decoder16_add_packet(qf_decoder16 *dec, uint64_t id, int is_systematic, const uint8_t *data,
                            uint32_t len, const uint8_t *coeffs, uint32_t coeff_len);
int qf_decoder16_is_decoded(const qf_decoder16 *dec);
/* replaces decoder.rs:643 get_decoded_packets: drains the k source packets in
 * index order (as qf_decoder_get_decoded_packets). */
int qf_decoder16_get_decoded_packets(qf_decoder16 *dec, uint8_t *out_data, uint32_t out_stride,
                                     uint32_t *out_len, uint64_t *out_ids, uint32_t *count);

/* ---------------------------------------------------------------------------
 * Synthetic payload (bench / tests): byte t of the region is byte (t & 7) of
 * splitmix64(seed + word_offset + t/8), little endian.  Device kernel.
 * ------------------------------------------------------------------------- */
int qf_fill_splitmix_dev(qf_ctx *ctx, uint8_t *dst_dev, size_t n, uint64_t seed,
                         uint64_t word_offset);

/* ---------------------------------------------------------------------------
 * Host self-test of the split-index v_perm tables the kernels use: checks
 * T0[x&7]^T1[x>>3&7]^T2[x>>6] == gf_mul_table(c, x) for all 65,536 (c, x)
 * with a host emulation of v_perm_b32.  Returns QF_OK or QF_EINVAL.
 * ------------------------------------------------------------------------- */
int qf_selftest_split_tables(void);

#ifdef __cplusplus
}
#endif
#endif /* QF_FEC_H */
