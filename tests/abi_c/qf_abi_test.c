/*
 * qf_abi_test.c -- drives libqf_fec.so through include/qf_fec.h from plain C
 * (TEST INFRASTRUCTURE: the caller a Rust / C integration would be), and
 * checks every result against the CPU oracle (oracle/liboracle.so).
 *
 *   batch     qf_encode_batch / qf_decode_batch       decoder.rs:172-275, 678-791
 *   desc      qf_encode_batch_desc / qf_decode_batch_desc (mixed windows)
 *   objects   qf_encoder_* / qf_decoder_*             decoder.rs:155-299, 658-791
 *   wiedemann qf_decoder_* with k > 256                decoder.rs:659-665, 794-975
 *   adaptive  qf_adaptive_on_send / on_receive / state adaptive.rs:508-599
 *             and their multi-connection batches (_on_send_batch / _on_receive_batch)
 *   framing   qf_packet_to_raw / from_raw / from_block encoder.rs:18-152
 *
 * Exit status 0 and "ALL OK" on success; the first mismatch is printed.
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/qf_fec.h"
#include "../../oracle/qf_oracle.h"

#define CHECK(cond, ...)                                            \
    do {                                                            \
        if (!(cond)) {                                              \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);    \
            fprintf(stderr, __VA_ARGS__);                           \
            fprintf(stderr, "\n");                                  \
            exit(1);                                                \
        }                                                           \
    } while (0)
#define QF(call) CHECK((call) == QF_OK, "%s -> %s", #call, qf_strerror(call))
#define HIP(call) CHECK((call) == hipSuccess, "%s", #call)

static uint64_t rng_state = 0x51464543u;
static uint8_t rnd8(void) {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint8_t)(rng_state >> 56);
}
static uint32_t rnd(uint32_t n) {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)((rng_state >> 33) % n);
}

static void *dev_alloc(size_t n) {
    void *p = NULL;
    HIP(hipMalloc(&p, n ? n : 16));
    return p;
}

/* e distinct sorted source indices < k */
static void erasures(uint32_t k, uint32_t e, uint32_t *E) {
    uint8_t taken[256] = {0};
    for (uint32_t q = 0; q < e;) {
        uint32_t i = rnd(k);
        if (!taken[i]) taken[i] = 1, ++q;
    }
    for (uint32_t i = 0, q = 0; i < k; ++i)
        if (taken[i]) E[q++] = i;
}

static void test_gf(void) {
    oracle_gf_init();
    QF(qf_gf256_init());
    for (int a = 0; a < 256; ++a)
        for (int b = 0; b < 256; ++b)
            CHECK(qf_gf256_mul((uint8_t)a, (uint8_t)b) == oracle_gf_mul((uint8_t)a, (uint8_t)b), "mul %d %d", a, b);
    uint8_t c[64 * 16], o[64 * 16];
    QF(qf_cauchy_coeffs(64, 16, c));
    CHECK(oracle_cauchy_coeffs(64, 16, o) == 0 && memcmp(c, o, sizeof c) == 0, "cauchy 64/16");
    uint8_t x;
    CHECK(qf_gf256_inv(0, &x) == QF_ERANGE, "inv(0) must be ERANGE (reference panics)");
}

static void test_batch(qf_ctx *ctx) {
    const uint32_t k = 64, r = 16, L = 1200, G = 48, e = 13, n = k - e + r, emax = 16;
    const size_t sb = (size_t)G * k * L, rb = (size_t)G * r * L;
    uint8_t *src = malloc(sb), *rep = malloc(rb), *want = malloc((size_t)r * L);
    for (size_t t = 0; t < sb; ++t) src[t] = rnd8();
    uint8_t *d_src = dev_alloc(sb), *d_rep = dev_alloc(rb);
    HIP(hipMemcpy(d_src, src, sb, hipMemcpyHostToDevice));
    qf_encode_shape sh = {k, r, L, 0, L, (uint64_t)k * L, L, (uint64_t)r * L};
    QF(qf_encode_batch(ctx, &sh, G, d_src, d_rep, NULL));
    QF(qf_sync(ctx));
    HIP(hipMemcpy(rep, d_rep, rb, hipMemcpyDeviceToHost));
    for (uint32_t g = 0; g < G; ++g) {
        CHECK(oracle_encode_window(k, r, L, src + (size_t)g * k * L, L, NULL, want, L) == 0, "oracle encode");
        CHECK(memcmp(want, rep + (size_t)g * r * L, (size_t)r * L) == 0, "encode generation %u", g);
    }
    /* decode: surviving sources then repairs, first k rows win */
    uint8_t *rows = malloc((size_t)G * n * L), *rec = malloc((size_t)G * emax * L), *sol = malloc((size_t)k * L);
    uint16_t *idx = malloc((size_t)G * n * 2), *ridx = malloc((size_t)G * emax * 2);
    uint32_t E[64], *nrec = malloc(G * 4);
    int32_t *st = malloc(G * 4);
    uint32_t *Es = malloc((size_t)G * e * 4);
    for (uint32_t g = 0; g < G; ++g) {
        erasures(k, e, E);
        memcpy(Es + g * e, E, e * 4);
        uint32_t s = 0;
        for (uint32_t i = 0, q = 0; i < k; ++i) {
            if (q < e && E[q] == i) { ++q; continue; }
            idx[g * n + s] = (uint16_t)i;
            memcpy(rows + ((size_t)g * n + s++) * L, src + ((size_t)g * k + i) * L, L);
        }
        for (uint32_t j = 0; j < r; ++j) {
            idx[g * n + s] = (uint16_t)(k + j);
            memcpy(rows + ((size_t)g * n + s++) * L, rep + ((size_t)g * r + j) * L, L);
        }
    }
    uint8_t *d_rows = dev_alloc((size_t)G * n * L), *d_rec = dev_alloc((size_t)G * emax * L);
    uint16_t *d_idx = dev_alloc((size_t)G * n * 2), *d_ridx = dev_alloc((size_t)G * emax * 2);
    uint32_t *d_nrec = dev_alloc(G * 4);
    int32_t *d_st = dev_alloc(G * 4);
    HIP(hipMemcpy(d_rows, rows, (size_t)G * n * L, hipMemcpyHostToDevice));
    HIP(hipMemcpy(d_idx, idx, (size_t)G * n * 2, hipMemcpyHostToDevice));
    qf_decode_shape dsh = {k, r, L, n, L, (uint64_t)n * L, L, (uint64_t)emax * L};
    QF(qf_decode_batch(ctx, &dsh, G, d_rows, d_idx, NULL, NULL, d_rec, d_ridx, d_nrec, d_st));
    QF(qf_sync(ctx));
    HIP(hipMemcpy(rec, d_rec, (size_t)G * emax * L, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(ridx, d_ridx, (size_t)G * emax * 2, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(nrec, d_nrec, G * 4, hipMemcpyDeviceToHost));
    HIP(hipMemcpy(st, d_st, G * 4, hipMemcpyDeviceToHost));
    uint8_t mask[64];
    for (uint32_t g = 0; g < G; ++g) {
        CHECK(st[g] == QF_OK && nrec[g] == e, "decode status %d / n_rec %u of generation %u", st[g], nrec[g], g);
        CHECK(oracle_decode_generation(k, L, n, idx + g * n, rows + (size_t)g * n * L, L, NULL, sol, L, mask) == 0,
              "oracle decode");
        for (uint32_t m = 0; m < e; ++m) {
            const uint32_t i = Es[g * e + m];
            CHECK(ridx[g * emax + m] == i && !mask[i], "rec index g %u m %u", g, m);
            CHECK(memcmp(rec + ((size_t)g * emax + m) * L, sol + (size_t)i * L, L) == 0, "recovered g %u row %u", g, i);
            CHECK(memcmp(sol + (size_t)i * L, src + ((size_t)g * k + i) * L, L) == 0, "oracle != source");
        }
    }
    hipFree(d_src); hipFree(d_rep); hipFree(d_rows); hipFree(d_rec); hipFree(d_idx); hipFree(d_ridx);
    hipFree(d_nrec); hipFree(d_st);
    free(src); free(rep); free(want); free(rows); free(rec); free(sol); free(idx); free(ridx); free(nrec);
    free(st); free(Es);
    printf("batch ok\n");
}

static void test_desc(qf_ctx *ctx) {
    /* two window shapes interleaved at reversed offsets (C5: Normal 64/10, Medium 160/48) */
    const uint32_t G = 6, L = 1200;
    const uint32_t ks[6] = {64, 160, 64, 160, 64, 160}, rs[6] = {10, 48, 10, 48, 10, 48};
    qf_gen_desc d[6];
    size_t so = 0, ro = 0;
    for (int q = 5; q >= 0; --q) {
        d[q].k = ks[q]; d[q].r = rs[q]; d[q].L = L; d[q].flags = 0;
        d[q].src_offset = so; d[q].src_row_stride = L;
        d[q].rep_offset = ro; d[q].rep_row_stride = L;
        so += (size_t)ks[q] * L + 64;
        ro += (size_t)rs[q] * L + 32;
    }
    uint8_t *src = malloc(so), *rep = malloc(ro), *want = malloc((size_t)48 * L);
    for (size_t t = 0; t < so; ++t) src[t] = rnd8();
    uint8_t *d_src = dev_alloc(so), *d_rep = dev_alloc(ro);
    HIP(hipMemcpy(d_src, src, so, hipMemcpyHostToDevice));
    QF(qf_encode_batch_desc(ctx, d, G, d_src, d_rep));
    QF(qf_sync(ctx));
    HIP(hipMemcpy(rep, d_rep, ro, hipMemcpyDeviceToHost));
    for (uint32_t q = 0; q < G; ++q) {
        CHECK(oracle_encode_window(ks[q], rs[q], L, src + d[q].src_offset, L, NULL, want, L) == 0, "oracle");
        CHECK(memcmp(want, rep + d[q].rep_offset, (size_t)rs[q] * L) == 0, "desc encode generation %u", q);
    }
    hipFree(d_src); hipFree(d_rep);
    free(src); free(rep); free(want);
    printf("desc ok\n");
}

static void test_objects(qf_ctx *ctx) {
    const uint32_t k = 16, n = 20, r = 4, L = 1200, T = 40;
    qf_encoder *enc;
    QF(qf_encoder_new(ctx, k, n, L, &enc));
    uint8_t *pk = malloc((size_t)T * L), out[4 * 1200], coeffs[4 * 16], want[4 * 1200];
    uint32_t lens[4];
    uint64_t ids[4];
    for (size_t t = 0; t < (size_t)T * L; ++t) pk[t] = rnd8();
    for (uint32_t t = 0; t < T; ++t) {
        QF(qf_encoder_add_source_packet(enc, 1000 + t, pk + (size_t)t * L, L));
        const int s = qf_encoder_generate_repairs(enc, 0, r, out, L, lens, coeffs, ids);
        if (t + 1 < k) {
            CHECK(s == QF_ENOTREADY, "window not full must be ENOTREADY (reference: None)");
            continue;
        }
        CHECK(s == QF_OK, "generate_repairs %d", s);
        CHECK(oracle_encode_window(k, r, L, pk + (size_t)(t + 1 - k) * L, L, NULL, want, L) == 0, "oracle");
        CHECK(memcmp(out, want, sizeof want) == 0, "object repairs after packet %u", t);
        for (uint32_t j = 0; j < r; ++j) CHECK(ids[j] == 1000 + t + 1 + j && lens[j] == L, "repair id / len");
    }
    /* decoder: generation = the last window (ids 1024..1039), 3 sources lost */
    qf_decoder *dec;
    QF(qf_decoder_new(ctx, k, L, &dec));
    const uint32_t lost[3] = {1, 7, 12};
    int decoded = 0;
    for (uint32_t i = 0; i < k; ++i) {
        if (i == lost[0] || i == lost[1] || i == lost[2]) continue;
        decoded = qf_decoder_add_packet(dec, 1024 + i, 1, pk + (size_t)(24 + i) * L, L, NULL, 0);
        CHECK(decoded == 0, "decoded too early");
    }
    CHECK(qf_decoder_add_packet(dec, 99, 0, out, L, NULL, 0) == QF_EINVAL,
          "repair without coefficients (decoder.rs:699)");
    for (uint32_t j = 0; j < 3; ++j) decoded = qf_decoder_add_packet(dec, 1040 + j, 0, out + j * L, L, coeffs + j * k, k);
    CHECK(decoded == 1 && qf_decoder_is_decoded(dec) == 1, "generation not decoded");
    uint8_t *got = malloc((size_t)k * L);
    uint32_t glen[16], cnt;
    uint64_t gid[16];
    QF(qf_decoder_get_decoded_packets(dec, got, L, glen, gid, &cnt));
    CHECK(cnt == k, "count %u", cnt);
    for (uint32_t i = 0; i < k; ++i) {
        const int was_lost = i == lost[0] || i == lost[1] || i == lost[2];
        CHECK(gid[i] == (was_lost ? i : 1024 + i), "id rule (decoder.rs:688/771) for packet %u: %llu", i,
              (unsigned long long)gid[i]);
        CHECK(glen[i] == L && memcmp(got + (size_t)i * L, pk + (size_t)(24 + i) * L, L) == 0, "packet %u", i);
    }
    QF(qf_decoder_get_decoded_packets(dec, got, L, glen, gid, &cnt));
    CHECK(cnt == 0, "get_decoded_packets drains (take())");
    QF(qf_decoder_free(dec));
    QF(qf_encoder_free(enc));
    free(pk); free(got);
    printf("objects ok\n");
}

/* decoder.rs:659-665 / 794-975: a k > 256 decoder takes the Wiedemann strategy;
 * repairs with explicit coefficients, checked against oracle_wiedemann_decode */
static void test_wiedemann(qf_ctx *ctx) {
    const uint32_t k = 300, e = 5, L = 200;
    qf_decoder *dec;
    QF(qf_decoder_new(ctx, k, L, &dec));
    CHECK(qf_decoder_strategy(dec) == QF_STRATEGY_WIEDEMANN, "strategy for k = %u", k);
    uint8_t *src = malloc((size_t)k * L), *coef = malloc((size_t)e * k), *rep = malloc((size_t)e * L);
    for (size_t t = 0; t < (size_t)k * L; ++t) src[t] = rnd8();
    for (size_t t = 0; t < (size_t)e * k; ++t) coef[t] = rnd8();
    CHECK(oracle_encode_window(k, e, L, src, L, coef, rep, L) == 0, "oracle encode");
    uint8_t lost[300] = {0};
    for (uint32_t q = 0; q < e;) {
        const uint32_t i = rnd(k);
        if (!lost[i]) lost[i] = 1, ++q;
    }
    /* arrival: surviving sources, then the repairs */
    uint16_t *idx = malloc(sizeof(uint16_t) * k);
    uint8_t *rows = malloc((size_t)k * L), *rc = calloc((size_t)k, k);
    uint32_t n = 0;
    int decoded = 0;
    for (uint32_t i = 0; i < k; ++i) {
        if (lost[i]) continue;
        idx[n] = (uint16_t)i;
        memcpy(rows + (size_t)n++ * L, src + (size_t)i * L, L);
        decoded = qf_decoder_add_packet(dec, i, 1, src + (size_t)i * L, L, NULL, 0);
        CHECK(decoded == 0, "decoded too early");
    }
    for (uint32_t j = 0; j < e; ++j) {
        idx[n] = (uint16_t)(k + j);
        memcpy(rows + (size_t)n * L, rep + (size_t)j * L, L);
        memcpy(rc + (size_t)n++ * k, coef + (size_t)j * k, k);
        decoded = qf_decoder_add_packet(dec, 5000 + j, 0, rep + (size_t)j * L, L, coef + (size_t)j * k, k);
    }
    CHECK(decoded == 1, "k = %u generation not decoded", k);
    uint8_t *want = malloc((size_t)k * L), *got = malloc((size_t)k * L);
    CHECK(oracle_wiedemann_decode(k, L, n, idx, rows, L, rc, want, L, NULL, NULL) == 0, "oracle wiedemann");
    uint32_t *glen = malloc(4 * k), cnt;
    uint64_t *gid = malloc(8 * k);
    QF(qf_decoder_get_decoded_packets(dec, got, L, glen, gid, &cnt));
    CHECK(cnt == k && memcmp(got, want, (size_t)k * L) == 0 && memcmp(got, src, (size_t)k * L) == 0,
          "k > 256 decode == oracle");
    QF(qf_decoder_free(dec));
    free(src); free(coef); free(rep); free(idx); free(rows); free(rc); free(want); free(got); free(glen); free(gid);
    printf("wiedemann ok\n");
}

static void test_adaptive(qf_ctx *ctx) {
    qf_fec_config cfg;
    qf_fec_config_default(&cfg);
    cfg.initial_mode = QF_MODE_NORMAL;
    cfg.max_len = 1200;
    QF(qf_fec_config_validate(&cfg));
    qf_adaptive *snd, *rcv;
    QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &snd));
    QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &rcv));
    int32_t mode, trans;
    uint32_t k, n;
    QF(qf_adaptive_state(snd, &mode, NULL, &k, &n, &trans, NULL, NULL));
    CHECK(mode == QF_MODE_NORMAL && k == 64 && n == 74 && !trans, "Normal mode params_for(64) = (64, 74)");
    const uint32_t L = 1000, cap = qf_adaptive_max_send_packets(snd);
    uint8_t *pk = malloc((size_t)k * L), *out = malloc((size_t)cap * 1200), *co = malloc((size_t)cap * 256);
    qf_packet_desc *desc = malloc(cap * sizeof(qf_packet_desc));
    uint8_t *want = malloc((size_t)10 * L);
    for (size_t t = 0; t < (size_t)k * L; ++t) pk[t] = rnd8();
    uint32_t nout = 0;
    CHECK(qf_adaptive_on_send(snd, 0, pk, L, out, L, co, 256, desc, cap, &nout) == QF_ETOOSMALL,
          "out_stride below max_len must fail before any state change");
    for (uint32_t i = 0; i < k; ++i) {
        QF(qf_adaptive_on_send(snd, i, pk + (size_t)i * L, L, out, 1200, co, 256, desc, cap, &nout));
        CHECK(desc[0].is_systematic && desc[0].id == i && memcmp(out, pk + (size_t)i * L, L) == 0, "systematic out");
        CHECK(nout == (i + 1 < k ? 1 : 1 + n - k), "packets out after %u: %u", i, nout);
    }
    CHECK(oracle_encode_window(k, n - k, L, pk, L, NULL, want, L) == 0, "oracle");
    for (uint32_t j = 0; j < n - k; ++j)
        CHECK(memcmp(out + (size_t)(1 + j) * 1200, want + (size_t)j * L, L) == 0 && desc[1 + j].coeff_len == k,
              "adaptive repair %u", j);
    /* receiver: 5 sources lost, then the repairs; recovery completes the generation */
    uint8_t *rout = malloc((size_t)k * 1200);
    qf_packet_desc *rdesc = malloc(k * sizeof(qf_packet_desc));
    uint32_t got = 0, m = 0;
    for (uint32_t i = 0; i < k; ++i) {
        if (i % 13 == 5) continue;
        QF(qf_adaptive_on_receive(rcv, i, 1, pk + (size_t)i * L, L, NULL, 0, rout, 1200, rdesc, k, &m));
        got += m;
    }
    for (uint32_t j = 0; j < n - k && !got; ++j) {
        QF(qf_adaptive_on_receive(rcv, k + j, 0, out + (size_t)(1 + j) * 1200, L, co + (size_t)(1 + j) * 256, k,
                                  rout, 1200, rdesc, k, &m));
        got += m;
    }
    CHECK(got == k, "recovered %u of %u", got, k);
    for (uint32_t i = 0; i < k; ++i)
        CHECK(rdesc[i].id == i && memcmp(rout + (size_t)i * 1200, pk + (size_t)i * L, L) == 0, "received %u", i);
    QF(qf_adaptive_free(snd));
    QF(qf_adaptive_free(rcv));
    free(pk); free(out); free(co); free(desc); free(want); free(rout); free(rdesc);
    printf("adaptive ok\n");
}

/* The buffer pattern of INTEGRATION.md's AdaptiveFec: output rows, coefficient
 * blocks and descriptors are owned by the connection, sized from
 * qf_adaptive_max_send_packets / _max_coeff_bytes / _max_receive_packets and
 * grown (never re-allocated per packet), across 16 generations = 1,024
 * on_receive calls.  After each generation both sides report the loss, which
 * rebuilds their codecs (adaptive.rs:602-630), as a connection's loss report
 * would; every recovered payload is checked. */
typedef struct {
    uint8_t *data, *coeffs;
    qf_packet_desc *desc;
    size_t rows, coeff_bytes, grows;
} reuse_bufs;

static void reuse_grow(reuse_bufs *b, size_t rows, size_t row_bytes, size_t coeff_bytes) {
    if (rows <= b->rows && coeff_bytes <= b->coeff_bytes) return;
    if (rows < b->rows) rows = b->rows;
    if (coeff_bytes < b->coeff_bytes) coeff_bytes = b->coeff_bytes;
    b->data = realloc(b->data, rows * row_bytes);
    b->coeffs = realloc(b->coeffs, rows * (coeff_bytes ? coeff_bytes : 1));
    b->desc = realloc(b->desc, rows * sizeof(qf_packet_desc));
    CHECK(b->data && b->coeffs && b->desc, "realloc");
    b->rows = rows, b->coeff_bytes = coeff_bytes, ++b->grows;
}

static void test_adaptive_reuse(qf_ctx *ctx) {
    qf_fec_config cfg;
    qf_fec_config_default(&cfg);
    cfg.initial_mode = QF_MODE_NORMAL;
    cfg.max_len = 1200;
    qf_adaptive *snd, *rcv;
    QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &snd));
    QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &rcv));
    uint32_t k, n;
    QF(qf_adaptive_state(snd, NULL, NULL, &k, &n, NULL, NULL, NULL));
    CHECK(qf_adaptive_max_receive_packets(rcv) == k, "max_receive_packets = k outside a cross-fade");
    CHECK(qf_adaptive_max_coeff_bytes(snd) == k, "max_coeff_bytes = k (GF(2^8))");
    const uint32_t L = 1200, gens = 16;
    reuse_bufs sb = {0}, rb = {0};
    uint8_t *pk = malloc((size_t)k * L), *rep = malloc((size_t)(n - k) * L), *rco = malloc((size_t)(n - k) * k);
    uint8_t *got_rows = malloc((size_t)k * L);
    uint32_t calls = 0;
    for (uint32_t g = 0; g < gens; ++g) {
        for (size_t t = 0; t < (size_t)k * L; ++t) pk[t] = rnd8();
        for (uint32_t i = 0; i < k; ++i) {
            reuse_grow(&sb, qf_adaptive_max_send_packets(snd), cfg.max_len, qf_adaptive_max_coeff_bytes(snd));
            uint32_t nout = 0;
            QF(qf_adaptive_on_send(snd, (uint64_t)g * k + i, pk + (size_t)i * L, L, sb.data, cfg.max_len, sb.coeffs,
                                   (uint32_t)sb.coeff_bytes, sb.desc, (uint32_t)sb.rows, &nout));
            CHECK(nout == (i + 1 < k ? 1u : 1 + n - k), "gen %u packet %u: %u out", g, i, nout);
            for (uint32_t j = 0; j + 1 < nout; ++j) {
                memcpy(rep + (size_t)j * L, sb.data + (size_t)(1 + j) * cfg.max_len, L);
                memcpy(rco + (size_t)j * k, sb.coeffs + (size_t)(1 + j) * sb.coeff_bytes, k);
            }
        }
        uint32_t got = 0, m = 0;
        uint8_t seen[256] = {0};
        for (uint32_t i = 0; i < k; ++i) {
            if ((i + g) % 13 == 5) continue;   /* lost */
            reuse_grow(&rb, qf_adaptive_max_receive_packets(rcv), cfg.max_len, 0);
            QF(qf_adaptive_on_receive(rcv, i, 1, pk + (size_t)i * L, L, NULL, 0, rb.data, cfg.max_len, rb.desc,
                                      (uint32_t)rb.rows, &m));
            ++calls;
            for (uint32_t q = 0; q < m; ++q) {
                const qf_packet_desc *d = &rb.desc[q];
                CHECK(d->id < k && d->len == L && !seen[d->id], "gen %u recovered id %llu", g, (unsigned long long)d->id);
                seen[d->id] = 1;
                memcpy(got_rows + (size_t)d->id * L, rb.data + (size_t)q * cfg.max_len, L);
            }
            got += m;
        }
        for (uint32_t j = 0; j < n - k && got < k; ++j) {
            reuse_grow(&rb, qf_adaptive_max_receive_packets(rcv), cfg.max_len, 0);
            QF(qf_adaptive_on_receive(rcv, k + j, 0, rep + (size_t)j * L, L, rco + (size_t)j * k, k, rb.data,
                                      cfg.max_len, rb.desc, (uint32_t)rb.rows, &m));
            ++calls;
            for (uint32_t q = 0; q < m; ++q) {
                const qf_packet_desc *d = &rb.desc[q];
                CHECK(d->id < k && d->len == L && !seen[d->id], "gen %u recovered id %llu", g, (unsigned long long)d->id);
                seen[d->id] = 1;
                memcpy(got_rows + (size_t)d->id * L, rb.data + (size_t)q * cfg.max_len, L);
            }
            got += m;
        }
        CHECK(got == k, "gen %u: recovered %u of %u", g, got, k);
        CHECK(memcmp(got_rows, pk, (size_t)k * L) == 0, "gen %u payloads", g);
        /* the next generation: a loss report rebuilds both codecs (no mode change in the dwell time) */
        QF(qf_adaptive_report_loss_at(snd, 0, 100, 0.0));
        QF(qf_adaptive_report_loss_at(rcv, 0, 100, 0.0));
    }
    CHECK(calls >= 1000, "only %u on_receive calls", calls);
    CHECK(sb.grows == 1 && rb.grows == 1, "buffers grown %zu / %zu times (expected once)", sb.grows, rb.grows);
    QF(qf_adaptive_free(snd));
    QF(qf_adaptive_free(rcv));
    free(sb.data); free(sb.coeffs); free(sb.desc); free(rb.data); free(rb.coeffs); free(rb.desc);
    free(pk); free(rep); free(rco); free(got_rows);
    printf("adaptive reuse ok (%u on_receive calls, one allocation per side)\n", calls);
}

/* qf_adaptive_on_send_batch / on_receive_batch over C connections: every
 * connection's repairs equal the oracle's encode of its window, and every
 * receiver recovers its generation. */
static void test_adaptive_batch(qf_ctx *ctx) {
    enum { C = 8 };
    qf_fec_config cfg;
    qf_fec_config_default(&cfg);
    cfg.initial_mode = QF_MODE_NORMAL;
    cfg.max_len = 1200;
    qf_adaptive *snd[C], *rcv[C];
    for (int c = 0; c < C; ++c) {
        QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &snd[c]));
        QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &rcv[c]));
    }
    uint32_t k, n;
    QF(qf_adaptive_state(snd[0], NULL, NULL, &k, &n, NULL, NULL, NULL));
    const uint32_t r = n - k, per = qf_adaptive_max_send_packets(snd[0]), cap = per * C;
    const uint32_t L = 1100;
    uint8_t *pk = malloc((size_t)C * k * L), *out = malloc((size_t)cap * 1200), *co = malloc((size_t)cap * 256);
    uint8_t *rep = malloc((size_t)C * r * 1200), *rco = malloc((size_t)C * r * 256), *want = malloc((size_t)r * L);
    qf_packet_desc *desc = malloc(cap * sizeof(qf_packet_desc));
    uint32_t n_out[C];
    int32_t st[C];
    for (size_t t = 0; t < (size_t)C * k * L; ++t) pk[t] = rnd8();
    for (uint32_t i = 0; i < k; ++i) {
        uint64_t ids[C];
        const uint8_t *data[C];
        uint32_t lens[C];
        for (int c = 0; c < C; ++c) ids[c] = i, data[c] = pk + ((size_t)c * k + i) * L, lens[c] = L;
        QF(qf_adaptive_on_send_batch(snd, C, ids, data, lens, out, 1200, co, 256, desc, cap, n_out, st));
        uint32_t pos = 0;
        for (int c = 0; c < C; ++c) {
            CHECK(st[c] == QF_OK && n_out[c] == (i + 1 < k ? 1 : 1 + r), "send batch count %u/%d: %u", i, c, n_out[c]);
            CHECK(desc[pos].is_systematic && desc[pos].id == i && memcmp(out + (size_t)pos * 1200, data[c], L) == 0,
                  "send batch systematic %u/%d", i, c);
            for (uint32_t j = 0; j + 1 < n_out[c]; ++j) {
                memcpy(rep + ((size_t)c * r + j) * 1200, out + (size_t)(pos + 1 + j) * 1200, 1200);
                memcpy(rco + ((size_t)c * r + j) * 256, co + (size_t)(pos + 1 + j) * 256, 256);
                CHECK(desc[pos + 1 + j].id == k + j && desc[pos + 1 + j].coeff_len == k, "repair desc");
            }
            pos += n_out[c];
        }
    }
    for (int c = 0; c < C; ++c) {
        CHECK(oracle_encode_window(k, r, L, pk + (size_t)c * k * L, L, NULL, want, L) == 0, "oracle");
        for (uint32_t j = 0; j < r; ++j)
            CHECK(memcmp(rep + ((size_t)c * r + j) * 1200, want + (size_t)j * L, L) == 0, "batch repair %d/%u", c, j);
    }
    /* receivers: connection c loses sources c + 7 q (q < 3), then gets the repairs */
    uint8_t *rout = malloc((size_t)C * k * 1200);
    qf_packet_desc *rdesc = malloc((size_t)C * k * sizeof(qf_packet_desc));
    uint32_t got[C] = {0};
    uint8_t *recv = calloc((size_t)C * k, 1200);
    for (uint32_t t = 0; t < k + r; ++t) {
        uint64_t ids[C];
        int32_t sys[C];
        const uint8_t *data[C], *cf[C];
        uint32_t lens[C], cl[C];
        uint32_t M = 0;
        qf_adaptive *conns[C];
        int which[C];
        for (int c = 0; c < C; ++c) {
            if (t < k && (t == (uint32_t)c || t == (uint32_t)c + 7 || t == (uint32_t)c + 14)) continue;  /* lost */
            conns[M] = rcv[c];
            which[M] = c;
            if (t < k) {
                ids[M] = t, sys[M] = 1, data[M] = pk + ((size_t)c * k + t) * L, lens[M] = L, cf[M] = NULL, cl[M] = 0;
            } else {
                const uint32_t j = t - k;
                ids[M] = k + j, sys[M] = 0, data[M] = rep + ((size_t)c * r + j) * 1200, lens[M] = L;
                cf[M] = rco + ((size_t)c * r + j) * 256, cl[M] = k;
            }
            ++M;
        }
        QF(qf_adaptive_on_receive_batch(conns, M, ids, sys, data, lens, cf, cl, rout, 1200, rdesc, C * k, n_out, st));
        uint32_t pos = 0;
        for (uint32_t q = 0; q < M; ++q) {
            CHECK(st[q] == QF_OK, "receive batch status %d", st[q]);
            for (uint32_t i = 0; i < n_out[q]; ++i) {
                const qf_packet_desc *d = &rdesc[pos + i];
                CHECK(d->id < k && d->len == L, "recovered id/len");
                memcpy(recv + ((size_t)which[q] * k + d->id) * 1200, rout + (size_t)(pos + i) * 1200, L);
            }
            got[which[q]] += n_out[q];
            pos += n_out[q];
        }
    }
    for (int c = 0; c < C; ++c) {
        CHECK(got[c] == k, "connection %d recovered %u of %u", c, got[c], k);
        for (uint32_t i = 0; i < k; ++i)
            CHECK(memcmp(recv + ((size_t)c * k + i) * 1200, pk + ((size_t)c * k + i) * L, L) == 0, "payload %d/%u", c, i);
        QF(qf_adaptive_free(snd[c]));
        QF(qf_adaptive_free(rcv[c]));
    }
    free(pk); free(out); free(co); free(rep); free(rco); free(want); free(desc); free(rout); free(rdesc); free(recv);
    printf("adaptive batch ok\n");
}

static void test_framing(void) {
    uint8_t payload[1200], coeffs[64], frame[1300], oframe[1300];
    for (int t = 0; t < 1200; ++t) payload[t] = rnd8();
    for (int t = 0; t < 64; ++t) coeffs[t] = rnd8();
    uint32_t len;
    size_t olen;
    QF(qf_packet_to_raw(0, coeffs, 64, payload, 1200, frame, sizeof frame, &len));
    CHECK(oracle_packet_to_raw(0, 1, coeffs, 64, 1, payload, 1200, oframe, sizeof oframe, &olen) == 0, "oracle");
    CHECK(len == 1267 && olen == len && memcmp(frame, oframe, len) == 0, "repair frame (1 + 2 + 64 + 1200 B)");
    CHECK(qf_packet_to_raw(0, coeffs, 64, payload, 1200, frame, 1266, &len) == QF_ETOOSMALL, "BufferTooShort");
    int sys;
    const uint8_t *c, *p;
    uint32_t cl, pl;
    QF(qf_packet_from_raw(oframe, (uint32_t)olen, &sys, &c, &cl, &p, &pl));
    CHECK(!sys && cl == 64 && pl == 1200 && memcmp(p, payload, 1200) == 0, "from_raw");
    uint8_t block[1300] = {0}, blk2[1300] = {0}, cout[64];
    memcpy(block, oframe, olen);
    memcpy(blk2, oframe, olen);
    uint32_t bcl, bpl;
    QF(qf_packet_from_block(block, sizeof block, (uint32_t)olen, &sys, cout, sizeof cout, &bcl, &bpl));
    int osys;
    uint32_t ocl;
    size_t opl;
    uint8_t ocout[64];
    CHECK(oracle_packet_from_block(blk2, sizeof blk2, olen, &osys, ocout, &ocl, &opl) == 0, "oracle from_block");
    CHECK(sys == osys && bcl == ocl && bpl == opl && memcmp(block, blk2, sizeof block) == 0 &&
          memcmp(cout, ocout, 64) == 0, "from_block == oracle");
    printf("framing ok\n");
}

/* qf_ctx_set_option / qf_ctx_get_option: ranges, unknown options, and the
 * batch codec on the coefficient-block kernels (QF_OPT_FFT_KERNELS = 0) and
 * the general v_perm paths (QF_OPT_BITSLICED = 0), both against the oracle */
static void test_options(qf_ctx *ctx) {
    int64_t v = -7;
    QF(qf_ctx_get_option(ctx, QF_OPT_FFT_KERNELS, &v));
    CHECK(v == 1, "fft_kernels default %lld", (long long)v);
    CHECK(qf_ctx_set_option(ctx, QF_OPT_COUNT, 1) == QF_EINVAL, "unknown option");
    CHECK(qf_ctx_get_option(ctx, -1, &v) == QF_EINVAL, "unknown option (get)");
    QF(qf_ctx_set_option(ctx, QF_OPT_SEND_CHUNKS, 99));
    QF(qf_ctx_get_option(ctx, QF_OPT_SEND_CHUNKS, &v));
    CHECK(v == 8, "send_chunks clamps to 8, got %lld", (long long)v);
    QF(qf_ctx_set_option(ctx, QF_OPT_SEND_CHUNKS, 1));
    QF(qf_ctx_set_option(ctx, QF_OPT_FFT_KERNELS, 0));
    test_batch(ctx);
    QF(qf_ctx_set_option(ctx, QF_OPT_BITSLICED, 0));
    test_batch(ctx);
    QF(qf_ctx_set_option(ctx, QF_OPT_BITSLICED, 1));
    QF(qf_ctx_set_option(ctx, QF_OPT_FFT_KERNELS, 1));
    printf("options ok\n");
}

int main(void) {
    CHECK(qf_abi_version() == QF_ABI_VERSION, "ABI version");
    test_gf();
    test_framing();
    qf_ctx *ctx;
    QF(qf_ctx_create(0, NULL, &ctx));
    test_batch(ctx);
    test_options(ctx);
    test_desc(ctx);
    test_objects(ctx);
    test_wiedemann(ctx);
    test_adaptive(ctx);
    test_adaptive_reuse(ctx);
    test_adaptive_batch(ctx);
    QF(qf_ctx_destroy(ctx));
    printf("ALL OK\n");
    return 0;
}
