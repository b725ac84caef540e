/*
 * qf_send_bench.c -- per-packet cost of the adaptive send path over many
 * connections: M connection states in Normal mode
 * (k = 64, n = 74, adaptive.rs:124-153) with full windows, each sending a
 * 1200-byte packet per round -- every send emits its window's 10 repairs
 * (adaptive.rs:519-562).  Timed two ways on the same connections:
 *   batch       one qf_adaptive_on_send_batch call per round (M packets)
 *   sequential  M qf_adaptive_on_send calls per round
 * Prints one JSON object per M on stdout (microseconds per source packet,
 * host wall clock around whole rounds: upload, encode, download, host copies).
 *
 * Receive side (--recv): M connections each receive one generation's stream
 * (k = 64 sources of 1,200 bytes with 6 lost, then the window's repairs, 68
 * packets), one packet per connection per round; timed with one
 * qf_adaptive_on_receive_batch per round and with per-packet
 * qf_adaptive_on_receive calls, each connection's generation recovered.
 *
 *   qf_send_bench [--recv] [M ...]        default: 1 64 1024
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/qf_fec.h"

#define QF(call)                                                                     \
    do {                                                                             \
        int s_ = (call);                                                             \
        if (s_ != QF_OK) {                                                           \
            fprintf(stderr, "FAIL %s:%d %s -> %s\n", __FILE__, __LINE__, #call,        \
                    qf_strerror(s_));                                                \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static uint64_t rng = 0x5eedu;
static uint8_t rnd8(void) {
    rng = rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint8_t)(rng >> 56);
}

static void run(qf_ctx *ctx, uint32_t M) {
    const uint32_t LEN = 1200, MAXLEN = 1500;
    qf_fec_config cfg;
    qf_fec_config_default(&cfg);
    cfg.initial_mode = QF_MODE_NORMAL;
    cfg.max_len = MAXLEN;
    qf_adaptive **conns = calloc(M, sizeof(*conns));
    for (uint32_t m = 0; m < M; ++m) QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &conns[m]));
    uint32_t k = 0, n = 0;
    QF(qf_adaptive_state(conns[0], NULL, NULL, &k, &n, NULL, NULL, NULL));
    const uint32_t per = qf_adaptive_max_send_packets(conns[0]);
    const uint32_t cap = per * M;
    uint8_t *src = malloc((size_t)M * LEN);
    for (size_t i = 0; i < (size_t)M * LEN; ++i) src[i] = rnd8();
    const uint8_t **data = malloc(M * sizeof(*data));
    uint32_t *lens = malloc(M * sizeof(*lens));
    uint64_t *ids = malloc(M * sizeof(*ids));
    for (uint32_t m = 0; m < M; ++m) data[m] = src + (size_t)m * LEN, lens[m] = LEN;
    uint8_t *out = malloc((size_t)cap * MAXLEN);
    uint8_t *co = malloc((size_t)cap * 256);
    qf_packet_desc *desc = malloc(cap * sizeof(*desc));
    uint32_t *n_out = malloc(M * sizeof(*n_out));
    uint64_t id = 0;
    /* fill the windows (and warm up the kernels) */
    for (uint32_t t = 0; t < k + 3; ++t) {
        for (uint32_t m = 0; m < M; ++m) ids[m] = id;
        ++id;
        QF(qf_adaptive_on_send_batch(conns, M, ids, data, lens, out, MAXLEN, co, 256, desc, cap, n_out, NULL));
    }
    const uint32_t rounds = M >= 512 ? 60 : M >= 64 ? 200 : 400;
    uint64_t emitted = 0;
    double t0 = now_s();
    for (uint32_t t = 0; t < rounds; ++t) {
        for (uint32_t m = 0; m < M; ++m) ids[m] = id;
        ++id;
        QF(qf_adaptive_on_send_batch(conns, M, ids, data, lens, out, MAXLEN, co, 256, desc, cap, n_out, NULL));
        for (uint32_t m = 0; m < M; ++m) emitted += n_out[m];
    }
    const double tb = now_s() - t0;
    if (emitted != (uint64_t)rounds * M * (1 + n - k)) {
        fprintf(stderr, "FAIL: emitted %llu packets\n", (unsigned long long)emitted);
        exit(1);
    }
    const uint32_t srounds = M >= 512 ? 3 : M >= 64 ? 20 : 400;
    t0 = now_s();
    for (uint32_t t = 0; t < srounds; ++t) {
        for (uint32_t m = 0; m < M; ++m) {
            uint32_t nn = 0;
            QF(qf_adaptive_on_send(conns[m], id, data[m], LEN, out, MAXLEN, co, 256, desc, per, &nn));
        }
        ++id;
    }
    const double ts = now_s() - t0;
    const double ub = 1e6 * tb / ((double)rounds * M), us = 1e6 * ts / ((double)srounds * M);
    printf("{\"M\": %u, \"k\": %u, \"n\": %u, \"len\": %u, \"rounds_batch\": %u, \"rounds_sequential\": %u, "
           "\"us_per_packet_batch\": %.3f, \"us_per_packet_sequential\": %.3f, \"speedup\": %.2f, "
           "\"repair_MiB_per_s_batch\": %.1f}\n",
           M, k, n, LEN, rounds, srounds, ub, us, us / ub, (double)(n - k) * LEN / ub / 1.048576);
    fflush(stdout);
    for (uint32_t m = 0; m < M; ++m) qf_adaptive_free(conns[m]);
    free(conns), free(src), free(data), free(lens), free(ids), free(out), free(co), free(desc), free(n_out);
}

/* one generation per connection: packets in arrival order */
typedef struct {
    uint32_t n;            /* packets */
    uint64_t *ids;
    int32_t *sys;
    uint8_t *data;         /* n x LEN */
    uint32_t *lens;
    uint8_t *coeffs;       /* n x 256 */
    uint32_t *clen;
} stream_t;

static double run_recv_leg(qf_ctx *ctx, uint32_t M, const stream_t *sm, int batch, uint64_t *recovered) {
    const uint32_t LEN = 1200, MAXLEN = 1500;
    qf_fec_config cfg;
    qf_fec_config_default(&cfg);
    cfg.initial_mode = QF_MODE_NORMAL;
    cfg.max_len = MAXLEN;
    qf_adaptive **conns = calloc(M, sizeof(*conns));
    for (uint32_t m = 0; m < M; ++m) QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &conns[m]));
    uint32_t k = 0;
    QF(qf_adaptive_state(conns[0], NULL, NULL, &k, NULL, NULL, NULL, NULL));
    const uint32_t cap = k * M;
    uint8_t *out = malloc((size_t)cap * MAXLEN);
    qf_packet_desc *desc = malloc(cap * sizeof(*desc));
    uint32_t *n_out = malloc(M * sizeof(*n_out));
    int32_t *st = malloc(M * sizeof(*st));
    uint64_t *ids = malloc(M * 8);
    int32_t *sys = malloc(M * 4);
    const uint8_t **data = malloc(M * sizeof(*data));
    uint32_t *lens = malloc(M * 4);
    const uint8_t **co = malloc(M * sizeof(*co));
    uint32_t *cl = malloc(M * 4);
    const uint32_t n = sm[0].n;
    *recovered = 0;
    double t0 = now_s();
    for (uint32_t t = 0; t < n; ++t) {
        if (batch) {
            for (uint32_t m = 0; m < M; ++m) {
                ids[m] = sm[m].ids[t];
                sys[m] = sm[m].sys[t];
                data[m] = sm[m].data + (size_t)t * LEN;
                lens[m] = sm[m].lens[t];
                co[m] = sm[m].clen[t] ? sm[m].coeffs + (size_t)t * 256 : NULL;
                cl[m] = sm[m].clen[t];
            }
            QF(qf_adaptive_on_receive_batch(conns, M, ids, sys, data, lens, co, cl, out, MAXLEN, desc, cap, n_out,
                                            st));
            for (uint32_t m = 0; m < M; ++m) {
                if (st[m] != QF_OK) { fprintf(stderr, "FAIL: status %d\n", st[m]); exit(1); }
                *recovered += n_out[m];
            }
        } else {
            for (uint32_t m = 0; m < M; ++m) {
                uint32_t nn = 0;
                QF(qf_adaptive_on_receive(conns[m], sm[m].ids[t], sm[m].sys[t], sm[m].data + (size_t)t * LEN,
                                          sm[m].lens[t], sm[m].clen[t] ? sm[m].coeffs + (size_t)t * 256 : NULL,
                                          sm[m].clen[t], out, MAXLEN, desc, k, &nn));
                *recovered += nn;
            }
        }
    }
    const double dt = now_s() - t0;
    for (uint32_t m = 0; m < M; ++m) qf_adaptive_free(conns[m]);
    free(conns), free(out), free(desc), free(n_out), free(st), free(ids), free(sys), free(data), free(lens);
    free(co), free(cl);
    return dt;
}

static void run_recv(qf_ctx *ctx, uint32_t M) {
    const uint32_t LEN = 1200, MAXLEN = 1500, LOST = 6;
    qf_fec_config cfg;
    qf_fec_config_default(&cfg);
    cfg.initial_mode = QF_MODE_NORMAL;
    cfg.max_len = MAXLEN;
    qf_adaptive **snd = calloc(M, sizeof(*snd));
    for (uint32_t m = 0; m < M; ++m) QF(qf_adaptive_new_at(ctx, &cfg, 0.0, &snd[m]));
    uint32_t k = 0, n = 0;
    QF(qf_adaptive_state(snd[0], NULL, NULL, &k, &n, NULL, NULL, NULL));
    const uint32_t per = qf_adaptive_max_send_packets(snd[0]), cap = per * M, npk = k - LOST + (n - k);
    stream_t *sm = calloc(M, sizeof(*sm));
    for (uint32_t m = 0; m < M; ++m) {
        sm[m].ids = malloc(npk * 8);
        sm[m].sys = malloc(npk * 4);
        sm[m].data = malloc((size_t)npk * LEN);
        sm[m].lens = malloc(npk * 4);
        sm[m].coeffs = malloc((size_t)npk * 256);
        sm[m].clen = malloc(npk * 4);
    }
    uint8_t *src = malloc((size_t)M * LEN), *out = malloc((size_t)cap * MAXLEN), *co = malloc((size_t)cap * 256);
    qf_packet_desc *desc = malloc(cap * sizeof(*desc));
    uint32_t *n_out = malloc(M * 4), *lens = malloc(M * 4);
    uint64_t *ids = malloc(M * 8);
    const uint8_t **data = malloc(M * sizeof(*data));
    for (uint32_t t = 0; t < k; ++t) {       /* the senders: one generation per connection */
        for (size_t i = 0; i < (size_t)M * LEN; ++i) src[i] = rnd8();
        for (uint32_t m = 0; m < M; ++m) ids[m] = t, data[m] = src + (size_t)m * LEN, lens[m] = LEN;
        QF(qf_adaptive_on_send_batch(snd, M, ids, data, lens, out, MAXLEN, co, 256, desc, cap, n_out, NULL));
        uint32_t pos = 0;
        for (uint32_t m = 0; m < M; ++m) {
            for (uint32_t i = pos; i < pos + n_out[m]; ++i) {
                /* lose sources 7 m + 3 q mod k (q < LOST) */
                int lost = 0;
                for (uint32_t q = 0; q < LOST; ++q) lost |= desc[i].is_systematic && desc[i].id == (7 * m + 11 * q) % k;
                if (lost) continue;
                stream_t *x = &sm[m];
                x->ids[x->n] = desc[i].id;
                x->sys[x->n] = desc[i].is_systematic;
                memcpy(x->data + (size_t)x->n * LEN, out + (size_t)i * MAXLEN, desc[i].len);
                x->lens[x->n] = desc[i].len;
                x->clen[x->n] = desc[i].coeff_len;
                if (desc[i].coeff_len) memcpy(x->coeffs + (size_t)x->n * 256, co + (size_t)i * 256, desc[i].coeff_len);
                x->n++;
            }
            pos += n_out[m];
        }
    }
    for (uint32_t m = 0; m < M; ++m)
        if (sm[m].n != npk) { fprintf(stderr, "FAIL: stream %u has %u packets\n", m, sm[m].n); exit(1); }
    uint64_t rb = 0, rs = 0;
    run_recv_leg(ctx, M < 64 ? M : 64, sm, 1, &rb);           /* warm-up */
    const double tb = run_recv_leg(ctx, M, sm, 1, &rb);
    const double ts = run_recv_leg(ctx, M, sm, 0, &rs);
    if (rb != (uint64_t)M * k || rs != (uint64_t)M * k) {
        fprintf(stderr, "FAIL: recovered %llu / %llu packets\n", (unsigned long long)rb, (unsigned long long)rs);
        exit(1);
    }
    const double ub = 1e6 * tb / ((double)M * npk), us = 1e6 * ts / ((double)M * npk);
    printf("{\"leg\": \"receive\", \"M\": %u, \"k\": %u, \"n\": %u, \"len\": %u, \"lost_per_generation\": %u, "
           "\"packets_per_connection\": %u, \"us_per_packet_batch\": %.3f, \"us_per_packet_sequential\": %.3f, "
           "\"speedup\": %.2f, \"generations_recovered\": %u}\n",
           M, k, n, LEN, LOST, npk, ub, us, us / ub, M);
    fflush(stdout);
    for (uint32_t m = 0; m < M; ++m) {
        qf_adaptive_free(snd[m]);
        free(sm[m].ids), free(sm[m].sys), free(sm[m].data), free(sm[m].lens), free(sm[m].coeffs), free(sm[m].clen);
    }
    free(snd), free(sm), free(src), free(out), free(co), free(desc), free(n_out), free(lens), free(ids), free(data);
}

int main(int argc, char **argv) {
    qf_ctx *ctx = NULL;
    QF(qf_ctx_create(0, NULL, &ctx));
    int recv = argc > 1 && strcmp(argv[1], "--recv") == 0;
    const int first = recv ? 2 : 1;
    const uint32_t Ms[3] = {1, 64, 1024};
    if (argc > first) {
        for (int i = first; i < argc; ++i) recv ? run_recv(ctx, (uint32_t)atoi(argv[i])) : run(ctx, (uint32_t)atoi(argv[i]));
    } else {
        for (int i = 0; i < 3; ++i) recv ? run_recv(ctx, Ms[i]) : run(ctx, Ms[i]);
    }
    qf_ctx_destroy(ctx);
    return 0;
}
