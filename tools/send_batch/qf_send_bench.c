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
 *   qf_send_bench [M ...]        default: 1 64 1024
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

int main(int argc, char **argv) {
    qf_ctx *ctx = NULL;
    QF(qf_ctx_create(0, NULL, &ctx));
    if (argc > 1) {
        for (int i = 1; i < argc; ++i) run(ctx, (uint32_t)atoi(argv[i]));
    } else {
        const uint32_t Ms[3] = {1, 64, 1024};
        for (int i = 0; i < 3; ++i) run(ctx, Ms[i]);
    }
    qf_ctx_destroy(ctx);
    return 0;
}
