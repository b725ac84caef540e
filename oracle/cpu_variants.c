/* cpu_variants.c -- CPU comparison encoders timed beside the GPU in bench.py
 * (SURVEY 8(d) "CPU timing beside the GPU").  BENCH / TEST INFRASTRUCTURE
 * ONLY: never linked into or called by the library.
 *
 *   cpu_encode_table  the reference's loop structure (decoder.rs:236-259:
 *                     repair j, source i, byte t; table gf_mul, gf_tables.rs:47-57)
 *   cpu_encode_avx2   optimized host SIMD: split-nibble pshufb tables per
 *                     coefficient, 32 bytes per step
 * Both take G dense generations (src[g][i][t], rep[g][j][t], row stride L) and
 * split the generations over `threads` pthreads.  Results equal
 * oracle_encode_window (checked by tests/test_oracle_golden.py).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "qf_oracle.h"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

typedef struct {
    uint32_t k, r, L, g0, g1;
    const uint8_t *src;
    uint8_t *rep;
    const uint8_t *coeff; /* r x k */
    int simd;
} job_t;

static void encode_table_gen(const job_t *j, uint32_t g) {
    const uint8_t *s = j->src + (size_t)g * j->k * j->L;
    uint8_t *o = j->rep + (size_t)g * j->r * j->L;
    for (uint32_t q = 0; q < j->r; ++q) {
        uint8_t *acc = o + (size_t)q * j->L;
        memset(acc, 0, j->L);
        for (uint32_t i = 0; i < j->k; ++i) {
            const uint8_t c = j->coeff[(size_t)q * j->k + i];
            const uint8_t *x = s + (size_t)i * j->L;
            for (uint32_t t = 0; t < j->L; ++t) acc[t] ^= oracle_gf_mul(c, x[t]);
        }
    }
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) static void encode_avx2_gen(const job_t *j, uint32_t g) {
    const uint8_t *s = j->src + (size_t)g * j->k * j->L;
    uint8_t *o = j->rep + (size_t)g * j->r * j->L;
    const __m256i nib = _mm256_set1_epi8(0x0F);
    for (uint32_t q = 0; q < j->r; ++q) {
        uint8_t *acc = o + (size_t)q * j->L;
        memset(acc, 0, j->L);
        for (uint32_t i = 0; i < j->k; ++i) {
            const uint8_t c = j->coeff[(size_t)q * j->k + i];
            uint8_t lo[16], hi[16];
            for (int v = 0; v < 16; ++v) {
                lo[v] = oracle_gf_mul(c, (uint8_t)v);
                hi[v] = oracle_gf_mul(c, (uint8_t)(v << 4));
            }
            const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
            const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
            const uint8_t *x = s + (size_t)i * j->L;
            uint32_t t = 0;
            for (; t + 32 <= j->L; t += 32) {
                const __m256i v = _mm256_loadu_si256((const __m256i *)(x + t));
                const __m256i pl = _mm256_shuffle_epi8(tlo, _mm256_and_si256(v, nib));
                const __m256i ph = _mm256_shuffle_epi8(thi, _mm256_and_si256(_mm256_srli_epi16(v, 4), nib));
                __m256i a = _mm256_loadu_si256((const __m256i *)(acc + t));
                a = _mm256_xor_si256(a, _mm256_xor_si256(pl, ph));
                _mm256_storeu_si256((__m256i *)(acc + t), a);
            }
            for (; t < j->L; ++t) acc[t] ^= oracle_gf_mul(c, x[t]);
        }
    }
}
#endif

static void *worker(void *arg) {
    const job_t *j = (const job_t *)arg;
    for (uint32_t g = j->g0; g < j->g1; ++g) {
#if defined(__x86_64__)
        if (j->simd) {
            encode_avx2_gen(j, g);
            continue;
        }
#endif
        encode_table_gen(j, g);
    }
    return NULL;
}

static int run(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src, uint8_t *rep,
               uint32_t threads, int simd) {
    if (k == 0 || k + r > 256 || threads == 0) return -1;
    uint8_t *coeff = (uint8_t *)malloc((size_t)k * r);
    if (!coeff) return -1;
    if (oracle_cauchy_coeffs(k, r, coeff) != 0) {
        free(coeff);
        return -2;
    }
    if (threads > G) threads = G ? G : 1;
    pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
    job_t *jobs = (job_t *)calloc(threads, sizeof(job_t));
    for (uint32_t w = 0; w < threads; ++w) {
        jobs[w] = (job_t){k, r, L, (uint32_t)((uint64_t)G * w / threads),
                          (uint32_t)((uint64_t)G * (w + 1) / threads), src, rep, coeff, simd};
        pthread_create(&th[w], NULL, worker, &jobs[w]);
    }
    for (uint32_t w = 0; w < threads; ++w) pthread_join(th[w], NULL);
    free(th);
    free(jobs);
    free(coeff);
    return 0;
}

int cpu_encode_table(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src,
                     uint8_t *rep, uint32_t threads) {
    return run(k, r, L, G, src, rep, threads, 0);
}

int cpu_has_avx2(void) {
#if defined(__x86_64__)
    return __builtin_cpu_supports("avx2");
#else
    return 0;
#endif
}

int cpu_encode_avx2(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src, uint8_t *rep,
                    uint32_t threads) {
    if (!cpu_has_avx2()) return -3;
    return run(k, r, L, G, src, rep, threads, 1);
}
