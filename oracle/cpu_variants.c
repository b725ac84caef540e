/* cpu_variants.c -- CPU comparison encoders timed beside the GPU in bench.py
 * (SURVEY 8(d) "CPU timing beside the GPU").  BENCH / TEST INFRASTRUCTURE
 * ONLY: never linked into or called by the library.
 *
 *   cpu_encode_table  the reference's loop structure (decoder.rs:236-259:
 *                     repair j, source i, byte t; table gf_mul, gf_tables.rs:47-57)
 *   cpu_encode_avx2   optimized host SIMD: split-nibble pshufb tables per
 *                     coefficient, 32 bytes per step
 *   cpu_encode_gfni   optimized host SIMD: AVX-512 GFNI affine transform with
 *                     the 8x8 GF(2) matrix of "multiply by c" over 0x11D (the
 *                     GF2P8MULB instruction itself is fixed to the AES poly
 *                     0x11B, so it cannot be used), 64 bytes per step
 *   cpu_encode_clmul  the reference AS WRITTEN, timing only: per byte
 *                     gf_mul_add -> gf_mul_bitsliced_sse2 (gf_tables.rs:129-141,
 *                     one PCLMULQDQ + XOR fold), same loop as decoder.rs:228-259
 *                     (skip c == 0, 4-byte unroll).  Its output is WRONG by
 *                     construction (the fold is a parity, not a
 *                     reduction mod 0x11D); the per-byte FeatureDetector/HashMap
 *                     dispatch of optimize.rs:385-408 is not modelled, so this
 *                     is a lower bound on the reference's cost.
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
    int simd;             /* 0 table, 1 avx2, 2 gfni, 3 clmul (as written) */
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

/* 8x8 GF(2) matrix of x -> c*x (poly 0x11D) in GF2P8AFFINEQB layout: result
 * bit i of each byte = parity(matrix byte (7 - i) & x), so byte 7 - i holds
 * row i, whose bit j is bit i of c * 2^j. */
static uint64_t affine_matrix(uint8_t c) {
    uint8_t col[8];
    for (int j = 0; j < 8; ++j) col[j] = oracle_gf_mul(c, (uint8_t)(1u << j));
    uint64_t m = 0;
    for (int i = 0; i < 8; ++i) {
        uint8_t row = 0;
        for (int j = 0; j < 8; ++j) row |= (uint8_t)(((col[j] >> i) & 1u) << j);
        m |= (uint64_t)row << (8 * (7 - i));
    }
    return m;
}

__attribute__((target("avx512f,avx512bw,gfni"))) static void encode_gfni_gen(const job_t *j, uint32_t g) {
    const uint8_t *s = j->src + (size_t)g * j->k * j->L;
    uint8_t *o = j->rep + (size_t)g * j->r * j->L;
    for (uint32_t q = 0; q < j->r; ++q) {
        uint8_t *acc = o + (size_t)q * j->L;
        memset(acc, 0, j->L);
        for (uint32_t i = 0; i < j->k; ++i) {
            const uint8_t c = j->coeff[(size_t)q * j->k + i];
            const __m512i m = _mm512_set1_epi64((long long)affine_matrix(c));
            const uint8_t *x = s + (size_t)i * j->L;
            uint32_t t = 0;
            for (; t + 64 <= j->L; t += 64) {
                const __m512i v = _mm512_loadu_si512((const void *)(x + t));
                const __m512i p = _mm512_gf2p8affine_epi64_epi8(v, m, 0);
                _mm512_storeu_si512((void *)(acc + t),
                                    _mm512_xor_si512(_mm512_loadu_si512((const void *)(acc + t)), p));
            }
            if (t < j->L) {
                const __mmask64 km = (__mmask64)((~0ULL) >> (64 - (j->L - t)));
                const __m512i v = _mm512_maskz_loadu_epi8(km, x + t);
                const __m512i a = _mm512_maskz_loadu_epi8(km, acc + t);
                _mm512_mask_storeu_epi8(acc + t, km,
                                        _mm512_xor_si512(a, _mm512_gf2p8affine_epi64_epi8(v, m, 0)));
            }
        }
    }
}

/* gf_tables.rs:129-141 as written (the SSE2/PCLMULQDQ member of the dispatch) */
__attribute__((target("sse2,pclmul"))) static inline uint8_t clmul_fold(uint8_t a, uint8_t b) {
    const __m128i p = _mm_clmulepi64_si128(_mm_set_epi64x(0, a), _mm_set_epi64x(0, b), 0x00);
    uint16_t t = (uint16_t)_mm_extract_epi16(p, 0);
    t ^= t >> 8;
    t ^= t >> 4;
    t ^= t >> 2;
    t ^= t >> 1;
    return (uint8_t)(t & 0xFF);
}

__attribute__((target("sse2,pclmul"))) static void encode_clmul_gen(const job_t *j, uint32_t g) {
    const uint8_t *s = j->src + (size_t)g * j->k * j->L;
    uint8_t *o = j->rep + (size_t)g * j->r * j->L;
    for (uint32_t q = 0; q < j->r; ++q) {
        uint8_t *acc = o + (size_t)q * j->L;
        memset(acc, 0, j->L);
        for (uint32_t i = 0; i < j->k; ++i) {
            const uint8_t c = j->coeff[(size_t)q * j->k + i];
            if (c == 0) continue;
            const uint8_t *x = s + (size_t)i * j->L;
            uint32_t t = 0;
            for (; t + 4 <= j->L; t += 4) {
                acc[t] ^= clmul_fold(c, x[t]);
                acc[t + 1] ^= clmul_fold(c, x[t + 1]);
                acc[t + 2] ^= clmul_fold(c, x[t + 2]);
                acc[t + 3] ^= clmul_fold(c, x[t + 3]);
            }
            for (; t < j->L; ++t) acc[t] ^= clmul_fold(c, x[t]);
        }
    }
}
#endif

static void *worker(void *arg) {
    const job_t *j = (const job_t *)arg;
    for (uint32_t g = j->g0; g < j->g1; ++g) {
#if defined(__x86_64__)
        if (j->simd == 1) {
            encode_avx2_gen(j, g);
            continue;
        }
        if (j->simd == 2) {
            encode_gfni_gen(j, g);
            continue;
        }
        if (j->simd == 3) {
            encode_clmul_gen(j, g);
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

int cpu_has_gfni(void) {
#if defined(__x86_64__)
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("gfni");
#else
    return 0;
#endif
}

int cpu_has_pclmul(void) {
#if defined(__x86_64__)
    return __builtin_cpu_supports("pclmul");
#else
    return 0;
#endif
}

int cpu_encode_gfni(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src, uint8_t *rep,
                    uint32_t threads) {
    if (!cpu_has_gfni()) return -3;
    return run(k, r, L, G, src, rep, threads, 2);
}

/* timing only: the output is the reference's defective fold */
int cpu_encode_clmul(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src, uint8_t *rep,
                     uint32_t threads) {
    if (!cpu_has_pclmul()) return -3;
    return run(k, r, L, G, src, rep, threads, 3);
}
