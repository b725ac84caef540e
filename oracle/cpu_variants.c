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
 *   cpu_encode_clmul_dispatch  the reference as written INCLUDING its per-byte
 *                     dispatch (timing only, same defective output): every
 *                     gf_mul (gf_tables.rs:283-300) calls
 *                     optimize::dispatch_bitslice (optimize.rs:385-408):
 *                     FeatureDetector::instance() (a Once, i.e. an acquire load,
 *                     optimize.rs:216-285), then has_feature lookups in a
 *                     HashMap<CpuFeature, bool> (std RandomState = SipHash-1-3
 *                     with random keys over the enum discriminant written as
 *                     isize; a SwissTable probe) -- AVX512F, AVX512VBMI and
 *                     PCLMULQDQ on an AVX-512 host, AVX2 + PCLMULQDQ or SSE2 +
 *                     PCLMULQDQ after a miss -- then the chosen member
 *                     (gf_mul_bitsliced_avx512: 512-bit broadcast + VPCLMULQDQ
 *                     + fold, gf_tables.rs:76-94; else the SSE2 member).
 * Both take G dense generations (src[g][i][t], rep[g][j][t], row stride L) and
 * split the generations over `threads` pthreads.  Results equal
 * oracle_encode_window (checked by tests/test_oracle_golden.py).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
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
    int simd;             /* 0 table, 1 avx2, 2 gfni, 3 clmul (as written), 4 clmul + dispatch */
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

/* ---- optimize.rs FeatureDetector + HashMap<CpuFeature, bool> model -------- */
/* CpuFeature discriminants (optimize.rs:186-202 declaration order) */
enum { F_AVX = 0, F_AVX2, F_SSE2, F_AVX512F, F_AVX512BW, F_AVX512VBMI, F_VAES, F_AESNI, F_PCLMULQDQ, F_NEON };

#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define SIPROUND                                                           \
    do {                                                                   \
        v0 += v1; v1 = ROTL(v1, 13); v1 ^= v0; v0 = ROTL(v0, 32);          \
        v2 += v3; v3 = ROTL(v3, 16); v3 ^= v2;                             \
        v0 += v3; v3 = ROTL(v3, 21); v3 ^= v0;                             \
        v2 += v1; v1 = ROTL(v1, 17); v1 ^= v2; v2 = ROTL(v2, 32);          \
    } while (0)

/* SipHash-1-3 of one 8-byte message (Hash::hash of a fieldless enum writes
 * its discriminant as isize) */
static inline uint64_t siphash13_u64(uint64_t k0, uint64_t k1, uint64_t m) {
    uint64_t v0 = k0 ^ 0x736f6d6570736575ULL, v1 = k1 ^ 0x646f72616e646f6dULL;
    uint64_t v2 = k0 ^ 0x6c7967656e657261ULL, v3 = k1 ^ 0x7465646279746573ULL;
    v3 ^= m;
    SIPROUND;
    v0 ^= m;
    const uint64_t b = (uint64_t)8 << 56; /* length byte, no tail */
    v3 ^= b;
    SIPROUND;
    v0 ^= b;
    v2 ^= 0xff;
    SIPROUND;
    SIPROUND;
    SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

typedef struct {
    uint64_t k0, k1;          /* RandomState keys */
    uint8_t ctrl[16];         /* SwissTable control bytes (h2 tag or 0xFF empty) */
    uint8_t key[16];
    uint8_t val[16];
} feature_map;

static feature_map g_features;
static int g_detector_state; /* Once: 0 new, 2 complete */
static int g_have_vpclmul;   /* this host can run the 512-bit member (avx512dq + vpclmulqdq) */
static int g_have_vpclmul256;   /* ... and the 256-bit member (avx2 + vpclmulqdq) */

static void map_insert(feature_map *m, uint8_t f, uint8_t v) {
    const uint64_t h = siphash13_u64(m->k0, m->k1, f);
    uint32_t pos = (uint32_t)h & 15;
    while (m->ctrl[pos] != 0xFF) pos = (pos + 1) & 15;
    m->ctrl[pos] = (uint8_t)(h >> 57);
    m->key[pos] = f;
    m->val[pos] = v;
}

/* FeatureDetector::instance (optimize.rs:216-285): Once + detection */
static const feature_map *detector_instance(void) {
    if (__atomic_load_n(&g_detector_state, __ATOMIC_ACQUIRE) != 2) {
        feature_map *m = &g_features;
        m->k0 = 0x0706050403020100ULL ^ (uint64_t)(uintptr_t)&g_features;
        m->k1 = 0x0f0e0d0c0b0a0908ULL ^ (uint64_t)(uintptr_t)&g_detector_state;
        memset(m->ctrl, 0xFF, sizeof m->ctrl);
        map_insert(m, F_AVX, (uint8_t)!!__builtin_cpu_supports("avx"));
        map_insert(m, F_AVX2, (uint8_t)!!__builtin_cpu_supports("avx2"));
        map_insert(m, F_SSE2, (uint8_t)!!__builtin_cpu_supports("sse2"));
        map_insert(m, F_AVX512F,
                   (uint8_t)(__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw")));
        map_insert(m, F_AVX512BW, (uint8_t)!!__builtin_cpu_supports("avx512bw"));
        map_insert(m, F_AVX512VBMI, (uint8_t)!!__builtin_cpu_supports("avx512vbmi"));
        map_insert(m, F_VAES, (uint8_t)!!__builtin_cpu_supports("vaes"));
        map_insert(m, F_AESNI, (uint8_t)!!__builtin_cpu_supports("aes"));
        map_insert(m, F_PCLMULQDQ, (uint8_t)!!__builtin_cpu_supports("pclmul"));
        g_have_vpclmul = __builtin_cpu_supports("avx512dq") && __builtin_cpu_supports("vpclmulqdq");
        g_have_vpclmul256 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("vpclmulqdq");
        __atomic_store_n(&g_detector_state, 2, __ATOMIC_RELEASE);
    }
    return &g_features;
}

/* FeatureDetector::has_feature (optimize.rs:288-290): hash, probe, compare */
static inline int has_feature(const feature_map *m, uint8_t f) {
    const uint64_t h = siphash13_u64(m->k0, m->k1, f);
    const uint8_t tag = (uint8_t)(h >> 57);
    uint32_t pos = (uint32_t)h & 15;
    for (int n = 0; n < 16; ++n, pos = (pos + 1) & 15) {
        if (m->ctrl[pos] == 0xFF) return 0;
        if (m->ctrl[pos] == tag && m->key[pos] == f) return m->val[pos];
    }
    return 0;
}

/* gf_tables.rs:76-94 gf_mul_bitsliced_avx512 as written */
__attribute__((target("avx512f,avx512dq,avx512vbmi,vpclmulqdq,pclmul"))) static uint8_t clmul_fold_avx512(uint8_t a,
                                                                                             uint8_t b) {
    const __m512i va = _mm512_broadcast_i64x2(_mm_set_epi64x(0, a));
    const __m512i vb = _mm512_broadcast_i64x2(_mm_set_epi64x(0, b));
    const __m512i prod = _mm512_clmulepi64_epi128(va, vb, 0x00);
    uint16_t t = (uint16_t)_mm_extract_epi16(_mm512_castsi512_si128(prod), 0);
    t ^= t >> 8;
    t ^= t >> 4;
    t ^= t >> 2;
    t ^= t >> 1;
    return (uint8_t)(t & 0xFF);
}

/* gf_tables.rs:102-118 gf_mul_bitsliced_avx2: both operands broadcast into a
 * 256-bit register, one 256-bit VPCLMULQDQ (_mm256_clmulepi64_epi128), the low
 * 16 bits of lane 0 folded as the other members do (the same defective fold,
 * SURVEY F3).  Needs avx2 + vpclmulqdq. */
__attribute__((target("avx2,vpclmulqdq,pclmul"))) static uint8_t clmul_fold_avx2(uint8_t a, uint8_t b) {
    const __m256i va = _mm256_broadcastsi128_si256(_mm_set_epi64x(0, a));
    const __m256i vb = _mm256_broadcastsi128_si256(_mm_set_epi64x(0, b));
    const __m256i prod = _mm256_clmulepi64_epi128(va, vb, 0x00);
    uint16_t t = (uint16_t)_mm_extract_epi16(_mm256_castsi256_si128(prod), 0);
    t ^= t >> 8;
    t ^= t >> 4;
    t ^= t >> 2;
    t ^= t >> 1;
    return (uint8_t)(t & 0xFF);
}

/* gf_tables.rs:283-300 gf_mul through optimize.rs:385-408 dispatch_bitslice */
__attribute__((noinline)) static uint8_t gf_mul_dispatched(uint8_t a, uint8_t b) {
    const feature_map *d = detector_instance();
    if (has_feature(d, F_AVX512F) && has_feature(d, F_AVX512VBMI) && has_feature(d, F_PCLMULQDQ))
        return g_have_vpclmul ? clmul_fold_avx512(a, b) : clmul_fold(a, b);
    if (has_feature(d, F_AVX2) && has_feature(d, F_PCLMULQDQ)) return clmul_fold(a, b);
    if (has_feature(d, F_SSE2) && has_feature(d, F_PCLMULQDQ)) return clmul_fold(a, b);
    return oracle_gf_mul(a, b);
}

static void encode_clmul_dispatch_gen(const job_t *j, uint32_t g) {
    const uint8_t *s = j->src + (size_t)g * j->k * j->L;
    uint8_t *o = j->rep + (size_t)g * j->r * j->L;
    for (uint32_t q = 0; q < j->r; ++q) {
        uint8_t *acc = o + (size_t)q * j->L;
        memset(acc, 0, j->L);
        for (uint32_t i = 0; i < j->k; ++i) {
            const uint8_t c = j->coeff[(size_t)q * j->k + i];
            if (c == 0) continue;
            const uint8_t *x = s + (size_t)i * j->L;
            for (uint32_t t = 0; t < j->L; ++t) acc[t] ^= gf_mul_dispatched(c, x[t]); /* gf_mul_add */
        }
    }
}
#endif

static int g_pin = 0;   /* cpu_set_pinning */

void cpu_set_pinning(int on) { g_pin = on != 0; }
int cpu_pinning(void) { return g_pin; }

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
        if (j->simd == 4) {
            encode_clmul_dispatch_gen(j, g);
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
    /* threads pinned, worker w to the w-th CPU this
     * process may run on (cpu_set_pinning) */
    cpu_set_t allowed;
    int ncpu = 0, cpus[1024];
    if (g_pin && sched_getaffinity(0, sizeof allowed, &allowed) == 0)
        for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; ++c)
            if (CPU_ISSET(c, &allowed)) cpus[ncpu++] = c;
    for (uint32_t w = 0; w < threads; ++w) {
        jobs[w] = (job_t){k, r, L, (uint32_t)((uint64_t)G * w / threads),
                          (uint32_t)((uint64_t)G * (w + 1) / threads), src, rep, coeff, simd};
        pthread_attr_t at;
        pthread_attr_init(&at);
        if (ncpu) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(cpus[w % (uint32_t)ncpu], &one);
            pthread_attr_setaffinity_np(&at, sizeof one, &one);
        }
        pthread_create(&th[w], &at, worker, &jobs[w]);
        pthread_attr_destroy(&at);
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

/* timing only: the as-written path with its per-byte dispatch (optimize.rs:385-408) */
int cpu_encode_clmul_dispatch(uint32_t k, uint32_t r, uint32_t L, uint32_t G, const uint8_t *src, uint8_t *rep,
                              uint32_t threads) {
    if (!cpu_has_pclmul()) return -3;
#if defined(__x86_64__)
    (void)detector_instance();
#endif
    return run(k, r, L, G, src, rep, threads, 4);
}

/* ---- decode on host threads (bench.py cpu_baseline) --------
 * The reference decodes one generation per Decoder (decoder.rs:658-791) and
 * fans its row operations out on rayon (decoder.rs:410-433, 479-489); here
 * the host cores each take whole generations (one generation per pinned
 * thread at a time), which is at least as parallel.
 *   kind 0 "table"     oracle_decode_generation: decoder.rs:720-783 with table
 *                      gf_mul (gf_tables.rs:47-57), F4 fixed -- its output is
 *                      compared with the GPU's recovered rows
 *   kind 4 "dispatch"  the same elimination with every product through the
 *                      reference's gf_mul -> dispatch_bitslice (optimize.rs:
 *                      385-408) -> CLMUL fold: the as-written per-byte cost,
 *                      timing only (the fold is not a field product)
 * rows: G generations of n_rows received rows (arrival order, row_index
 * G x n_rows), L bytes each, dense; out: G x k x L (every source row). */
typedef struct {
    uint32_t k, L, n_rows, g0, g1;
    const uint16_t *row_index;
    const uint8_t *rows;
    uint8_t *out;
    int kind;
    int status;
} dec_job_t;

#if defined(__x86_64__)
/* decoder.rs:720-783 (pivot search, swap, scale_row, add_scaled_row on every
 * other row, early exit at rank k) over dense rows, products dispatched */
static int decode_dispatch_gen(uint32_t k, uint32_t L, uint32_t n_rows, const uint16_t *ri, const uint8_t *rows,
                               uint8_t *out) {
    uint8_t *m = (uint8_t *)calloc((size_t)k, (size_t)k + L);
    uint8_t **row = (uint8_t **)malloc(sizeof(uint8_t *) * k);
    uint8_t present[256] = {0};
    if (!m || !row) { free(m); free(row); return -1; }
    uint32_t n = 0;
    for (uint32_t s = 0; s < n_rows && n < k; ++s) {
        const uint32_t idx = ri[s];
        uint8_t *c = m + (size_t)n * (k + L);
        if (idx < k) {
            if (present[idx]) continue;
            present[idx] = 1;
            c[idx] = 1;
        } else {
            const uint8_t y = (uint8_t)idx;
            for (uint32_t i = 0; i < k; ++i) oracle_gf_inv((uint8_t)((uint8_t)i ^ y), &c[i]);
        }
        memcpy(c + k, rows + (size_t)s * L, L);
        row[n++] = c;
    }
    int st = n < k ? -2 : 0;
    for (uint32_t i = 0; i < k && !st; ++i) {
        uint32_t p = k;
        for (uint32_t r = i; r < k; ++r)
            if (row[r][i]) { p = r; break; }
        if (p == k) { st = -3; break; }
        uint8_t *t = row[i]; row[i] = row[p]; row[p] = t;
        uint8_t inv;
        oracle_gf_inv(row[i][i], &inv);
        for (uint32_t c = 0; c < k + L; ++c) row[i][c] = gf_mul_dispatched(row[i][c], inv);
        for (uint32_t r = 0; r < k; ++r) {
            const uint8_t f = row[r][i];
            if (r == i || f == 0) continue;
            for (uint32_t c = 0; c < k + L; ++c) row[r][c] ^= gf_mul_dispatched(f, row[i][c]);
        }
    }
    for (uint32_t i = 0; i < k && !st; ++i) memcpy(out + (size_t)i * L, row[i] + k, L);
    free(m);
    free(row);
    return st;
}
#endif

static void *dec_worker(void *arg) {
    dec_job_t *j = (dec_job_t *)arg;
    for (uint32_t g = j->g0; g < j->g1; ++g) {
        const uint16_t *ri = j->row_index + (size_t)g * j->n_rows;
        const uint8_t *rows = j->rows + (size_t)g * j->n_rows * j->L;
        uint8_t *out = j->out + (size_t)g * j->k * j->L;
        int st = -1;
#if defined(__x86_64__)
        if (j->kind == 4) st = decode_dispatch_gen(j->k, j->L, j->n_rows, ri, rows, out);
#endif
        if (j->kind == 0)
            st = oracle_decode_generation(j->k, j->L, j->n_rows, ri, rows, j->L, NULL, out, j->L, NULL);
        if (st != 0 && j->status == 0) j->status = st;
    }
    return NULL;
}

int cpu_decode(int kind, uint32_t k, uint32_t L, uint32_t G, uint32_t n_rows, const uint16_t *row_index,
               const uint8_t *rows, uint8_t *out, uint32_t threads) {
    if (k == 0 || k > 256 || threads == 0 || (kind != 0 && kind != 4)) return -1;
    if (kind == 4 && !cpu_has_pclmul()) return -3;
#if defined(__x86_64__)
    if (kind == 4) (void)detector_instance();
#endif
    if (threads > G) threads = G ? G : 1;
    pthread_t *th = (pthread_t *)calloc(threads, sizeof(pthread_t));
    dec_job_t *jobs = (dec_job_t *)calloc(threads, sizeof(dec_job_t));
    if (!th || !jobs) { free(th); free(jobs); return -1; }
    cpu_set_t allowed;
    int ncpu = 0, cpus[1024];
    if (g_pin && sched_getaffinity(0, sizeof allowed, &allowed) == 0)
        for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; ++c)
            if (CPU_ISSET(c, &allowed)) cpus[ncpu++] = c;
    for (uint32_t w = 0; w < threads; ++w) {
        jobs[w] = (dec_job_t){k, L, n_rows, (uint32_t)((uint64_t)G * w / threads),
                              (uint32_t)((uint64_t)G * (w + 1) / threads), row_index, rows, out, kind, 0};
        pthread_attr_t at;
        pthread_attr_init(&at);
        if (ncpu) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(cpus[w % (uint32_t)ncpu], &one);
            pthread_attr_setaffinity_np(&at, sizeof one, &one);
        }
        pthread_create(&th[w], &at, dec_worker, &jobs[w]);
        pthread_attr_destroy(&at);
    }
    int st = 0;
    for (uint32_t w = 0; w < threads; ++w) {
        pthread_join(th[w], NULL);
        if (jobs[w].status && !st) st = jobs[w].status;
    }
    free(th);
    free(jobs);
    return st;
}

/* benches/gf_bitslice_bench.rs:17-102 restated (the
 * only published numbers of the path): a[i] = i, b[i] = 255 - i for i < 1024
 * (as u8), acc ^= mul(a[i], b[i]), `iters` passes; every operand goes
 * through a compiler barrier (criterion::black_box).
 *   kind 0 "table"    gf_mul_table (gf_tables.rs:47-57)
 *   kind 1 "dispatch" gf_mul -> dispatch_bitslice per byte (gf_tables.rs:283-300,
 *                     optimize.rs:385-408: FeatureDetector + HashMap lookups,
 *                     then the CLMUL member) -- the reference's own gf_mul
 *   kind 2 "sse2"     gf_mul_bitsliced_sse2 (gf_tables.rs:129-141, one PCLMULQDQ + fold)
 *   kind 3 "avx512"   gf_mul_bitsliced_avx512 (gf_tables.rs:76-94, VPCLMULQDQ)
 *   kind 4 "avx2"     gf_mul_bitsliced_avx2 (gf_tables.rs:102-118, 256-bit VPCLMULQDQ)
 * Kinds 1-4 compute the reference's defective fold: timing only.
 * Returns the final acc (>= 0), or -3 when this host lacks the instructions. */
#define BB(x) __asm__ volatile("" : "+r"(x))
/* one product of a CLMUL member (2 sse2, 3 avx512, 4 avx2), for the test that
 * the three members compute the same fold; -3 when the host lacks it */
int cpu_clmul_fold_pair(int kind, uint8_t a, uint8_t b) {
#if defined(__x86_64__)
    (void)detector_instance();
    if (!cpu_has_pclmul()) return -3;
    if (kind == 2) return clmul_fold(a, b);
    if (kind == 3) return g_have_vpclmul ? clmul_fold_avx512(a, b) : -3;
    if (kind == 4) return g_have_vpclmul256 ? clmul_fold_avx2(a, b) : -3;
#else
    (void)a, (void)b;
#endif
    (void)kind;
    return -3;
}

int cpu_gf_mul_loop(int kind, uint64_t iters) {
    uint8_t a[1024], b[1024];
    for (int i = 0; i < 1024; ++i) {
        a[i] = (uint8_t)i;
        b[i] = (uint8_t)(255 - i);
    }
    uint8_t acc = 0;
    if (kind == 0) {
        for (uint64_t it = 0; it < iters; ++it) {
            for (int i = 0; i < 1024; ++i) {
                uint8_t x = a[i], y = b[i];
                BB(x);
                BB(y);
                acc ^= oracle_gf_mul(x, y);
            }
            BB(acc);
        }
        return acc;
    }
#if defined(__x86_64__)
    if (!cpu_has_pclmul()) return -3;
    if (kind == 1) {
        (void)detector_instance();
        for (uint64_t it = 0; it < iters; ++it) {
            for (int i = 0; i < 1024; ++i) {
                uint8_t x = a[i], y = b[i];
                BB(x);
                BB(y);
                acc ^= gf_mul_dispatched(x, y);
            }
            BB(acc);
        }
        return acc;
    }
    if (kind == 2) {
        for (uint64_t it = 0; it < iters; ++it) {
            for (int i = 0; i < 1024; ++i) {
                uint8_t x = a[i], y = b[i];
                BB(x);
                BB(y);
                acc ^= clmul_fold(x, y);
            }
            BB(acc);
        }
        return acc;
    }
    if (kind == 3) {
        (void)detector_instance();
        if (!g_have_vpclmul) return -3;
        for (uint64_t it = 0; it < iters; ++it) {
            for (int i = 0; i < 1024; ++i) {
                uint8_t x = a[i], y = b[i];
                BB(x);
                BB(y);
                acc ^= clmul_fold_avx512(x, y);
            }
            BB(acc);
        }
        return acc;
    }
    if (kind == 4) {
        (void)detector_instance();
        if (!g_have_vpclmul256) return -3;
        for (uint64_t it = 0; it < iters; ++it) {
            for (int i = 0; i < 1024; ++i) {
                uint8_t x = a[i], y = b[i];
                BB(x);
                BB(y);
                acc ^= clmul_fold_avx2(x, y);
            }
            BB(acc);
        }
        return acc;
    }
#endif
    return -3;
}
