/*
 * fec_cpu_simd.c — the CPU baseline codec (BASELINE.md "CPU baseline plan"):
 * the same coding contract as fec_oracle.c, vectorised
 * the way a tuned CPU FEC library is (ISA-L style):
 *   level 1  AVX2: GF(2^8) products by split-nibble tables (vpshufb), several
 *            repair / recovered rows accumulated per pass over an input row;
 *   level 2  AVX2 + GFNI: one vgf2p8affineqb per product (the multiply-by-c
 *            bit matrix; GFNI's own field polynomial is not used);
 *   level 0  scalar (fec_oracle.c's byte loops).
 * TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg times it
 * and tests/test_oracle_simd.py checks it against the scalar oracle.  The
 * product (libfecgpu.so) never links it.
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fec_oracle.h"

static int g_level = -1;  /* -1: detect */
#define ORC_SIMD_MAX_N 256  /* k + r of the block codes (Cauchy rows exist up to 256) */

int orc_simd_detect(void) {
    __builtin_cpu_init();
    if (!__builtin_cpu_supports("avx2")) return 0;
    return __builtin_cpu_supports("gfni") ? 2 : 1;
}

int orc_simd_level(void) { return g_level < 0 ? orc_simd_detect() : g_level; }

/* force a level (tests); -1 restores detection.  Clamped to what the CPU has. */
void orc_simd_set_level(int level) {
    const int hw = orc_simd_detect();
    g_level = level < 0 ? -1 : (level > hw ? hw : level);
}

/* ------------------------------------------------------------ tables --- */
static uint8_t LG[256], EX[512];  /* local log / exp tables (0x11D, generator 2) */

static void tables_init(void) {
    if (EX[0]) return;
    int x = 1;
    for (int i = 0; i < 255; i++) {
        EX[i] = EX[i + 255] = (uint8_t)x;
        LG[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    EX[510] = EX[0];
}

static inline uint8_t gmul(uint8_t a, uint8_t b) { return (a && b) ? EX[LG[a] + LG[b]] : 0; }
static inline uint8_t ginv(uint8_t a) { return EX[255 - LG[a]]; }

/* 8x8 bit-matrix transpose of the bytes of x (Hacker's Delight transpose8) */
static inline uint64_t transpose8(uint64_t x) {
    uint64_t t;
    t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x = x ^ t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x = x ^ t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    x = x ^ t ^ (t << 28);
    return x;
}
/* per coefficient: 32-B low-nibble and high-nibble product tables (the 16-B
 * table twice, one per AVX2 lane) and the GFNI 8x8 bit matrix */
typedef struct {
    uint8_t lo[32], hi[32];
    uint64_t gfni;
} coef_t;

static void coef_make(uint8_t c, coef_t *t) {
    uint8_t p[8];  /* c * 2^b: the product is linear in the bits of x */
    p[0] = c;
    for (int b = 1; b < 8; b++) p[b] = (uint8_t)((p[b - 1] << 1) ^ ((p[b - 1] & 0x80) ? 0x1D : 0));
    t->lo[0] = t->hi[0] = 0;
    for (int x = 1; x < 16; x++) {
        const int b = __builtin_ctz(x);
        t->lo[x] = (uint8_t)(t->lo[x & (x - 1)] ^ p[b]);
        t->hi[x] = (uint8_t)(t->hi[x & (x - 1)] ^ p[b + 4]);
    }
    memcpy(t->lo + 16, t->lo, 16);
    memcpy(t->hi + 16, t->hi, 16);
    /* vgf2p8affineqb: result bit i = parity(qword byte (7 - i) & x), so byte
     * 7 - i holds row i = sum_b bit_i(c * 2^b) << b: the transpose of the
     * matrix whose byte b is c * 2^b, bytes reversed */
    uint64_t m = 0;
    for (int b = 0; b < 8; b++) m |= (uint64_t)p[b] << (8 * b);
    t->gfni = __builtin_bswap64(transpose8(m));
}

/* out[m] = sum_j tab[j * nout + m] * in[j] over bytes [0, n) for nout <= 8;
 * always inlined into a switch on nout so the accumulators stay in registers */
__attribute__((target("avx2"), always_inline)) static inline void dot_avx2_n(
    int nin, const uint8_t *const *in, const int nout, uint8_t *const *out, const coef_t *tab,
    uint32_t n) {
    const __m256i mask = _mm256_set1_epi8(0x0f);
    uint32_t p = 0;
    for (; p + 32 <= n; p += 32) {
        __m256i acc[8];
        for (int m = 0; m < nout; m++) acc[m] = _mm256_setzero_si256();
        for (int j = 0; j < nin; j++) {
            const __m256i d = _mm256_loadu_si256((const __m256i *)(in[j] + p));
            const __m256i lo = _mm256_and_si256(d, mask);
            const __m256i hi = _mm256_and_si256(_mm256_srli_epi64(d, 4), mask);
            const coef_t *t = tab + (size_t)j * nout;
            for (int m = 0; m < nout; m++) {
                const __m256i pl = _mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i *)t[m].lo), lo);
                const __m256i ph = _mm256_shuffle_epi8(_mm256_loadu_si256((const __m256i *)t[m].hi), hi);
                acc[m] = _mm256_xor_si256(acc[m], _mm256_xor_si256(pl, ph));
            }
        }
        for (int m = 0; m < nout; m++) _mm256_storeu_si256((__m256i *)(out[m] + p), acc[m]);
    }
    for (; p < n; p++)  /* tail bytes */
        for (int m = 0; m < nout; m++) {
            uint8_t v = 0;
            for (int j = 0; j < nin; j++) v ^= (uint8_t)(tab[(size_t)j * nout + m].lo[in[j][p] & 15] ^
                                                         tab[(size_t)j * nout + m].hi[in[j][p] >> 4]);
            out[m][p] = v;
        }
}

__attribute__((target("avx2,gfni"), always_inline)) static inline void dot_gfni_n(
    int nin, const uint8_t *const *in, const int nout, uint8_t *const *out, const coef_t *tab,
    uint32_t n) {
    uint32_t p = 0;
    for (; p + 32 <= n; p += 32) {
        __m256i acc[8];
        for (int m = 0; m < nout; m++) acc[m] = _mm256_setzero_si256();
        for (int j = 0; j < nin; j++) {
            const __m256i d = _mm256_loadu_si256((const __m256i *)(in[j] + p));
            const coef_t *t = tab + (size_t)j * nout;
            for (int m = 0; m < nout; m++)
                acc[m] = _mm256_xor_si256(
                    acc[m], _mm256_gf2p8affine_epi64_epi8(d, _mm256_set1_epi64x((long long)t[m].gfni), 0));
        }
        for (int m = 0; m < nout; m++) _mm256_storeu_si256((__m256i *)(out[m] + p), acc[m]);
    }
    for (; p < n; p++)
        for (int m = 0; m < nout; m++) {
            uint8_t v = 0;
            for (int j = 0; j < nin; j++) v ^= (uint8_t)(tab[(size_t)j * nout + m].lo[in[j][p] & 15] ^
                                                         tab[(size_t)j * nout + m].hi[in[j][p] >> 4]);
            out[m][p] = v;
        }
}

static void dot_scalar(int nin, const uint8_t *const *in, int nout, uint8_t *const *out,
                       const coef_t *tab, uint32_t n) {
    for (uint32_t p = 0; p < n; p++)
        for (int m = 0; m < nout; m++) {
            uint8_t v = 0;
            for (int j = 0; j < nin; j++) v ^= (uint8_t)(tab[(size_t)j * nout + m].lo[in[j][p] & 15] ^
                                                         tab[(size_t)j * nout + m].hi[in[j][p] >> 4]);
            out[m][p] = v;
        }
}

#define DOT_SWITCH(FN)                                                   \
    switch (nout) {                                                      \
        case 1: FN(nin, in, 1, out, tab, n); break;                      \
        case 2: FN(nin, in, 2, out, tab, n); break;                      \
        case 3: FN(nin, in, 3, out, tab, n); break;                      \
        case 4: FN(nin, in, 4, out, tab, n); break;                      \
        case 5: FN(nin, in, 5, out, tab, n); break;                      \
        case 6: FN(nin, in, 6, out, tab, n); break;                      \
        case 7: FN(nin, in, 7, out, tab, n); break;                      \
        default: FN(nin, in, 8, out, tab, n); break;                     \
    }

__attribute__((target("avx2"))) static void dot_avx2(int nin, const uint8_t *const *in, int nout,
                                                     uint8_t *const *out, const coef_t *tab,
                                                     uint32_t n) {
    DOT_SWITCH(dot_avx2_n)
}

__attribute__((target("avx2,gfni"))) static void dot_gfni(int nin, const uint8_t *const *in, int nout,
                                                          uint8_t *const *out, const coef_t *tab,
                                                          uint32_t n) {
    DOT_SWITCH(dot_gfni_n)
}

static void dot(int level, int nin, const uint8_t *const *in, int nout, uint8_t *const *out,
                const coef_t *tab, uint32_t n) {
    if (level >= 2) dot_gfni(nin, in, nout, out, tab, n);
    else if (level == 1) dot_avx2(nin, in, nout, out, tab, n);
    else dot_scalar(nin, in, nout, out, tab, n);
}

/* dst ^= src over n bytes (XOR scheme) */
__attribute__((target("avx2"))) static void xor_into_avx2(uint8_t *dst, const uint8_t *src, uint32_t n) {
    uint32_t p = 0;
    for (; p + 32 <= n; p += 32)
        _mm256_storeu_si256((__m256i *)(dst + p),
                            _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(dst + p)),
                                             _mm256_loadu_si256((const __m256i *)(src + p))));
    for (; p < n; p++) dst[p] ^= src[p];
}

static void xor_into(int level, uint8_t *dst, const uint8_t *src, uint32_t n) {
    if (level >= 1) xor_into_avx2(dst, src, n);
    else for (uint32_t p = 0; p < n; p++) dst[p] ^= src[p];
}

/* ----------------------------------------------------------- windows --- */
static void encode_window(int level, int scheme, int k, int r, const coef_t *tab, uint32_t S,
                          uint32_t stride, uint8_t *win) {
    if (scheme == ORC_XOR) {
        for (int g = 0; g < r; g++) {
            uint8_t *R = win + (size_t)(k + g) * stride;
            memcpy(R, win + (size_t)g * stride, S);
            for (int j = g + r; j < k; j += r) xor_into(level, R, win + (size_t)j * stride, S);
        }
        return;
    }
    const uint8_t *in[ORC_SIMD_MAX_N];
    uint8_t *out[8];
    for (int j = 0; j < k; j++) in[j] = win + (size_t)j * stride;
    for (int i = 0; i < r; i++) out[i] = win + (size_t)(k + i) * stride;
    dot(level, k, in, r, out, tab, S);
}

/* GF(2^8) inverse of an e x e matrix (e <= 8) by Gauss-Jordan; 0 if singular */
static int inv_small(int e, uint8_t *A, uint8_t *Ai) {
    uint8_t M[8][16];
    for (int i = 0; i < e; i++)
        for (int j = 0; j < 2 * e; j++) M[i][j] = j < e ? A[i * e + j] : (uint8_t)(j - e == i);
    for (int c = 0; c < e; c++) {
        int p = c;
        while (p < e && !M[p][c]) p++;
        if (p == e) return 0;
        if (p != c)
            for (int j = 0; j < 2 * e; j++) { uint8_t t = M[c][j]; M[c][j] = M[p][j]; M[p][j] = t; }
        const uint8_t iv = ginv(M[c][c]);
        for (int j = 0; j < 2 * e; j++) M[c][j] = gmul(M[c][j], iv);
        for (int i = 0; i < e; i++) {
            if (i == c || !M[i][c]) continue;
            const uint8_t f = M[i][c];
            for (int j = 0; j < 2 * e; j++) M[i][j] ^= gmul(f, M[c][j]);
        }
    }
    for (int i = 0; i < e; i++)
        for (int j = 0; j < e; j++) Ai[i * e + j] = M[i][e + j];
    return 1;
}

/* orc_select_rows over multi-word present masks (bit i in word i / 64; codes
 * with k + r up to 256): the missing sources and e present repairs whose rows
 * restricted to them are independent, greedily in repair order */
static int pbit(const uint64_t *pw, int i) { return (int)((pw[i >> 6] >> (i & 63)) & 1u); }
static int select_rows_w(int k, int r, const uint8_t *C, const uint64_t *pw, int *miss, int *sel) {
    int e = 0, n = 0;
    for (int j = 0; j < k; j++)
        if (!pbit(pw, j)) miss[e++] = j;
    if (e == 0) return 0;
    if (e > 8) return -1;
    uint8_t basis[8][8];
    int pivc[8];
    for (int i = 0; i < r && n < e; i++) {
        if (!pbit(pw, k + i)) continue;
        uint8_t v[8];
        for (int u = 0; u < e; u++) v[u] = C[i * k + miss[u]];
        for (int b = 0; b < n; b++) {
            const uint8_t f = v[pivc[b]];
            if (!f) continue;
            for (int u = 0; u < e; u++) v[u] ^= gmul(f, basis[b][u]);
        }
        int pc = -1;
        for (int u = 0; u < e; u++)
            if (v[u]) { pc = u; break; }
        if (pc < 0) continue;
        const uint8_t iv = ginv(v[pc]);
        for (int u = 0; u < e; u++) basis[n][u] = gmul(v[u], iv);
        pivc[n] = pc;
        sel[n++] = i;
    }
    return n == e ? e : -1;
}

static int decode_window(int level, int scheme, int k, int r, const uint8_t *C, uint32_t S,
                         uint32_t stride, const uint64_t *pw, uint8_t *win) {
    const uint64_t present = pw[0];  /* XOR codes: k + r <= 64 */
    if (scheme == ORC_XOR) {
        int status = ORC_OK;
        for (int g = 0; g < r; g++) {
            int miss = -1, nmiss = 0;
            for (int j = g; j < k; j += r)
                if (!((present >> j) & 1)) { miss = j; nmiss++; }
            if (nmiss == 0) continue;
            if (nmiss > 1 || !((present >> (k + g)) & 1)) { status = ORC_UNRECOVERABLE; continue; }
            uint8_t *out = win + (size_t)miss * stride;
            memcpy(out, win + (size_t)(k + g) * stride, S);
            for (int j = g; j < k; j += r)
                if (j != miss) xor_into(level, out, win + (size_t)j * stride, S);
        }
        return status;
    }
    int miss[ORC_SIMD_MAX_N], sel[8];
    const int e = select_rows_w(k, r, C, pw, miss, sel);
    if (e == 0) return ORC_OK;
    if (e < 0 || e > 8) return ORC_UNRECOVERABLE;
    /* A[t][u] = C[sel_t][miss_u]; recovered_u = sum_t Ainv[u][t] (R_sel_t + sum_j C[sel_t][j] S_j)
     * folded into one dot product over the k inputs (received sources, chosen repairs) */
    uint8_t A[64], Ai[64];
    for (int t = 0; t < e; t++)
        for (int u = 0; u < e; u++) A[t * e + u] = C[sel[t] * k + miss[u]];
    if (!inv_small(e, A, Ai)) return ORC_UNRECOVERABLE;
    const uint8_t *in[ORC_SIMD_MAX_N];
    uint8_t *out[8];
    coef_t tab[ORC_SIMD_MAX_N * 8];
    int q = 0;
    for (int j = 0; j < k; j++) {
        if (!pbit(pw, j)) continue;
        for (int u = 0; u < e; u++) {
            uint8_t c = 0;
            for (int t = 0; t < e; t++) c ^= gmul(Ai[u * e + t], C[sel[t] * k + j]);
            coef_make(c, &tab[q * e + u]);
        }
        in[q++] = win + (size_t)j * stride;
    }
    for (int t = 0; t < e; t++) {
        for (int u = 0; u < e; u++) coef_make(Ai[u * e + t], &tab[q * e + u]);
        in[q++] = win + (size_t)(k + sel[t]) * stride;
    }
    for (int u = 0; u < e; u++) out[u] = win + (size_t)miss[u] * stride;
    dot(level, q, in, e, out, tab, S);
    return ORC_OK;
}

/* -------------------------------------------------------------- batch --- */
typedef struct {
    int op, level, scheme, k, r, nw;
    const uint32_t *S;
    uint32_t stride;
    uint64_t lo, hi;
    const uint64_t *present;  /* nw words per window */
    uint8_t *status, *wins;
    const coef_t *tab;
    const uint8_t *C;
} sjob_t;

static void *run_sjob(void *p) {
    sjob_t *j = (sjob_t *)p;
    const size_t wbytes = (size_t)(j->k + j->r) * j->stride;
    for (uint64_t w = j->lo; w < j->hi; w++) {
        uint8_t *win = j->wins + w * wbytes;
        if (j->op == 0)
            encode_window(j->level, j->scheme, j->k, j->r, j->tab, j->S[w], j->stride, win);
        else
            j->status[w] = (uint8_t)decode_window(j->level, j->scheme, j->k, j->r, j->C, j->S[w],
                                                  j->stride, j->present + w * (uint64_t)j->nw, win);
    }
    return NULL;
}

static void run_sbatch(int op, int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                       uint64_t nwin, int nw, const uint64_t *present, uint8_t *status, uint8_t *wins,
                       int nthreads) {
    uint8_t *C = (uint8_t *)calloc((size_t)k * r + 1, 1);
    coef_t *tab = NULL;
    tables_init();
    if (scheme != ORC_XOR) {
        orc_matrix(scheme, k, r, C);
        tab = (coef_t *)malloc(sizeof(coef_t) * (size_t)k * r);
        for (int j = 0; j < k; j++)
            for (int i = 0; i < r; i++) coef_make(C[i * k + j], &tab[(size_t)j * r + i]);
    }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    sjob_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        sjob_t x = {op, orc_simd_level(), scheme, k, r, nw, S, stride,
                    nwin * (uint64_t)t / (uint64_t)nthreads, nwin * (uint64_t)(t + 1) / (uint64_t)nthreads,
                    present, status, wins, tab, C};
        jobs[t] = x;
        if (nthreads == 1) run_sjob(&jobs[t]);
        else pthread_create(&th[t], NULL, run_sjob, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(tab);
    free(C);
}

/* k + r <= ORC_SIMD_MAX_N (256) for the GF schemes (the systematic Vandermonde
 * rows: k <= 64), 64 for XOR */
void orc_encode_batch_simd(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                           uint64_t nwin, uint8_t *wins, int nthreads) {
    run_sbatch(0, scheme, k, r, S, stride, nwin, 1, NULL, NULL, wins, nthreads);
}

void orc_decode_batch_simd(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                           uint64_t nwin, const uint64_t *present, uint8_t *status, uint8_t *wins,
                           int nthreads) {
    run_sbatch(1, scheme, k, r, S, stride, nwin, 1, present, status, wins, nthreads);
}

/* present: nw = ceil((k + r) / 64) words per window (bit i in word i / 64) */
void orc_decode_batch_simd_w(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                             uint64_t nwin, int nw, const uint64_t *present, uint8_t *status, uint8_t *wins,
                             int nthreads) {
    run_sbatch(1, scheme, k, r, S, stride, nwin, nw, present, status, wins, nthreads);
}

/* ------------------------------------------ sliding-window RLC (cfg7) --- */
/* The CPU baseline of the sliding-window code (RFC 8681, m = 8): encode is a
 * dot product per repair over its window; decode splits the lost sources into
 * linked systems, gives each thread a run of whole systems and solves them by
 * the banded elimination of fec_sw_banded.c (forward elimination with the
 * earliest-ending pivot, null-space sweep, back substitution), with every data
 * row operation vectorised.  Outputs equal orc_sw_encode / orc_sw_decode
 * (tests/test_oracle_simd.py). */

/* y ^= c * x over n bytes */
__attribute__((target("avx2,gfni"))) static void axpy_gfni(uint8_t *y, uint8_t c, const uint8_t *x, uint32_t n,
                                                           const coef_t *t) {
    uint32_t p = 0;
    const __m256i m = _mm256_set1_epi64x((long long)t->gfni);
    for (; p + 32 <= n; p += 32) {
        const __m256i d = _mm256_loadu_si256((const __m256i *)(x + p));
        _mm256_storeu_si256((__m256i *)(y + p), _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(y + p)),
                                                                 _mm256_gf2p8affine_epi64_epi8(d, m, 0)));
    }
    for (; p < n; p++) y[p] ^= gmul(c, x[p]);
}
__attribute__((target("avx2"))) static void axpy_avx2(uint8_t *y, uint8_t c, const uint8_t *x, uint32_t n,
                                                      const coef_t *t) {
    const __m256i mask = _mm256_set1_epi8(0x0f);
    const __m256i tl = _mm256_loadu_si256((const __m256i *)t->lo), th = _mm256_loadu_si256((const __m256i *)t->hi);
    uint32_t p = 0;
    for (; p + 32 <= n; p += 32) {
        const __m256i d = _mm256_loadu_si256((const __m256i *)(x + p));
        const __m256i pr = _mm256_xor_si256(_mm256_shuffle_epi8(tl, _mm256_and_si256(d, mask)),
                                            _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi64(d, 4), mask)));
        _mm256_storeu_si256((__m256i *)(y + p), _mm256_xor_si256(_mm256_loadu_si256((const __m256i *)(y + p)), pr));
    }
    for (; p < n; p++) y[p] ^= gmul(c, x[p]);
}
static void axpy(int level, uint8_t *y, uint8_t c, const uint8_t *x, uint32_t n) {
    if (!c) return;
    if (level == 0) {
        for (uint32_t p = 0; p < n; p++) y[p] ^= gmul(c, x[p]);
        return;
    }
    coef_t t;
    coef_make(c, &t);
    if (level >= 2) axpy_gfni(y, c, x, n, &t);
    else axpy_avx2(y, c, x, n, &t);
}

typedef struct {
    const uint8_t *src;
    uint32_t S, stride;
    const orc_sw_repair *hdr;
    uint64_t lo, hi;
    uint8_t *rep;
    int level;
} swenc_t;

static void *run_swenc(void *p) {
    const swenc_t *j = (const swenc_t *)p;
    uint8_t cc[256];
    coef_t tab[256];
    const uint8_t *in[256];
    for (uint64_t t = j->lo; t < j->hi; t++) {
        const orc_sw_repair *h = &j->hdr[t];
        orc_rlc_coefs(h->key, h->nss, h->dt, cc);
        for (int q = 0; q < h->nss; q++) {
            coef_make(cc[q], &tab[q]);
            in[q] = j->src + (h->fss + (uint64_t)q) * j->stride;
        }
        uint8_t *out = j->rep + t * j->stride;
        dot(j->level, h->nss, in, 1, &out, tab, j->S);
    }
    return NULL;
}

void orc_sw_encode_simd(const uint8_t *src, uint64_t nsrc, uint32_t S, uint32_t stride, const orc_sw_repair *hdr,
                        uint64_t nrep, uint8_t *rep, int nthreads) {
    (void)nsrc;
    tables_init();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    swenc_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        swenc_t x = {src, S, stride, hdr, nrep * (uint64_t)t / (uint64_t)nthreads,
                     nrep * (uint64_t)(t + 1) / (uint64_t)nthreads, rep, orc_simd_level()};
        jobs[t] = x;
        if (nthreads == 1) run_swenc(&jobs[t]);
        else pthread_create(&th[t], NULL, run_swenc, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

typedef struct {
    int64_t lo, hi;  /* unknown range (system-local indices) */
    uint8_t *a;      /* coefficients of unknowns lo..hi */
    uint8_t *s;      /* right-hand side */
} srow_t;

typedef struct {
    uint8_t *src;
    const uint8_t *src_present, *rep, *rep_present;
    const orc_sw_repair *hdr;
    uint64_t nrep;
    uint32_t S, stride;
    uint8_t *status;
    const int64_t *lost, *rank;  /* lost sources; rank[i] = lost sources before i */
    int64_t xa, xb;              /* this part's lost range (whole systems) */
    uint64_t ta, tb;             /* candidate repairs (fss in the part's span) */
    int level;
    int64_t rec;
} swdec_t;

static uint8_t scoef(const srow_t *r, int64_t c) { return (c < r->lo || c > r->hi) ? 0 : r->a[c - r->lo]; }

static void *run_swdec(void *pp) {
    swdec_t *J = (swdec_t *)pp;
    const int64_t x0 = J->xa, e = J->xb - J->xa;
    const uint32_t S = J->S;
    if (e <= 0) return NULL;
    srow_t *R = calloc(J->tb - J->ta + 1, sizeof(srow_t));
    int64_t p = 0;
    uint8_t cc[256];
    for (uint64_t t = J->ta; t < J->tb; t++) {
        if (!J->rep_present[t]) continue;
        const orc_sw_repair *h = &J->hdr[t];
        const int64_t r0 = J->rank[h->fss], r1 = J->rank[h->fss + h->nss];
        if (r1 <= r0 || r0 >= J->xb || r1 <= J->xa) continue;  /* holds none of this part's unknowns */
        srow_t *r = &R[p++];
        r->lo = r0 - x0;
        r->hi = r1 - 1 - x0;
        r->a = calloc((size_t)(r->hi - r->lo + 1), 1);
        r->s = malloc(S);
        memcpy(r->s, J->rep + t * J->stride, S);
        orc_rlc_coefs(h->key, h->nss, h->dt, cc);
        /* syndrome: the received sources' terms, one vectorised dot */
        const uint8_t *in[257];
        coef_t tab[257];
        int nin = 0;
        in[nin] = r->s;
        coef_make(1, &tab[nin++]);
        for (int j = 0; j < h->nss; j++) {
            const uint64_t i = h->fss + (uint64_t)j;
            if (!J->src_present[i]) {
                r->a[J->rank[i] - x0 - r->lo] = cc[j];
            } else if (cc[j]) {
                in[nin] = J->src + i * J->stride;
                coef_make(cc[j], &tab[nin++]);
            }
        }
        uint8_t *out = r->s;  /* in place: the dot reads each 32-B block before writing it */
        dot(J->level, nin, in, 1, &out, tab, S);
    }
    /* forward elimination (rows in order of lo: repairs are in fss order) */
    int64_t *piv = malloc(sizeof(int64_t) * e), *act = malloc(sizeof(int64_t) * (p ? p : 1));
    int64_t nact = 0, next = 0, B = 1;
    for (int64_t c = 0; c < e; c++) {
        while (next < p && R[next].lo == c) act[nact++] = next++;
        int64_t P = -1;
        for (int64_t x = 0; x < nact; x++)
            if (scoef(&R[act[x]], c) && (P < 0 || R[act[x]].hi < R[P].hi)) P = act[x];
        piv[c] = P;
        if (P >= 0) {
            const srow_t *rp = &R[P];
            const uint8_t ip = ginv(scoef(rp, c));
            for (int64_t x = 0; x < nact; x++) {
                srow_t *r = &R[act[x]];
                if (act[x] == P || !scoef(r, c)) continue;
                const uint8_t f = gmul(scoef(r, c), ip);
                for (int64_t jj = c; jj <= rp->hi; jj++) r->a[jj - r->lo] ^= gmul(f, scoef(rp, jj));
                axpy(J->level, r->s, f, rp->s, S);
            }
            if (rp->hi - c + 1 > B) B = rp->hi - c + 1;
        }
        int64_t w = 0;
        for (int64_t x = 0; x < nact; x++)
            if (act[x] != P && R[act[x]].hi > c) act[w++] = act[x];
        nact = w;
    }
    /* null-space sweep (vectors over coordinates c .. c + 255, slot j % 256) */
    uint8_t *det = calloc(e, 1);
    int64_t cap = 64, nv = 0;
    uint8_t *V = malloc((size_t)cap * 256);
    for (int64_t c = e - 1; c >= 0; c--) {
        const int sc = (int)(c & 255);
        const int64_t P = piv[c];
        if (P < 0) {
            for (int64_t v = 0; v < nv; v++) V[v * 256 + sc] = 0;
            if (nv == cap) { cap *= 2; V = realloc(V, (size_t)cap * 256); }
            memset(V + nv * 256, 0, 256);
            V[nv * 256 + sc] = 1;
            nv++;
        } else {
            const srow_t *rp = &R[P];
            const uint8_t ip = ginv(scoef(rp, c));
            int zero = 1;
            for (int64_t v = 0; v < nv; v++) {
                uint8_t acc = 0;
                for (int64_t j = c + 1; j <= rp->hi; j++) acc ^= gmul(scoef(rp, j), V[v * 256 + (j & 255)]);
                acc = gmul(acc, ip);
                V[v * 256 + sc] = acc;
                zero &= acc == 0;
            }
            det[c] = (uint8_t)zero;
        }
        if (nv > 2 * B + 8) {  /* basis of the projection on [c, c + B) */
            int64_t rank = 0;
            for (int64_t jj = 0; jj < B && rank < nv; jj++) {
                const int s = (int)((c + jj) & 255);
                int64_t pv = -1;
                for (int64_t v = rank; v < nv; v++)
                    if (V[v * 256 + s]) { pv = v; break; }
                if (pv < 0) continue;
                if (pv != rank)
                    for (int b = 0; b < 256; b++) {
                        uint8_t tt = V[pv * 256 + b]; V[pv * 256 + b] = V[rank * 256 + b]; V[rank * 256 + b] = tt;
                    }
                const uint8_t iv = ginv(V[rank * 256 + s]);
                for (int64_t v = rank + 1; v < nv; v++) {
                    const uint8_t f = gmul(V[v * 256 + s], iv);
                    if (!f) continue;
                    for (int64_t j2 = 0; j2 < B; j2++) {
                        const int s2 = (int)((c + j2) & 255);
                        V[v * 256 + s2] ^= gmul(f, V[rank * 256 + s2]);
                    }
                }
                rank++;
            }
            nv = rank;
        }
    }
    /* back substitution (free unknowns 0): one vectorised dot per pivot */
    uint8_t *X = calloc(256, S ? S : 1);
    const uint8_t *in[257];
    coef_t tab[257];
    for (int64_t c = e - 1; c >= 0; c--) {
        uint8_t *x = X + (size_t)(c & 255) * S;
        const int64_t P = piv[c];
        if (P < 0) {
            memset(x, 0, S);
            continue;
        }
        const srow_t *rp = &R[P];
        const uint8_t ip = ginv(scoef(rp, c));
        int nin = 0;
        in[nin] = rp->s;
        coef_make(ip, &tab[nin++]);
        for (int64_t j = c + 1; j <= rp->hi; j++) {
            const uint8_t a = scoef(rp, j);
            if (!a) continue;
            in[nin] = X + (size_t)(j & 255) * S;
            coef_make(gmul(a, ip), &tab[nin++]);
        }
        dot(J->level, nin, in, 1, &x, tab, S);
        if (det[c]) {
            memcpy(J->src + (uint64_t)J->lost[x0 + c] * J->stride, x, S);
            J->status[J->lost[x0 + c]] = ORC_OK;
            J->rec++;
        }
    }
    for (int64_t q = 0; q < p; q++) { free(R[q].a); free(R[q].s); }
    free(R); free(piv); free(act); free(det); free(V); free(X);
    return NULL;
}

/* Headers must be in fss order (the API's order); returns #recovered. */
int64_t orc_sw_decode_simd(uint8_t *src, const uint8_t *src_present, uint64_t nsrc, const uint8_t *rep,
                           const uint8_t *rep_present, const orc_sw_repair *hdr, uint64_t nrep, uint32_t S,
                           uint32_t stride, uint8_t *status, int nthreads) {
    tables_init();
    int64_t *rank = malloc(sizeof(int64_t) * (nsrc + 1)), *lost = malloc(sizeof(int64_t) * (nsrc ? nsrc : 1));
    int64_t e = 0;
    for (uint64_t i = 0; i < nsrc; i++) {
        rank[i] = e;
        status[i] = src_present[i] ? ORC_OK : ORC_UNRECOVERABLE;
        if (!src_present[i]) lost[e++] = (int64_t)i;
    }
    rank[nsrc] = e;
    /* system starts: lost[x] starts a system iff no received repair starting at
     * or before lost[x - 1] reaches past lost[x] (reach = prefix max of ends) */
    uint64_t wmax = 1;
    for (uint64_t t = 0; t < nrep; t++)
        if (hdr[t].nss > wmax) wmax = hdr[t].nss;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    int64_t cut[257];
    cut[0] = 0;
    {
        uint64_t t = 0, reach = 0;
        int part = 1;
        for (int64_t x = 1; x < e && part < nthreads; x++) {
            for (; t < nrep && hdr[t].fss <= (uint64_t)lost[x - 1]; t++)
                if (rep_present[t] && hdr[t].fss + hdr[t].nss > reach) reach = hdr[t].fss + hdr[t].nss;
            if (reach <= (uint64_t)lost[x] && x >= e * part / nthreads) cut[part++] = x;
        }
        for (; part <= nthreads; part++) cut[part] = e;
    }
    pthread_t th[256];
    swdec_t jobs[256];
    int64_t rec = 0;
    for (int t = 0; t < nthreads; t++) {
        swdec_t x = {src, src_present, rep, rep_present, hdr, nrep, S, stride, status, lost, rank,
                     cut[t], cut[t + 1], 0, 0, orc_simd_level(), 0};
        if (x.xb > x.xa) {
            const uint64_t a = (uint64_t)lost[x.xa], b = (uint64_t)lost[x.xb - 1];
            uint64_t lo = 0, hi = nrep;  /* first repair with fss >= a - wmax + 1 */
            const uint64_t key = a >= wmax ? a - wmax + 1 : 0;
            while (lo < hi) { const uint64_t m = (lo + hi) / 2; if (hdr[m].fss < key) lo = m + 1; else hi = m; }
            x.ta = lo;
            hi = nrep;
            while (lo < hi) { const uint64_t m = (lo + hi) / 2; if (hdr[m].fss <= b) lo = m + 1; else hi = m; }
            x.tb = lo;
        }
        jobs[t] = x;
        if (nthreads == 1) run_swdec(&jobs[t]);
        else pthread_create(&th[t], NULL, run_swdec, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        rec += jobs[t].rec;
    }
    free(rank);
    free(lost);
    return rec;
}
