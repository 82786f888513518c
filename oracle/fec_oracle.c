/*
 * fec_oracle.c — CPU restatement of the FEC coding contract.
 * TEST INFRASTRUCTURE ONLY (see fec_oracle.h).  PARITY UNPINNED.
 *
 * What it follows.  The reference fec branch is not mounted
 * (/root/reference/README.md:1-8 is the whole reference; the branch is named
 * only by URL at README.md:7), so nothing here can cite a reference file:line
 * for the arithmetic.  Every function cites the clause of the build-owned
 * contract it restates: SURVEY.md Appendix A (A.1 field, A.2 matrices, A.3
 * framing, A.4 layout, A.5 PRNG, A.6 digest) and SURVEY.md §8a rows a1-a9.
 * Workload definitions (payload, MTU, shortening, erasure streams) are
 * DESIGN.md §Workloads.
 *
 * Deliberately written the slow, obvious way: byte loops, log/exp tables,
 * textbook Gauss-Jordan with pivot search.  It shares no code with the HIP
 * product (quic-fec-eps_amd/csrc).
 */
#include "fec_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- A.1 --- */
/* GF(2^8), reduction polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2.
 * SURVEY.md Appendix A.1; §8a a1. */
static uint8_t g_exp[512];
static int     g_log[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_build(void) {
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (uint8_t)x;
        g_log[x] = i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) g_exp[i] = g_exp[i - 255];
    g_log[0] = -1;
}
static void gf_init(void) { pthread_once(&g_once, gf_build); }

uint8_t orc_gf_exp(int i) { gf_init(); return g_exp[((i % 255) + 255) % 255]; }
int     orc_gf_log(uint8_t a) { gf_init(); return g_log[a]; }

uint8_t orc_gf_mul(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0 || b == 0) return 0;
    return g_exp[g_log[a] + g_log[b]];
}

uint8_t orc_gf_inv(uint8_t a) {
    gf_init();
    if (a == 0) return 0; /* undefined; callers never ask */
    return g_exp[255 - g_log[a]];
}

/* ---------------------------------------------------------------- A.2 --- */
/* Systematic Cauchy generator rows: C[i][j] = inv((k+i) xor j), i<r, j<k
 * (ISA-L gf_gen_cauchy1_matrix layout).  SURVEY.md Appendix A.2; §8a a5. */
void orc_cauchy(int k, int r, uint8_t *C) {
    for (int i = 0; i < r; i++)
        for (int j = 0; j < k; j++) C[i * k + j] = orc_gf_inv((uint8_t)((k + i) ^ j));
}

/* Gauss-Jordan inverse of an n x n matrix (n <= 64) with row pivoting;
 * returns 0 if singular. */
static int gf_invert64(int n, const uint8_t *A, uint8_t *Ainv) {
    static __thread uint8_t M[64][128];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 2 * n; j++)
            M[i][j] = j < n ? A[i * n + j] : (uint8_t)(j - n == i);
    for (int c = 0; c < n; c++) {
        int p = -1;
        for (int i = c; i < n; i++)
            if (M[i][c]) { p = i; break; }
        if (p < 0) return 0;
        if (p != c)
            for (int j = 0; j < 2 * n; j++) { uint8_t t = M[c][j]; M[c][j] = M[p][j]; M[p][j] = t; }
        const uint8_t iv = orc_gf_inv(M[c][c]);
        for (int j = 0; j < 2 * n; j++) M[c][j] = orc_gf_mul(M[c][j], iv);
        for (int i = 0; i < n; i++) {
            if (i == c || !M[i][c]) continue;
            const uint8_t f = M[i][c];
            for (int j = 0; j < 2 * n; j++) M[i][j] ^= orc_gf_mul(f, M[c][j]);
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) Ainv[i * n + j] = M[i][n + j];
    return 1;
}

/* a^n in the field, with 0^0 = 1 (Backblaze Galois.exp) */
static uint8_t gf_pow(uint8_t a, int n) {
    if (n == 0) return 1;
    if (a == 0) return 0;
    return orc_gf_exp((orc_gf_log(a) * n) % 255);
}

/* Systematic Vandermonde generator (FECGPU_MATRIX_VANDERMONDE): the (k+r) x k
 * Vandermonde matrix V[i][j] = i^j (points 0..k+r-1) times the inverse of its
 * top k x k block; rows k.. of the product are the parity rows P[r][k].  The
 * construction of Backblaze's JavaReedSolomon (ReedSolomon.buildMatrix), the
 * default matrix of klauspost/reedsolomon and of the Rust crate
 * reed-solomon-erasure; pinned by their published 5+5 known answer
 * (tests/test_oracle_field.py::test_vandermonde_kat).  MDS (distinct points). */
void orc_vandermonde(int k, int r, uint8_t *P) {
    static __thread uint8_t top[64 * 64], inv[64 * 64];
    for (int i = 0; i < k; i++)
        for (int j = 0; j < k; j++) top[i * k + j] = gf_pow((uint8_t)i, j);
    (void)gf_invert64(k, top, inv);  /* distinct points: never singular */
    for (int i = 0; i < r; i++)
        for (int j = 0; j < k; j++) {
            uint8_t v = 0;
            for (int t = 0; t < k; t++) v ^= orc_gf_mul(gf_pow((uint8_t)(k + i), t), inv[t * k + j]);
            P[i * k + j] = v;
        }
}

/* RFC 8682 TinyMT32, parameter set mat1 = 0x8f7011ee, mat2 = 0xfc78ff1f,
 * tmat = 0x3793fdff, restated from the RFC's reference code (tinymt32_init,
 * next_state, temper).  Pinned by the RFC's seed-1 output list
 * (tests/test_rlc_spec.py).  FECGPU_MATRIX_RLC, SURVEY.md Appendix A.2
 * "seeded RLC" / Appendix B q6. */
typedef struct { uint32_t st[4]; } tmt_t;

static void tmt_next(tmt_t *t) {
    uint32_t y = t->st[3];
    uint32_t x = (t->st[0] & 0x7fffffffu) ^ t->st[1] ^ t->st[2];
    x ^= x << 1;
    y ^= (y >> 1) ^ x;
    t->st[0] = t->st[1];
    t->st[1] = t->st[2];
    t->st[2] = x ^ (y << 10);
    t->st[3] = y;
    if (y & 1) {
        t->st[1] ^= 0x8f7011eeu;
        t->st[2] ^= 0xfc78ff1fu;
    }
}

static uint32_t tmt_u32(tmt_t *t) {
    tmt_next(t);
    uint32_t t0 = t->st[3];
    uint32_t t1 = t->st[0] + (t->st[2] >> 8);
    t0 ^= t1;
    if (t1 & 1) t0 ^= 0x3793fdffu;
    return t0;
}

static void tmt_init(tmt_t *t, uint32_t seed) {
    t->st[0] = seed;
    t->st[1] = 0x8f7011eeu;
    t->st[2] = 0xfc78ff1fu;
    t->st[3] = 0x3793fdffu;
    for (uint32_t i = 1; i < 8; i++)
        t->st[i & 3] ^= i + 1812433253u * (t->st[(i - 1) & 3] ^ (t->st[(i - 1) & 3] >> 30));
    if ((t->st[0] & 0x7fffffffu) == 0 && t->st[1] == 0 && t->st[2] == 0 && t->st[3] == 0) {
        t->st[0] = 'T'; t->st[1] = 'I'; t->st[2] = 'N'; t->st[3] = 'Y';
    }
    for (int i = 0; i < 8; i++) tmt_next(t);
}

void orc_tinymt32(uint32_t seed, int n, uint32_t *out) {
    tmt_t t;
    tmt_init(&t, seed);
    for (int i = 0; i < n; i++) out[i] = tmt_u32(&t);
}

/* RFC 8681 §3.6 generate_coding_coefficients() for m = 8: rand16() = u32 &
 * 0xF, rand256() = u32 & 0xFF; dt = 15: every coefficient a nonzero
 * rand256(); else coefficient i is nonzero iff rand16() <= dt. */
int orc_rlc_coefs(uint32_t key, int n, int dt, uint8_t *cc) {
    if (dt < 0 || dt > 15) return -1;
    tmt_t t;
    tmt_init(&t, key & 0xFFFFu);
    for (int i = 0; i < n; i++) {
        cc[i] = 0;
        if (dt == 15 || (int)(tmt_u32(&t) & 0xFu) <= dt) {
            do cc[i] = (uint8_t)(tmt_u32(&t) & 0xFFu); while (cc[i] == 0);
        }
    }
    return 0;
}

/* parity rows of the scheme's generator (GF schemes); RLC: row i from
 * repair_key key0 + i (ORC_RLC(key0, dt)) */
void orc_matrix(int scheme, int k, int r, uint8_t *C) {
    if (ORC_KIND(scheme) == ORC_GF256_RLC) {
        for (int i = 0; i < r; i++)
            orc_rlc_coefs((uint32_t)(ORC_RLC_KEY(scheme) + i), k, ORC_RLC_DT(scheme), C + i * k);
        return;
    }
    if (scheme == ORC_GF256_VDM) orc_vandermonde(k, r, C);
    else orc_cauchy(k, r, C);
}

/* a6/a7: the missing sources miss[0..e) and e present repairs sel[0..e) whose
 * rows restricted to the missing columns are independent, chosen greedily in
 * repair order (for an MDS matrix: the first e present repairs).  Returns e,
 * or -1 if the present repairs have rank < e (unrecoverable). */
int orc_select_rows(int k, int r, const uint8_t *C, uint64_t present, int *miss, int *sel) {
    int e = 0, n = 0;
    for (int j = 0; j < k; j++)
        if (!((present >> j) & 1)) miss[e++] = j;
    if (e == 0) return 0;
    if (e > 16) return -1;
    uint8_t basis[16][16];
    int pivc[16];
    for (int i = 0; i < r && n < e; i++) {
        if (!((present >> (k + i)) & 1)) continue;
        uint8_t v[16];
        for (int u = 0; u < e; u++) v[u] = C[i * k + miss[u]];
        for (int b = 0; b < n; b++) {
            const uint8_t f = v[pivc[b]];
            if (!f) continue;
            for (int u = 0; u < e; u++) v[u] ^= orc_gf_mul(f, basis[b][u]);
        }
        int pc = -1;
        for (int u = 0; u < e; u++)
            if (v[u]) { pc = u; break; }
        if (pc < 0) continue;  /* dependent on the rows chosen so far */
        const uint8_t iv = orc_gf_inv(v[pc]);
        for (int u = 0; u < e; u++) basis[n][u] = orc_gf_mul(v[u], iv);
        pivc[n] = pc;
        sel[n++] = i;
    }
    return n == e ? e : -1;
}

/* ---------------------------------------------------------------- A.5 --- */
uint64_t orc_sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* sub-stream seeds */
#define TAG_PAY 0x5041594C4F414400ull
#define TAG_MTU 0x4D54550000000000ull
#define TAG_LEN 0x4C454E0000000000ull
#define TAG_ERA 0x4552415345000000ull
#define P10 429496730u /* 0.1 * 2^32, rounded */

uint32_t orc_pkt_len(int workload, uint64_t seed, uint64_t w, int j, int k, uint32_t L) {
    (void)k;
    if (workload == 0) return L; /* fixed */
    uint32_t mtu = (orc_sm64(orc_sm64(seed ^ TAG_MTU) + w) & 1) ? 9000u : 1200u;
    uint64_t h = orc_sm64(orc_sm64(seed ^ TAG_LEN) + ((w << 8) | (uint64_t)j));
    if ((uint32_t)h < P10) return 64u + (uint32_t)((h >> 32) % (uint64_t)(mtu - 63u));
    return mtu;
}

uint32_t orc_sym_len(int workload, uint64_t seed, uint64_t w, int k, uint32_t L) {
    if (workload == 0) return L;
    uint32_t mx = 0;
    for (int j = 0; j < k; j++) {
        uint32_t l = orc_pkt_len(workload, seed, w, j, k, L);
        if (l > mx) mx = l;
    }
    return 2u + mx; /* A.3 LENPREFIX: u16be len || payload || 0-pad */
}

static uint8_t payload_byte(uint64_t spay, uint64_t w, int j, uint32_t o) {
    uint64_t word = orc_sm64(spay + ((w << 24) | ((uint64_t)j << 16) | (uint64_t)(o >> 3)));
    return (uint8_t)(word >> (8 * (o & 7)));
}

/* A.3 framing + A.4 layout, one window's sources. */
void orc_fill_window(int workload, uint64_t seed, uint64_t w, int k, int r, uint32_t L,
                     uint32_t stride, uint8_t *win) {
    uint64_t spay = orc_sm64(seed ^ TAG_PAY);
    memset(win, 0, (size_t)(k + r) * stride);
    for (int j = 0; j < k; j++) {
        uint8_t *s = win + (size_t)j * stride;
        uint32_t len = orc_pkt_len(workload, seed, w, j, k, L);
        if (workload == 0) {
            for (uint32_t o = 0; o < len; o++) s[o] = payload_byte(spay, w, j, o);
        } else {
            s[0] = (uint8_t)(len >> 8);
            s[1] = (uint8_t)len;
            for (uint32_t o = 0; o < len; o++) s[2 + o] = payload_byte(spay, w, j, o);
        }
    }
}

/* erasure streams: 0 none, 1 exactly-r (GF: partial Fisher-Yates over
 * sources; XOR: one source per group), 2 i.i.d. p=0.1 over all k+r symbols */
uint64_t orc_present(int erasure, uint64_t seed, uint64_t w, int scheme, int k, int r) {
    uint64_t all = (k + r >= 64) ? ~0ull : ((1ull << (k + r)) - 1);
    uint64_t sera = orc_sm64(seed ^ TAG_ERA);
    if (erasure == 0) return all;
    if (erasure == 2) {
        uint64_t p = all;
        for (int i = 0; i < k + r; i++)
            if ((uint32_t)orc_sm64(sera + ((w << 8) | (uint64_t)i)) < P10) p &= ~(1ull << i);
        return p;
    }
    uint64_t p = all;
    if (scheme != ORC_XOR) {
        int perm[64];
        for (int j = 0; j < k; j++) perm[j] = j;
        int e = r < k ? r : k;
        for (int t = 0; t < e; t++) {
            uint64_t h = orc_sm64(sera + ((w << 8) | (uint64_t)t));
            int u = t + (int)(h % (uint64_t)(k - t));
            int tmp = perm[t]; perm[t] = perm[u]; perm[u] = tmp;
            p &= ~(1ull << perm[t]);
        }
    } else {
        for (int g = 0; g < r; g++) {
            int n = (k - g + r - 1) / r;
            if (n <= 0) continue;
            int idx = (int)(orc_sm64(sera + ((w << 8) | (uint64_t)g)) % (uint64_t)n);
            p &= ~(1ull << (g + idx * r));
        }
    }
    return p;
}

/* ----------------------------------------------------------- a4 / a5 --- */
void orc_encode(int scheme, int k, int r, uint32_t S, uint32_t stride, uint8_t *win) {
    if (scheme == ORC_XOR) {
        /* a4: R_g = xor of S_j, j = g (mod r) */
        for (int g = 0; g < r; g++) {
            uint8_t *R = win + (size_t)(k + g) * stride;
            memset(R, 0, S);
            for (int j = g; j < k; j += r) {
                const uint8_t *s = win + (size_t)j * stride;
                for (uint32_t p = 0; p < S; p++) R[p] ^= s[p];
            }
        }
        return;
    }
    /* a5: R_i = sum_j C[i][j] * S_j */
    uint8_t C[64 * 64];
    orc_matrix(scheme, k, r, C);
    for (int i = 0; i < r; i++) {
        uint8_t *R = win + (size_t)(k + i) * stride;
        memset(R, 0, S);
        for (int j = 0; j < k; j++) {
            const uint8_t *s = win + (size_t)j * stride;
            uint8_t c = C[i * k + j];
            for (uint32_t p = 0; p < S; p++) R[p] ^= orc_gf_mul(c, s[p]);
        }
    }
}

/* Gauss-Jordan inverse of an n x n matrix over GF(2^8); returns 0 if singular. */
static int gf_invert(int n, const uint8_t *A, uint8_t *Ainv) {
    uint8_t M[16][32];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 2 * n; j++)
            M[i][j] = j < n ? A[i * n + j] : (uint8_t)(j - n == i);
    for (int c = 0; c < n; c++) {
        int p = -1;
        for (int i = c; i < n; i++)
            if (M[i][c]) { p = i; break; }
        if (p < 0) return 0;
        if (p != c)
            for (int j = 0; j < 2 * n; j++) { uint8_t t = M[c][j]; M[c][j] = M[p][j]; M[p][j] = t; }
        uint8_t iv = orc_gf_inv(M[c][c]);
        for (int j = 0; j < 2 * n; j++) M[c][j] = orc_gf_mul(M[c][j], iv);
        for (int i = 0; i < n; i++) {
            if (i == c || !M[i][c]) continue;
            uint8_t f = M[i][c];
            for (int j = 0; j < 2 * n; j++) M[i][j] ^= orc_gf_mul(f, M[c][j]);
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) Ainv[i * n + j] = M[i][n + j];
    return 1;
}

/* ----------------------------------------------------- a6 / a7 / a8 --- */
int orc_decode(int scheme, int k, int r, uint32_t S, uint32_t stride, uint64_t present,
               uint8_t *win) {
    if (scheme == ORC_XOR) {
        /* a8: a group with exactly one missing source and its repair present */
        int status = ORC_OK;
        for (int g = 0; g < r; g++) {
            int miss = -1, nmiss = 0;
            for (int j = g; j < k; j += r)
                if (!((present >> j) & 1)) { miss = j; nmiss++; }
            if (nmiss == 0) continue;
            if (nmiss > 1 || !((present >> (k + g)) & 1)) { status = ORC_UNRECOVERABLE; continue; }
            uint8_t *out = win + (size_t)miss * stride;
            memcpy(out, win + (size_t)(k + g) * stride, S);
            for (int j = g; j < k; j += r) {
                if (j == miss) continue;
                const uint8_t *s = win + (size_t)j * stride;
                for (uint32_t p = 0; p < S; p++) out[p] ^= s[p];
            }
        }
        return status;
    }
    /* a7: solve with e present repairs independent on the missing columns
     * (an MDS matrix: the first e present) */
    int miss[64], sel[64];
    uint8_t C[64 * 64], A[16 * 16], Ai[16 * 16];
    orc_matrix(scheme, k, r, C);
    const int e = orc_select_rows(k, r, C, present, miss, sel);
    if (e == 0) return ORC_OK;
    if (e < 0) return ORC_UNRECOVERABLE;
    for (int t = 0; t < e; t++)
        for (int u = 0; u < e; u++) A[t * e + u] = C[sel[t] * k + miss[u]];
    if (!gf_invert(e, A, Ai)) return ORC_UNRECOVERABLE;
    uint8_t s[16];
    for (uint32_t p = 0; p < S; p++) {
        for (int t = 0; t < e; t++) {
            uint8_t v = win[(size_t)(k + sel[t]) * stride + p];
            for (int j = 0; j < k; j++)
                if ((present >> j) & 1) v ^= orc_gf_mul(C[sel[t] * k + j], win[(size_t)j * stride + p]);
            s[t] = v;
        }
        for (int u = 0; u < e; u++) {
            uint8_t v = 0;
            for (int t = 0; t < e; t++) v ^= orc_gf_mul(Ai[u * e + t], s[t]);
            win[(size_t)miss[u] * stride + p] = v;
        }
    }
    return ORC_OK;
}

/* ---------------------------------------------------------------- A.6 --- */
/* Window digest: XOR over symbols i and 8-byte little-endian words t of
 * sm64(word ^ (w-independent key (i<<16)|t)); bytes >= S count as zero. The
 * batch digest XORs window digests mixed with the window id. */
uint64_t orc_window_digest(int k, int r, uint32_t S, uint32_t stride, const uint8_t *win) {
    uint64_t d = 0;
    for (int i = 0; i < k + r; i++) {
        const uint8_t *s = win + (size_t)i * stride;
        for (uint32_t t = 0; t * 8 < S; t++) {
            uint64_t word = 0;
            for (int b = 0; b < 8; b++) {
                uint32_t o = t * 8 + b;
                if (o < S) word |= (uint64_t)s[o] << (8 * b);
            }
            d ^= orc_sm64(word ^ (((uint64_t)i << 16) | t));
        }
    }
    return d;
}

/* --------------------------------------------------------------- batch --- */
typedef struct {
    int op, scheme, k, r;
    const uint32_t *S;
    uint32_t stride;
    uint64_t lo, hi;
    const uint64_t *present;
    uint8_t *status, *wins;
} job_t;

static void *run_job(void *p) {
    job_t *j = (job_t *)p;
    size_t wbytes = (size_t)(j->k + j->r) * j->stride;
    for (uint64_t w = j->lo; w < j->hi; w++) {
        uint8_t *win = j->wins + w * wbytes;
        if (j->op == 0)
            orc_encode(j->scheme, j->k, j->r, j->S[w], j->stride, win);
        else
            j->status[w] = (uint8_t)orc_decode(j->scheme, j->k, j->r, j->S[w], j->stride,
                                               j->present[w], win);
    }
    return NULL;
}

static void run_batch(job_t proto, uint64_t nwin, int nthreads) {
    gf_init();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto;
        jobs[t].lo = nwin * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].hi = nwin * (uint64_t)(t + 1) / (uint64_t)nthreads;
        if (nthreads == 1) run_job(&jobs[t]);
        else pthread_create(&th[t], NULL, run_job, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void orc_encode_batch(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                      uint64_t nwin, uint8_t *wins, int nthreads) {
    job_t j = {0, scheme, k, r, S, stride, 0, 0, NULL, NULL, wins};
    run_batch(j, nwin, nthreads);
}

void orc_decode_batch(int scheme, int k, int r, const uint32_t *S, uint32_t stride,
                      uint64_t nwin, const uint64_t *present, uint8_t *status, uint8_t *wins,
                      int nthreads) {
    job_t j = {1, scheme, k, r, S, stride, 0, 0, present, status, wins};
    run_batch(j, nwin, nthreads);
}

/* ------------------------------------------------ batch workload fill --- */
typedef struct {
    int workload, scheme, erasure, k, r;
    uint64_t seed, w0, lo, hi;
    uint32_t L, stride;
    uint8_t *wins;
    uint32_t *S;
    uint64_t *present;
    uint64_t src_bytes;
} fill_t;

static void *run_fill(void *p) {
    fill_t *f = (fill_t *)p;
    size_t wbytes = (size_t)(f->k + f->r) * f->stride;
    f->src_bytes = 0;
    for (uint64_t i = f->lo; i < f->hi; i++) {
        uint64_t w = f->w0 + i;
        orc_fill_window(f->workload, f->seed, w, f->k, f->r, f->L, f->stride, f->wins + i * wbytes);
        f->S[i] = orc_sym_len(f->workload, f->seed, w, f->k, f->L);
        f->present[i] = orc_present(f->erasure, f->seed, w, f->scheme, f->k, f->r);
        for (int j = 0; j < f->k; j++) f->src_bytes += orc_pkt_len(f->workload, f->seed, w, j, f->k, f->L);
    }
    return NULL;
}

/* Fill nwin windows (sources, S, present masks) in parallel; returns the sum
 * of packet lengths (source-packet bytes). */
uint64_t orc_make_batch(int workload, uint64_t seed, uint64_t w0, uint64_t nwin, int scheme,
                        int erasure, int k, int r, uint32_t L, uint32_t stride, uint8_t *wins,
                        uint32_t *S, uint64_t *present, int nthreads) {
    gf_init();
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    fill_t f[256];
    for (int t = 0; t < nthreads; t++) {
        fill_t x = {workload, scheme, erasure, k, r, seed, w0,
                    nwin * (uint64_t)t / (uint64_t)nthreads, nwin * (uint64_t)(t + 1) / (uint64_t)nthreads,
                    L, stride, wins, S, present, 0};
        f[t] = x;
        pthread_create(&th[t], NULL, run_fill, &f[t]);
    }
    uint64_t total = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        total += f[t].src_bytes;
    }
    return total;
}

/* ------------------------------------------ sliding-window RLC (RFC 8681) --- */
/* a5 for the sliding-window scheme: repair t combines
 * the nss_t sources of its encoding window with RFC 8681 §3.6 coefficients. */
void orc_sw_encode(const uint8_t *src, uint64_t nsrc, uint32_t S, uint32_t stride,
                   const orc_sw_repair *hdr, uint64_t nrep, uint8_t *rep) {
    uint8_t cc[256];
    (void)nsrc;
    for (uint64_t t = 0; t < nrep; t++) {
        uint8_t *out = rep + t * stride;
        memset(out, 0, S);
        orc_rlc_coefs(hdr[t].key, hdr[t].nss, hdr[t].dt, cc);
        for (int j = 0; j < hdr[t].nss; j++) {
            const uint8_t *s = src + (hdr[t].fss + (uint64_t)j) * stride;
            for (uint32_t b = 0; b < S; b++) out[b] ^= orc_gf_mul(cc[j], s[b]);
        }
    }
}

/* a7 for the sliding-window scheme: unknowns = lost sources, equations = the
 * received repairs whose windows hold at least one unknown, with right-hand
 * side s_t = rep_t + sum over the window's received sources of cc * src.
 * Gauss-Jordan with pivot search on [A | I]; a pivot column is determined iff
 * its pivot row is zero on every free column, and then x = (I part) * s. */
int64_t orc_sw_decode(uint8_t *src, const uint8_t *src_present, uint64_t nsrc, const uint8_t *rep,
                      const uint8_t *rep_present, const orc_sw_repair *hdr, uint64_t nrep,
                      uint32_t S, uint32_t stride, uint8_t *status) {
    int64_t e = 0;
    for (uint64_t i = 0; i < nsrc; i++) {
        status[i] = src_present[i] ? 0 : 1;
        e += !src_present[i];
    }
    if (e == 0) return 0;
    if (e > 4096) return -1;
    int64_t *unk = malloc(sizeof(int64_t) * e), *col = malloc(sizeof(int64_t) * nsrc);
    e = 0;
    for (uint64_t i = 0; i < nsrc; i++) {
        col[i] = -1;
        if (!src_present[i]) { col[i] = e; unk[e++] = (int64_t)i; }
    }
    int64_t *eq = malloc(sizeof(int64_t) * (nrep ? nrep : 1)), p = 0;
    uint8_t cc[256];
    for (uint64_t t = 0; t < nrep; t++) {
        if (!rep_present[t]) continue;
        int any = 0;
        for (int j = 0; j < hdr[t].nss; j++) any |= col[hdr[t].fss + j] >= 0;
        if (any) eq[p++] = (int64_t)t;
    }
    const int64_t w = e + p;
    uint8_t *M = calloc((size_t)p * w, 1), *s = calloc((size_t)p * S, 1);
    for (int64_t q = 0; q < p; q++) {
        const orc_sw_repair *h = &hdr[eq[q]];
        orc_rlc_coefs(h->key, h->nss, h->dt, cc);
        memcpy(s + q * S, rep + eq[q] * stride, S);
        for (int j = 0; j < h->nss; j++) {
            const uint64_t i = h->fss + j;
            if (col[i] >= 0) { M[q * w + col[i]] = cc[j]; continue; }
            for (uint32_t b = 0; b < S; b++) s[q * S + b] ^= orc_gf_mul(cc[j], src[i * stride + b]);
        }
        M[q * w + e + q] = 1;
    }
    int64_t *pivrow = malloc(sizeof(int64_t) * e), nused = 0;
    char *isfree = calloc(e, 1);
    for (int64_t c = 0; c < e; c++) {
        int64_t pr = -1;
        for (int64_t q = nused; q < p; q++)
            if (M[q * w + c]) { pr = q; break; }
        if (pr < 0) { isfree[c] = 1; pivrow[c] = -1; continue; }
        if (pr != nused)
            for (int64_t j = 0; j < w; j++) { uint8_t x = M[pr * w + j]; M[pr * w + j] = M[nused * w + j]; M[nused * w + j] = x; }
        pr = nused++;
        const uint8_t iv = orc_gf_inv(M[pr * w + c]);
        for (int64_t j = 0; j < w; j++) M[pr * w + j] = orc_gf_mul(M[pr * w + j], iv);
        for (int64_t q = 0; q < p; q++) {
            const uint8_t f = M[q * w + c];
            if (q == pr || !f) continue;
            for (int64_t j = 0; j < w; j++) M[q * w + j] ^= orc_gf_mul(f, M[pr * w + j]);
        }
        pivrow[c] = pr;
    }
    int64_t rec = 0;
    for (int64_t c = 0; c < e; c++) {
        if (isfree[c]) continue;
        const int64_t pr = pivrow[c];
        int det = 1;
        for (int64_t j = 0; j < e; j++)
            if (isfree[j] && M[pr * w + j]) { det = 0; break; }
        if (!det) continue;
        uint8_t *out = src + unk[c] * stride;
        memset(out, 0, S);
        for (int64_t q = 0; q < p; q++) {
            const uint8_t f = M[pr * w + e + q];
            if (!f) continue;
            for (uint32_t b = 0; b < S; b++) out[b] ^= orc_gf_mul(f, s[q * S + b]);
        }
        status[unk[c]] = 0;
        rec++;
    }
    free(unk); free(col); free(eq); free(M); free(s); free(pivrow); free(isfree);
    return rec;
}
