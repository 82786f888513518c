/*
 * fec_sw_banded.c — sliding-window RLC decode (RFC 8681, m = 8) by banded
 * elimination.  TEST INFRASTRUCTURE ONLY (see fec_oracle.h).  PARITY UNPINNED
 * (the fec branch is named only by URL at /root/reference/README.md:7).
 *
 * Same contract and results as orc_sw_decode (fec_oracle.c: one dense
 * identity-augmented Gauss-Jordan over every lost source), without its size
 * limit: statuses and recovered bytes are equal for every input
 * (tests/test_sw_oracle.py checks the two against each other on i.i.d.,
 * burst and rank-deficient cases).  It is the CPU statement of the algorithm
 * the GPU runs for long linked systems (DESIGN.md §4b "Long systems"), and the
 * oracle the GPU tests use where the dense one would take minutes.
 *
 * Structure used.  Unknowns are the lost sources in stream order; an equation
 * is a received repair whose window holds at least one of them, and its
 * nonzero coefficients lie in the unknown range [lo, hi] of the lost sources
 * inside its window (at most 255 of them).
 *  1. Forward elimination in column order.  The pivot of column c is, among
 *     the unfinished rows with a nonzero entry there, the one whose range ends
 *     first (smallest hi).  Eliminating with it never widens a row: every row
 *     stays inside its own [lo, hi], so the rows alive at column c are the
 *     equations whose range holds c.
 *  2. Which unknowns are determined.  x_c is determined iff every vector of
 *     the null space N of the system is zero at c.  N is swept from the last
 *     column down: a free column adds its unit vector, a pivot column gets its
 *     coordinate from the pivot row (a_Pc x_c = sum_{j > c} a_Pj x_j).  Only
 *     the coordinates [c, c + B) matter below column c (B = the widest pivot
 *     row), so the vectors are kept as their projections there, and reduced to
 *     a basis of that projection when they pile up.
 *  3. Back substitution over the data with every free unknown set to 0: a
 *     particular solution, whose determined entries are the only ones written.
 */
#include <stdlib.h>
#include <string.h>

#include "fec_oracle.h"

typedef struct {
    int64_t lo, hi;  /* unknown range of the row */
    uint8_t *a;      /* coefficients of unknowns lo..hi */
    uint8_t *s;      /* right-hand side (S bytes) */
} brow;

static uint8_t coef(const brow *r, int64_t c) { return (c < r->lo || c > r->hi) ? 0 : r->a[c - r->lo]; }

static void row_axpy(uint8_t *y, uint8_t f, const uint8_t *x, uint32_t n) {
    if (!f) return;
    for (uint32_t b = 0; b < n; b++) y[b] ^= orc_gf_mul(f, x[b]);
}

int64_t orc_sw_decode_banded(uint8_t *src, const uint8_t *src_present, uint64_t nsrc, const uint8_t *rep,
                             const uint8_t *rep_present, const orc_sw_repair *hdr, uint64_t nrep, uint32_t S,
                             uint32_t stride, uint8_t *status) {
    int64_t e = 0;
    for (uint64_t i = 0; i < nsrc; i++) {
        status[i] = src_present[i] ? ORC_OK : ORC_UNRECOVERABLE;
        e += !src_present[i];
    }
    if (e == 0) return 0;
    /* nl[i] = index of the first unknown at source >= i */
    int64_t *U = malloc(sizeof(int64_t) * e), *nl = malloc(sizeof(int64_t) * (nsrc + 1));
    {
        int64_t u = e;
        nl[nsrc] = e;
        for (uint64_t i = nsrc; i-- > 0;) {
            if (!src_present[i]) U[--u] = (int64_t)i;
            nl[i] = u;
        }
    }
    /* equations, sorted by lo (stable: qsort on (lo, position) keys) */
    brow *R = calloc(nrep ? nrep : 1, sizeof(brow));
    int64_t p = 0;
    uint8_t cc[256];
    for (uint64_t t = 0; t < nrep; t++) {
        if (!rep_present[t]) continue;
        const orc_sw_repair *h = &hdr[t];
        const int64_t lo = nl[h->fss], hi = nl[h->fss + h->nss] - 1;
        if (lo > hi) continue;
        brow *r = &R[p++];
        r->lo = lo;
        r->hi = hi;
        r->a = calloc((size_t)(hi - lo + 1), 1);
        r->s = malloc(S);
        memcpy(r->s, rep + t * stride, S);
        orc_rlc_coefs(h->key, h->nss, h->dt, cc);
        for (int j = 0; j < h->nss; j++) {
            const uint64_t i = h->fss + (uint64_t)j;
            if (!src_present[i]) r->a[nl[i] - lo] = cc[j];
            else row_axpy(r->s, cc[j], src + i * stride, S);
        }
    }
    /* rows in order of lo (nondecreasing already when the headers' fss are, as
     * the API asks; otherwise a stable insertion sort, test sizes) */
    for (int64_t q = 1; q < p; q++) {
        const brow x = R[q];
        int64_t j = q - 1;
        while (j >= 0 && R[j].lo > x.lo) { R[j + 1] = R[j]; j--; }
        R[j + 1] = x;
    }
    /* 1. forward elimination */
    int64_t *piv = malloc(sizeof(int64_t) * e);
    int64_t *act = malloc(sizeof(int64_t) * (p ? p : 1)), nact = 0, next = 0;
    int64_t B = 1;  /* widest pivot row: hi - c + 1 */
    for (int64_t c = 0; c < e; c++) {
        while (next < p && R[next].lo == c) act[nact++] = next++;
        int64_t P = -1;
        for (int64_t x = 0; x < nact; x++) {
            const brow *r = &R[act[x]];
            if (coef(r, c) && (P < 0 || r->hi < R[P].hi)) P = act[x];
        }
        piv[c] = P;
        if (P >= 0) {
            const brow *rp = &R[P];
            const uint8_t ip = orc_gf_inv(coef(rp, c));
            for (int64_t x = 0; x < nact; x++) {
                brow *r = &R[act[x]];
                if (act[x] == P || !coef(r, c)) continue;
                const uint8_t f = orc_gf_mul(coef(r, c), ip);
                for (int64_t j = c; j <= rp->hi; j++) r->a[j - r->lo] ^= orc_gf_mul(f, coef(rp, j));
                row_axpy(r->s, f, rp->s, S);
            }
            if (rp->hi - c + 1 > B) B = rp->hi - c + 1;
        }
        /* retire the pivot and the rows whose range ends here (now zero) */
        int64_t w = 0;
        for (int64_t x = 0; x < nact; x++)
            if (act[x] != P && R[act[x]].hi > c) act[w++] = act[x];
        nact = w;
    }
    /* 2. null-space sweep: vectors over coordinates c .. c + 255 (slot j % 256) */
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
            det[c] = 0;
        } else {
            const brow *rp = &R[P];
            const uint8_t ip = orc_gf_inv(coef(rp, c));
            int zero = 1;
            for (int64_t v = 0; v < nv; v++) {
                uint8_t acc = 0;
                for (int64_t j = c + 1; j <= rp->hi; j++) acc ^= orc_gf_mul(coef(rp, j), V[v * 256 + (j & 255)]);
                acc = orc_gf_mul(acc, ip);
                V[v * 256 + sc] = acc;
                zero &= acc == 0;
            }
            det[c] = (uint8_t)zero;
        }
        /* keep a basis of the projection on [c, c + B): eliminate, drop zeros */
        if (nv > 2 * B + 8) {
            int64_t rank = 0;
            for (int64_t jj = 0; jj < B && rank < nv; jj++) {
                const int s = (int)((c + jj) & 255);
                int64_t pv = -1;
                for (int64_t v = rank; v < nv; v++)
                    if (V[v * 256 + s]) { pv = v; break; }
                if (pv < 0) continue;
                if (pv != rank)
                    for (int b = 0; b < 256; b++) {
                        uint8_t t = V[pv * 256 + b]; V[pv * 256 + b] = V[rank * 256 + b]; V[rank * 256 + b] = t;
                    }
                const uint8_t iv = orc_gf_inv(V[rank * 256 + s]);
                for (int64_t v = rank + 1; v < nv; v++) {
                    const uint8_t f = orc_gf_mul(V[v * 256 + s], iv);
                    if (!f) continue;
                    for (int64_t j2 = 0; j2 < B; j2++) {
                        const int s2 = (int)((c + j2) & 255);
                        V[v * 256 + s2] ^= orc_gf_mul(f, V[rank * 256 + s2]);
                    }
                }
                rank++;
            }
            nv = rank;  /* rows past the rank are zero on the window */
        }
    }
    /* 3. back substitution with free unknowns 0; write the determined ones */
    uint8_t *X = calloc(256, S ? S : 1);
    int64_t rec = 0;
    for (int64_t c = e - 1; c >= 0; c--) {
        uint8_t *x = X + (size_t)(c & 255) * S;
        const int64_t P = piv[c];
        if (P < 0) {
            memset(x, 0, S);
            continue;
        }
        const brow *rp = &R[P];
        memcpy(x, rp->s, S);
        for (int64_t j = c + 1; j <= rp->hi; j++) row_axpy(x, coef(rp, j), X + (size_t)(j & 255) * S, S);
        const uint8_t ip = orc_gf_inv(coef(rp, c));
        for (uint32_t b = 0; b < S; b++) x[b] = orc_gf_mul(x[b], ip);
        if (det[c]) {
            memcpy(src + (uint64_t)U[c] * stride, x, S);
            status[U[c]] = ORC_OK;
            rec++;
        }
    }
    for (int64_t q = 0; q < p; q++) { free(R[q].a); free(R[q].s); }
    free(R); free(U); free(nl); free(piv); free(act); free(det); free(V); free(X);
    return rec;
}
