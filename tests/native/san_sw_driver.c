/* san_sw_driver.c — host-side sanitizer run over the sliding-window CPU code
 * (ADVICE r03): the banded decoder (oracle/fec_sw_banded.c, the
 * CPU statement of the GPU's long-system path) and the threaded AVX2 / GFNI
 * codec (oracle/fec_cpu_simd.c, the bench's CPU baseline).  Built by
 * tests/test_sanitizers.py twice: ASan + UBSan, and ThreadSanitizer (the SIMD
 * codec's worker threads).  Every buffer is an exact-size heap block, so a read
 * or write past a stream, a repair row or a status array is caught.
 * Exercises, on random streams with odd symbol sizes:
 *   - banded decode == dense Gauss-Jordan (statuses, count, bytes) under i.i.d.
 *     loss, bursts, sparse coefficients (rank-deficient systems), and a stream
 *     whose lost sources form one long system;
 *   - more than 256 repairs alive at one column (two repairs per step at
 *     W = 255, and 300 repairs sharing one fss): banded only;
 *   - the SIMD sliding-window encode / decode at every level the host has and
 *     1 / 3 / 8 threads == the scalar oracle;
 *   - the SIMD block codec (XOR, GF) with threads == the scalar one.
 * Exit 0 and "sw sanitizers ok" on success; any report makes it non-zero. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/fec_oracle.h"

static uint64_t rng = 0x5EEDFEC5ull;
static uint64_t next(void) { rng = orc_sm64(rng); return rng; }

#define CHECK(c)                                                                           \
    do {                                                                                   \
        if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); exit(2); } \
    } while (0)

typedef struct {
    uint64_t nsrc, nrep;
    uint32_t S, stride;
    uint8_t *src, *rep, *sp, *rp;
    orc_sw_repair *hdr;
} stream_t;

/* a repair after every k sources over the last W (mult repairs per step) */
static stream_t make_stream(uint64_t nsrc, int k, int W, int mult, int dt, uint32_t S) {
    stream_t s;
    s.nsrc = nsrc;
    s.S = S;
    s.stride = (S + 15u) & ~15u;
    s.nrep = (nsrc / (uint64_t)k) * (uint64_t)mult;
    s.src = malloc(nsrc * s.stride);
    s.rep = malloc(s.nrep ? s.nrep * s.stride : 1);
    s.sp = malloc(nsrc);
    s.rp = malloc(s.nrep ? s.nrep : 1);
    s.hdr = calloc(s.nrep ? s.nrep : 1, sizeof(orc_sw_repair));
    for (uint64_t i = 0; i < nsrc * s.stride; i++) s.src[i] = (uint8_t)next();
    for (uint64_t t = 0; t < s.nrep; t++) {
        const uint64_t end = (t / (uint64_t)mult + 1) * (uint64_t)k;
        const uint64_t fss = end > (uint64_t)W ? end - (uint64_t)W : 0;
        s.hdr[t].fss = fss;
        s.hdr[t].nss = (uint16_t)(end - fss);
        s.hdr[t].key = (uint16_t)(t * 7 + 3);
        s.hdr[t].dt = (uint8_t)dt;
    }
    orc_sw_encode(s.src, nsrc, S, s.stride, s.hdr, s.nrep, s.rep);
    return s;
}

static void lose(stream_t *s, double p, int burst) {
    const uint64_t thr = (uint64_t)(p * 18446744073709551615.0);
    for (uint64_t i = 0; i < s->nsrc; i++) s->sp[i] = next() >= thr;
    for (uint64_t t = 0; t < s->nrep; t++) s->rp[t] = next() >= thr;
    if (burst && s->nsrc > (uint64_t)burst) {
        const uint64_t b = next() % (s->nsrc - (uint64_t)burst);
        memset(s->sp + b, 0, (size_t)burst);
    }
}

static void free_stream(stream_t *s) {
    free(s->src);
    free(s->rep);
    free(s->sp);
    free(s->rp);
    free(s->hdr);
}

/* decode a poisoned copy with `which` (0 dense, 1 banded, 2 simd) */
static int64_t decode_copy(const stream_t *s, int which, int threads, uint8_t **out, uint8_t **st) {
    *out = malloc(s->nsrc * s->stride);
    *st = malloc(s->nsrc);
    memcpy(*out, s->src, s->nsrc * s->stride);
    for (uint64_t i = 0; i < s->nsrc; i++)
        if (!s->sp[i]) memset(*out + i * s->stride, 0xAB, s->stride);
    if (which == 0) return orc_sw_decode(*out, s->sp, s->nsrc, s->rep, s->rp, s->hdr, s->nrep, s->S, s->stride, *st);
    if (which == 1)
        return orc_sw_decode_banded(*out, s->sp, s->nsrc, s->rep, s->rp, s->hdr, s->nrep, s->S, s->stride, *st);
    return orc_sw_decode_simd(*out, s->sp, s->nsrc, s->rep, s->rp, s->hdr, s->nrep, s->S, s->stride, *st, threads);
}

static void same_decode(const stream_t *s, int wa, int ta, int wb, int tb) {
    uint8_t *da, *sa, *db, *sb;
    const int64_t na = decode_copy(s, wa, ta, &da, &sa), nb = decode_copy(s, wb, tb, &db, &sb);
    CHECK(na >= 0 && na == nb);
    CHECK(!memcmp(sa, sb, s->nsrc));
    for (uint64_t i = 0; i < s->nsrc; i++) {
        if (sa[i]) continue;
        CHECK(!memcmp(da + i * s->stride, db + i * s->stride, s->S));
        CHECK(!memcmp(da + i * s->stride, s->src + i * s->stride, s->S));
    }
    free(da);
    free(sa);
    free(db);
    free(sb);
}

static void sw_cases(void) {
    /* banded == dense on small streams */
    for (int it = 0; it < 40; it++) {
        const int k = 1 + (int)(next() % 8), W = k + (int)(next() % 60);
        const int dt = (it % 4 == 0) ? (int)(next() % 4) : 15;
        stream_t s = make_stream(150 + next() % 400, k, W, 1, dt, 1 + (uint32_t)(next() % 70));
        lose(&s, (it % 3) * 0.08 + 0.02, (it % 5 == 0) ? 40 : 0);
        same_decode(&s, 0, 1, 1, 1);
        free_stream(&s);
    }
    /* long systems and > 256 alive rows: banded vs the SIMD decoder */
    {
        stream_t s = make_stream(1500, 1, 255, 2, 15, 9);  /* ~500 repairs cover each source */
        lose(&s, 0.15, 0);
        same_decode(&s, 1, 1, 2, 3);
        free_stream(&s);
    }
    {
        stream_t s = make_stream(900, 4, 32, 1, 15, 13);
        /* 300 extra repairs over one 255-source window */
        const uint64_t extra = 300, n = s.nrep + extra;
        orc_sw_repair *h = calloc(n, sizeof *h);
        uint64_t o = 0, e = 0;
        for (uint64_t t = 0; t < s.nrep; t++) {
            while (e < extra && s.hdr[t].fss > 300) {
                h[o].fss = 300;
                h[o].nss = 255;
                h[o].key = (uint16_t)(5000 + e);
                h[o].dt = 15;
                o++;
                e++;
            }
            h[o++] = s.hdr[t];
        }
        CHECK(o == n);
        free(s.hdr);
        free(s.rep);
        free(s.rp);
        s.hdr = h;
        s.nrep = n;
        s.rep = malloc(n * s.stride);
        s.rp = malloc(n);
        orc_sw_encode(s.src, s.nsrc, s.S, s.stride, s.hdr, s.nrep, s.rep);
        lose(&s, 0.03, 0);
        memset(s.sp + 300, 0, 120);
        same_decode(&s, 1, 1, 2, 8);
        free_stream(&s);
    }
    /* SIMD encode / decode at every level and thread count */
    const int top = orc_simd_detect();
    for (int lvl = 0; lvl <= top; lvl++) {
        orc_simd_set_level(lvl);
        static const int threads[] = {1, 3, 8};
        for (int ti = 0; ti < 3; ti++) {
            const int th = threads[ti];
            stream_t s = make_stream(700, 8, 32, 1, lvl == 1 ? 5 : 15, 1 + (uint32_t)(next() % 200));
            uint8_t *r2 = malloc(s.nrep * s.stride);
            memset(r2, 0, s.nrep * s.stride);
            orc_sw_encode_simd(s.src, s.nsrc, s.S, s.stride, s.hdr, s.nrep, r2, th);
            for (uint64_t t = 0; t < s.nrep; t++) CHECK(!memcmp(r2 + t * s.stride, s.rep + t * s.stride, s.S));
            free(r2);
            lose(&s, 0.1, 30);
            same_decode(&s, 1, 1, 2, th);
            free_stream(&s);
        }
    }
    orc_simd_set_level(-1);
}

static void block_cases(void) {
    const int top = orc_simd_detect();
    for (int lvl = 0; lvl <= top; lvl++) {
        orc_simd_set_level(lvl);
        for (int it = 0; it < 6; it++) {
            const int scheme = it & 1, r = 1 + (int)(next() % 8);
            const int k = (scheme == ORC_XOR ? r : 1) + (int)(next() % (uint64_t)(40 - r));
            const uint64_t nwin = 3 + next() % 60;
            const uint32_t Smax = 1 + (uint32_t)(next() % 600), stride = (Smax + 15u) & ~15u;
            const size_t wb = (size_t)(k + r) * stride;
            uint32_t *S = malloc(nwin * 4);
            uint64_t *pres = malloc(nwin * 8);
            uint8_t *a = malloc(nwin * wb), *b = malloc(nwin * wb), *sa = malloc(nwin), *sb = malloc(nwin);
            for (uint64_t w = 0; w < nwin; w++) {
                S[w] = 1 + (uint32_t)(next() % Smax);
                pres[w] = ((1ull << (k + r)) - 1) & ~(next() & next() & next());
            }
            for (size_t i = 0; i < nwin * wb; i++) a[i] = (uint8_t)next();
            for (uint64_t w = 0; w < nwin; w++)  /* bytes past S are zero (A.3) */
                for (int j = 0; j < k + r; j++) memset(a + w * wb + (size_t)j * stride + S[w], 0, stride - S[w]);
            memcpy(b, a, nwin * wb);
            orc_encode_batch(scheme, k, r, S, stride, nwin, a, 1);
            orc_encode_batch_simd(scheme, k, r, S, stride, nwin, b, 1 + it % 4);
            CHECK(!memcmp(a, b, nwin * wb));
            orc_decode_batch(scheme, k, r, S, stride, nwin, pres, sa, a, 1);
            orc_decode_batch_simd(scheme, k, r, S, stride, nwin, pres, sb, b, 1 + it % 4);
            CHECK(!memcmp(sa, sb, nwin));
            for (uint64_t w = 0; w < nwin; w++)
                if (!sa[w])
                    for (int j = 0; j < k; j++)
                        CHECK(!memcmp(a + w * wb + (size_t)j * stride, b + w * wb + (size_t)j * stride, S[w]));
            free(S);
            free(pres);
            free(a);
            free(b);
            free(sa);
            free(sb);
        }
    }
    orc_simd_set_level(-1);
}

int main(void) {
    sw_cases();
    block_cases();
    puts("sw sanitizers ok");
    return 0;
}
