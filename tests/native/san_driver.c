/* san_driver.c — host-side sanitizer run (SURVEY.md §5 "race detection /
 * sanitizers": ASan + UBSan on the CPU codec and the host-only ABI code).
 * Built by tests/test_sanitizers.py with -fsanitize=address,undefined together
 * with oracle/fec_oracle.c (test infrastructure) and
 * quic-fec-eps_amd/csrc/fec_frame.cpp (the product's wire-format code, which
 * has no device calls).  Exercises:
 *   - encode -> erase -> decode over every present mask of small codes and
 *     random masks of large ones, ragged symbol lengths (odd S, S < 16);
 *   - frame write/parse round trips at varint boundaries;
 *   - the frame parser on every truncation of valid frames and on random bytes
 *     (no read may leave the buffer: ASan aborts the run if one does).
 * Exit 0 on success; any sanitizer report makes it non-zero. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "../../include/fecgpu.h"
#include "../../oracle/fec_oracle.h"

static uint64_t rng = 0x5EEDFEC0ull;
static uint64_t next(void) { rng = orc_sm64(rng); return rng; }

#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); exit(2); } \
    } while (0)

static void codec_case(int scheme, int k, int r, uint32_t S, uint64_t present) {
    const uint32_t stride = (S + 15u) & ~15u;
    const size_t n = (size_t)(k + r) * stride;
    /* exact-size heap blocks: any overrun of [0, (k+r)*stride) is caught */
    uint8_t *win = malloc(n), *ref = malloc(n);
    memset(win, 0, n);
    for (int j = 0; j < k; j++)
        for (uint32_t b = 0; b < S; b++) win[(size_t)j * stride + b] = (uint8_t)next();
    orc_encode(scheme, k, r, S, stride, win);
    memcpy(ref, win, n);
    for (int i = 0; i < k + r; i++)
        if (!((present >> i) & 1)) memset(win + (size_t)i * stride, 0xAB, stride);
    const int st = orc_decode(scheme, k, r, S, stride, present, win);
    if (st == ORC_OK)
        for (int j = 0; j < k; j++) CHECK(!memcmp(win + (size_t)j * stride, ref + (size_t)j * stride, S));
    free(win);
    free(ref);
}

static void frames(void) {
    static const uint64_t wins[] = {0, 63, 64, 16383, 16384, (1ull << 30) - 1, 1ull << 30, (1ull << 62) - 1};
    uint8_t sym[1300], buf[1400];
    for (size_t i = 0; i < sizeof sym; i++) sym[i] = (uint8_t)next();
    for (size_t w = 0; w < sizeof wins / sizeof wins[0]; w++) {
        for (size_t len = 0; len < sizeof sym; len += 97) {
            ssize_t m = fecgpu_frame_write_repair(buf, sizeof buf, wins[w], 32, 8, 17, 5, sym, len);
            CHECK(m > 0);
            for (ssize_t cut = 0; cut <= m; cut++) {
                /* a heap copy of exactly `cut` bytes: the parser may not read past it */
                uint8_t *t = malloc(cut ? (size_t)cut : 1);
                memcpy(t, buf, (size_t)cut);
                fecgpu_frame f;
                ssize_t rc = fecgpu_frame_parse(t, (size_t)cut, &f);
                if (cut < m) CHECK(rc < 0);
                else CHECK(rc == m && f.win == wins[w] && f.nsrc == 17 && f.payload_len == len &&
                           !memcmp(f.payload, sym, len));
                free(t);
            }
        }
        ssize_t m = fecgpu_frame_write_source_id(buf, sizeof buf, wins[w], 1000);
        CHECK(m > 0);
        fecgpu_frame f;
        CHECK(fecgpu_frame_parse(buf, (size_t)m, &f) == m && f.idx == 1000);
    }
    for (int it = 0; it < 200000; it++) {  /* random bytes, random lengths */
        size_t len = next() % 24;
        uint8_t *t = malloc(len ? len : 1);
        for (size_t i = 0; i < len; i++) t[i] = (uint8_t)next();
        if (len && (next() & 1)) t[0] = 0x80 | (uint8_t)(next() & 1);  /* bias to our types */
        fecgpu_frame f;
        (void)fecgpu_frame_parse(t, len, &f);
        free(t);
    }
}

int main(void) {
    static const int small[][2] = {{1, 1}, {3, 2}, {4, 3}, {5, 3}, {2, 6}};
    static const uint32_t lens[] = {1, 7, 16, 33, 1200};
    for (int s = 0; s < 2; s++)
        for (size_t c = 0; c < sizeof small / sizeof small[0]; c++) {
            const int k = small[c][0], r = small[c][1];
            if (s == ORC_XOR && r > k) continue;
            for (uint64_t p = 0; p < (1ull << (k + r)); p++) codec_case(s, k, r, lens[p % 5], p);
        }
    for (int it = 0; it < 300; it++) {
        const int s = it & 1, r = 1 + (int)(next() % 8);
        const int k = (s == ORC_XOR ? r : 1) + (int)(next() % (uint64_t)(56 - r));
        const uint64_t all = (1ull << (k + r)) - 1;
        codec_case(s, k, r, 1 + (uint32_t)(next() % 1500), all & ~(next() & next()));
    }
    frames();
    puts("sanitizers ok");
    return 0;
}
