// many_conn.cpp — a server's many connections on one ctx, driven from C++:
// C connections each send W windows of k packets through their own encoder,
// a seeded channel drops sources and repairs, and every connection's decoder
// files what arrives.  Senders are flushed together (fecgpu_encoder_flush_many),
// receivers likewise (fecgpu_decoder_flush_many); then every packet is checked
// byte for byte and the unrecovered count against what the loss pattern
// allows.  R rounds close every connection and open new ones (pinned-block
// cache, shared stream pool).  Exercised under host ASan as many_conn_asan.
//   run : scripts/many_conn <xor|gf256> k r L conns windows loss rounds
// Exit 3 on a corrupt packet or an unexpected unrecovered count.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/fecgpu.h"

namespace {

uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

#define CK(x)                                                                           \
    do {                                                                                \
        ssize_t rc_ = (x);                                                              \
        if (rc_ < 0) {                                                                  \
            fprintf(stderr, "%s:%d %s -> %zd (%s: %s)\n", __FILE__, __LINE__, #x, rc_,   \
                    fecgpu_strerror(rc_), fecgpu_last_error());                         \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

// payload of packet j of window w of connection c (LENPREFIX: length 1..L)
uint32_t plen(uint64_t c, uint64_t w, int j, uint32_t L, bool lp) {
    return lp ? 1 + (uint32_t)(sm64((c << 40) ^ (w << 16) ^ (uint64_t)j) % L) : L;
}
void fill(uint8_t *d, uint64_t c, uint64_t w, int j, uint32_t n) {
    const uint64_t s = sm64(~((c << 40) ^ (w << 16) ^ (uint64_t)j));
    for (uint32_t o = 0; o < n; o++) d[o] = (uint8_t)(sm64(s + o / 8) >> (8 * (o % 8)));
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 9) {
        fprintf(stderr, "usage: %s <xor|gf256> k r L conns windows loss rounds\n", argv[0]);
        return 2;
    }
    const bool gf = !strcmp(argv[1], "gf256");
    const int k = atoi(argv[2]), r = atoi(argv[3]);
    const uint32_t L = (uint32_t)atoi(argv[4]);
    const int C = atoi(argv[5]), W = atoi(argv[6]);
    const double loss = atof(argv[7]);
    const int rounds = atoi(argv[8]);
    const bool lp = gf;  // GF runs with LENPREFIX lengths, XOR with FIXED
    fecgpu_code code{};
    code.scheme = gf ? FECGPU_SCHEME_GF256 : FECGPU_SCHEME_XOR;
    code.matrix = FECGPU_MATRIX_CAUCHY;
    code.framing = lp ? FECGPU_FRAMING_LENPREFIX : FECGPU_FRAMING_FIXED;
    code.k = (uint16_t)k;
    code.r = (uint16_t)r;
    CK(fecgpu_code_check(&code));
    fecgpu_ctx *ctx = nullptr;
    CK(fecgpu_ctx_new(nullptr, 0, &ctx));

    std::vector<uint8_t> pkt(L + 2), out(L + 2), rep(L + 2);
    size_t bad = 0, missing = 0, expect_missing = 0, lost = 0, recovered = 0;
    double t_enc = 0, t_dec = 0;
    auto dropped = [&](uint64_t c, uint64_t w, int i, int round) {
        return (double)(sm64(0xD00Dull ^ ((uint64_t)round << 56) ^ (c << 32) ^ (w << 8) ^ (uint64_t)i) >> 11) *
                   0x1.0p-53 < loss;
    };
    for (int round = 0; round < rounds; round++) {
        std::vector<fecgpu_encoder *> encs(C);
        std::vector<fecgpu_decoder *> decs(C);
        for (int c = 0; c < C; c++) {
            // batches larger than the traffic: no automatic launch or flush, the
            // windows go through the flush_many calls
            CK(fecgpu_encoder_new(ctx, &code, L, (uint32_t)W + 1, &encs[c]));
            CK(fecgpu_decoder_new(ctx, &code, L, 4 * (uint32_t)W, &decs[c]));
        }
        // senders: W windows each, queued
        std::vector<uint64_t> win0(C);
        for (int c = 0; c < C; c++)
            for (int w = 0; w < W; w++)
                for (int j = 0; j < k; j++) {
                    const uint32_t n = plen(c, w, j, L, lp);
                    fill(pkt.data(), c, w, j, n);
                    uint64_t wi;
                    uint16_t ji;
                    CK(fecgpu_encoder_add_source(encs[c], pkt.data(), n, &wi, &ji));
                    if (w == 0 && j == 0) win0[c] = wi;
                }
        auto t0 = std::chrono::steady_clock::now();
        CK(fecgpu_encoder_flush_many(encs.data(), (size_t)C));
        auto t1 = std::chrono::steady_clock::now();
        // channel + receivers
        for (int c = 0; c < C; c++)
            for (int w = 0; w < W; w++) {
                const uint64_t wi = win0[c] + (uint64_t)w;
                for (int j = 0; j < k; j++) {
                    if (dropped(c, w, j, round)) continue;
                    const uint32_t n = plen(c, w, j, L, lp);
                    fill(pkt.data(), c, w, j, n);
                    CK(fecgpu_decoder_add_source(decs[c], wi, (uint16_t)j, pkt.data(), n));
                }
                for (int i = 0; i < r; i++) {
                    const ssize_t n = fecgpu_encoder_repair(encs[c], wi, (uint16_t)i, rep.data(), rep.size());
                    CK(n);
                    if (!dropped(c, w, k + i, round))
                        CK(fecgpu_decoder_add_repair(decs[c], wi, (uint16_t)i, rep.data(), (size_t)n));
                }
            }
        auto t2 = std::chrono::steady_clock::now();
        CK(fecgpu_decoder_flush_many(decs.data(), (size_t)C));
        auto t3 = std::chrono::steady_clock::now();
        t_enc += std::chrono::duration<double>(t1 - t0).count();
        t_dec += std::chrono::duration<double>(t3 - t2).count();
        // delivery and the expected outcome
        for (int c = 0; c < C; c++)
            for (int w = 0; w < W; w++) {
                const uint64_t wi = win0[c] + (uint64_t)w;
                int nl = 0, rp = 0;
                std::vector<int> lo(k, 0);
                for (int j = 0; j < k; j++) nl += lo[j] = dropped(c, w, j, round);
                for (int i = 0; i < r; i++) rp += !dropped(c, w, k + i, round);
                lost += nl;
                if (gf) {
                    if (nl > rp) expect_missing += nl;
                } else {
                    for (int g = 0; g < r; g++) {
                        int ng = 0;
                        for (int j = g; j < k; j += r) ng += lo[j];
                        if (!(ng == 1 && !dropped(c, w, k + g, round))) expect_missing += ng;
                    }
                }
                for (int j = 0; j < k; j++) {
                    if (!lo[j]) continue;
                    const ssize_t n = fecgpu_decoder_recovered(decs[c], wi, (uint16_t)j, out.data(), out.size());
                    if (n == FECGPU_ERR_DONE) {
                        missing++;
                        continue;
                    }
                    CK(n);
                    const uint32_t want = plen(c, w, j, L, lp);
                    fill(pkt.data(), c, w, j, want);
                    if ((uint32_t)n != want || memcmp(out.data(), pkt.data(), want)) bad++;
                    else recovered++;
                }
            }
        for (int c = 0; c < C; c++) {
            fecgpu_encoder_free(encs[c]);
            fecgpu_decoder_free(decs[c]);
        }
    }
    fecgpu_ctx_free(ctx);
    printf("{\"what\": \"many connections, encoder/decoder flush_many\", \"scheme\": \"%s\", \"k\": %d, "
           "\"r\": %d, \"L\": %u, \"conns\": %d, \"windows\": %d, \"rounds\": %d, \"loss\": %.3f, \"lost\": %zu, "
           "\"recovered\": %zu, \"unrecovered\": %zu, \"expected_unrecovered\": %zu, \"corrupt\": %zu, "
           "\"encode_flush_ms\": %.3f, \"decode_flush_ms\": %.3f}\n",
           gf ? "gf256" : "xor", k, r, L, C, W, rounds, loss, lost, recovered, missing, expect_missing, bad,
           t_enc * 1e3 / rounds, t_dec * 1e3 / rounds);
    return (bad || missing != expect_missing) ? 3 : 0;
}
