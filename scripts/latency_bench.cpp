// latency_bench.cpp — GPU round-trip latency of the per-connection path
// (when batches reach the GPU).  For a batch of B windows:
//   encode: time from the add_source that closes the batch's last window (it
//           launches the batch) until that window's repairs are readable;
//   decode: time of the flush that recovers the batch (2 sources lost per
//           window, both repairs received).
// Median of 31 rounds per batch size; one JSON line per (code, B).
//   run: scripts/latency_bench <xor|gf256> k r mtu
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/fecgpu.h"

#define CK(x)                                                                          \
    do {                                                                               \
        ssize_t rc_ = (x);                                                             \
        if (rc_ < 0) {                                                                 \
            fprintf(stderr, "%s:%d %s -> %zd (%s)\n", __FILE__, __LINE__, #x, rc_,     \
                    fecgpu_last_error());                                              \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

using clk = std::chrono::steady_clock;

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s <xor|gf256> k r mtu\n", argv[0]);
        return 2;
    }
    const bool gf = !strcmp(argv[1], "gf256");
    const int k = atoi(argv[2]), r = atoi(argv[3]);
    const uint32_t mtu = (uint32_t)atoi(argv[4]);
    fecgpu_code code{};
    code.scheme = gf ? FECGPU_SCHEME_GF256 : FECGPU_SCHEME_XOR;
    code.framing = FECGPU_FRAMING_FIXED;
    code.k = (uint16_t)k;
    code.r = (uint16_t)r;
    fecgpu_ctx *ctx = nullptr;
    CK(fecgpu_ctx_new(nullptr, 0, &ctx));
    std::vector<uint8_t> pkt(mtu), rep((size_t)r * mtu);
    for (uint32_t i = 0; i < mtu; i++) pkt[i] = (uint8_t)(i * 131 + 7);
    for (uint32_t B : {1u, 4u, 16u, 64u, 256u, 1024u}) {
        fecgpu_encoder *enc = nullptr;
        fecgpu_decoder *dec = nullptr;
        CK(fecgpu_encoder_new(ctx, &code, mtu, B, &enc));
        CK(fecgpu_decoder_new(ctx, &code, mtu, 1u << 30, &dec));  // flush only when asked
        std::vector<double> te, td;
        uint64_t w = 0, idw = 0;
        uint16_t idx = 0;
        for (int round = 0; round < 33; round++) {
            // encode: fill B windows; the last add_source launches the batch
            clk::time_point t0;
            const uint64_t w0 = idw;
            for (uint32_t b = 0; b < B; b++)
                for (int j = 0; j < k; j++) {
                    if (b == B - 1 && j == k - 1) t0 = clk::now();
                    CK(fecgpu_encoder_add_source(enc, pkt.data(), mtu, &w, &idx));
                }
            for (int i = 0; i < r; i++) CK(fecgpu_encoder_repair(enc, w, (uint16_t)i, &rep[(size_t)i * mtu], mtu));
            const double e_us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
            // decode: the same windows with sources 0 and 1 lost
            for (uint64_t x = w0; x <= w; x++) {
                for (int j = 2; j < k; j++) CK(fecgpu_decoder_add_source(dec, x, (uint16_t)j, pkt.data(), mtu));
                for (int i = 0; i < r; i++) {
                    CK(fecgpu_encoder_repair(enc, x, (uint16_t)i, &rep[(size_t)i * mtu], mtu));
                    CK(fecgpu_decoder_add_repair(dec, x, (uint16_t)i, &rep[(size_t)i * mtu], mtu));
                }
            }
            auto t1 = clk::now();
            CK(fecgpu_decoder_flush(dec));
            const double d_us = std::chrono::duration<double, std::micro>(clk::now() - t1).count();
            for (uint64_t x = w0; x <= w; x++) {
                CK(fecgpu_encoder_release(enc, x));
                CK(fecgpu_decoder_release(dec, x));
            }
            idw = w + 1;
            if (round >= 2) {  // warm-up rounds: pinned buffers, code objects
                te.push_back(e_us);
                td.push_back(d_us);
            }
        }
        printf("{\"what\": \"per-connection GPU round trip\", \"scheme\": \"%s\", \"k\": %d, \"r\": %d, "
               "\"mtu\": %u, \"batch_windows\": %u, \"encode_us\": %.1f, \"decode_flush_us\": %.1f, "
               "\"encode_us_per_window\": %.2f, \"decode_us_per_window\": %.2f}\n",
               gf ? "gf256" : "xor", k, r, mtu, B, median(te), median(td), median(te) / B, median(td) / B);
        fflush(stdout);
        fecgpu_encoder_free(enc);
        fecgpu_decoder_free(dec);
    }
    fecgpu_ctx_free(ctx);
    return 0;
}
