// conn_bench.cpp — per-connection path (fecgpu_encoder_* / fecgpu_decoder_*,
// SURVEY.md §8b item 2, §8f-2/f-3) driven packet by packet from C++, as a QUIC
// Connection would call it: sender appends payloads and reads repairs, a seeded
// lossy channel drops sources and repairs, receiver files what arrives and reads
// lost packets back.  Verifies every packet of every recoverable window and
// reports packets/s and GB/s of payload for each side.
//   build: g++ -O2 -std=c++17 -o scripts/conn_bench scripts/conn_bench.cpp
//          -Lquic-fec-eps_amd/lib -lfecgpu -Wl,-rpath,'$ORIGIN/../quic-fec-eps_amd/lib'
//   run  : scripts/conn_bench <xor|gf256> k r mtu MB loss batch [vary]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/fecgpu.h"

static uint64_t sm64(uint64_t x) {
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

int main(int argc, char **argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: %s <xor|gf256> k r mtu MB loss batch [vary]\n", argv[0]);
        return 2;
    }
    const bool gf = !strcmp(argv[1], "gf256");
    const int k = atoi(argv[2]), r = atoi(argv[3]);
    const uint32_t mtu = (uint32_t)atoi(argv[4]);
    const size_t total = (size_t)(atof(argv[5]) * (1 << 20));
    const double loss = atof(argv[6]);
    const uint32_t batch = (uint32_t)atoi(argv[7]);
    const bool vary = argc > 8 && atoi(argv[8]);
    fecgpu_code code{};
    code.scheme = gf ? FECGPU_SCHEME_GF256 : FECGPU_SCHEME_XOR;
    code.matrix = FECGPU_MATRIX_CAUCHY;
    code.framing = vary ? FECGPU_FRAMING_LENPREFIX : FECGPU_FRAMING_FIXED;
    code.k = (uint16_t)k;
    code.r = (uint16_t)r;
    code.poly = 0x11D;

    // the stream, cut into packets (FIXED: every packet mtu bytes, zero-padded tail)
    std::vector<uint8_t> data(total + mtu, 0);
    for (size_t i = 0; i < total; i += 8) {
        const uint64_t v = sm64(i);
        memcpy(&data[i], &v, 8);
    }
    std::vector<size_t> off, len;
    uint64_t h = 0x5EEDFEC0ull;
    for (size_t p = 0; p < total;) {
        h = sm64(h);
        const size_t n = vary ? 1 + h % mtu : mtu;
        off.push_back(p);
        len.push_back(n);
        p += n;
    }
    const size_t npk = off.size();

    fecgpu_ctx *ctx = nullptr;
    CK(fecgpu_ctx_new(nullptr, 0, &ctx));
    fecgpu_encoder *enc = nullptr;
    fecgpu_decoder *dec = nullptr;
    CK(fecgpu_encoder_new(ctx, &code, mtu, batch, &enc));
    CK(fecgpu_decoder_new(ctx, &code, mtu, batch, &dec));

    // warm-up window (ctx tables, code objects, staging): not timed
    {
        std::vector<uint8_t> z(mtu, 1);
        uint64_t w;
        uint16_t i;
        for (int j = 0; j < k; j++) CK(fecgpu_encoder_add_source(enc, z.data(), mtu, &w, &i));
        CK(fecgpu_encoder_flush(enc));
        CK(fecgpu_encoder_release(enc, w));
    }

    // ---- sender
    std::vector<uint64_t> pw(npk);
    std::vector<uint16_t> pi(npk);
    const uint32_t smax = mtu + (vary ? 2 : 0);
    // repairs go "on the wire" (into reps) once the window's batch was encoded;
    // the sender keeps at most ~2 batches of windows alive (steady state)
    const uint64_t nw_max = (npk + k - 1) / k + 1;
    std::vector<uint8_t> reps(nw_max * (size_t)r * smax);
    std::vector<uint32_t> replen(nw_max * (size_t)r);
    uint64_t w_sent = 0;  // windows whose repairs were read and released
    auto send_repairs = [&](uint64_t upto) {
        for (; w_sent < upto; w_sent++) {
            for (int i = 0; i < r; i++) {
                const size_t s = w_sent * r + i;
                ssize_t n = fecgpu_encoder_repair(enc, w_sent + 1, (uint16_t)i, &reps[s * smax], smax);
                CK(n);
                replen[s] = (uint32_t)n;
            }
            CK(fecgpu_encoder_release(enc, w_sent + 1));
        }
    };
    auto t0 = std::chrono::steady_clock::now();
    for (size_t p = 0; p < npk; p++) {
        CK(fecgpu_encoder_add_source(enc, &data[off[p]], len[p], &pw[p], &pi[p]));
        // window ids start at 1 (0 was the warm-up); batches [1 + j*batch, ...) launch when full
        if (pi[p] == k - 1 && pw[p] % batch == 0 && pw[p] >= 2 * (uint64_t)batch)
            send_repairs(pw[p] - batch);
    }
    ssize_t last = fecgpu_encoder_close_window(enc);
    CK(fecgpu_encoder_flush(enc));
    const uint64_t w_first = pw[0], w_last = last >= 0 ? (uint64_t)last : pw[npk - 1];
    send_repairs(w_last);
    auto t1 = std::chrono::steady_clock::now();

    // ---- channel + receiver
    uint64_t ch = 0xC0FFEEull;
    auto drop = [&]() { ch = sm64(ch); return (double)(ch >> 11) * 0x1.0p-53 < loss; };
    std::vector<uint8_t> lost(npk, 0);
    for (size_t p = 0; p < npk; p++) lost[p] = drop();
    std::vector<uint8_t> replost((w_last - w_first + 1) * (size_t)r);
    for (auto &x : replost) x = drop();
    auto t2 = std::chrono::steady_clock::now();
    size_t recovered = 0, missing = 0, bad = 0;
    std::vector<uint8_t> out(mtu);
    size_t p = 0, q = 0;
    uint64_t w_done = w_first;  // windows delivered and released
    // hand lost packets of windows < upto to the application, release them
    auto deliver = [&](uint64_t upto) {
        for (; q < npk && pw[q] < upto; q++) {
            if (!lost[q]) continue;
            ssize_t n = fecgpu_decoder_recovered(dec, pw[q], pi[q], out.data(), mtu);
            if (n == FECGPU_ERR_DONE) { missing++; continue; }
            CK(n);
            if ((size_t)n != len[q] || memcmp(out.data(), &data[off[q]], len[q])) bad++;
            else recovered++;
        }
        for (; w_done < upto; w_done++) (void)fecgpu_decoder_release(dec, w_done);
    };
    for (uint64_t w = w_first; w <= w_last; w++) {
        for (; p < npk && pw[p] == w; p++)
            if (!lost[p]) CK(fecgpu_decoder_add_source(dec, w, pi[p], &data[off[p]], len[p]));
        for (int i = 0; i < r; i++) {
            const size_t s = (w - w_first) * r + i;
            if (!replost[s]) CK(fecgpu_decoder_add_repair(dec, w, (uint16_t)i, &reps[s * smax], replen[s]));
        }
        // auto-flushes run every batch*k symbols; windows 3 batches back are final
        if (w >= w_first + 3 * (uint64_t)batch && (w - w_first) % batch == 0) deliver(w - 3 * (uint64_t)batch);
    }
    CK(fecgpu_decoder_flush(dec));
    deliver(w_last + 1);
    auto t3 = std::chrono::steady_clock::now();

    const double ts = std::chrono::duration<double>(t1 - t0).count();
    const double tr = std::chrono::duration<double>(t3 - t2).count();
    size_t lost_n = 0;
    for (auto x : lost) lost_n += x;
    printf("{\"what\": \"per-connection encoder/decoder (C ABI, packet by packet)\", "
           "\"scheme\": \"%s\", \"k\": %d, \"r\": %d, \"mtu\": %u, \"vary\": %d, \"batch\": %u, "
           "\"bytes\": %zu, \"packets\": %zu, \"loss\": %.3f, \"lost\": %zu, \"recovered\": %zu, "
           "\"unrecovered\": %zu, \"corrupt\": %zu, \"send_s\": %.4f, \"recv_s\": %.4f, "
           "\"send_Mpps\": %.3f, \"recv_Mpps\": %.3f, \"send_GBps\": %.3f, \"recv_GBps\": %.3f}\n",
           gf ? "gf256" : "xor", k, r, mtu, (int)vary, batch, total, npk, loss, lost_n, recovered,
           missing, bad, ts, tr, npk / ts / 1e6, npk / tr / 1e6, total / ts / 1e9, total / tr / 1e9);
    fecgpu_encoder_free(enc);
    fecgpu_decoder_free(dec);
    fecgpu_ctx_free(ctx);
    return bad ? 3 : 0;
}
