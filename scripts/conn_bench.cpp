// conn_bench.cpp — per-connection path (fecgpu_encoder_* / fecgpu_decoder_*,
// SURVEY.md §8b item 2, §8f-2/f-3) driven packet by packet from C++, as a QUIC
// Connection would call it: sender appends payloads and reads repairs, a seeded
// lossy channel drops sources and repairs, receiver files what arrives and reads
// lost packets back.  Verifies every packet of every recoverable window and
// reports packets/s and GB/s of payload for each side.
//   build: g++ -O2 -std=c++17 -o scripts/conn_bench scripts/conn_bench.cpp
//          -Lquic-fec-eps_amd/lib -lfecgpu -Wl,-rpath,'$ORIGIN/../quic-fec-eps_amd/lib'
//   run  : scripts/conn_bench <xor|gf256> k r mtu MB loss batch [vary [reorder [dup]]]
//          vary: LENPREFIX lengths 1..mtu; reorder: symbols arrive shuffled within
//          blocks of that many windows; dup: fraction of symbols delivered twice.
// Exit status 3 if a delivered packet differs or the number of unrecovered
// packets differs from what the loss pattern allows (MDS count for GF, one
// loss per group with its repair for XOR).
#include <algorithm>
#include <chrono>
#include <cstdint>
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
    const uint32_t reorder = argc > 9 ? (uint32_t)atoi(argv[9]) : 0;
    const double dup = argc > 10 ? atof(argv[10]) : 0.0;
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
    std::vector<uint16_t> wnsrc(nw_max);  // the REPAIR frames' nsrc (real sources per window)
    uint64_t w_sent = 0;  // windows whose repairs were read and released
    auto send_repairs = [&](uint64_t upto) {
        for (; w_sent < upto; w_sent++) {
            const ssize_t ns = fecgpu_encoder_window_sources(enc, w_sent + 1);
            CK(ns);
            wnsrc[w_sent] = (uint16_t)ns;
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
    size_t p = 0, q = 0;  // next packet to file / to deliver
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
    // symbol events: (window, index); index < k source (packet number p), >= k repair
    struct Ev { uint64_t w; uint32_t i; size_t p; };
    std::vector<Ev> evs;
    auto feed = [&](const Ev &e) {
        ssize_t rc;
        if (e.i < (uint32_t)k) {
            rc = fecgpu_decoder_add_source(dec, e.w, (uint16_t)e.i, &data[off[e.p]], len[e.p]);
        } else {
            const size_t s = (e.w - w_first) * r + (e.i - k);
            // a REPAIR frame of a window closed early names its real sources:
            // the padding indices are not losses (fec_frame.cpp)
            const uint16_t ns = wnsrc[e.w - w_first];
            if (ns < k) CK(fecgpu_decoder_set_window_sources(dec, e.w, ns));
            rc = fecgpu_decoder_add_repair(dec, e.w, (uint16_t)(e.i - k), &reps[s * smax], replen[s]);
        }
        if (rc != FECGPU_ERR_DONE) CK(rc);  // DONE: a duplicate
    };
    const uint32_t blk = reorder ? reorder : 1;
    for (uint64_t w0 = w_first; w0 <= w_last; w0 += blk) {
        evs.clear();
        const uint64_t w1 = std::min<uint64_t>(w_last + 1, w0 + blk);
        for (uint64_t w = w0; w < w1; w++) {
            for (; p < npk && pw[p] == w; p++)
                if (!lost[p]) evs.push_back({w, pi[p], p});
            for (int i = 0; i < r; i++)
                if (!replost[(w - w_first) * r + i]) evs.push_back({w, (uint32_t)(k + i), 0});
        }
        if (reorder)
            for (size_t i = evs.size(); i > 1; i--) {
                ch = sm64(ch);
                std::swap(evs[i - 1], evs[ch % i]);
            }
        for (const Ev &e : evs) {
            feed(e);
            if (dup > 0) {
                ch = sm64(ch);
                if ((double)(ch >> 11) * 0x1.0p-53 < dup) feed(e);
            }
        }
        // auto-flushes run every batch*k symbols; windows 3 batches back are final
        const uint64_t lag = 3 * (uint64_t)batch + blk;
        if (w1 > w_first + lag) deliver(w1 - lag);
    }
    CK(fecgpu_decoder_flush(dec));
    deliver(w_last + 1);
    auto t3 = std::chrono::steady_clock::now();

    // what the loss pattern allows
    size_t expect_missing = 0;
    for (size_t a = 0, b = 0; a < npk; a = b) {
        const uint64_t w = pw[a];
        while (b < npk && pw[b] == w) b++;
        std::vector<int> lo(k, 0);
        for (size_t t = a; t < b; t++) lo[pi[t]] = lost[t];
        int nl = 0;
        for (int j = 0; j < k; j++) nl += lo[j];
        const uint8_t *rl = &replost[(w - w_first) * r];
        if (gf) {
            int rp = 0;
            for (int i = 0; i < r; i++) rp += !rl[i];
            if (nl > rp) expect_missing += nl;
        } else {
            for (int g = 0; g < r; g++) {
                int ng = 0;
                for (int j = g; j < k; j += r) ng += lo[j];
                if (!(ng == 1 && !rl[g])) expect_missing += ng;
            }
        }
    }

    const double ts = std::chrono::duration<double>(t1 - t0).count();
    const double tr = std::chrono::duration<double>(t3 - t2).count();
    size_t lost_n = 0;
    for (auto x : lost) lost_n += x;
    printf("{\"what\": \"per-connection encoder/decoder (C ABI, packet by packet)\", "
           "\"scheme\": \"%s\", \"k\": %d, \"r\": %d, \"mtu\": %u, \"vary\": %d, \"batch\": %u, "
           "\"bytes\": %zu, \"packets\": %zu, \"loss\": %.3f, \"lost\": %zu, \"recovered\": %zu, "
           "\"unrecovered\": %zu, \"expected_unrecovered\": %zu, \"reorder\": %u, \"dup\": %.3f, "
           "\"corrupt\": %zu, \"send_s\": %.4f, \"recv_s\": %.4f, "
           "\"send_Mpps\": %.3f, \"recv_Mpps\": %.3f, \"send_GBps\": %.3f, \"recv_GBps\": %.3f}\n",
           gf ? "gf256" : "xor", k, r, mtu, (int)vary, batch, total, npk, loss, lost_n, recovered,
           missing, expect_missing, reorder, dup, bad, ts, tr, npk / ts / 1e6, npk / tr / 1e6, total / ts / 1e9, total / tr / 1e9);
    fecgpu_encoder_free(enc);
    fecgpu_decoder_free(dec);
    fecgpu_ctx_free(ctx);
    return (bad || missing != expect_missing) ? 3 : 0;
}
