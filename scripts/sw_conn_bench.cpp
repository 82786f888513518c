// sw_conn_bench.cpp — the sliding-window per-connection path (fecgpu_sw_encoder_* /
// fecgpu_sw_decoder_*, RFC 8681 with m = 8) driven packet by packet from C++, as
// a QUIC Connection would call it: the sender appends payloads and reads repairs
// as they are encoded, a seeded lossy channel drops sources and repairs, the
// receiver files what arrives and reads lost packets back as they are recovered.
// Every packet the receiver returns is checked byte for byte; reports packets/s
// and GB/s of payload per side and the fraction of losses recovered.
//   build: g++ -O2 -std=c++17 -o scripts/sw_conn_bench scripts/sw_conn_bench.cpp
//          -Lquic-fec-eps_amd/lib -lfecgpu -Wl,-rpath,'$ORIGIN/../quic-fec-eps_amd/lib'
//   run  : scripts/sw_conn_bench E W step MB loss batch [span]
//          E: symbol size (LENPREFIX, payloads 1..E-2 bytes); a repair after every
//          `step` sources over the last W.  SW_GROUP=1|2|4: the ctx's "sw_group".
// Exit status 3 if a returned packet differs from the one sent.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s E W step MB loss batch [span]\n", argv[0]);
        return 2;
    }
    const uint32_t E = (uint32_t)atoi(argv[1]);
    const uint16_t W = (uint16_t)atoi(argv[2]), step = (uint16_t)atoi(argv[3]);
    const double mb = atof(argv[4]), loss = atof(argv[5]);
    const uint32_t batch = (uint32_t)atoi(argv[6]), span = argc > 7 ? (uint32_t)atoi(argv[7]) : 0;
    const uint64_t seed = 0x5EEDFEC0;
    fecgpu_ctx *ctx = nullptr;
    CK(fecgpu_ctx_new(nullptr, 0, &ctx));
    if (const char *g = getenv("SW_GROUP")) CK(fecgpu_ctx_set_tuning(ctx, "sw_group", atoi(g)));
    fecgpu_sw_params p{};
    p.framing = FECGPU_FRAMING_LENPREFIX;
    p.symbol_size = E;
    p.window = W;
    p.step = step;
    p.dt = 15;
    p.batch = batch;
    p.span = span;
    fecgpu_sw_encoder *enc = nullptr;
    fecgpu_sw_decoder *dec = nullptr;
    CK(fecgpu_sw_encoder_new(ctx, &p, &enc));
    CK(fecgpu_sw_decoder_new(ctx, &p, &dec));
    // the stream: payload lengths 1..E-2, bytes from (esi, offset)
    std::vector<uint32_t> len;
    uint64_t total = 0;
    while (total < (uint64_t)(mb * 1e6)) {
        const uint32_t l = 1 + (uint32_t)(sm64(seed ^ len.size()) % (E - 2));
        len.push_back(l);
        total += l;
    }
    const uint64_t n = len.size();
    // payload of ESI i: a 4 KiB-pool slice chosen by i, its first 8 bytes = i
    // (cheap to make and to check, so the timings are the library's)
    std::vector<uint8_t> pool(4096 + E);
    for (size_t o = 0; o < pool.size(); o++) pool[o] = (uint8_t)(sm64(seed + (o >> 3)) >> (8 * (o & 7)));
    auto fill = [&](uint64_t esi, uint8_t *b) {
        memcpy(b, pool.data() + (sm64(esi) & 4095), len[esi]);
        memcpy(b, &esi, len[esi] < 8 ? len[esi] : 8);
    };
    // the sender's output, held so both sides are timed separately: sources, then
    // repairs in the order the encoder emits them, interleaved as on the wire
    struct Rep {
        fecgpu_sw_repair h;
        std::vector<uint8_t> sym;
        uint64_t after;  // the source count when it was read
    };
    std::vector<Rep> reps;
    std::vector<uint8_t> pkt(E), sym(E);
    double t0 = now();
    for (uint64_t i = 0; i < n; i++) {
        fill(i, pkt.data());
        uint64_t esi = 0;
        ssize_t rc;
        while ((rc = fecgpu_sw_encoder_add_source(enc, pkt.data(), len[i], &esi)) == FECGPU_ERR_LIMIT) {
            fecgpu_sw_repair h{};
            while (fecgpu_sw_encoder_next_repair(enc, &h, sym.data(), E) > 0) reps.push_back({h, sym, i});
        }
        CK(rc);
        fecgpu_sw_repair h{};
        while (fecgpu_sw_encoder_next_repair(enc, &h, sym.data(), E) > 0) reps.push_back({h, sym, i + 1});
    }
    CK(fecgpu_sw_encoder_flush(enc));
    {
        fecgpu_sw_repair h{};
        while (fecgpu_sw_encoder_next_repair(enc, &h, sym.data(), E) > 0) reps.push_back({h, sym, n});
    }
    const double t_send = now() - t0;
    // receiver: sources in order with the repairs that were emitted after them
    uint64_t lost = 0, rec = 0, bad = 0, ri = 0, late = 0;
    auto file_repair = [&](const Rep &r) {
        const ssize_t rc = fecgpu_sw_decoder_add_repair(dec, &r.h, r.sym.data(), E);
        if (rc == FECGPU_ERR_DONE) late++;  // its window starts before the receiver's span
        else CK(rc);
    };
    std::vector<uint8_t> got(E), ref(E);
    auto drain = [&]() {
        uint64_t e;
        while (fecgpu_sw_decoder_next_recovered(dec, &e) == 0) {
            const ssize_t m = fecgpu_sw_decoder_recovered(dec, e, got.data(), E);
            if (m < 0) continue;  // given up since
            fill(e, ref.data());
            if ((uint32_t)m != len[e] || memcmp(got.data(), ref.data(), m)) bad++;
            rec++;
        }
    };
    t0 = now();
    for (uint64_t i = 0; i < n; i++) {
        const bool drop = (uint32_t)sm64(seed ^ 0xD0D0 ^ i) < (uint32_t)(loss * 4294967296.0);
        if (drop) {
            lost++;
        } else {
            fill(i, pkt.data());
            CK(fecgpu_sw_decoder_add_source(dec, i, pkt.data(), len[i]));
        }
        for (; ri < reps.size() && reps[ri].after <= i + 1; ri++) {
            if ((uint32_t)sm64(seed ^ 0xBEEF ^ ri) < (uint32_t)(loss * 4294967296.0)) continue;
            file_repair(reps[ri]);
        }
        drain();
    }
    for (; ri < reps.size(); ri++) file_repair(reps[ri]);
    CK(fecgpu_sw_decoder_flush(dec));
    drain();
    const double t_recv = now() - t0;
    printf("{\"E\": %u, \"W\": %u, \"step\": %u, \"batch\": %u, \"packets\": %llu, \"payload_MB\": %.1f, "
           "\"repairs\": %zu, \"send_Mpps\": %.3f, \"send_GBps\": %.3f, \"recv_Mpps\": %.3f, \"recv_GBps\": %.3f, "
           "\"loss\": %.3f, \"lost\": %llu, \"recovered\": %llu, \"late_repairs\": %llu, \"mismatch\": %llu}\n",
           E, W, step, batch, (unsigned long long)n, total / 1e6, reps.size(), n / t_send / 1e6,
           total / t_send / 1e9, n / t_recv / 1e6, total / t_recv / 1e9, loss, (unsigned long long)lost,
           (unsigned long long)rec, (unsigned long long)late, (unsigned long long)bad);
    fecgpu_sw_encoder_free(enc);
    fecgpu_sw_decoder_free(dec);
    fecgpu_ctx_free(ctx);
    return bad ? 3 : 0;
}
