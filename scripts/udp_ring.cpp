// udp_ring.cpp — real UDP sockets -> pinned window ring -> GPU batch encode ->
// UDP frames -> per-connection decoder (SURVEY.md §8f-4 "zero-copy NIC/socket
// -> pinned ring integration", §8f-3 over a real socket path instead of a
// simulated channel).  One process, four threads, loopback 127.0.0.1:
//
//   gen : sends `packets` datagrams of L bytes (payload p: its packet number
//         and a pattern derived from it) to the FEC sender's ingress socket;
//   tx  : recvmmsg() with one iovec per datagram pointing straight at its row
//         of a pinned, GPU-mapped window buffer (fecgpu_host_alloc): the
//         kernel's copy out of the socket buffer is the only copy before the
//         GPU reads the sources.  A full buffer (`batch` windows) goes to enc;
//   enc : fecgpu_encode_batch(FECGPU_F_HOST_PTRS | SYNC) on the buffer, then
//         sendmmsg() of SOURCE_ID + source row and REPAIR header + repair row
//         as two-iovec gather sends, again straight from the pinned rows;
//         a seeded channel drops each datagram with probability `loss`;
//   rx  : recvmmsg() of the frames, fecgpu_frame_parse, fecgpu_decoder_add_*,
//         and in-order delivery of every packet (received, or recovered with
//         fecgpu_decoder_recovered) checked byte for byte.
//
// Flow control is closed-loop (credits below the sockets' receive buffers),
// so the kernel never drops a datagram: every loss is the seeded channel's.
//   run : scripts/udp_ring <xor|gf256> k r L packets loss batch
// Exit 3 if a delivered packet differs or the unrecovered count differs from
// what the loss pattern allows; 4 on a socket stall.
#include <arpa/inet.h>
#include <time.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
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
#define SYS(x)                                                            \
    do {                                                                  \
        if ((x) < 0) {                                                    \
            perror(#x);                                                   \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

constexpr int kVlen = 64;  // datagrams per recvmmsg / sendmmsg

// payload of packet p: word 0 = p, word t = sm64(p) + t * golden (cheap to check)
void fill(uint8_t *d, uint64_t p, uint32_t L) {
    const uint64_t s = sm64(p);
    uint64_t w = p;
    uint32_t o = 0;
    for (uint64_t t = 0; o + 8 <= L; t++, o += 8) {
        memcpy(d + o, &w, 8);
        w = s + (t + 1) * 0x9E3779B97F4A7C15ull;
    }
    for (; o < L; o++) d[o] = (uint8_t)(w >> (8 * (o & 7)));
}

bool check(const uint8_t *d, uint64_t p, uint32_t L) {
    uint8_t tmp[65536];
    fill(tmp, p, L);
    return !memcmp(tmp, d, L);
}

int udp_socket(uint16_t *port, int rcvbuf) {
    const int s = socket(AF_INET, SOCK_DGRAM, 0);
    SYS(s);
    if (rcvbuf) {
        SYS(setsockopt(s, SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof(rcvbuf)));
        SYS(setsockopt(s, SOL_SOCKET, SO_SNDBUF, &rcvbuf, sizeof(rcvbuf)));
    }
    timeval tv{5, 0};  // a stall (a lost datagram despite the credits) ends the run
    SYS(setsockopt(s, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv)));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = 0;
    SYS(bind(s, (sockaddr *)&a, sizeof(a)));
    socklen_t al = sizeof(a);
    SYS(getsockname(s, (sockaddr *)&a, &al));
    *port = ntohs(a.sin_port);
    return s;
}

// datagrams a socket can queue without dropping (skb truesize ~ payload + 1 KiB)
int credits_for(int s, uint32_t L) {
    int v = 0;
    socklen_t n = sizeof(v);
    SYS(getsockopt(s, SOL_SOCKET, SO_RCVBUF, &v, &n));
    return std::max(8, std::min(4096, v / (int)(2 * (L + 1024))));
}

sockaddr_in to_port(uint16_t port) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = htons(port);
    return a;
}

// blocks until n more datagrams fit in the receiver's credit (n <= credit)
void wait_credit(const std::atomic<uint64_t> &consumed, uint64_t sent, uint64_t n, uint64_t credit) {
    while (sent + n - consumed.load(std::memory_order_acquire) > credit) std::this_thread::yield();
}

// buffer queue between tx and enc
struct Queue {
    std::mutex m;
    std::condition_variable cv;
    std::deque<int> q;
    void push(int v) {
        { std::lock_guard<std::mutex> g(m); q.push_back(v); }
        cv.notify_one();
    }
    int pop() {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return !q.empty(); });
        const int v = q.front();
        q.pop_front();
        return v;
    }
};

double thread_cpu_s() {
    timespec ts;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double secs(std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: %s <xor|gf256> k r L packets loss batch\n", argv[0]);
        return 2;
    }
    const bool gf = !strcmp(argv[1], "gf256");
    const int k = atoi(argv[2]), r = atoi(argv[3]);
    const uint32_t L = (uint32_t)atoi(argv[4]);
    const uint64_t npk = strtoull(argv[5], nullptr, 10);
    const double loss = atof(argv[6]);
    const uint32_t batch = (uint32_t)atoi(argv[7]);
    if (k < 1 || r < 1 || L < 8 || L > 65000 || npk == 0 || batch == 0) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    fecgpu_code code{};
    code.scheme = gf ? FECGPU_SCHEME_GF256 : FECGPU_SCHEME_XOR;
    code.matrix = FECGPU_MATRIX_CAUCHY;
    code.framing = FECGPU_FRAMING_FIXED;
    code.k = (uint16_t)k;
    code.r = (uint16_t)r;
    code.poly = 0x11D;
    CK(fecgpu_code_check(&code));

    const uint32_t stride = (L + 15) & ~15u;
    const size_t wbytes = (size_t)(k + r) * stride, bbytes = wbytes * batch;
    constexpr int kBufs = 4;
    uint8_t *buf[kBufs];
    fecgpu_ctx *ctx = nullptr;
    CK(fecgpu_ctx_new(nullptr, 0, &ctx));
    for (auto &b : buf) CK(fecgpu_host_alloc(bbytes, (void **)&b));
    fecgpu_decoder *dec = nullptr;
    CK(fecgpu_decoder_new(ctx, &code, L, batch, &dec));
    {  // warm-up (code objects, tables, mapping of every buffer): not timed
        for (auto &b : buf) {
            memset(b, 1, bbytes);
            CK(fecgpu_encode_batch(ctx, &code, b, nullptr, nullptr, L, stride, batch,
                                   FECGPU_F_HOST_PTRS | FECGPU_F_SYNC, nullptr));
        }
    }

    const int sockbuf = 8 << 20;
    uint16_t p_gen, p_in, p_enc, p_rx;
    const int s_gen = udp_socket(&p_gen, 0), s_in = udp_socket(&p_in, sockbuf);
    const int s_enc = udp_socket(&p_enc, sockbuf), s_rx = udp_socket(&p_rx, sockbuf);
    const uint64_t credit_in = (uint64_t)credits_for(s_in, L), credit_rx = (uint64_t)credits_for(s_rx, L);
    const sockaddr_in a_in = to_port(p_in), a_rx = to_port(p_rx);

    const uint64_t nwin = (npk + k - 1) / k;            // windows 1..nwin (the last may be short)
    auto dropped = [&](uint64_t w, int i) {              // seeded channel: symbol i of window w
        return (double)(sm64(0xC0FFEEull ^ (w * 64 + (uint64_t)i)) >> 11) * 0x1.0p-53 < loss;
    };
    std::atomic<uint64_t> in_consumed{0}, rx_consumed{0}, enc_sent{0};
    std::atomic<bool> enc_done{false};
    std::atomic<int> stall{0};
    Queue full, freeq;
    for (int i = 0; i < kBufs; i++) freeq.push(i);
    std::vector<int> buf_nwin(kBufs, 0);
    std::vector<uint64_t> buf_w0(kBufs, 0);
    double enc_gpu_s = 0;
    double cpu_s[4] = {0, 0, 0, 0};  // gen, tx, enc, rx thread CPU time

    auto t0 = std::chrono::steady_clock::now();

    std::thread gen([&] {
        std::vector<uint8_t> pk((size_t)kVlen * L);
        mmsghdr m[kVlen];
        iovec iv[kVlen];
        for (uint64_t p = 0; p < npk;) {
            const int n = (int)std::min<uint64_t>(std::min<uint64_t>(kVlen, credit_in), npk - p);
            wait_credit(in_consumed, p, (uint64_t)n, credit_in);
            for (int i = 0; i < n; i++) {
                fill(&pk[(size_t)i * L], p + i, L);
                iv[i] = {&pk[(size_t)i * L], L};
                m[i].msg_hdr = {};
                m[i].msg_hdr.msg_name = (void *)&a_in;
                m[i].msg_hdr.msg_namelen = sizeof(a_in);
                m[i].msg_hdr.msg_iov = &iv[i];
                m[i].msg_hdr.msg_iovlen = 1;
            }
            int sent = 0;
            while (sent < n) {
                const int rc = sendmmsg(s_gen, m + sent, n - sent, 0);
                SYS(rc);
                sent += rc;
            }
            p += n;
        }
        cpu_s[0] = thread_cpu_s();
    });

    std::thread tx([&] {  // ingress datagrams -> pinned window rows
        mmsghdr m[kVlen];
        iovec iv[kVlen];
        uint64_t p = 0;
        for (uint64_t w0 = 1; p < npk; w0 += batch) {
            const int b = freeq.pop();
            const uint64_t nb = std::min<uint64_t>(batch, nwin - (w0 - 1));
            const uint64_t p_end = std::min<uint64_t>(npk, p + nb * k);
            const uint64_t p_first = p;
            while (p < p_end) {
                const int n = (int)std::min<uint64_t>(kVlen, p_end - p);
                for (int i = 0; i < n; i++) {
                    const uint64_t q = p + i - p_first;  // row of this batch
                    iv[i] = {buf[b] + (q / k) * wbytes + (q % k) * stride, L};
                    m[i].msg_hdr = {};
                    m[i].msg_hdr.msg_iov = &iv[i];
                    m[i].msg_hdr.msg_iovlen = 1;
                }
                const int rc = recvmmsg(s_in, m, n, MSG_WAITFORONE, nullptr);
                if (rc < 0) { stall = 1; fprintf(stderr, "tx: ingress stalled at packet %lu\n", (unsigned long)p); exit(4); }
                for (int i = 0; i < rc; i++)
                    if (m[i].msg_len != L || (m[i].msg_hdr.msg_flags & MSG_TRUNC)) {
                        fprintf(stderr, "tx: datagram of %u bytes (FIXED framing wants %u)\n", m[i].msg_len, L);
                        exit(1);
                    }
                p += rc;
                in_consumed.fetch_add(rc, std::memory_order_release);
            }
            // a short last window: its missing sources are empty (zero) packets
            for (uint64_t q = p_end - p_first; q < nb * k; q++)
                memset(buf[b] + (q / k) * wbytes + (q % k) * stride, 0, stride);
            buf_nwin[b] = (int)nb;
            buf_w0[b] = w0;
            full.push(b);
        }
        full.push(-1);
        cpu_s[1] = thread_cpu_s();
    });

    const int vlen_rx = (int)std::min<uint64_t>(kVlen, credit_rx);
    std::thread enc([&] {  // GPU encode, then gather sends straight from the rows
        std::vector<uint8_t> hdr((size_t)kVlen * 32);
        mmsghdr m[kVlen];
        iovec iv[2 * kVlen];
        uint64_t sent = 0;
        for (;;) {
            const int b = full.pop();
            if (b < 0) break;
            const auto ta = std::chrono::steady_clock::now();
            CK(fecgpu_encode_batch(ctx, &code, buf[b], nullptr, nullptr, L, stride, (uint64_t)buf_nwin[b],
                                   FECGPU_F_HOST_PTRS | FECGPU_F_SYNC, nullptr));
            enc_gpu_s += secs(ta, std::chrono::steady_clock::now());
            int n = 0;
            auto flush = [&] {
                int done = 0;
                wait_credit(rx_consumed, sent, (uint64_t)n, credit_rx);
                while (done < n) {
                    const int rc = sendmmsg(s_enc, m + done, n - done, 0);
                    SYS(rc);
                    done += rc;
                }
                sent += n;
                enc_sent.store(sent, std::memory_order_release);
                n = 0;
            };
            for (int wl = 0; wl < buf_nwin[b]; wl++) {
                const uint64_t w = buf_w0[b] + wl;
                const int nsrc = (int)std::min<uint64_t>(k, npk - (w - 1) * k);
                for (int i = 0; i < nsrc + r; i++) {
                    if (dropped(w, i < nsrc ? i : k + (i - nsrc))) continue;
                    uint8_t *h = &hdr[(size_t)n * 32];
                    ssize_t hl;
                    uint8_t *row;
                    if (i < nsrc) {
                        hl = fecgpu_frame_write_source_id(h, 32, w, (uint16_t)i);
                        row = buf[b] + wl * wbytes + (size_t)i * stride;
                    } else {
                        const int ri = i - nsrc;
                        hl = fecgpu_frame_write_repair_header(h, 32, w, (uint16_t)k, (uint16_t)r, (uint16_t)nsrc,
                                                              (uint16_t)ri, L);
                        row = buf[b] + wl * wbytes + (size_t)(k + ri) * stride;
                    }
                    CK(hl);
                    iv[2 * n] = {h, (size_t)hl};
                    iv[2 * n + 1] = {row, L};
                    m[n].msg_hdr = {};
                    m[n].msg_hdr.msg_name = (void *)&a_rx;
                    m[n].msg_hdr.msg_namelen = sizeof(a_rx);
                    m[n].msg_hdr.msg_iov = &iv[2 * n];
                    m[n].msg_hdr.msg_iovlen = 2;
                    if (++n == vlen_rx) flush();
                }
            }
            if (n) flush();
            freeq.push(b);
        }
        enc_done.store(true, std::memory_order_release);
        cpu_s[2] = thread_cpu_s();
        SYS(sendto(s_enc, "", 0, 0, (const sockaddr *)&a_rx, sizeof(a_rx)));  // FIN: wakes rx
    });

    // rx (this thread): frames -> decoder -> in-order delivery
    size_t delivered = 0, recovered = 0, missing = 0, bad = 0;
    const double rx_cpu0 = thread_cpu_s();  // the main thread also did the set-up
    {
        std::vector<uint8_t> rb((size_t)kVlen * (L + 64)), out(L);
        mmsghdr m[kVlen];
        iovec iv[kVlen];
        uint64_t got = 0, w_max = 0, w_next = 1;
        std::vector<uint8_t> have;  // per (window - w_next) bitmap of received sources, ring
        const uint64_t lag = 3 * (uint64_t)batch + 1;
        const size_t ring = (size_t)(lag + 4 * batch) * 64;
        have.assign(ring, 0);
        auto slot = [&](uint64_t w, int i) -> uint8_t & { return have[((w % (ring / 64)) * 64) + i]; };
        auto deliver = [&](uint64_t upto) {
            for (; w_next < upto && w_next <= nwin; w_next++) {
                const int nsrc = (int)std::min<uint64_t>(k, npk - (w_next - 1) * k);
                for (int i = 0; i < nsrc; i++) {
                    uint8_t &h = slot(w_next, i);
                    if (h) { h = 0; delivered++; continue; }  // checked on arrival
                    const ssize_t n = fecgpu_decoder_recovered(dec, w_next, (uint16_t)i, out.data(), L);
                    if (n == FECGPU_ERR_DONE) { missing++; continue; }
                    CK(n);
                    if ((uint32_t)n != L || !check(out.data(), (w_next - 1) * k + i, L)) bad++;
                    else { recovered++; delivered++; }
                }
                (void)fecgpu_decoder_release(dec, w_next);
            }
        };
        bool fin = false;
        for (;;) {
            if (fin && enc_done.load(std::memory_order_acquire) && got == enc_sent.load(std::memory_order_acquire)) break;
            for (int i = 0; i < kVlen; i++) {
                iv[i] = {&rb[(size_t)i * (L + 64)], L + 64};
                m[i].msg_hdr = {};
                m[i].msg_hdr.msg_iov = &iv[i];
                m[i].msg_hdr.msg_iovlen = 1;
            }
            const int rc = recvmmsg(s_rx, m, kVlen, MSG_WAITFORONE, nullptr);
            if (rc < 0) {
                fprintf(stderr, "rx: stalled after %lu datagrams\n", (unsigned long)got);
                exit(4);
            }
            int nfin = 0;
            for (int i = 0; i < rc; i++) {
                const uint8_t *d = &rb[(size_t)i * (L + 64)];
                if (m[i].msg_len == 0) { fin = true; nfin++; continue; }
                fecgpu_frame f;
                const ssize_t h = fecgpu_frame_parse(d, m[i].msg_len, &f);
                CK(h);
                if (f.type == FECGPU_FRAME_SOURCE_ID) {
                    if (m[i].msg_len - (size_t)h != L || !check(d + h, (f.win - 1) * k + f.idx, L)) { bad++; continue; }
                    CK(fecgpu_decoder_add_source(dec, f.win, f.idx, d + h, L));
                    slot(f.win, f.idx) = 1;
                } else {
                    // the short last window's REPAIR frames carry nsrc < k: its
                    // padding sources never go on the wire and are not losses
                    if (f.nsrc < k) CK(fecgpu_decoder_set_window_sources(dec, f.win, f.nsrc));
                    CK(fecgpu_decoder_add_repair(dec, f.win, f.idx, f.payload, f.payload_len));
                }
                w_max = std::max<uint64_t>(w_max, f.win);
            }
            got += rc - nfin;
            rx_consumed.store(got, std::memory_order_release);
            if (w_max > lag) deliver(w_max - lag);
        }
        CK(fecgpu_decoder_flush(dec));
        deliver(nwin + 1);
        cpu_s[3] = thread_cpu_s() - rx_cpu0;
    }
    auto t1 = std::chrono::steady_clock::now();
    gen.join();
    tx.join();
    enc.join();

    // what the loss pattern allows (MDS count for GF; one loss per group with its repair for XOR)
    size_t expect_missing = 0, lost = 0;
    for (uint64_t w = 1; w <= nwin; w++) {
        const int nsrc = (int)std::min<uint64_t>(k, npk - (w - 1) * k);
        std::vector<int> lo(k, 0);
        int nl = 0, rp = 0;
        for (int j = 0; j < nsrc; j++) nl += lo[j] = dropped(w, j);
        lost += nl;
        if (gf) {
            for (int i = 0; i < r; i++) rp += !dropped(w, k + i);
            if (nl > rp) expect_missing += nl;
        } else {
            for (int g = 0; g < r; g++) {
                int ng = 0;
                for (int j = g; j < k; j += r) ng += lo[j];
                if (!(ng == 1 && !dropped(w, k + g))) expect_missing += ng;
            }
        }
    }
    const double t = secs(t0, t1);
    printf("{\"what\": \"UDP loopback -> pinned window ring -> GPU encode -> UDP frames -> decoder\", "
           "\"scheme\": \"%s\", \"k\": %d, \"r\": %d, \"L\": %u, \"batch\": %u, \"packets\": %lu, "
           "\"loss\": %.3f, \"lost\": %zu, \"delivered\": %zu, \"recovered\": %zu, \"unrecovered\": %zu, "
           "\"expected_unrecovered\": %zu, \"corrupt\": %zu, \"credits\": [%lu, %lu], \"seconds\": %.4f, "
           "\"Mpps\": %.3f, \"Gbps_payload\": %.3f, \"encode_call_s\": %.4f, "
           "\"thread_cpu_s\": {\"gen\": %.3f, \"tx\": %.3f, \"enc\": %.3f, \"rx\": %.3f}}\n",
           gf ? "gf256" : "xor", k, r, L, batch, (unsigned long)npk, loss, lost, delivered, recovered, missing,
           expect_missing, bad, (unsigned long)credit_in, (unsigned long)credit_rx, t, npk / t / 1e6,
           npk * (double)L * 8 / t / 1e9, enc_gpu_s, cpu_s[0], cpu_s[1], cpu_s[2], cpu_s[3]);
    fecgpu_decoder_free(dec);
    for (auto &b : buf) fecgpu_host_free(b);
    fecgpu_ctx_free(ctx);
    close(s_gen); close(s_in); close(s_enc); close(s_rx);
    return (bad || missing != expect_missing || delivered + missing != npk) ? 3 : 0;
}
