// fec_conn.cpp — per-connection encoder / decoder objects of the C ABI
// (include/fecgpu.h, "per-packet API"; SURVEY.md §8b item 2, §3 call stacks
// A and B, §8f-2/f-3).
//
// These are the calls a QUIC Connection makes one packet at a time: the
// sender appends each protected payload as a source symbol and reads repair
// symbols back; the receiver files sources and repairs by (window, index) and
// reads recovered packets back.  Framing: FIXED —
// every packet of a window has the same length, symbol = packet; LENPREFIX —
// symbol = u16be(len) || payload || zero pad to S = 2 + max len of the window.
//
// Zero-copy design.  Every symbol is written exactly once, by the add call,
// into pinned host memory that the GPU maps, at its final place in a window
// of (k + r) rows of a fixed pitch `stride` = round_up(max symbol, 16):
//   sender   — a ring of batch buffers of `batch` windows each.  Closing the
//              last window of a buffer launches its encode (uniform layout,
//              per-window S) on the encoder's stream and the sender moves on
//              to the next buffer; the kernel reads the sources and writes
//              the repairs over PCIe.  A buffer is recycled once every one of
//              its windows has been released.
//   receiver — a pool of window slots.  flush() collects the windows that can
//              recover something and decodes them in one launch over the pool
//              (ragged layout with a fixed pitch: slot offsets from the first
//              chunk, 64-bit wrap-around), the kernel writing recovered rows
//              in place.  No staging buffers, no H2D / D2H copies.
//              The automatic flush (every batch*k filed symbols) does not
//              wait: its windows are marked in flight and the next call that
//              touches one of them (or the next flush) completes it, so the
//              receiver keeps filing packets while the GPU decodes.  The
//              window that triggered it stays open for the next flush (its
//              remaining repairs are likely still arriving).  fecgpu_decoder_
//              flush() and tick() complete everything before returning.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <vector>

#include "../../include/fecgpu.h"
#include "fec_internal.h"

using fecgpu::BatchArgs;

namespace {

inline uint32_t rup16(uint32_t x) { return (x + 15u) & ~15u; }
inline bool is_lenprefix(const fecgpu_code &c) { return c.framing == FECGPU_FRAMING_LENPREFIX; }

// Pinned host block mapped into the device's address space.
struct Pinned {
    uint8_t *host = nullptr, *dev = nullptr;
    size_t bytes = 0;
};

// Pinned blocks come from the ctx's cache of blocks freed by earlier objects
// (connection churn would otherwise pin and unpin pages per connection).
ssize_t pinned_alloc(fecgpu_ctx *ctx, size_t bytes, Pinned &p) {
    void *h = nullptr, *d = nullptr;
    ssize_t rc = fecgpu::ctx_pinned_get(ctx, bytes, &h);
    if (rc) return rc;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
        fecgpu::ctx_pinned_put(ctx, h, bytes);
        return FECGPU_ERR_DEVICE;
    }
    p.host = static_cast<uint8_t *>(h);
    p.dev = static_cast<uint8_t *>(d);
    p.bytes = bytes;
    return 0;
}

void pinned_free(fecgpu_ctx *ctx, Pinned &p) {
    if (p.host) fecgpu::ctx_pinned_put(ctx, p.host, p.bytes);
    p = Pinned{};
}

// Makes `dev` the current device for the guard's scope.
struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DevGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int ctx_device() {
    int d = 0;
    (void)hipGetDevice(&d);
    return d;
}

// ------------------------------------------------------------ encoder ---
struct EncBatch {
    Pinned mem;               // batch x (k + r) x stride window bytes, then S[batch]
    uint32_t *S = nullptr;    // host view of the per-window symbol lengths
    uint32_t *S_dev = nullptr;
    hipEvent_t done = nullptr;
    uint64_t first = 0;       // window id of slot 0
    uint32_t nwin = 0;        // closed windows
    uint32_t live = 0;        // closed and not released
    bool launched = false;
    std::vector<uint8_t> released;
    std::vector<uint16_t> nsrc;  // real sources per window (k unless closed early)
};

}  // namespace

struct fecgpu_encoder {
    fecgpu_ctx *ctx = nullptr;
    fecgpu_code code{};
    uint32_t max_len = 0, batch = 0, stride = 0;
    size_t wbytes = 0;
    int dev = 0;
    hipStream_t stream = nullptr;  // of the ctx's pool
    hipEvent_t last_done = nullptr; // recorded after the latest launched batch
    uint64_t next_win = 0;
    int open_n = 0;           // sources in the open window
    uint32_t open_max = 0;
    uint32_t open_len[FECGPU_MAX_K] = {};
    EncBatch *cur = nullptr;  // being filled (its windows [first, first + nwin) closed)
    fecgpu_policy policy{};
    uint64_t now = 0;         // latest caller clock (tick)
    uint64_t open_t = 0;      // when the open window got its first packet
    uint64_t cur_t = 0;       // when cur's first window closed
    std::deque<EncBatch *> active;  // window order: launched batches, then cur
    std::vector<EncBatch *> spare;
    std::vector<EncBatch *> all;
};

namespace {

ssize_t enc_take_batch(fecgpu_encoder *e) {
    EncBatch *b = nullptr;
    if (!e->spare.empty()) {
        b = e->spare.back();
        e->spare.pop_back();
        if (b->done) (void)hipEventSynchronize(b->done);  // the GPU is done with it
    } else {
        b = new EncBatch();
        const size_t wb = (size_t)e->batch * e->wbytes;
        ssize_t rc = pinned_alloc(e->ctx, wb + (size_t)e->batch * 4, b->mem);
        if (rc) {
            delete b;
            return rc;
        }
        b->S = reinterpret_cast<uint32_t *>(b->mem.host + wb);
        b->S_dev = reinterpret_cast<uint32_t *>(b->mem.dev + wb);
        if (hipEventCreateWithFlags(&b->done, hipEventDisableTiming) != hipSuccess) {
            pinned_free(e->ctx, b->mem);
            delete b;
            return FECGPU_ERR_DEVICE;
        }
        b->released.assign(e->batch, 0);
        b->nsrc.assign(e->batch, 0);
        e->all.push_back(b);
    }
    b->first = e->next_win;
    b->nwin = 0;
    b->live = 0;
    b->launched = false;
    std::fill(b->released.begin(), b->released.end(), 0);
    e->cur = b;
    e->active.push_back(b);
    return 0;
}

// Encode the current batch's closed windows on the encoder's stream (async).
ssize_t enc_launch(fecgpu_encoder *e) {
    EncBatch *b = e->cur;
    if (!b || b->nwin == 0) return 0;
    BatchArgs a{};
    a.win = b->mem.dev;
    a.sym_len = b->S_dev;
    a.stride = e->stride;
    a.nwin = b->nwin;
    ssize_t rc = fecgpu::launch_batch(e->ctx, &e->code, false, a, e->stream, true, e->dev);
    if (rc) return rc;
    DevGuard g(e->dev);
    if (hipEventRecord(b->done, e->stream) != hipSuccess) return FECGPU_ERR_DEVICE;
    e->last_done = b->done;
    b->launched = true;
    e->cur = nullptr;
    if (b->live == 0) {  // every window already released (never read): recycle
        e->active.pop_back();
        e->spare.push_back(b);
    }
    return (ssize_t)b->nwin;
}

uint8_t *enc_row(fecgpu_encoder *e, EncBatch *b, uint32_t slot, int row) {
    return b->mem.host + (size_t)slot * e->wbytes + (size_t)row * e->stride;
}

ssize_t enc_close(fecgpu_encoder *e) {
    const int k = e->code.k;
    const bool lp = is_lenprefix(e->code);
    EncBatch *b = e->cur;
    const uint32_t slot = b->nwin;
    if (!lp && e->open_n < k) {  // FIXED: missing sources are zero packets of length L
        const uint32_t L = e->open_len[0];
        for (int j = e->open_n; j < k; j++) e->open_len[j] = L;
    }
    const uint32_t S = lp ? 2 + e->open_max : std::max<uint32_t>(e->open_max, 1);
    const uint32_t S16 = rup16(S);
    for (int j = 0; j < k; j++) {
        uint8_t *row = enc_row(e, b, slot, j);
        uint32_t used = 0;
        if (j < e->open_n) used = lp ? 2 + e->open_len[j] : e->open_len[j];
        // zero padding of the symbol (and of its last 16-byte column)
        std::memset(row + used, 0, S16 - used);
    }
    b->S[slot] = S;
    b->nsrc[slot] = (uint16_t)e->open_n;
    if (b->nwin == 0) e->cur_t = e->now;
    b->nwin++;
    b->live++;
    e->next_win++;
    e->open_n = 0;
    e->open_max = 0;
    if (b->nwin == e->batch) return enc_launch(e);  // windows launched, or an error
    return 0;
}

EncBatch *enc_find(fecgpu_encoder *e, uint64_t win, uint32_t &slot) {
    // active batches cover increasing, contiguous window ranges
    auto it = std::upper_bound(e->active.begin(), e->active.end(), win,
                               [](uint64_t w, const EncBatch *b) { return w < b->first; });
    if (it == e->active.begin()) return nullptr;
    EncBatch *b = *(it - 1);
    if (win >= b->first + b->nwin) return nullptr;
    slot = (uint32_t)(win - b->first);
    return b;
}

}  // namespace

extern "C" {

ssize_t fecgpu_encoder_new(fecgpu_ctx *ctx, const fecgpu_code *code, uint32_t max_len,
                           uint32_t batch, fecgpu_encoder **out) {
    if (!ctx || !out || max_len == 0 || batch == 0) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = fecgpu::code_check_narrow(code);
    if (rc) return rc;
    if (is_lenprefix(*code) && max_len > 65535) return FECGPU_ERR_INVALID_ARG;
    auto *e = new fecgpu_encoder();
    e->ctx = ctx;
    e->code = *code;
    e->max_len = max_len;
    e->batch = batch;
    e->stride = rup16(max_len + (is_lenprefix(*code) ? 2 : 0));
    e->wbytes = (size_t)(code->k + code->r) * e->stride;
    e->dev = ctx_device();
    rc = fecgpu::ctx_conn_stream(ctx, e->dev, &e->stream);  // shared, owned by the ctx
    if (rc) {
        delete e;
        return rc;
    }
    *out = e;
    return 0;
}

void fecgpu_encoder_free(fecgpu_encoder *e) {
    if (!e) return;
    DevGuard g(e->dev);
    if (e->last_done) (void)hipEventSynchronize(e->last_done);  // its launches, in stream order
    for (EncBatch *b : e->all) {
        if (b->done) (void)hipEventDestroy(b->done);
        pinned_free(e->ctx, b->mem);
        delete b;
    }
    delete e;
}

ssize_t fecgpu_encoder_add_source(fecgpu_encoder *e, const uint8_t *pkt, size_t len,
                                  uint64_t *win, uint16_t *idx) {
    if (!e || (!pkt && len)) return FECGPU_ERR_INVALID_ARG;
    if (len > e->max_len) return FECGPU_ERR_BUFFER_TOO_SHORT;
    const bool lp = is_lenprefix(e->code);
    if (!lp) {
        if (len == 0) return FECGPU_ERR_INVALID_ARG;
        if (e->open_n && e->open_len[0] != len) return FECGPU_ERR_INVALID_ARG;
    }
    if (e->cur && e->cur->nwin >= e->batch) {
        // a full batch whose launch failed earlier: launch it before taking
        // a new source (never index a slot past the batch)
        ssize_t rc = enc_launch(e);
        if (rc < 0) return rc;
    }
    if (!e->cur) {
        ssize_t rc = enc_take_batch(e);
        if (rc) return rc;
    }
    uint8_t *row = enc_row(e, e->cur, e->cur->nwin, e->open_n);
    if (lp) {
        row[0] = (uint8_t)(len >> 8);
        row[1] = (uint8_t)len;
        if (len) std::memcpy(row + 2, pkt, len);
    } else {
        std::memcpy(row, pkt, len);
    }
    if (win) *win = e->next_win;
    if (idx) *idx = (uint16_t)e->open_n;
    if (e->open_n == 0) e->open_t = e->now;
    e->open_len[e->open_n++] = (uint32_t)len;
    e->open_max = std::max<uint32_t>(e->open_max, (uint32_t)len);
    if (e->open_n == e->code.k) {
        ssize_t rc = enc_close(e);
        if (rc < 0) return rc;
    }
    return 0;
}

ssize_t fecgpu_encoder_close_window(fecgpu_encoder *e) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    if (e->open_n == 0) return FECGPU_ERR_DONE;
    const uint64_t id = e->next_win;
    ssize_t rc = enc_close(e);  // missing sources become empty (zero) packets
    return rc < 0 ? rc : (ssize_t)id;
}

ssize_t fecgpu_encoder_flush(fecgpu_encoder *e) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    ssize_t n = enc_launch(e);
    if (n < 0) return n;
    DevGuard g(e->dev);
    // the stream is shared with other connections: wait for this encoder's
    // last launch only (its earlier ones precede it on the same stream)
    if (e->last_done && hipEventSynchronize(e->last_done) != hipSuccess) return FECGPU_ERR_DEVICE;
    return n;
}

ssize_t fecgpu_encoder_flush_many(fecgpu_encoder *const *encs, size_t n) {
    if (!encs || n == 0) return FECGPU_ERR_INVALID_ARG;
    fecgpu_encoder *e0 = encs[0];
    for (size_t i = 0; i < n; i++) {
        const fecgpu_encoder *e = encs[i];
        if (!e || !e0 || e->ctx != e0->ctx || e->dev != e0->dev || e->stride != e0->stride ||
            std::memcmp(&e->code, &e0->code, sizeof(fecgpu_code)) != 0)
            return FECGPU_ERR_INVALID_ARG;
        for (size_t j = 0; j < i; j++)
            if (encs[j] == e) return FECGPU_ERR_INVALID_ARG;  // listed twice
    }
    // every encoder's queued windows, as ragged windows (fixed pitch) of one launch
    uint64_t total = 0, base = 0;
    for (size_t i = 0; i < n; i++)
        if (encs[i]->cur && encs[i]->cur->nwin) {
            total += encs[i]->cur->nwin;
            if (!base) base = reinterpret_cast<uint64_t>(encs[i]->cur->mem.dev);
        }
    DevGuard g(e0->dev);
    if (total) {
        const size_t o_len = (total * 8 + 255) & ~size_t(255);
        size_t bytes = (size_t)64 << 10;  // power-of-two sizes: the ctx cache finds it next time
        while (bytes < o_len + total * 4) bytes <<= 1;
        Pinned arg;
        ssize_t rc = pinned_alloc(e0->ctx, bytes, arg);
        if (rc) return rc;
        uint64_t *off = reinterpret_cast<uint64_t *>(arg.host);
        uint32_t *len = reinterpret_cast<uint32_t *>(arg.host + o_len);
        uint64_t i0 = 0;
        for (size_t i = 0; i < n; i++) {
            const EncBatch *b = encs[i]->cur;
            if (!b) continue;
            for (uint32_t w = 0; w < b->nwin; w++, i0++) {
                off[i0] = reinterpret_cast<uint64_t>(b->mem.dev) + (uint64_t)w * e0->wbytes - base;
                len[i0] = b->S[w];
            }
        }
        BatchArgs a{};
        a.win = reinterpret_cast<uint8_t *>(base);
        a.win_off = reinterpret_cast<const uint64_t *>(arg.dev);
        a.sym_len = reinterpret_cast<const uint32_t *>(arg.dev + o_len);
        a.stride = e0->stride;
        a.off_stride = e0->stride;
        a.nwin = total;
        rc = fecgpu::launch_batch(e0->ctx, &e0->code, false, a, e0->stream, true, e0->dev);  // one launch
        if (rc == 0) {
            // no per-batch events: this call waits for the stream before it
            // returns, so every batch is complete before anyone looks at it
            // (an event record per batch cost ~5 us each on the host)
            for (size_t i = 0; i < n; i++) {
                fecgpu_encoder *e = encs[i];
                EncBatch *b = e->cur;
                if (!b || !b->nwin) continue;
                b->launched = true;
                e->cur = nullptr;
                if (b->live == 0) {  // every window already released: recycle
                    e->active.pop_back();
                    e->spare.push_back(b);
                }
            }
        }
        if (hipStreamSynchronize(e0->stream) != hipSuccess && rc == 0) rc = FECGPU_ERR_DEVICE;
        pinned_free(e0->ctx, arg);
        if (rc) return rc;
    }
    for (size_t i = 0; i < n; i++)  // launches of earlier batches, possibly on other streams
        if (encs[i]->last_done && hipEventSynchronize(encs[i]->last_done) != hipSuccess)
            return FECGPU_ERR_DEVICE;
    return (ssize_t)total;
}

ssize_t fecgpu_encoder_set_policy(fecgpu_encoder *e, const fecgpu_policy *p) {
    if (!e || !p) return FECGPU_ERR_INVALID_ARG;
    e->policy = *p;
    return 0;
}

ssize_t fecgpu_encoder_tick(fecgpu_encoder *e, uint64_t now_us) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    e->now = std::max(e->now, now_us);
    ssize_t launched = 0;
    const uint64_t wt = e->policy.window_timeout_us, bt = e->policy.batch_timeout_us;
    if (wt && e->open_n && e->now - e->open_t >= wt) {
        ssize_t rc = enc_close(e);  // may launch a now-full batch
        if (rc < 0) return rc;
        launched += rc;
    }
    if (bt && e->cur && e->cur->nwin && e->now - e->cur_t >= bt) {
        ssize_t rc = enc_launch(e);
        if (rc < 0) return rc;
        launched += rc;
    }
    return launched;
}

ssize_t fecgpu_encoder_window_sources(fecgpu_encoder *e, uint64_t win) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    uint32_t slot = 0;
    EncBatch *b = enc_find(e, win, slot);
    if (!b || b->released[slot]) return FECGPU_ERR_DONE;
    return (ssize_t)b->nsrc[slot];
}

ssize_t fecgpu_encoder_repair(fecgpu_encoder *e, uint64_t win, uint16_t i, uint8_t *out,
                              size_t cap) {
    if (!e || i >= e->code.r) return FECGPU_ERR_INVALID_ARG;
    uint32_t slot = 0;
    EncBatch *b = enc_find(e, win, slot);
    if (!b || b->released[slot]) return win <= e->next_win ? FECGPU_ERR_DONE : FECGPU_ERR_INVALID_ARG;
    if (!b->launched) return FECGPU_ERR_DONE;  // not encoded yet
    if (hipEventQuery(b->done) != hipSuccess) {
        DevGuard g(e->dev);
        if (hipEventSynchronize(b->done) != hipSuccess) return FECGPU_ERR_DEVICE;
    }
    const uint32_t S = b->S[slot];
    if (!out || cap < S) return FECGPU_ERR_BUFFER_TOO_SHORT;
    std::memcpy(out, enc_row(e, b, slot, e->code.k + i), S);
    return (ssize_t)S;
}

ssize_t fecgpu_encoder_release(fecgpu_encoder *e, uint64_t win) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    uint32_t slot = 0;
    EncBatch *b = enc_find(e, win, slot);
    if (!b || !b->launched || b->released[slot]) return FECGPU_ERR_DONE;
    b->released[slot] = 1;
    if (--b->live == 0) {
        e->active.erase(std::find(e->active.begin(), e->active.end(), b));
        e->spare.push_back(b);
    }
    return 0;
}

}  // extern "C"

// ------------------------------------------------------------ decoder ---
namespace {

struct DecSlot {
    uint64_t win = 0;
    uint64_t present = 0;  // bit i: symbol i held (received or recovered)
    uint32_t S = 0;        // known once a repair (or FIXED source) arrives
    uint16_t nsrc = 0;     // real sources (REPAIR frame nsrc); 0 = not told (k)
    bool used = false;
    bool cand = false;     // touched since the last flush
    bool inflight = false; // in the launched, not yet completed decode
};

// window slots per pinned chunk of the decoder's pool: 4 batches, 16..256
// (a low-rate connection with small batches keeps a small footprint)
uint32_t dec_chunk_slots(uint32_t batch) { return std::min<uint32_t>(256, std::max<uint32_t>(16, 4 * batch)); }

}  // namespace

struct fecgpu_decoder {
    fecgpu_ctx *ctx = nullptr;
    fecgpu_code code{};
    uint32_t max_len = 0, batch = 0, stride = 0;
    size_t wbytes = 0;
    int dev = 0;
    hipStream_t stream = nullptr;
    uint32_t chunk_slots = 256;        // windows per pinned chunk (dec_chunk_slots)
    std::vector<Pinned> chunks;        // chunk_slots windows each
    std::vector<DecSlot> slots;
    std::vector<uint32_t> plen;        // [slot * k + j] payload length
    std::vector<uint32_t> free_slots;
    std::unordered_map<uint64_t, uint32_t> map;
    std::vector<uint32_t> cand;
    Pinned arg;                        // flush arrays: off, S, present, status
    size_t arg_cap = 0;
    uint64_t dirty = 0;
    fecgpu_policy policy{};
    uint64_t now = 0;                  // latest caller clock (tick)
    uint64_t dirty_t = 0;              // when the first symbol since the last flush was filed
    std::vector<uint32_t> sel;         // windows of the launched decode (in arg order)
    bool pending = false;              // a launched decode awaits completion
    hipEvent_t done = nullptr;         // recorded after the pending decode
    uint64_t max_windows = 4096;       // open-window limit (0 = none)
    ssize_t rec_acc = 0;               // recovered since flush / tick last returned
    std::deque<std::pair<uint64_t, uint16_t>> rec_q;  // recovered (win, idx), oldest first
};

namespace {

uint8_t *dec_row(fecgpu_decoder *d, uint32_t s, int row) {
    return d->chunks[s / d->chunk_slots].host + (size_t)(s % d->chunk_slots) * d->wbytes +
           (size_t)row * d->stride;
}
uint64_t dec_dev_addr(fecgpu_decoder *d, uint32_t s) {
    return reinterpret_cast<uint64_t>(d->chunks[s / d->chunk_slots].dev) +
           (uint64_t)(s % d->chunk_slots) * d->wbytes;
}

ssize_t dec_slot(fecgpu_decoder *d, uint64_t win, uint32_t &out) {
    auto it = d->map.find(win);
    if (it != d->map.end()) {
        out = it->second;
        return 0;
    }
    // a peer controls the window ids it sends: bound what it can make us pin
    if (d->max_windows && d->map.size() >= d->max_windows) return FECGPU_ERR_LIMIT;
    if (d->free_slots.empty()) {
        Pinned p;
        ssize_t rc = pinned_alloc(d->ctx, (size_t)d->chunk_slots * d->wbytes, p);
        if (rc) return rc;
        const uint32_t base = (uint32_t)d->slots.size();
        d->chunks.push_back(p);
        d->slots.resize(base + d->chunk_slots);
        d->plen.resize((size_t)(base + d->chunk_slots) * d->code.k, 0);
        for (uint32_t i = d->chunk_slots; i-- > 0;) d->free_slots.push_back(base + i);
    }
    const uint32_t s = d->free_slots.back();
    d->free_slots.pop_back();
    DecSlot &w = d->slots[s];
    w = DecSlot{};
    w.win = win;
    w.used = true;
    d->map.emplace(win, s);
    out = s;
    return 0;
}

void dec_touch(fecgpu_decoder *d, uint32_t s) {
    if (d->dirty == 0) d->dirty_t = d->now;
    if (!d->slots[s].cand) {
        d->slots[s].cand = true;
        d->cand.push_back(s);
    }
}

// decodable now: some missing source can be recovered by the next flush
bool decodable(const fecgpu_code &c, const DecSlot &w) {
    const int k = c.k, r = c.r;
    if (w.S == 0) return false;
    const uint64_t kmask = (k >= 64) ? ~0ull : (1ull << k) - 1;
    const uint64_t miss = ~w.present & kmask;
    if (!miss) return false;
    if (c.scheme == FECGPU_SCHEME_GF256)
        return __builtin_popcountll(miss) <= __builtin_popcountll((w.present >> k) & ((1ull << r) - 1));
    for (int g = 0; g < r; g++) {
        int nm = 0;
        for (int j = g; j < k; j += r) nm += !((w.present >> j) & 1);
        if (nm == 1 && ((w.present >> (k + g)) & 1)) return true;
    }
    return false;
}

}  // namespace

extern "C" {

ssize_t fecgpu_decoder_new(fecgpu_ctx *ctx, const fecgpu_code *code, uint32_t max_len,
                           uint32_t batch, fecgpu_decoder **out) {
    if (!ctx || !out || max_len == 0 || batch == 0) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = fecgpu::code_check_narrow(code);
    if (rc) return rc;
    if (is_lenprefix(*code) && max_len > 65535) return FECGPU_ERR_INVALID_ARG;
    auto *d = new fecgpu_decoder();
    d->ctx = ctx;
    d->code = *code;
    d->max_len = max_len;
    d->batch = batch;
    d->stride = rup16(max_len + (is_lenprefix(*code) ? 2 : 0));
    d->wbytes = (size_t)(code->k + code->r) * d->stride;
    d->chunk_slots = dec_chunk_slots(batch);
    d->dev = ctx_device();
    rc = fecgpu::ctx_conn_stream(ctx, d->dev, &d->stream);  // shared, owned by the ctx
    if (rc) {
        delete d;
        return rc;
    }
    if (hipEventCreateWithFlags(&d->done, hipEventDisableTiming) != hipSuccess) {
        delete d;
        return FECGPU_ERR_DEVICE;
    }
    *out = d;
    return 0;
}

void fecgpu_decoder_free(fecgpu_decoder *d) {
    if (!d) return;
    DevGuard g(d->dev);
    if (d->pending) (void)hipEventSynchronize(d->done);  // its launch (the stream is shared)
    for (Pinned &p : d->chunks) pinned_free(d->ctx, p);
    pinned_free(d->ctx, d->arg);
    (void)hipEventDestroy(d->done);
    delete d;
}

}  // extern "C"

namespace {

// Marks what a decode recovered in the windows of d->sel, whose status bytes
// are status[0 .. |sel|) (ok: the launch completed).  Returns the number of
// recovered sources.
ssize_t dec_apply(fecgpu_decoder *d, const uint8_t *status, bool ok) {
    const int k = d->code.k, r = d->code.r;
    const bool lp = is_lenprefix(d->code);
    ssize_t recovered = 0;
    for (size_t i = 0; i < d->sel.size(); i++) {
        const uint32_t s = d->sel[i];
        DecSlot &w = d->slots[s];
        w.inflight = false;
        if (!ok) continue;
        uint64_t got_mask = 0;
        for (int j = 0; j < k; j++) {
            if ((w.present >> j) & 1) continue;
            // XOR windows recover group by group; a source is valid iff its group was solvable
            bool got = status[i] == FECGPU_STATUS_OK;
            if (!got && d->code.scheme == FECGPU_SCHEME_XOR) {
                const int grp = j % r;
                int nm = 0;
                for (int x = grp; x < k; x += r) nm += !((w.present >> x) & 1);
                got = nm == 1 && ((w.present >> (k + grp)) & 1);
            }
            if (!got) continue;
            uint32_t pl = w.S;
            if (lp) {
                const uint8_t *row = dec_row(d, s, j);
                pl = ((uint32_t)row[0] << 8) | row[1];
                if (pl + 2 > w.S) pl = w.S - 2;  // corrupt prefix: clamp
            }
            d->plen[(size_t)s * k + j] = pl;
            got_mask |= 1ull << j;
            recovered++;
            d->rec_q.emplace_back(w.win, (uint16_t)j);
        }
        w.present |= got_mask;
    }
    d->sel.clear();
    // the queue is for callers that poll it; bounded for those that do not
    const size_t qcap = std::max<size_t>(4096, (size_t)k * (d->max_windows ? d->max_windows : d->slots.size()));
    while (d->rec_q.size() > qcap) d->rec_q.pop_front();
    d->rec_acc += recovered;
    return recovered;
}

// Recovered count since the last flush / tick returned (every completed
// decode adds to it, whichever call completed it), and reset it.
ssize_t dec_take(fecgpu_decoder *d) {
    const ssize_t n = d->rec_acc;
    d->rec_acc = 0;
    return n;
}

// Completes the pending decode: waits for it and marks what it recovered.
// Returns the number of recovered sources (0 if nothing was pending).
ssize_t dec_complete(fecgpu_decoder *d) {
    if (!d->pending) return 0;
    d->pending = false;
    DevGuard g(d->dev);
    const hipError_t e = hipEventSynchronize(d->done);
    const ssize_t rec = dec_apply(d, d->arg.host + d->arg_cap / 2, e == hipSuccess);  // see dec_args
    return e == hipSuccess ? rec : FECGPU_ERR_DEVICE;
}

// A call about to read or write slot s first completes a decode that owns it.
ssize_t dec_ready(fecgpu_decoder *d, uint32_t s) {
    return d->slots[s].inflight ? dec_complete(d) : 0;
}

// The candidate windows that can recover something now go to d->sel (all but
// `keep`, which stays a candidate).  Returns |sel|.
size_t dec_select(fecgpu_decoder *d, uint32_t keep) {
    std::vector<uint32_t> &sel = d->sel;
    sel.clear();
    bool kept = false;
    for (uint32_t s : d->cand) {
        DecSlot &w = d->slots[s];
        if (!w.cand) continue;  // released (or a duplicate entry) since
        if (s == keep) {
            kept = true;
            continue;
        }
        w.cand = false;
        if (w.used && decodable(d->code, w)) sel.push_back(s);
    }
    d->cand.clear();
    d->dirty = 0;
    if (kept) {
        d->cand.push_back(keep);
        d->dirty = 1;
        d->dirty_t = d->now;
    }
    return sel.size();
}

// Per-window launch arguments for n windows in d's pinned argument block, which
// the kernel reads directly: win_off, sym_len, present, and the status bytes
// in the upper half (dec_complete finds them at arg_cap / 2).
struct DecArgs {
    uint64_t *off;
    uint32_t *len;
    uint64_t *pres;
    uint8_t *status;
    size_t o_len, o_pres, o_stat;
};

ssize_t dec_args(fecgpu_decoder *d, size_t n, DecArgs &a) {
    a.o_len = (n * 8 + 255) & ~size_t(255);
    a.o_pres = a.o_len + ((n * 4 + 255) & ~size_t(255));
    const size_t need = a.o_pres + n * 8;
    if (d->arg_cap / 2 < std::max(need, n)) {
        pinned_free(d->ctx, d->arg);
        d->arg_cap = 0;
        ssize_t rc = pinned_alloc(d->ctx, std::max(need, (size_t)64 << 10) * 2, d->arg);
        if (rc) return rc;
        d->arg_cap = d->arg.bytes;
    }
    a.o_stat = d->arg_cap / 2;
    a.off = reinterpret_cast<uint64_t *>(d->arg.host);
    a.len = reinterpret_cast<uint32_t *>(d->arg.host + a.o_len);
    a.pres = reinterpret_cast<uint64_t *>(d->arg.host + a.o_pres);
    a.status = d->arg.host + a.o_stat;
    return 0;
}

// Fills argument rows [i0, i0 + |d->sel|) for d's selected windows, as
// offsets from `base` (64-bit wrap: any pinned chunk of any decoder), and
// zero-pads their received LENPREFIX sources (A.3).
void dec_fill(fecgpu_decoder *d, uint64_t base, size_t i0, const DecArgs &a) {
    const int k = d->code.k;
    const bool lp = is_lenprefix(d->code);
    for (size_t i = 0; i < d->sel.size(); i++) {
        const uint32_t s = d->sel[i];
        DecSlot &w = d->slots[s];
        const uint32_t S16 = rup16(w.S);
        const int nsrc = w.nsrc ? w.nsrc : k;
        if (lp) {
            for (int j = 0; j < nsrc; j++)
                if ((w.present >> j) & 1) {
                    const uint32_t used = 2 + d->plen[(size_t)s * k + j];
                    std::memset(dec_row(d, s, j) + used, 0, S16 - used);
                }
        }
        // padding sources of a window closed early: empty (LENPREFIX) / zero
        // (FIXED) packets, i.e. all-zero rows, as the sender encoded them
        for (int j = nsrc; j < k; j++) std::memset(dec_row(d, s, j), 0, S16);
        a.off[i0 + i] = dec_dev_addr(d, s) - base;
        a.len[i0 + i] = w.S;
        a.pres[i0 + i] = w.present;
        a.status[i0 + i] = 0xFF;
        w.inflight = true;
    }
}

// Launches the decode of n argument rows on d's stream and records d->done.
ssize_t dec_launch_args(fecgpu_decoder *d, uint64_t base, size_t n, const DecArgs &da) {
    BatchArgs a{};
    a.win = reinterpret_cast<uint8_t *>(base);
    a.win_off = reinterpret_cast<const uint64_t *>(d->arg.dev);
    a.sym_len = reinterpret_cast<const uint32_t *>(d->arg.dev + da.o_len);
    a.present = reinterpret_cast<const uint64_t *>(d->arg.dev + da.o_pres);
    a.status = d->arg.dev + da.o_stat;
    a.stride = d->stride;
    a.off_stride = d->stride;
    a.nwin = n;
    ssize_t rc = fecgpu::launch_batch(d->ctx, &d->code, true, a, d->stream, true, d->dev);
    if (rc == 0 && hipEventRecord(d->done, d->stream) != hipSuccess) rc = FECGPU_ERR_DEVICE;
    return rc;
}

void dec_unselect(fecgpu_decoder *d) {
    for (uint32_t s : d->sel) d->slots[s].inflight = false;
    d->sel.clear();
}

// Launches one decode over the candidate windows that can recover something
// (all but `keep`, which stays a candidate).  The caller completes any
// pending decode first.  Returns the number of windows launched.
ssize_t dec_launch(fecgpu_decoder *d, uint32_t keep) {
    const size_t n = dec_select(d, keep);
    if (n == 0) return 0;
    DevGuard g(d->dev);
    DecArgs a;
    ssize_t rc = dec_args(d, n, a);
    if (rc) {
        d->sel.clear();
        return rc;
    }
    const uint64_t base = reinterpret_cast<uint64_t>(d->chunks[0].dev);
    dec_fill(d, base, 0, a);
    rc = dec_launch_args(d, base, n, a);
    if (rc) {
        dec_unselect(d);
        return rc;
    }
    d->pending = true;
    return (ssize_t)n;
}

// The automatic flush after `batch`*k filed symbols: launch without waiting.
ssize_t dec_auto_flush(fecgpu_decoder *d, uint32_t s) {
    if (++d->dirty < (uint64_t)d->batch * d->code.k) return 0;
    ssize_t rc = dec_complete(d);  // its recovered count stays in rec_acc
    if (rc >= 0) rc = dec_launch(d, s);
    return rc < 0 ? FECGPU_ERR_DEVICE : 0;
}

}  // namespace

extern "C" {

ssize_t fecgpu_decoder_flush(fecgpu_decoder *d) {
    if (!d) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = dec_complete(d);
    if (rc < 0) return rc;
    rc = dec_launch(d, UINT32_MAX);
    if (rc < 0) return rc;
    if (rc > 0) {
        rc = dec_complete(d);
        if (rc < 0) return rc;
    }
    return dec_take(d);
}

ssize_t fecgpu_decoder_flush_many(fecgpu_decoder *const *decs, size_t n) {
    if (!decs || n == 0) return FECGPU_ERR_INVALID_ARG;
    fecgpu_decoder *d0 = decs[0];
    for (size_t i = 0; i < n; i++) {
        const fecgpu_decoder *d = decs[i];
        if (!d || !d0 || d->ctx != d0->ctx || d->dev != d0->dev || d->stride != d0->stride ||
            std::memcmp(&d->code, &d0->code, sizeof(fecgpu_code)) != 0)
            return FECGPU_ERR_INVALID_ARG;
        for (size_t j = 0; j < i; j++)
            if (decs[j] == d) return FECGPU_ERR_INVALID_ARG;  // listed twice
    }
    auto take_all = [&]() {
        ssize_t t = 0;
        for (size_t i = 0; i < n; i++) t += dec_take(decs[i]);
        return t;
    };
    for (size_t i = 0; i < n; i++) {  // automatic flushes still in flight
        const ssize_t rc = dec_complete(decs[i]);
        if (rc < 0) return rc;
    }
    size_t total = 0;
    uint64_t base = 0;
    for (size_t i = 0; i < n; i++) {
        total += dec_select(decs[i], UINT32_MAX);
        if (!base && !decs[i]->chunks.empty()) base = reinterpret_cast<uint64_t>(decs[i]->chunks[0].dev);
    }
    if (total == 0) return take_all();
    DevGuard g(d0->dev);
    DecArgs a;
    ssize_t rc = dec_args(d0, total, a);
    if (rc) {
        for (size_t i = 0; i < n; i++) decs[i]->sel.clear();
        return rc;
    }
    std::vector<size_t> at(n);
    for (size_t i = 0, i0 = 0; i < n; i0 += decs[i]->sel.size(), i++) {
        at[i] = i0;
        dec_fill(decs[i], base, i0, a);
    }
    rc = dec_launch_args(d0, base, total, a);  // one launch for every decoder
    const bool ok = rc == 0 && hipEventSynchronize(d0->done) == hipSuccess;
    for (size_t i = 0; i < n; i++) (void)dec_apply(decs[i], a.status + at[i], ok);
    if (rc) return rc;
    return ok ? take_all() : FECGPU_ERR_DEVICE;
}

ssize_t fecgpu_decoder_add_source(fecgpu_decoder *d, uint64_t win, uint16_t idx, const uint8_t *pkt,
                                  size_t len) {
    if (!d || idx >= d->code.k || (!pkt && len)) return FECGPU_ERR_INVALID_ARG;
    if (len > d->max_len) return FECGPU_ERR_BUFFER_TOO_SHORT;
    uint32_t s = 0;
    ssize_t rc = dec_slot(d, win, s);
    if (rc) return rc;
    if (dec_ready(d, s) < 0) return FECGPU_ERR_DEVICE;
    DecSlot &w = d->slots[s];
    if (w.nsrc && idx >= w.nsrc) return FECGPU_ERR_INVALID_ARG;  // a padding index
    if ((w.present >> idx) & 1) return FECGPU_ERR_DONE;  // duplicate
    uint8_t *row = dec_row(d, s, idx);
    if (is_lenprefix(d->code)) {
        if (w.S && 2 + len > w.S) return FECGPU_ERR_INVALID_ARG;
        row[0] = (uint8_t)(len >> 8);
        row[1] = (uint8_t)len;
        if (len) std::memcpy(row + 2, pkt, len);
    } else {
        if (w.S && len != w.S) return FECGPU_ERR_INVALID_ARG;
        std::memcpy(row, pkt, len);
        w.S = (uint32_t)len;
    }
    d->plen[(size_t)s * d->code.k + idx] = (uint32_t)len;
    w.present |= 1ull << idx;
    dec_touch(d, s);
    return dec_auto_flush(d, s);
}

ssize_t fecgpu_decoder_add_repair(fecgpu_decoder *d, uint64_t win, uint16_t idx, const uint8_t *sym,
                                  size_t len) {
    if (!d || idx >= d->code.r || !sym || len == 0) return FECGPU_ERR_INVALID_ARG;
    if (len > (size_t)d->max_len + (is_lenprefix(d->code) ? 2 : 0)) return FECGPU_ERR_BUFFER_TOO_SHORT;
    uint32_t s = 0;
    ssize_t rc = dec_slot(d, win, s);
    if (rc) return rc;
    if (dec_ready(d, s) < 0) return FECGPU_ERR_DEVICE;
    DecSlot &w = d->slots[s];
    const int k = d->code.k;
    if ((w.present >> (k + idx)) & 1) return FECGPU_ERR_DONE;
    if (w.S && w.S != len) return FECGPU_ERR_INVALID_ARG;
    if (!w.S) {
        // LENPREFIX: the repair length fixes S; sources received so far must fit
        for (int j = 0; j < (w.nsrc ? w.nsrc : k); j++)
            if (((w.present >> j) & 1) && 2 + d->plen[(size_t)s * k + j] > len) return FECGPU_ERR_INVALID_ARG;
        w.S = (uint32_t)len;
    }
    std::memcpy(dec_row(d, s, k + idx), sym, len);
    w.present |= 1ull << (k + idx);
    dec_touch(d, s);
    return dec_auto_flush(d, s);
}

ssize_t fecgpu_decoder_set_policy(fecgpu_decoder *d, const fecgpu_policy *p) {
    if (!d || !p) return FECGPU_ERR_INVALID_ARG;
    d->policy = *p;
    return 0;
}

ssize_t fecgpu_decoder_tick(fecgpu_decoder *d, uint64_t now_us) {
    if (!d) return FECGPU_ERR_INVALID_ARG;
    d->now = std::max(d->now, now_us);
    const uint64_t bt = d->policy.batch_timeout_us;
    if (bt && d->dirty && d->now - d->dirty_t >= bt) return fecgpu_decoder_flush(d);
    // an automatic flush that has finished by now is completed here
    if (d->pending && hipEventQuery(d->done) != hipErrorNotReady) {
        const ssize_t rc = dec_complete(d);
        if (rc < 0) return rc;
    }
    return dec_take(d);
}

ssize_t fecgpu_decoder_set_window_sources(fecgpu_decoder *d, uint64_t win, uint16_t nsrc) {
    if (!d || nsrc == 0 || nsrc > d->code.k) return FECGPU_ERR_INVALID_ARG;
    uint32_t s = 0;
    ssize_t rc = dec_slot(d, win, s);
    if (rc) return rc;
    if (dec_ready(d, s) < 0) return FECGPU_ERR_DEVICE;
    DecSlot &w = d->slots[s];
    const int k = d->code.k;
    if (w.nsrc) return w.nsrc == nsrc ? 0 : FECGPU_ERR_INVALID_ARG;
    if (nsrc == k) {
        w.nsrc = nsrc;
        return 0;
    }
    const uint64_t kmask = (k >= 64) ? ~0ull : (1ull << k) - 1;
    const uint64_t pad = kmask & ~((1ull << nsrc) - 1);
    if (w.present & pad) return FECGPU_ERR_INVALID_ARG;  // a source filed at a padding index
    w.nsrc = nsrc;
    w.present |= pad;
    for (int j = nsrc; j < k; j++) d->plen[(size_t)s * k + j] = 0;
    dec_touch(d, s);
    return 0;
}

ssize_t fecgpu_decoder_set_max_windows(fecgpu_decoder *d, uint64_t max_windows) {
    if (!d) return FECGPU_ERR_INVALID_ARG;
    d->max_windows = max_windows;
    return 0;
}

ssize_t fecgpu_decoder_next_recovered(fecgpu_decoder *d, uint64_t *win, uint16_t *idx) {
    if (!d || !win || !idx) return FECGPU_ERR_INVALID_ARG;
    // a finished automatic flush contributes without the caller flushing
    if (d->pending && hipEventQuery(d->done) != hipErrorNotReady && dec_complete(d) < 0)
        return FECGPU_ERR_DEVICE;
    while (!d->rec_q.empty()) {
        const auto [w, j] = d->rec_q.front();
        d->rec_q.pop_front();
        auto it = d->map.find(w);
        if (it == d->map.end() || !((d->slots[it->second].present >> j) & 1)) continue;  // released
        *win = w;
        *idx = j;
        return 0;
    }
    return FECGPU_ERR_DONE;
}

ssize_t fecgpu_decoder_recovered(fecgpu_decoder *d, uint64_t win, uint16_t idx, uint8_t *out,
                                 size_t cap) {
    if (!d || idx >= d->code.k) return FECGPU_ERR_INVALID_ARG;
    auto it = d->map.find(win);
    if (it == d->map.end()) return FECGPU_ERR_DONE;
    const uint32_t s = it->second;
    if (dec_ready(d, s) < 0) return FECGPU_ERR_DEVICE;
    if (!((d->slots[s].present >> idx) & 1)) return FECGPU_ERR_DONE;
    if (d->slots[s].nsrc && idx >= d->slots[s].nsrc) return FECGPU_ERR_DONE;  // padding, not a packet
    const uint32_t n = d->plen[(size_t)s * d->code.k + idx];
    if (cap < n || (!out && n)) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (n) std::memcpy(out, dec_row(d, s, idx) + (is_lenprefix(d->code) ? 2 : 0), n);
    return (ssize_t)n;
}

ssize_t fecgpu_decoder_release(fecgpu_decoder *d, uint64_t win) {
    if (!d) return FECGPU_ERR_INVALID_ARG;
    auto it = d->map.find(win);
    if (it == d->map.end()) return FECGPU_ERR_DONE;
    if (dec_ready(d, it->second) < 0) return FECGPU_ERR_DEVICE;
    DecSlot &w = d->slots[it->second];
    w.used = false;
    w.cand = false;
    d->free_slots.push_back(it->second);
    d->map.erase(it);
    return 0;
}

}  // extern "C"
