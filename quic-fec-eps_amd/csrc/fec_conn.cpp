// fec_conn.cpp — per-connection encoder / decoder objects of the C ABI
// (include/fecgpu.h, "per-packet API"; SURVEY.md §8b item 2, §3 call stacks
// A and B).
//
// These are the calls a QUIC Connection makes one packet at a time: the
// sender appends each protected payload as a source symbol and reads repair
// symbols back; the receiver files sources and repairs by (window, index) and
// reads recovered packets back.  Both sides queue complete windows and hand
// them to the GPU hot path in batches (fecgpu_encode_batch /
// fecgpu_decode_batch with FECGPU_F_HOST_PTRS, ragged window layout), so a
// connection pays one H2D/kernel/D2H round trip per `batch` windows, not per
// packet.  Framing: FIXED — every packet of a window
// has the same length, symbol = packet; LENPREFIX — symbol = u16be(len) ||
// payload || zero pad to S = 2 + max len of the window.
#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <vector>

#include "../../include/fecgpu.h"

namespace {

inline uint32_t rup16(uint32_t x) { return (x + 15u) & ~15u; }

struct EncWin {
    uint64_t id = 0;
    uint32_t S = 0;
    std::vector<uint8_t> sym;  // (k + r) * rup16(S): sources then repairs
};

struct DecWin {
    uint32_t S = 0;                       // known once a repair (or FIXED source) arrives
    uint64_t present = 0;                 // bit i: symbol i held (received or recovered)
    std::vector<std::vector<uint8_t>> src;  // framed source symbols (length S once known)
    std::vector<std::vector<uint8_t>> rep;
    std::vector<uint32_t> plen;           // payload length per source (LENPREFIX: from prefix)
};

bool is_lenprefix(const fecgpu_code &c) { return c.framing == FECGPU_FRAMING_LENPREFIX; }

}  // namespace

struct fecgpu_encoder {
    fecgpu_ctx *ctx;
    fecgpu_code code;
    uint32_t max_len, batch;
    uint64_t next_win = 0;
    std::vector<std::vector<uint8_t>> open;  // payloads of the open window
    std::deque<EncWin> pending;              // closed, not yet encoded
    std::map<uint64_t, EncWin> done;         // encoded, repairs readable
};

struct fecgpu_decoder {
    fecgpu_ctx *ctx;
    fecgpu_code code;
    uint32_t max_len, batch;
    std::map<uint64_t, DecWin> wins;
    uint64_t dirty = 0;  // windows changed since the last flush
};

namespace {

// Pack windows into one ragged host batch (win_off layout) and run the hot path.
ssize_t run_host_batch(fecgpu_ctx *ctx, const fecgpu_code &code, bool decode,
                       std::vector<uint8_t> &buf, std::vector<uint64_t> &off,
                       std::vector<uint32_t> &len, std::vector<uint64_t> &pres,
                       std::vector<uint8_t> &status) {
    const uint64_t n = off.size();
    if (n == 0) return 0;
    if (decode)
        return fecgpu_decode_batch(ctx, &code, buf.data(), off.data(), len.data(), 0, 0, n,
                                   pres.data(), status.data(), FECGPU_F_HOST_PTRS, nullptr);
    return fecgpu_encode_batch(ctx, &code, buf.data(), off.data(), len.data(), 0, 0, n,
                               FECGPU_F_HOST_PTRS, nullptr);
}

void close_window(fecgpu_encoder *e) {
    const int k = e->code.k, r = e->code.r;
    const bool lp = is_lenprefix(e->code);
    uint32_t mx = 0;
    for (auto &p : e->open) mx = std::max<uint32_t>(mx, (uint32_t)p.size());
    EncWin w;
    w.id = e->next_win++;
    w.S = lp ? 2 + mx : std::max<uint32_t>(mx, 1);
    const uint32_t st = rup16(w.S);
    w.sym.assign((size_t)(k + r) * st, 0);
    for (int j = 0; j < (int)e->open.size(); j++) {
        uint8_t *s = w.sym.data() + (size_t)j * st;
        const auto &p = e->open[j];
        if (lp) {
            s[0] = (uint8_t)(p.size() >> 8);
            s[1] = (uint8_t)p.size();
            std::memcpy(s + 2, p.data(), p.size());
        } else {
            std::memcpy(s, p.data(), p.size());
        }
    }
    e->open.clear();
    e->pending.push_back(std::move(w));
}

}  // namespace

extern "C" {

ssize_t fecgpu_encoder_new(fecgpu_ctx *ctx, const fecgpu_code *code, uint32_t max_len,
                           uint32_t batch, fecgpu_encoder **out) {
    if (!ctx || !out || max_len == 0 || batch == 0) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = fecgpu_code_check(code);
    if (rc) return rc;
    if (is_lenprefix(*code) && max_len > 65535) return FECGPU_ERR_INVALID_ARG;
    auto *e = new fecgpu_encoder();
    e->ctx = ctx;
    e->code = *code;
    e->max_len = max_len;
    e->batch = batch;
    *out = e;
    return 0;
}

void fecgpu_encoder_free(fecgpu_encoder *enc) { delete enc; }

ssize_t fecgpu_encoder_flush(fecgpu_encoder *e) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    const int n = e->code.k + e->code.r;
    std::vector<uint64_t> off, pres;
    std::vector<uint32_t> len;
    std::vector<uint8_t> buf, status;
    uint64_t pos = 0;
    for (auto &w : e->pending) {
        off.push_back(pos);
        len.push_back(w.S);
        pos += (uint64_t)n * rup16(w.S);
    }
    buf.resize(pos);
    for (size_t i = 0; i < e->pending.size(); i++)
        std::memcpy(buf.data() + off[i], e->pending[i].sym.data(), e->pending[i].sym.size());
    ssize_t rc = run_host_batch(e->ctx, e->code, false, buf, off, len, pres, status);
    if (rc < 0) return rc;
    const ssize_t nw = (ssize_t)e->pending.size();
    for (size_t i = 0; i < e->pending.size(); i++) {
        EncWin &w = e->pending[i];
        std::memcpy(w.sym.data(), buf.data() + off[i], w.sym.size());
        const uint64_t id = w.id;
        e->done[id] = std::move(w);
    }
    e->pending.clear();
    return nw;
}

ssize_t fecgpu_encoder_add_source(fecgpu_encoder *e, const uint8_t *pkt, size_t len,
                                  uint64_t *win, uint16_t *idx) {
    if (!e || (!pkt && len)) return FECGPU_ERR_INVALID_ARG;
    if (len > e->max_len) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (!is_lenprefix(e->code)) {
        if (len == 0) return FECGPU_ERR_INVALID_ARG;
        if (!e->open.empty() && e->open[0].size() != len) return FECGPU_ERR_INVALID_ARG;
    }
    if (win) *win = e->next_win;
    if (idx) *idx = (uint16_t)e->open.size();
    e->open.emplace_back(pkt, pkt + len);
    if ((int)e->open.size() == e->code.k) {
        close_window(e);
        if (e->pending.size() >= e->batch) {
            ssize_t rc = fecgpu_encoder_flush(e);
            if (rc < 0) return rc;
        }
    }
    return 0;
}

ssize_t fecgpu_encoder_close_window(fecgpu_encoder *e) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    if (e->open.empty()) return FECGPU_ERR_DONE;
    const size_t L = e->open[0].size();
    while ((int)e->open.size() < e->code.k)
        e->open.emplace_back(is_lenprefix(e->code) ? 0 : L, 0);  // zero padding symbols
    close_window(e);
    return (ssize_t)(e->next_win - 1);
}

ssize_t fecgpu_encoder_repair(fecgpu_encoder *e, uint64_t win, uint16_t i, uint8_t *out,
                              size_t cap) {
    if (!e || i >= e->code.r) return FECGPU_ERR_INVALID_ARG;
    auto it = e->done.find(win);
    if (it == e->done.end()) return win <= e->next_win ? FECGPU_ERR_DONE : FECGPU_ERR_INVALID_ARG;
    const EncWin &w = it->second;
    if (!out || cap < w.S) return FECGPU_ERR_BUFFER_TOO_SHORT;
    std::memcpy(out, w.sym.data() + (size_t)(e->code.k + i) * rup16(w.S), w.S);
    return (ssize_t)w.S;
}

ssize_t fecgpu_encoder_release(fecgpu_encoder *e, uint64_t win) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    return e->done.erase(win) ? 0 : FECGPU_ERR_DONE;
}

// ------------------------------------------------------------- decoder ---

ssize_t fecgpu_decoder_new(fecgpu_ctx *ctx, const fecgpu_code *code, uint32_t max_len,
                           uint32_t batch, fecgpu_decoder **out) {
    if (!ctx || !out || max_len == 0 || batch == 0) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = fecgpu_code_check(code);
    if (rc) return rc;
    if (is_lenprefix(*code) && max_len > 65535) return FECGPU_ERR_INVALID_ARG;
    auto *d = new fecgpu_decoder();
    d->ctx = ctx;
    d->code = *code;
    d->max_len = max_len;
    d->batch = batch;
    *out = d;
    return 0;
}

void fecgpu_decoder_free(fecgpu_decoder *d) { delete d; }

static DecWin &dwin(fecgpu_decoder *d, uint64_t win) {
    DecWin &w = d->wins[win];
    if (w.src.empty()) {
        w.src.resize(d->code.k);
        w.rep.resize(d->code.r);
        w.plen.assign(d->code.k, 0);
    }
    return w;
}

// decodable now: some missing source can be recovered by the next flush
static bool decodable(const fecgpu_code &c, const DecWin &w) {
    const int k = c.k, r = c.r;
    if (w.S == 0) return false;
    const uint64_t kmask = (1ull << k) - 1;
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

ssize_t fecgpu_decoder_flush(fecgpu_decoder *d) {
    if (!d) return FECGPU_ERR_INVALID_ARG;
    const int k = d->code.k, r = d->code.r, n = k + r;
    const bool lp = is_lenprefix(d->code);
    std::vector<uint64_t> ids, off, pres;
    std::vector<uint32_t> len;
    uint64_t pos = 0;
    for (auto &kv : d->wins) {
        if (!decodable(d->code, kv.second)) continue;
        ids.push_back(kv.first);
        off.push_back(pos);
        len.push_back(kv.second.S);
        pres.push_back(kv.second.present);
        pos += (uint64_t)n * rup16(kv.second.S);
    }
    std::vector<uint8_t> buf(pos, 0), status(ids.size(), 0);
    for (size_t i = 0; i < ids.size(); i++) {
        DecWin &w = d->wins[ids[i]];
        const uint32_t st = rup16(w.S);
        for (int j = 0; j < k; j++)
            if ((w.present >> j) & 1) std::memcpy(buf.data() + off[i] + (size_t)j * st, w.src[j].data(), w.S);
        for (int t = 0; t < r; t++)
            if ((w.present >> (k + t)) & 1)
                std::memcpy(buf.data() + off[i] + (size_t)(k + t) * st, w.rep[t].data(), w.S);
    }
    ssize_t rc = run_host_batch(d->ctx, d->code, true, buf, off, len, pres, status);
    if (rc < 0) return rc;
    ssize_t recovered = 0;
    for (size_t i = 0; i < ids.size(); i++) {
        DecWin &w = d->wins[ids[i]];
        const uint32_t st = rup16(w.S);
        const uint64_t kmask = (1ull << k) - 1;
        for (int j = 0; j < k; j++) {
            if ((w.present >> j) & 1) continue;
            // XOR windows recover group by group; a source is valid iff its group was solvable
            bool got = status[i] == FECGPU_STATUS_OK;
            if (!got && d->code.scheme == FECGPU_SCHEME_XOR) {
                const int g = j % r;
                int nm = 0;
                for (int x = g; x < k; x += r) nm += !((w.present >> x) & 1);
                got = nm == 1 && ((w.present >> (k + g)) & 1);
            }
            if (!got) continue;
            const uint8_t *s = buf.data() + off[i] + (size_t)j * st;
            w.src[j].assign(s, s + w.S);
            w.plen[j] = lp ? (((uint32_t)s[0] << 8) | s[1]) : w.S;
            if (lp && w.plen[j] + 2 > w.S) w.plen[j] = w.S - 2;  // corrupt prefix: clamp
            recovered++;
        }
        for (int j = 0; j < k; j++)
            if (!w.src[j].empty()) w.present |= 1ull << j;
        (void)kmask;
    }
    d->dirty = 0;
    return recovered;
}

ssize_t fecgpu_decoder_add_source(fecgpu_decoder *d, uint64_t win, uint16_t idx, const uint8_t *pkt,
                                  size_t len) {
    if (!d || idx >= d->code.k || (!pkt && len)) return FECGPU_ERR_INVALID_ARG;
    if (len > d->max_len) return FECGPU_ERR_BUFFER_TOO_SHORT;
    DecWin &w = dwin(d, win);
    if ((w.present >> idx) & 1) return FECGPU_ERR_DONE;  // duplicate
    const bool lp = is_lenprefix(d->code);
    std::vector<uint8_t> sym;
    if (lp) {
        sym.assign(2 + len, 0);
        sym[0] = (uint8_t)(len >> 8);
        sym[1] = (uint8_t)len;
        if (len) std::memcpy(sym.data() + 2, pkt, len);
    } else {
        if (w.S && len != w.S) return FECGPU_ERR_INVALID_ARG;
        sym.assign(pkt, pkt + len);
        w.S = (uint32_t)len;
    }
    if (w.S) {
        if (sym.size() > w.S) return FECGPU_ERR_INVALID_ARG;
        sym.resize(w.S, 0);
    }
    w.src[idx] = std::move(sym);
    w.plen[idx] = (uint32_t)len;
    w.present |= 1ull << idx;
    if (++d->dirty >= (uint64_t)d->batch * d->code.k) return fecgpu_decoder_flush(d) < 0 ? FECGPU_ERR_DEVICE : 0;
    return 0;
}

ssize_t fecgpu_decoder_add_repair(fecgpu_decoder *d, uint64_t win, uint16_t idx, const uint8_t *sym,
                                  size_t len) {
    if (!d || idx >= d->code.r || !sym || len == 0) return FECGPU_ERR_INVALID_ARG;
    if (len > (size_t)d->max_len + (is_lenprefix(d->code) ? 2 : 0)) return FECGPU_ERR_BUFFER_TOO_SHORT;
    DecWin &w = dwin(d, win);
    const int k = d->code.k;
    if ((w.present >> (k + idx)) & 1) return FECGPU_ERR_DONE;
    if (w.S && w.S != len) return FECGPU_ERR_INVALID_ARG;
    if (!w.S) {
        // LENPREFIX: the repair length fixes S; pad sources received so far
        for (int j = 0; j < k; j++) {
            if (!((w.present >> j) & 1)) continue;
            if (w.src[j].size() > len) return FECGPU_ERR_INVALID_ARG;
            w.src[j].resize(len, 0);
        }
        w.S = (uint32_t)len;
    }
    w.rep[idx].assign(sym, sym + len);
    w.present |= 1ull << (k + idx);
    if (++d->dirty >= (uint64_t)d->batch * d->code.k) return fecgpu_decoder_flush(d) < 0 ? FECGPU_ERR_DEVICE : 0;
    return 0;
}

ssize_t fecgpu_decoder_recovered(fecgpu_decoder *d, uint64_t win, uint16_t idx, uint8_t *out,
                                 size_t cap) {
    if (!d || idx >= d->code.k) return FECGPU_ERR_INVALID_ARG;
    auto it = d->wins.find(win);
    if (it == d->wins.end() || !((it->second.present >> idx) & 1)) return FECGPU_ERR_DONE;
    const DecWin &w = it->second;
    const uint32_t n = w.plen[idx];
    if (cap < n || (!out && n)) return FECGPU_ERR_BUFFER_TOO_SHORT;
    const uint8_t *s = w.src[idx].data() + (is_lenprefix(d->code) ? 2 : 0);
    if (n) std::memcpy(out, s, n);
    return (ssize_t)n;
}

ssize_t fecgpu_decoder_release(fecgpu_decoder *d, uint64_t win) {
    if (!d) return FECGPU_ERR_INVALID_ARG;
    return d->wins.erase(win) ? 0 : FECGPU_ERR_DONE;
}

}  // extern "C"
