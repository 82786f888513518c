// fec_frame.cpp — FEC frame wire format.
//
// The fec branch's frame types and header fields are not mounted
// (/root/reference/README.md:7), so this is the build's
// own encoding, written in QUIC's idiom: every integer is a QUIC
// variable-length integer (RFC 9000 §16) and a frame is
//   SOURCE_ID: type | window | index
//   REPAIR   : type | window | k | r | nsrc | index | length | repair symbol bytes
// with frame types in the reserved-for-extensions space.  nsrc is the number
// of real sources of the window (1..k): a window closed early (close_window,
// window timeout) is padded with empty sources that never go on the wire, and
// the receiver marks indices >= nsrc as present and empty
// (fecgpu_decoder_set_window_sources) instead of counting them as lost.  A
// Connection puts a SOURCE_ID frame next to each protected payload and carries
// repair symbols in REPAIR frames; the receiver parses both and feeds
// fecgpu_decoder_*.
// Sliding-window frames carry RFC 8681's FEC payload IDs in the same idiom:
//   SW_SOURCE: type | esi
//   SW_REPAIR: type | fss | nss | repair_key | dt | length | repair symbol bytes
// Pure host code: no device calls.
#include <cstring>

#include "../../include/fecgpu.h"

namespace {

size_t varint_len(uint64_t v) {
    if (v < (1ull << 6)) return 1;
    if (v < (1ull << 14)) return 2;
    if (v < (1ull << 30)) return 4;
    return 8;
}

uint8_t *varint_put(uint8_t *p, uint64_t v) {
    const size_t n = varint_len(v);
    const uint64_t tag = n == 1 ? 0 : n == 2 ? 1 : n == 4 ? 2 : 3;
    for (size_t i = 0; i < n; i++) p[i] = (uint8_t)(v >> (8 * (n - 1 - i)));
    p[0] = (uint8_t)((p[0] & 0x3F) | (tag << 6));
    return p + n;
}

// returns bytes consumed, 0 if truncated
size_t varint_get(const uint8_t *p, size_t len, uint64_t *v) {
    if (len == 0) return 0;
    const size_t n = (size_t)1 << (p[0] >> 6);
    if (len < n) return 0;
    uint64_t x = p[0] & 0x3F;
    for (size_t i = 1; i < n; i++) x = (x << 8) | p[i];
    *v = x;
    return n;
}

}  // namespace

extern "C" {

ssize_t fecgpu_frame_source_id_len(uint64_t win, uint16_t idx) {
    return (ssize_t)(varint_len(FECGPU_FRAME_SOURCE_ID) + varint_len(win) + varint_len(idx));
}

ssize_t fecgpu_frame_write_source_id(uint8_t *buf, size_t cap, uint64_t win, uint16_t idx) {
    if (!buf || win >= (1ull << 62)) return FECGPU_ERR_INVALID_ARG;
    const size_t n = (size_t)fecgpu_frame_source_id_len(win, idx);
    if (cap < n) return FECGPU_ERR_BUFFER_TOO_SHORT;
    uint8_t *p = varint_put(buf, FECGPU_FRAME_SOURCE_ID);
    p = varint_put(p, win);
    p = varint_put(p, idx);
    return (ssize_t)(p - buf);
}

ssize_t fecgpu_frame_repair_len(uint64_t win, uint16_t k, uint16_t r, uint16_t nsrc, uint16_t idx,
                                size_t sym_len) {
    return (ssize_t)(varint_len(FECGPU_FRAME_REPAIR) + varint_len(win) + varint_len(k) + varint_len(r) +
                     varint_len(nsrc) + varint_len(idx) + varint_len(sym_len) + sym_len);
}

ssize_t fecgpu_frame_write_repair_header(uint8_t *buf, size_t cap, uint64_t win, uint16_t k,
                                         uint16_t r, uint16_t nsrc, uint16_t idx, size_t sym_len) {
    if (!buf || win >= (1ull << 62) || idx >= r || k == 0 || r == 0 || nsrc == 0 || nsrc > k ||
        sym_len >= (1ull << 62))
        return FECGPU_ERR_INVALID_ARG;
    const size_t n = (size_t)fecgpu_frame_repair_len(win, k, r, nsrc, idx, sym_len) - sym_len;
    if (cap < n) return FECGPU_ERR_BUFFER_TOO_SHORT;
    uint8_t *p = varint_put(buf, FECGPU_FRAME_REPAIR);
    p = varint_put(p, win);
    p = varint_put(p, k);
    p = varint_put(p, r);
    p = varint_put(p, nsrc);
    p = varint_put(p, idx);
    p = varint_put(p, sym_len);
    return (ssize_t)(p - buf);
}

ssize_t fecgpu_frame_write_repair(uint8_t *buf, size_t cap, uint64_t win, uint16_t k, uint16_t r,
                                  uint16_t nsrc, uint16_t idx, const uint8_t *sym, size_t sym_len) {
    if (!buf || (!sym && sym_len)) return FECGPU_ERR_INVALID_ARG;
    const ssize_t h = fecgpu_frame_write_repair_header(buf, cap, win, k, r, nsrc, idx, sym_len);
    if (h < 0) return h;
    if (cap - (size_t)h < sym_len) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (sym_len) std::memcpy(buf + h, sym, sym_len);
    return h + (ssize_t)sym_len;
}

ssize_t fecgpu_frame_write_sw_source(uint8_t *buf, size_t cap, uint64_t esi) {
    if (!buf || esi >= (1ull << 62)) return FECGPU_ERR_INVALID_ARG;
    const size_t n = varint_len(FECGPU_FRAME_SW_SOURCE) + varint_len(esi);
    if (cap < n) return FECGPU_ERR_BUFFER_TOO_SHORT;
    uint8_t *p = varint_put(buf, FECGPU_FRAME_SW_SOURCE);
    p = varint_put(p, esi);
    return (ssize_t)(p - buf);
}

ssize_t fecgpu_frame_write_sw_repair(uint8_t *buf, size_t cap, const struct fecgpu_sw_repair *hdr,
                                     const uint8_t *sym, size_t sym_len) {
    if (!buf || !hdr || (!sym && sym_len) || hdr->fss >= (1ull << 62) || hdr->nss == 0 ||
        hdr->nss > FECGPU_SW_MAX_WINDOW || hdr->dt > 15 || sym_len >= (1ull << 62))
        return FECGPU_ERR_INVALID_ARG;
    const size_t n = varint_len(FECGPU_FRAME_SW_REPAIR) + varint_len(hdr->fss) + varint_len(hdr->nss) +
                     varint_len(hdr->key) + varint_len(hdr->dt) + varint_len(sym_len) + sym_len;
    if (cap < n) return FECGPU_ERR_BUFFER_TOO_SHORT;
    uint8_t *p = varint_put(buf, FECGPU_FRAME_SW_REPAIR);
    p = varint_put(p, hdr->fss);
    p = varint_put(p, hdr->nss);
    p = varint_put(p, hdr->key);
    p = varint_put(p, hdr->dt);
    p = varint_put(p, sym_len);
    if (sym_len) std::memcpy(p, sym, sym_len);
    return (ssize_t)(p + sym_len - buf);
}

ssize_t fecgpu_frame_parse(const uint8_t *buf, size_t len, fecgpu_frame *out) {
    if (!buf || !out) return FECGPU_ERR_INVALID_ARG;
    std::memset(out, 0, sizeof(*out));
    size_t pos = 0, n;
    uint64_t v;
#define GET(dst)                                              \
    do {                                                      \
        n = varint_get(buf + pos, len - pos, &v);             \
        if (!n) return FECGPU_ERR_BUFFER_TOO_SHORT;           \
        pos += n;                                             \
        dst = v;                                              \
    } while (0)
    uint64_t type;
    GET(type);
    if (type != FECGPU_FRAME_SOURCE_ID && type != FECGPU_FRAME_REPAIR && type != FECGPU_FRAME_SW_SOURCE &&
        type != FECGPU_FRAME_SW_REPAIR)
        return FECGPU_ERR_INVALID_ARG;
    out->type = type;
    GET(out->win);
    if (type == FECGPU_FRAME_SW_SOURCE) return (ssize_t)pos;
    if (type == FECGPU_FRAME_SW_REPAIR) {
        uint64_t nss, key, dt, sl;
        GET(nss);
        GET(key);
        GET(dt);
        GET(sl);
        if (nss == 0 || nss > FECGPU_SW_MAX_WINDOW || key > 0xFFFF || dt > 15) return FECGPU_ERR_INVALID_ARG;
        if (sl > len - pos) return FECGPU_ERR_BUFFER_TOO_SHORT;
        out->nsrc = (uint16_t)nss;
        out->key = (uint16_t)key;
        out->dt = (uint8_t)dt;
        out->payload = buf + pos;
        out->payload_len = sl;
        return (ssize_t)(pos + sl);
    }
    if (type == FECGPU_FRAME_SOURCE_ID) {
        uint64_t idx;
        GET(idx);
        if (idx > 0xFFFF) return FECGPU_ERR_INVALID_ARG;
        out->idx = (uint16_t)idx;
        return (ssize_t)pos;
    }
    uint64_t k, r, nsrc, idx, sl;
    GET(k);
    GET(r);
    GET(nsrc);
    GET(idx);
    GET(sl);
#undef GET
    if (k == 0 || r == 0 || k > 0xFFFF || r > 0xFFFF || idx >= r || nsrc == 0 || nsrc > k)
        return FECGPU_ERR_INVALID_ARG;
    if (sl > len - pos) return FECGPU_ERR_BUFFER_TOO_SHORT;
    out->k = (uint16_t)k;
    out->r = (uint16_t)r;
    out->nsrc = (uint16_t)nsrc;
    out->idx = (uint16_t)idx;
    out->payload = buf + pos;
    out->payload_len = sl;
    return (ssize_t)(pos + sl);
}

}  // extern "C"
