// fec_swconn.cpp — per-connection objects of the sliding-window code
// (include/fecgpu.h fecgpu_sw_encoder_* / fecgpu_sw_decoder_*; RFC 8681 with
// m = 8): the per-packet API a Connection calls, over
// the batch entry points of fec_sw.cpp.
//
// Sender: source symbols (A.3 framing, E bytes each) are written once into a
// pinned host buffer the GPU maps, at their ESI's row.  Repairs are scheduled
// every `step` sources over the last `window`; `batch` of them go to the GPU in
// one asynchronous launch (the kernel reads the sources over PCIe, writes the
// repairs into pinned rows); four launch slots hold repairs until they are
// read back, in order.  Launched repairs only read rows below the newest
// source, which are never rewritten except by a compaction: when the buffer
// fills, the rows still needed move to its front, after the launches in
// flight finish.
// Receiver: sources and repairs are filed into pinned rows (sources by ESI in a
// buffer over [base, base + cap)); a flush runs fecgpu_sw_decode over the
// buffer's live span with the GPU reading the rows in place.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <vector>

#include "../../include/fecgpu.h"
#include "fec_internal.h"

using namespace fecgpu;

namespace {

#define SWC_TRY(expr, what)                                     \
    do {                                                        \
        hipError_t e_ = (expr);                                 \
        if (e_ != hipSuccess) return set_dev_error(e_, what);   \
    } while (0)

constexpr int kSlots = 4;  // encoder launch slots (launched batches whose repairs are not all read)

ssize_t check_params(const fecgpu_sw_params *p) {
    if (!p) return FECGPU_ERR_INVALID_ARG;
    if (p->framing != FECGPU_FRAMING_FIXED && p->framing != FECGPU_FRAMING_LENPREFIX) return FECGPU_ERR_INVALID_ARG;
    if (p->symbol_size == 0 || p->symbol_size > 65537 || (p->framing == FECGPU_FRAMING_LENPREFIX && p->symbol_size < 2))
        return FECGPU_ERR_INVALID_ARG;
    if (p->window == 0 || p->window > FECGPU_SW_MAX_WINDOW || p->step == 0 || p->dt > 15 || p->batch == 0 ||
        p->batch > (1u << 16))
        return FECGPU_ERR_INVALID_ARG;
    return 0;
}

// A.3 symbol of a payload into row (E bytes, zero padded); false if it does not fit
bool frame_into(const fecgpu_sw_params &p, uint8_t *row, const uint8_t *pkt, size_t len) {
    const uint32_t E = p.symbol_size;
    if (p.framing == FECGPU_FRAMING_LENPREFIX) {
        if (len + 2 > E) return false;
        row[0] = (uint8_t)(len >> 8);
        row[1] = (uint8_t)len;
        if (len) std::memcpy(row + 2, pkt, len);
        std::memset(row + 2 + len, 0, E - 2 - len);
        return true;
    }
    if (len != E) return false;  // FIXED: the payload is the symbol
    std::memcpy(row, pkt, len);
    return true;
}

}  // namespace

struct fecgpu_sw_encoder {
    fecgpu_ctx *ctx = nullptr;
    int dev = 0;
    hipStream_t s = nullptr;
    fecgpu_sw_params p{};
    uint32_t stride = 0;
    // sources of ESI [base, base + cap) at rows esi - base
    uint8_t *src = nullptr;
    uint64_t cap = 0, base = 0, next = 0;
    std::vector<fecgpu_sw_repair> sched;  // scheduled, not launched (absolute fss)
    uint32_t key = 0;
    int group = 1;   // repairs per combine job (ctx "sw_group")
    int stream = 0;  // streaming encode (ctx "sw_stream")
    struct Slot {
        fecgpu_sw_repair *hdr = nullptr;  // pinned, fss relative to the base at launch
        uint8_t *rep = nullptr;           // pinned rows
        void *jobs = nullptr, *coef = nullptr, *outs = nullptr;  // device scratch
        hipEvent_t ev = nullptr;
        std::vector<fecgpu_sw_repair> abs;
        size_t n = 0, popped = 0;
        bool used = false;
    } slot[kSlots];
    std::deque<int> order;  // launched slots, oldest first
};

struct fecgpu_sw_decoder {
    fecgpu_ctx *ctx = nullptr;
    int dev = 0;
    hipStream_t s = nullptr;
    fecgpu_sw_params p{};
    uint32_t stride = 0;
    uint64_t cap = 0, base = 0, hi = 0;  // sources [base, base + cap); hi = 1 + newest ESI
    uint8_t *src = nullptr;              // pinned rows
    std::vector<uint8_t> have;           // per row: received or recovered
    uint8_t *rep = nullptr;              // pinned repair rows
    uint32_t rcap = 0;
    std::vector<fecgpu_sw_repair> rh;    // headers of the filed repairs (absolute fss), row i
    uint32_t nrep = 0;
    uint32_t since = 0;                  // repairs filed since the last flush
    std::deque<uint64_t> rec_q;
    std::vector<uint8_t> st;             // decode scratch
};

namespace {

// Launches up to `batch` scheduled repairs (the oldest) in a free slot
// (ERR_LIMIT: none free).  On a failed launch nothing is consumed: the repairs
// stay scheduled, the slot stays free (its kernels, if any ran, are waited for
// first, so a retry never overlaps them).
ssize_t enc_launch(fecgpu_sw_encoder *e) {
    if (e->sched.empty()) return 0;
    int k = -1;
    for (int i = 0; i < kSlots; i++)
        if (!e->slot[i].used) { k = i; break; }
    if (k < 0) return FECGPU_ERR_LIMIT;
    auto &S = e->slot[k];
    const size_t n = std::min<size_t>(e->sched.size(), e->p.batch);  // the slot's rows
    for (size_t t = 0; t < n; t++) {
        S.hdr[t] = e->sched[t];
        S.hdr[t].fss -= e->base;
    }
    const uint8_t *rlc = nullptr;
    ChkRec *chk = nullptr;  // FECGPU_CHECK builds: faults surface at the ctx's next checked call
    ssize_t rc = ctx_fault_take(e->ctx) ? (ssize_t)FECGPU_ERR_DEVICE : ctx_rlc_table(e->ctx, e->s, &rlc);
    if (rc >= 0) rc = ctx_chk_record(e->ctx, &chk);
    if (rc >= 0)
        rc = sw_encode_core(e->src, e->cap, S.rep, S.hdr, n, e->p.window, e->p.symbol_size, e->stride, S.jobs, S.coef,
                            S.outs, e->s, e->group, S.hdr, e->stream, rlc, chk);
    if (rc >= 0) {
        const hipError_t er = hipEventRecord(S.ev, e->s);
        if (er != hipSuccess) rc = set_dev_error(er, "hipEventRecord");
    }
    if (rc < 0) {
        (void)hipStreamSynchronize(e->s);
        return rc;
    }
    S.n = n;
    S.popped = 0;
    S.abs.assign(e->sched.begin(), e->sched.begin() + n);
    S.used = true;
    e->order.push_back(k);
    e->sched.erase(e->sched.begin(), e->sched.begin() + n);
    return (ssize_t)n;
}

// Room for the next source: move the rows still needed to the front.
ssize_t enc_compact(fecgpu_sw_encoder *e) {
    for (int i : e->order) SWC_TRY(hipEventSynchronize(e->slot[i].ev), "hipEventSynchronize");
    uint64_t keep = e->next > e->p.window ? e->next - e->p.window : 0;
    for (const auto &h : e->sched) keep = std::min(keep, h.fss);
    keep = std::max(keep, e->base);
    const uint64_t shift = keep - e->base;
    if (shift == 0) return FECGPU_ERR_LIMIT;  // cannot happen: cap > window + batch * step
    std::memmove(e->src, e->src + shift * e->stride, (e->next - keep) * e->stride);
    e->base = keep;
    return 0;
}

bool enc_slot_free(const fecgpu_sw_encoder *e) {
    for (int i = 0; i < kSlots; i++)
        if (!e->slot[i].used) return true;
    return false;
}

// Repairs of the decoder's rows that can still matter (window end above base).
void dec_drop_old(fecgpu_sw_decoder *d) {
    uint32_t w = 0;
    for (uint32_t i = 0; i < d->nrep; i++) {
        const fecgpu_sw_repair &h = d->rh[i];
        if (h.fss < d->base) continue;
        bool useful = false;  // a source of the window still missing
        for (uint64_t x = h.fss; x < h.fss + h.nss && !useful; x++)
            useful = x >= d->hi || !d->have[x - d->base];
        if (!useful) continue;
        if (w != i) {
            d->rh[w] = h;
            std::memcpy(d->rep + (size_t)w * d->stride, d->rep + (size_t)i * d->stride, d->stride);
        }
        w++;
    }
    d->nrep = w;
}

// Advance base so that ESI `esi` fits: sources more than `span` behind are given up.
void dec_advance(fecgpu_sw_decoder *d, uint64_t esi) {
    const uint64_t keep = d->cap / 2;
    const uint64_t nb = esi + 1 > keep ? esi + 1 - keep : 0;
    if (nb <= d->base) return;
    const uint64_t shift = nb - d->base;
    if (shift < d->cap) {
        std::memmove(d->src, d->src + shift * d->stride, (d->cap - shift) * d->stride);
        std::memmove(d->have.data(), d->have.data() + shift, d->cap - shift);
        std::memset(d->have.data() + d->cap - shift, 0, shift);
    } else {
        std::memset(d->have.data(), 0, d->cap);
    }
    d->base = nb;
    d->hi = std::max(d->hi, nb);
    dec_drop_old(d);
}

}  // namespace

extern "C" {

ssize_t fecgpu_sw_encoder_new(fecgpu_ctx *ctx, const fecgpu_sw_params *p, fecgpu_sw_encoder **out) {
    if (!ctx || !out) return FECGPU_ERR_INVALID_ARG;
    *out = nullptr;
    ssize_t rc = check_params(p);
    if (rc) return rc;
    auto *e = new fecgpu_sw_encoder();
    e->ctx = ctx;
    e->p = *p;
    e->group = ctx_sw_group(ctx);
    e->stream = ctx_sw_stream(ctx);
    e->stride = (p->symbol_size + 15u) & ~15u;
    e->cap = 4ull * (p->window + (uint64_t)p->batch * p->step);
    rc = [&]() -> ssize_t {
        SWC_TRY(hipGetDevice(&e->dev), "hipGetDevice");
        rc = ctx_conn_stream(ctx, e->dev, &e->s);
        if (rc) return rc;
        rc = ctx_pinned_get(ctx, e->cap * e->stride, reinterpret_cast<void **>(&e->src));
        if (rc) return rc;
        std::memset(e->src, 0, e->cap * e->stride);
        for (auto &S : e->slot) {
            rc = ctx_pinned_get(ctx, p->batch * (sizeof(fecgpu_sw_repair) + e->stride), reinterpret_cast<void **>(&S.hdr));
            if (rc) return rc;
            S.rep = reinterpret_cast<uint8_t *>(S.hdr + p->batch);
            SWC_TRY(hipMalloc(&S.jobs, sw_enc_jobs(p->batch, e->group) * sizeof(CombJob)), "hipMalloc");
            SWC_TRY(hipMalloc(&S.coef, p->batch * (size_t)kSwCoefPitch), "hipMalloc");
            SWC_TRY(hipMalloc(&S.outs, p->batch * sizeof(uint64_t)), "hipMalloc");
            SWC_TRY(hipEventCreateWithFlags(&S.ev, hipEventDisableTiming), "hipEventCreate");
        }
        return 0;
    }();
    if (rc) {
        fecgpu_sw_encoder_free(e);
        return rc;
    }
    *out = e;
    return 0;
}

void fecgpu_sw_encoder_free(fecgpu_sw_encoder *e) {
    if (!e) return;
    if (e->s) (void)hipStreamSynchronize(e->s);
    for (auto &S : e->slot) {
        if (S.hdr) ctx_pinned_put(e->ctx, S.hdr, e->p.batch * (sizeof(fecgpu_sw_repair) + e->stride));
        if (S.jobs) (void)hipFree(S.jobs);
        if (S.coef) (void)hipFree(S.coef);
        if (S.outs) (void)hipFree(S.outs);
        if (S.ev) (void)hipEventDestroy(S.ev);
    }
    if (e->src) ctx_pinned_put(e->ctx, e->src, e->cap * e->stride);
    delete e;
}

ssize_t fecgpu_sw_encoder_add_source(fecgpu_sw_encoder *e, const uint8_t *pkt, size_t len, uint64_t *esi) {
    if (!e || (!pkt && len)) return FECGPU_ERR_INVALID_ARG;
    if (e->p.framing == FECGPU_FRAMING_LENPREFIX ? len + 2 > e->p.symbol_size : len != e->p.symbol_size)
        return FECGPU_ERR_BUFFER_TOO_SHORT;
    const bool schedules = (e->next + 1) % e->p.step == 0;
    if (schedules && e->sched.size() >= e->p.batch) {
        // a full batch left behind by a failed launch: it goes first (or the
        // call fails with nothing consumed), so a slot never takes more than batch
        if (!enc_slot_free(e)) return FECGPU_ERR_LIMIT;
        const ssize_t rc = enc_launch(e);
        if (rc < 0) return rc;
    }
    if (schedules && e->sched.size() + 1 >= e->p.batch && !enc_slot_free(e)) return FECGPU_ERR_LIMIT;
    if (e->next == e->base + e->cap) {
        const ssize_t rc = enc_compact(e);
        if (rc) return rc;
    }
    (void)frame_into(e->p, e->src + (e->next - e->base) * e->stride, pkt, len);
    if (esi) *esi = e->next;
    e->next++;
    if (schedules) {
        fecgpu_sw_repair h{};
        const uint64_t W = e->p.window;
        h.fss = e->next > W ? e->next - W : 0;
        h.nss = (uint16_t)(e->next - h.fss);
        h.key = (uint16_t)(e->key++ & 0xFFFF);
        h.dt = e->p.dt;
        e->sched.push_back(h);
        // the source is stored and its repair scheduled: a failed launch leaves
        // the batch scheduled, and the next call that schedules (or a flush)
        // launches it first or fails with nothing consumed
        if (e->sched.size() >= e->p.batch) (void)enc_launch(e);
    }
    return 0;
}

ssize_t fecgpu_sw_encoder_flush(fecgpu_sw_encoder *e) {
    if (!e) return FECGPU_ERR_INVALID_ARG;
    while (!e->sched.empty() && enc_slot_free(e)) {  // else the rest waits for a slot (read repairs first)
        const ssize_t rc = enc_launch(e);
        if (rc < 0) return rc;
    }
    SWC_TRY(hipStreamSynchronize(e->s), "hipStreamSynchronize");
    size_t ready = 0;
    for (int i : e->order) ready += e->slot[i].n - e->slot[i].popped;
    return (ssize_t)ready;
}

ssize_t fecgpu_sw_encoder_next_repair(fecgpu_sw_encoder *e, fecgpu_sw_repair *hdr, uint8_t *out, size_t cap) {
    if (!e || !hdr || !out) return FECGPU_ERR_INVALID_ARG;
    if (cap < e->p.symbol_size) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (e->order.empty()) return FECGPU_ERR_DONE;
    auto &S = e->slot[e->order.front()];
    const hipError_t q = hipEventQuery(S.ev);
    if (q == hipErrorNotReady) return FECGPU_ERR_DONE;
    if (q != hipSuccess) return set_dev_error(q, "sliding-window encode");
    *hdr = S.abs[S.popped];
    std::memcpy(out, S.rep + S.popped * e->stride, e->p.symbol_size);
    if (++S.popped == S.n) {
        S.used = false;
        e->order.pop_front();
    }
    return (ssize_t)e->p.symbol_size;
}

ssize_t fecgpu_sw_decoder_new(fecgpu_ctx *ctx, const fecgpu_sw_params *p, fecgpu_sw_decoder **out) {
    if (!ctx || !out) return FECGPU_ERR_INVALID_ARG;
    *out = nullptr;
    ssize_t rc = check_params(p);
    if (rc) return rc;
    auto *d = new fecgpu_sw_decoder();
    d->ctx = ctx;
    d->p = *p;
    d->stride = (p->symbol_size + 15u) & ~15u;
    // default span: 16 windows, plus the sender's batching delay.  A repair of
    // the same parameters is sent once its batch is read from the sender: up to
    // kSlots launched batches plus the one filling, each batch * step sources
    // (at 2 batches, r02's 5 % loss / batch 64 run gave up 108 repairs as late)
    const uint64_t span = p->span ? std::max<uint64_t>(p->span, 2ull * p->window)
                                  : 16ull * p->window + (uint64_t)(kSlots + 1) * p->batch * p->step;
    d->cap = 2 * span;
    d->rcap = (uint32_t)std::min<uint64_t>(1u << 20, d->cap / p->step + 2ull * p->batch + 16);
    d->have.assign(d->cap, 0);
    d->rh.resize(d->rcap);
    rc = [&]() -> ssize_t {
        SWC_TRY(hipGetDevice(&d->dev), "hipGetDevice");
        rc = ctx_conn_stream(ctx, d->dev, &d->s);
        if (rc) return rc;
        rc = ctx_pinned_get(ctx, d->cap * d->stride, reinterpret_cast<void **>(&d->src));
        if (rc) return rc;
        return ctx_pinned_get(ctx, (size_t)d->rcap * d->stride, reinterpret_cast<void **>(&d->rep));
    }();
    if (rc) {
        fecgpu_sw_decoder_free(d);
        return rc;
    }
    *out = d;
    return 0;
}

void fecgpu_sw_decoder_free(fecgpu_sw_decoder *d) {
    if (!d) return;
    if (d->s) (void)hipStreamSynchronize(d->s);
    if (d->src) ctx_pinned_put(d->ctx, d->src, d->cap * d->stride);
    if (d->rep) ctx_pinned_put(d->ctx, d->rep, (size_t)d->rcap * d->stride);
    delete d;
}

ssize_t fecgpu_sw_decoder_add_source(fecgpu_sw_decoder *d, uint64_t esi, const uint8_t *pkt, size_t len) {
    if (!d || (!pkt && len) || esi >= (1ull << 62)) return FECGPU_ERR_INVALID_ARG;
    if (d->p.framing == FECGPU_FRAMING_LENPREFIX ? len + 2 > d->p.symbol_size : len != d->p.symbol_size)
        return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (esi < d->base) return FECGPU_ERR_DONE;  // given up already
    if (esi >= d->base + d->cap) dec_advance(d, esi);
    const uint64_t row = esi - d->base;
    (void)frame_into(d->p, d->src + row * d->stride, pkt, len);
    d->have[row] = 1;
    d->hi = std::max(d->hi, esi + 1);
    return 0;
}

ssize_t fecgpu_sw_decoder_add_repair(fecgpu_sw_decoder *d, const fecgpu_sw_repair *h, const uint8_t *sym,
                                     size_t len) {
    if (!d || !h || !sym || h->nss == 0 || h->nss > FECGPU_SW_MAX_WINDOW || h->dt > 15 || h->fss >= (1ull << 62))
        return FECGPU_ERR_INVALID_ARG;
    // a window longer than the session's W is malformed: rejected before it can
    // move the span (advancing first would give up every buffered source)
    if (h->nss > d->p.window) return FECGPU_ERR_INVALID_ARG;
    if (len != d->p.symbol_size) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (h->fss < d->base) return FECGPU_ERR_DONE;  // its window reaches behind the kept span
    // nss <= W <= cap / 2, so after the advance the whole window is inside the span
    if (h->fss + h->nss > d->base + d->cap) dec_advance(d, h->fss + h->nss - 1);
    if (d->nrep == d->rcap) {
        dec_drop_old(d);
        if (d->nrep == d->rcap) {  // still full: the oldest repair goes
            std::memmove(d->rh.data(), d->rh.data() + 1, (d->nrep - 1) * sizeof(fecgpu_sw_repair));
            std::memmove(d->rep, d->rep + d->stride, (size_t)(d->nrep - 1) * d->stride);
            d->nrep--;
        }
    }
    // keep the rows in fss order (fecgpu_sw_decode's headers are nondecreasing)
    uint32_t at = d->nrep;
    while (at > 0 && d->rh[at - 1].fss > h->fss) at--;
    if (at < d->nrep) {
        std::memmove(d->rh.data() + at + 1, d->rh.data() + at, (d->nrep - at) * sizeof(fecgpu_sw_repair));
        std::memmove(d->rep + (size_t)(at + 1) * d->stride, d->rep + (size_t)at * d->stride,
                     (size_t)(d->nrep - at) * d->stride);
    }
    d->rh[at] = *h;
    std::memcpy(d->rep + (size_t)at * d->stride, sym, len);
    if (d->stride > len) std::memset(d->rep + (size_t)at * d->stride + len, 0, d->stride - len);
    d->nrep++;
    d->hi = std::max(d->hi, h->fss + h->nss);
    if (++d->since >= d->p.batch) {
        const ssize_t rc = fecgpu_sw_decoder_flush(d);
        if (rc < 0) return rc;
    }
    return 0;
}

ssize_t fecgpu_sw_decoder_flush(fecgpu_sw_decoder *d) {
    if (!d) return FECGPU_ERR_INVALID_ARG;
    d->since = 0;
    dec_drop_old(d);
    if (d->nrep == 0 || d->hi <= d->base) return 0;
    const uint64_t n = d->hi - d->base;
    std::vector<fecgpu_sw_repair> rel(d->rh.begin(), d->rh.begin() + d->nrep);
    for (auto &h : rel) h.fss -= d->base;
    std::vector<uint8_t> rp(d->nrep, 1);
    d->st.assign(n, 0);
    const ssize_t rc = fecgpu_sw_decode(d->ctx, d->src, d->have.data(), n, d->rep, rp.data(), rel.data(), d->nrep,
                                        d->p.symbol_size, d->stride, d->st.data(), 0, d->s);
    if (rc < 0) return rc;
    for (uint64_t i = 0; i < n; i++)
        if (!d->have[i] && d->st[i] == FECGPU_STATUS_OK) {
            d->have[i] = 1;
            d->rec_q.push_back(d->base + i);
        }
    while (d->rec_q.size() > d->cap) d->rec_q.pop_front();
    dec_drop_old(d);
    return rc;
}

ssize_t fecgpu_sw_decoder_recovered(fecgpu_sw_decoder *d, uint64_t esi, uint8_t *out, size_t cap) {
    if (!d || !out) return FECGPU_ERR_INVALID_ARG;
    if (esi < d->base || esi >= d->base + d->cap || !d->have[esi - d->base]) return FECGPU_ERR_DONE;
    const uint8_t *row = d->src + (esi - d->base) * d->stride;
    size_t n = d->p.symbol_size;
    const uint8_t *pl = row;
    if (d->p.framing == FECGPU_FRAMING_LENPREFIX) {
        n = std::min<size_t>(((size_t)row[0] << 8) | row[1], d->p.symbol_size - 2);
        pl = row + 2;
    }
    if (cap < n) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (n) std::memcpy(out, pl, n);
    return (ssize_t)n;
}

ssize_t fecgpu_sw_decoder_next_recovered(fecgpu_sw_decoder *d, uint64_t *esi) {
    if (!d || !esi) return FECGPU_ERR_INVALID_ARG;
    if (d->rec_q.empty()) return FECGPU_ERR_DONE;
    *esi = d->rec_q.front();
    d->rec_q.pop_front();
    return 0;
}

}  // extern "C"
