// fec_sw.cpp — sliding-window random linear code entry points (include/fecgpu.h
// fecgpu_sw_encode / fecgpu_sw_decode; RFC 8681 with m = 8; SURVEY.md Appendix
// B q6).  Host side: argument checks, staging, the decode's split of the lost
// sources into linked systems, and the launches of fec_kernels.hip's
// sliding-window kernels.  No CPU fallback: every symbol byte is computed on
// the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/fecgpu.h"
#include "fec_internal.h"

using namespace fecgpu;

namespace {

#define SW_TRY(expr, what)                                      \
    do {                                                        \
        hipError_t e_ = (expr);                                 \
        if (e_ != hipSuccess) return set_dev_error(e_, what);   \
    } while (0)
#define RC_TRY(expr)               \
    do {                           \
        ssize_t r_ = (expr);       \
        if (r_ < 0) return r_;     \
    } while (0)

constexpr uint32_t kCombBudget = 40u << 10;  // LDS of one combine workgroup's job tables
constexpr int kSwSolveOut = 8;               // recovered sources per solve job

ssize_t check_geometry(uint32_t sym_len, uint32_t stride, const void *a, const void *b) {
    if (stride == 0 || (stride & 15) || sym_len == 0 || sym_len > stride) return FECGPU_ERR_INVALID_ARG;
    if (stride > FECGPU_MAX_SYMBOL) return FECGPU_ERR_UNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(a) & 15) || (reinterpret_cast<uintptr_t>(b) & 15))
        return FECGPU_ERR_INVALID_ARG;
    return 0;
}

bool header_ok(const fecgpu_sw_repair &h, uint64_t nsrc) {
    return h.nss >= 1 && h.nss <= kSwMaxWindow && h.dt <= 15 && h.fss <= nsrc && nsrc - h.fss >= h.nss;
}

// One combine launch (fec_internal.h CombJob) over njobs jobs (plus *extra
// more, at most extra_max, when extra is given).
ssize_t run_comb(const CombJob *jobs, uint64_t njobs, const uint8_t *coef, const uint64_t *outs,
                 const uint8_t *in_base, uint8_t *out_base, const uint8_t *xor_base, uint32_t S,
                 uint32_t stride, int R, int nin_max, hipStream_t s, const uint32_t *extra = nullptr,
                 uint64_t extra_max = 0, bool skip = false) {
    CombArgs a{};
    a.jobs = jobs;
    a.coef = coef;
    a.outs = outs;
    a.in_base = in_base;
    a.out_base = out_base;
    a.xor_base = xor_base;
    a.njobs = njobs;
    a.extra = extra;
    a.extra_max = extra_max;
    a.skip = skip;
    a.ncol = (S + 15u) >> 4;
    a.stride = stride;
    a.nin_max = std::max(1, nin_max);
    a.nout_max = R;
    a.job_lds = comb_job_lds(a.nin_max, R);
    // groups of 8 have 8-output tables over a wider span: a larger share of the CU's LDS
    const uint32_t budget = skip && R == 8 ? kCombBudget * 2 : kCombBudget;
    a.wpb = std::max(1, std::min(kMaxWpb, choose_wpb_for(a.ncol, a.job_lds, budget)));
    SW_TRY(launch_comb(a, R, s), "sliding-window combine launch");
    return 0;
}

}  // namespace

namespace fecgpu {

// Repairs per group and the union span a group may cover: W + 3 steps for
// 4 repairs at W / step = 4, so 2 * max_window keeps the overlapping stream
// shapes grouped and the job tables small (comb_job_lds).
int sw_span_max(int max_window, int group) {
    // groups of 8: W + 7 steps at W / step = 4, within 3 * max_window
    return std::min<int>(kSwCoefPitch, (group > 4 ? 3 : 2) * std::max(1, max_window));
}

// Host replica of sw_enc_group's fit test: every group's clipped windows span
// at most span_max sources (then the per-repair tail is not launched).
bool sw_groups_fit(const fecgpu_sw_repair *h, uint64_t nrep, uint64_t nsrc, int max_window, int group,
                   int span_max) {
    for (uint64_t t0 = 0; t0 < nrep; t0 += group) {
        const int n = (int)std::min<uint64_t>(group, nrep - t0);
        uint64_t lo = ~0ull, hi = 0;
        for (int u = 0; u < n; u++) {
            const uint64_t fss = std::min<uint64_t>(h[t0 + u].fss, nsrc);
            const uint64_t nss = std::min<uint64_t>(std::min<int>(h[t0 + u].nss, max_window), nsrc - fss);
            lo = std::min(lo, fss);
            hi = std::max(hi, fss + nss);
        }
        if (hi - lo > (uint64_t)span_max || (hi - lo) * (uint64_t)n > (uint64_t)group * kSwCoefPitch)
            return false;
    }
    return true;
}

ssize_t sw_encode_core(const uint8_t *src, uint64_t nsrc, uint8_t *rep, const fecgpu_sw_repair *hdr,
                       uint64_t nrep, int max_window, uint32_t S, uint32_t stride, void *pj, void *pc,
                       void *po, hipStream_t s, int group, const fecgpu_sw_repair *hdr_host) {
    SwEncCoefArgs ca{};
    ca.hdr = hdr;
    ca.nrep = nrep;
    ca.nsrc = nsrc;
    ca.stride = stride;
    ca.max_window = max_window;
    ca.group = nrep > 1 && group > 1 ? group : 1;
    ca.span_max = sw_span_max(max_window, ca.group);
    ca.jobs = static_cast<CombJob *>(pj);
    ca.coef = static_cast<uint8_t *>(pc);
    ca.outs = static_cast<uint64_t *>(po);
    if (ca.group == 1) {
        SW_TRY(launch_sw_enc_coef(ca, s), "sliding-window coefficient launch");
        return run_comb(ca.jobs, nrep, ca.coef, ca.outs, src, rep, nullptr, S, stride, 1, max_window, s);
    }
    // the tail counter sits after the jobs (sw_enc_jobs leaves room); the host
    // copy of the headers, when given, says whether a tail can occur at all
    const uint64_t ngroups = (nrep + ca.group - 1) / ca.group;
    const bool tail = !hdr_host || !sw_groups_fit(hdr_host, nrep, nsrc, max_window, ca.group, ca.span_max);
    ca.tail = reinterpret_cast<uint32_t *>(ca.jobs + ngroups + nrep);
    SW_TRY(hipMemsetAsync(ca.tail, 0, sizeof(uint32_t), s), "sliding-window tail reset");
    SW_TRY(launch_sw_enc_coef(ca, s), "sliding-window coefficient launch");
    return run_comb(ca.jobs, ngroups, ca.coef, ca.outs, src, rep, nullptr, S, stride, ca.group,
                    std::max(ca.span_max, max_window), s, tail ? ca.tail : nullptr, nrep, true);
}

}  // namespace fecgpu

namespace {

ssize_t sw_encode_dev(fecgpu_ctx *ctx, const uint8_t *src, uint64_t nsrc, uint8_t *rep,
                      const fecgpu_sw_repair *hdr, uint64_t nrep, int max_window, uint32_t S,
                      uint32_t stride, hipStream_t s, const fecgpu_sw_repair *hdr_host = nullptr) {
    void *pj = nullptr, *pc = nullptr, *po = nullptr;
    const int group = ctx_sw_group(ctx);
    RC_TRY(ctx_sw_scratch(ctx, 0, sw_enc_jobs(nrep, group) * sizeof(CombJob), &pj));
    RC_TRY(ctx_sw_scratch(ctx, 1, nrep * kSwCoefPitch, &pc));
    RC_TRY(ctx_sw_scratch(ctx, 2, nrep * sizeof(uint64_t), &po));
    return sw_encode_core(src, nsrc, rep, hdr, nrep, max_window, S, stride, pj, pc, po, s, group, hdr_host);
}

// Host arrays of a decode's linked systems (see fecgpu_sw_decode).
struct SwPlan {
    std::vector<SwComp> comps;
    std::vector<uint64_t> unk, eqr;
    std::vector<uint32_t> eqc;
    std::vector<fecgpu_sw_repair> eqh;
    uint64_t amat = 0, nsolve = 0, tcoef = 0;
    int max_nss = 1, max_p = 1;
};

// Lost sources, ascending, split into linked systems: consecutive lost sources
// a < b are linked iff a received repair's window holds both, i.e. some
// received repair with fss <= a ends past b (windows are intervals, so this
// links every pair a repair holds).  Each system's equations are the received
// repairs whose windows hold one of its lost sources (the first kSwMaxEq).
// Systems of more than kSwMaxUnknowns lost sources, or with no equation, are
// left out (their sources stay lost).
void sw_build_plan(const uint8_t *src_present, uint64_t nsrc, const uint8_t *rep_present,
                   const fecgpu_sw_repair *hdr, uint64_t nrep, SwPlan &P) {
    // lost sources: 8 flags at a time, skipping words with no zero byte
    std::vector<uint64_t> lost;
    uint64_t i = 0;
    for (; i + 8 <= nsrc; i += 8) {
        uint64_t v;
        std::memcpy(&v, src_present + i, 8);
        if (!((v - 0x0101010101010101ull) & ~v & 0x8080808080808080ull)) continue;
        for (int b = 0; b < 8; b++)
            if (!src_present[i + b]) lost.push_back(i + b);
    }
    for (; i < nsrc; i++)
        if (!src_present[i]) lost.push_back(i);
    std::vector<uint64_t> pr;  // received repairs, fss ascending (headers are sorted)
    pr.reserve(nrep);
    uint64_t wmax = 1;  // longest received window: a repair holding source i has fss > i - wmax
    for (uint64_t t = 0; t < nrep; t++)
        if (rep_present[t]) {
            pr.push_back(t);
            wmax = std::max<uint64_t>(wmax, hdr[t].nss);
        }
    size_t ip = 0;
    uint64_t max_end = 0;
    size_t start = 0;
    std::vector<uint64_t> eq;  // one system's equations (reused)
    size_t jp = 0;             // first received repair that can hold the next system's sources
    P.unk.reserve(lost.size());
    P.comps.reserve(lost.size());
    P.eqr.reserve(4 * lost.size());
    P.eqc.reserve(4 * lost.size());
    P.eqh.reserve(4 * lost.size());
    for (size_t x = 0; x < lost.size(); x++) {
        while (ip < pr.size() && hdr[pr[ip]].fss <= lost[x]) {
            max_end = std::max(max_end, hdr[pr[ip]].fss + hdr[pr[ip]].nss);
            ip++;
        }
        if (x + 1 < lost.size() && max_end > lost[x + 1]) continue;
        // system = lost[start .. x]
        const uint64_t *U = lost.data() + start;
        const size_t e = x + 1 - start;
        start = x + 1;
        if (e > (size_t)kSwMaxUnknowns) continue;
        // systems come in ascending order, so the first candidate repair only
        // moves forward (a sweep, not a search per system)
        const uint64_t lo = U[0] >= wmax ? U[0] - wmax + 1 : 0;
        while (jp < pr.size() && hdr[pr[jp]].fss < lo) jp++;
        eq.clear();
        for (size_t it = jp; it < pr.size() && hdr[pr[it]].fss <= U[e - 1] && eq.size() < (size_t)kSwMaxEq; ++it) {
            const fecgpu_sw_repair &h = hdr[pr[it]];
            const uint64_t *u = e == 1 ? U : std::lower_bound(U, U + e, h.fss);
            if (u != U + e && *u >= h.fss && *u < h.fss + h.nss) eq.push_back(pr[it]);
        }
        if (eq.empty()) continue;
        SwComp c{};
        c.u_off = P.unk.size();
        c.q_off = P.eqr.size();
        c.a_off = P.amat;
        c.j_off = P.nsolve;
        c.t_off = P.tcoef;  // relative; the syndrome coefficients go first
        c.o_off = c.u_off;  // relative; the syndrome outputs go first
        c.e = (uint32_t)e;
        c.p = (uint32_t)eq.size();
        P.amat += (uint64_t)c.e * c.p;
        P.nsolve += (e + kSwSolveOut - 1) / kSwSolveOut;
        P.tcoef += (uint64_t)((e + kSwSolveOut - 1) / kSwSolveOut * kSwSolveOut) * c.p;
        P.max_p = std::max(P.max_p, (int)c.p);
        const uint32_t ci = (uint32_t)P.comps.size();
        for (size_t j = 0; j < e; j++) P.unk.push_back(U[j]);
        for (uint64_t t : eq) {
            P.eqr.push_back(t);
            P.eqc.push_back(ci);
            P.eqh.push_back(hdr[t]);
            P.max_nss = std::max(P.max_nss, (int)hdr[t].nss);
        }
        P.comps.push_back(c);
    }
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Device part of a decode: src / rep device pointers, plan P on the host.
ssize_t sw_decode_dev(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *rep, SwPlan &P, uint32_t S,
                      uint32_t stride, const uint8_t **ustat, hipStream_t s) {
    const uint64_t neq = P.eqr.size(), nunk = P.unk.size(), ncomp = P.comps.size();
    const uint64_t coef_syn = neq * kSwCoefPitch;
    for (SwComp &c : P.comps) {
        c.t_off += coef_syn;
        c.o_off += neq;
    }
    // one metadata block: comps | unk | eqr | eqc | eqh, then amat, ustat, syndrome rows
    const size_t o_unk = align256(ncomp * sizeof(SwComp));
    const size_t o_eqr = o_unk + align256(nunk * 8);
    const size_t o_eqc = o_eqr + align256(neq * 8);
    const size_t o_eqh = o_eqc + align256(neq * 4);
    const size_t o_amat = o_eqh + align256(neq * sizeof(fecgpu_sw_repair));
    const size_t o_ust = o_amat + align256(P.amat);
    const size_t o_syn = o_ust + align256(nunk);
    const size_t total = o_syn + neq * (size_t)stride;
    // the plan goes up from (and the statuses come back to) the ctx's pinned
    // staging block: a pageable copy of ~2 MB was a third of the call
    void *ph = nullptr;
    RC_TRY(ctx_sw_host(ctx, o_amat + nunk, &ph));
    uint8_t *meta = static_cast<uint8_t *>(ph);
    std::memcpy(meta, P.comps.data(), ncomp * sizeof(SwComp));
    std::memcpy(meta + o_unk, P.unk.data(), nunk * 8);
    std::memcpy(meta + o_eqr, P.eqr.data(), neq * 8);
    std::memcpy(meta + o_eqc, P.eqc.data(), neq * 4);
    std::memcpy(meta + o_eqh, P.eqh.data(), neq * sizeof(fecgpu_sw_repair));
    void *pm = nullptr, *pj = nullptr, *pc = nullptr, *po = nullptr;
    RC_TRY(ctx_sw_scratch(ctx, 6, total, &pm));
    RC_TRY(ctx_sw_scratch(ctx, 0, (neq + P.nsolve) * sizeof(CombJob), &pj));
    RC_TRY(ctx_sw_scratch(ctx, 1, coef_syn + P.tcoef, &pc));
    RC_TRY(ctx_sw_scratch(ctx, 2, (neq + nunk) * sizeof(uint64_t), &po));
    uint8_t *m = static_cast<uint8_t *>(pm);
    SW_TRY(hipMemcpyAsync(m, meta, o_amat, hipMemcpyHostToDevice, s), "H2D sw plan");
    CombJob *jobs = static_cast<CombJob *>(pj);
    uint8_t *coef = static_cast<uint8_t *>(pc);
    uint64_t *outs = static_cast<uint64_t *>(po);
    uint8_t *synd = m + o_syn;

    SwSynArgs ya{};
    ya.eqh = reinterpret_cast<const fecgpu_sw_repair *>(m + o_eqh);
    ya.eqr = reinterpret_cast<const uint64_t *>(m + o_eqr);
    ya.eqc = reinterpret_cast<const uint32_t *>(m + o_eqc);
    ya.comps = reinterpret_cast<const SwComp *>(m);
    ya.unk = reinterpret_cast<const uint64_t *>(m + o_unk);
    ya.neq = neq;
    ya.stride = stride;
    ya.jobs = jobs;
    ya.coef = coef;
    ya.outs = outs;
    ya.amat = m + o_amat;
    SW_TRY(launch_sw_syn(ya, s), "sliding-window syndrome coefficient launch");

    SwPlanArgs pa{};
    pa.comps = ya.comps;
    pa.ncomp = ncomp;
    pa.amat = m + o_amat;
    pa.unk = ya.unk;
    pa.stride = stride;
    pa.jobs = jobs + neq;
    pa.syn_jobs = jobs;
    pa.coef = coef;
    pa.outs = outs;
    pa.ustat = m + o_ust;
    SW_TRY(launch_sw_plan(pa, s), "sliding-window plan launch");
    RC_TRY(run_comb(jobs, neq, coef, outs, src, synd, rep, S, stride, 1, P.max_nss, s));
    RC_TRY(run_comb(jobs + neq, P.nsolve, coef, outs, synd, src, nullptr, S, stride, kSwSolveOut,
                    P.max_p, s));
    SW_TRY(hipMemcpyAsync(meta + o_amat, m + o_ust, nunk, hipMemcpyDeviceToHost, s), "D2H sw status");
    *ustat = meta + o_amat;  // valid once the stream has completed
    return 0;
}

}  // namespace

extern "C" {

ssize_t fecgpu_sw_encode(fecgpu_ctx *ctx, const uint8_t *src, uint64_t nsrc, uint8_t *rep,
                         const fecgpu_sw_repair *hdr, uint64_t nrep, uint32_t max_window,
                         uint32_t sym_len, uint32_t stride, uint32_t flags, void *stream) {
    if (!ctx) return FECGPU_ERR_INVALID_ARG;
    if (nrep == 0) return 0;
    if (!src || !rep || !hdr || nsrc == 0) return FECGPU_ERR_INVALID_ARG;
    if (max_window > (uint32_t)kSwMaxWindow) return FECGPU_ERR_INVALID_ARG;
    RC_TRY(check_geometry(sym_len, stride, src, rep));
    int mw = max_window ? (int)max_window : kSwMaxWindow;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (flags & FECGPU_F_HOST_PTRS) {
        int hmax = 1;
        for (uint64_t t = 0; t < nrep; t++) {
            if (!header_ok(hdr[t], nsrc) || hdr[t].nss > mw) return FECGPU_ERR_INVALID_ARG;
            hmax = std::max(hmax, (int)hdr[t].nss);
        }
        RC_TRY(ctx_sw_begin(ctx, s));
        void *ds = nullptr, *dr = nullptr, *dh = nullptr;
        RC_TRY(ctx_sw_scratch(ctx, 3, nsrc * stride, &ds));
        RC_TRY(ctx_sw_scratch(ctx, 4, nrep * stride, &dr));
        RC_TRY(ctx_sw_scratch(ctx, 5, nrep * sizeof(fecgpu_sw_repair), &dh));
        SW_TRY(hipMemcpyAsync(ds, src, nsrc * stride, hipMemcpyHostToDevice, s), "H2D sw sources");
        SW_TRY(hipMemcpyAsync(dh, hdr, nrep * sizeof(fecgpu_sw_repair), hipMemcpyHostToDevice, s), "H2D sw headers");
        RC_TRY(sw_encode_dev(ctx, static_cast<uint8_t *>(ds), nsrc, static_cast<uint8_t *>(dr),
                             static_cast<fecgpu_sw_repair *>(dh), nrep, hmax, sym_len, stride, s, hdr));
        SW_TRY(hipMemcpyAsync(rep, dr, nrep * stride, hipMemcpyDeviceToHost, s), "D2H sw repairs");
        RC_TRY(ctx_sw_end(ctx, s));
        SW_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
        return (ssize_t)nrep;
    }
    RC_TRY(ctx_sw_begin(ctx, s));
    RC_TRY(sw_encode_dev(ctx, src, nsrc, rep, hdr, nrep, mw, sym_len, stride, s));
    RC_TRY(ctx_sw_end(ctx, s));
    if (flags & FECGPU_F_SYNC) SW_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    return (ssize_t)nrep;
}

ssize_t fecgpu_sw_decode(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *src_present, uint64_t nsrc,
                         const uint8_t *rep, const uint8_t *rep_present,
                         const fecgpu_sw_repair *hdr, uint64_t nrep, uint32_t sym_len,
                         uint32_t stride, uint8_t *src_status, uint32_t flags, void *stream) {
    if (!ctx || !src || !src_present || !src_status || nsrc == 0) return FECGPU_ERR_INVALID_ARG;
    if (nrep && (!rep || !rep_present || !hdr)) return FECGPU_ERR_INVALID_ARG;
    RC_TRY(check_geometry(sym_len, stride, src, nrep ? rep : src));
    for (uint64_t t = 0; t < nrep; t++) {
        if (!header_ok(hdr[t], nsrc)) return FECGPU_ERR_INVALID_ARG;
        if (t && hdr[t].fss < hdr[t - 1].fss) return FECGPU_ERR_INVALID_ARG;  // fss nondecreasing
    }
    uint64_t nlost = 0;
    for (uint64_t i = 0; i < nsrc; i++) {
        src_status[i] = src_present[i] ? FECGPU_STATUS_OK : FECGPU_STATUS_UNRECOVERABLE;
        nlost += !src_present[i];
    }
    if (nlost == 0 || nrep == 0) return 0;
    SwPlan P;
    sw_build_plan(src_present, nsrc, rep_present, hdr, nrep, P);
    if (P.comps.empty()) return 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    RC_TRY(ctx_sw_begin(ctx, s));
    uint8_t *dsrc = src;
    const uint8_t *drep = rep;
    if (flags & FECGPU_F_HOST_PTRS) {
        void *ds = nullptr, *dr = nullptr;
        RC_TRY(ctx_sw_scratch(ctx, 3, nsrc * stride, &ds));
        RC_TRY(ctx_sw_scratch(ctx, 4, nrep * stride, &dr));
        SW_TRY(hipMemcpyAsync(ds, src, nsrc * stride, hipMemcpyHostToDevice, s), "H2D sw sources");
        SW_TRY(hipMemcpyAsync(dr, rep, nrep * stride, hipMemcpyHostToDevice, s), "H2D sw repairs");
        dsrc = static_cast<uint8_t *>(ds);
        drep = static_cast<uint8_t *>(dr);
    }
    const uint8_t *ustat = nullptr;
    RC_TRY(sw_decode_dev(ctx, dsrc, drep, P, sym_len, stride, &ustat, s));
    if (flags & FECGPU_F_HOST_PTRS)
        SW_TRY(hipMemcpyAsync(src, dsrc, nsrc * stride, hipMemcpyDeviceToHost, s), "D2H sw sources");
    RC_TRY(ctx_sw_end(ctx, s));
    SW_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    ssize_t rec = 0;
    for (size_t u = 0; u < P.unk.size(); u++)
        if (ustat[u] == 0) {
            src_status[P.unk[u]] = FECGPU_STATUS_OK;
            rec++;
        }
    return rec;
}

}  // extern "C"
