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

// A decode's linked systems (see fecgpu_sw_decode).  The arrays the GPU reads
// (comps | unk | eqr | eqc | eqh) are written straight into the ctx's pinned
// staging block at offsets sized for the worst case (sw_plan_layout), so the
// plan goes up with one copy per array and no host-side repacking; the device
// block uses the same offsets.  lost / eq are per-thread scratch
// (sw_plan_scratch) that keeps its capacity from call to call.
struct SwPlan {
    SwComp *comps = nullptr;
    uint64_t *unk = nullptr, *eqr = nullptr;
    uint32_t *eqc = nullptr;
    fecgpu_sw_repair *eqh = nullptr;
    uint8_t *ustat = nullptr;  // statuses of the unknowns, copied back
    uint64_t ncomp = 0, nunk = 0, neq = 0;
    std::vector<uint64_t> lost, eq;  // lost sources ascending; one system's equations
    uint64_t amat = 0, nsolve = 0, tcoef = 0;
    int max_nss = 1, max_p = 1;
};

SwPlan &sw_plan_scratch() {
    thread_local SwPlan P;
    std::vector<uint64_t> lost = std::move(P.lost), eq = std::move(P.eq);
    lost.clear();
    eq.clear();
    P = SwPlan{};
    P.lost = std::move(lost);
    P.eq = std::move(eq);
    return P;
}

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Offsets of the plan arrays for nlost lost sources and nrep repairs: at most
// nlost systems and unknowns, and at most nrep equations (a received repair
// holding lost sources of two systems would link them, so each repair is an
// equation of one system at most).
struct SwLayout {
    size_t o_unk, o_eqr, o_eqc, o_eqh, meta, o_ust, host;
};
SwLayout sw_plan_layout(uint64_t nlost, uint64_t nrep) {
    SwLayout L;
    L.o_unk = align256(nlost * sizeof(SwComp));
    L.o_eqr = L.o_unk + align256(nlost * 8);
    L.o_eqc = L.o_eqr + align256(nrep * 8);
    L.o_eqh = L.o_eqc + align256(nrep * 4);
    L.meta = L.o_eqh + align256(nrep * sizeof(fecgpu_sw_repair));
    L.o_ust = L.meta;  // host only: the unknowns' statuses
    L.host = L.o_ust + nlost;
    return L;
}

// Per-source statuses (0 present, 1 lost) and the lost sources, ascending, in
// one pass over the arrival flags, 8 at a time: bit 7 of byte b of
// ((v & 0x7f..) + 0x7f..) | v is set iff flag b is nonzero (no carries cross
// bytes), so the status word is its complement shifted down.
uint64_t sw_scan_lost(const uint8_t *src_present, uint64_t nsrc, uint8_t *src_status,
                      std::vector<uint64_t> &lost) {
    constexpr uint64_t k7f = 0x7f7f7f7f7f7f7f7full, k01 = 0x0101010101010101ull;
    uint64_t i = 0;
    for (; i + 8 <= nsrc; i += 8) {
        uint64_t v;
        std::memcpy(&v, src_present + i, 8);
        const uint64_t st = ~((((v & k7f) + k7f) | v) >> 7) & k01;
        std::memcpy(src_status + i, &st, 8);
        for (uint64_t m = st; m; m &= m - 1) lost.push_back(i + ((uint64_t)__builtin_ctzll(m) >> 3));
    }
    for (; i < nsrc; i++) {
        src_status[i] = src_present[i] ? FECGPU_STATUS_OK : FECGPU_STATUS_UNRECOVERABLE;
        if (!src_present[i]) lost.push_back(i);
    }
    return lost.size();
}

// P.lost (ascending) split into linked systems: consecutive lost sources
// a < b are linked iff a received repair's window holds both, i.e. some
// received repair with fss <= a ends past b (windows are intervals, so this
// links every pair a repair holds).  Each system's equations are the received
// repairs whose windows hold one of its lost sources (the first kSwMaxEq).
// Systems of more than kSwMaxUnknowns lost sources, or with no equation, are
// left out (their sources stay lost).  wmax: an upper bound of the received
// windows' nss (a repair holding source i has fss > i - wmax).  Headers are in
// fss order, so the repairs are walked directly with their arrival flags.
void sw_build_plan(const uint8_t *rep_present, const fecgpu_sw_repair *hdr, uint64_t nrep,
                   uint64_t wmax, SwPlan &P) {
    const std::vector<uint64_t> &lost = P.lost;
    std::vector<uint64_t> &eq = P.eq;
    uint64_t ip = 0;  // repairs with fss <= the current lost source are folded into max_end
    uint64_t max_end = 0;
    size_t start = 0;
    uint64_t jp = 0;  // first repair that can hold the next system's sources
    for (size_t x = 0; x < lost.size(); x++) {
        for (; ip < nrep && hdr[ip].fss <= lost[x]; ip++)
            if (rep_present[ip]) max_end = std::max(max_end, hdr[ip].fss + hdr[ip].nss);
        if (x + 1 < lost.size() && max_end > lost[x + 1]) continue;
        // system = lost[start .. x]
        const uint64_t *U = lost.data() + start;
        const size_t e = x + 1 - start;
        start = x + 1;
        if (e > (size_t)kSwMaxUnknowns) continue;
        // systems come in ascending order, so the first candidate repair only
        // moves forward (a sweep, not a search per system)
        const uint64_t lo = U[0] >= wmax ? U[0] - wmax + 1 : 0;
        while (jp < nrep && hdr[jp].fss < lo) jp++;
        eq.clear();
        for (uint64_t it = jp; it < nrep && hdr[it].fss <= U[e - 1] && eq.size() < (size_t)kSwMaxEq; ++it) {
            if (!rep_present[it]) continue;
            const fecgpu_sw_repair &h = hdr[it];
            const uint64_t *u = e == 1 ? U : std::lower_bound(U, U + e, h.fss);
            if (u != U + e && *u >= h.fss && *u < h.fss + h.nss) eq.push_back(it);
        }
        if (eq.empty()) continue;
        SwComp c{};
        c.u_off = P.nunk;
        c.q_off = P.neq;
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
        const uint32_t ci = (uint32_t)P.ncomp;
        for (size_t j = 0; j < e; j++) P.unk[P.nunk++] = U[j];
        for (uint64_t t : eq) {
            P.eqr[P.neq] = t;
            P.eqc[P.neq] = ci;
            P.eqh[P.neq++] = hdr[t];
            P.max_nss = std::max(P.max_nss, (int)hdr[t].nss);
        }
        P.comps[P.ncomp++] = c;
    }
}

// Device part of a decode: src / rep device pointers, plan P in the pinned
// staging block at layout L.
ssize_t sw_decode_dev(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *rep, SwPlan &P, const SwLayout &L,
                      uint32_t S, uint32_t stride, hipStream_t s) {
    const uint64_t neq = P.neq, nunk = P.nunk, ncomp = P.ncomp;
    const uint64_t coef_syn = neq * kSwCoefPitch;
    for (uint64_t c = 0; c < ncomp; c++) {
        P.comps[c].t_off += coef_syn;
        P.comps[c].o_off += neq;
    }
    // device block: the plan arrays at L's offsets, then amat, ustat, syndrome rows
    const size_t o_unk = L.o_unk, o_eqr = L.o_eqr, o_eqc = L.o_eqc, o_eqh = L.o_eqh;
    const size_t o_amat = L.meta;
    const size_t o_ust = o_amat + align256(P.amat);
    const size_t o_syn = o_ust + align256(nunk);
    const size_t total = o_syn + neq * (size_t)stride;
    const uint8_t *meta = reinterpret_cast<const uint8_t *>(P.comps);
    void *pm = nullptr, *pj = nullptr, *pc = nullptr, *po = nullptr;
    RC_TRY(ctx_sw_scratch(ctx, 6, total, &pm));
    RC_TRY(ctx_sw_scratch(ctx, 0, (neq + P.nsolve) * sizeof(CombJob), &pj));
    RC_TRY(ctx_sw_scratch(ctx, 1, coef_syn + P.tcoef, &pc));
    RC_TRY(ctx_sw_scratch(ctx, 2, (neq + nunk) * sizeof(uint64_t), &po));
    uint8_t *m = static_cast<uint8_t *>(pm);
    // the used part of each array (from pinned memory: a pageable copy of
    // ~2 MB was a third of the call)
    const size_t part[5][2] = {{0, ncomp * sizeof(SwComp)}, {o_unk, nunk * 8}, {o_eqr, neq * 8},
                               {o_eqc, neq * 4}, {o_eqh, neq * sizeof(fecgpu_sw_repair)}};
    for (const auto &pt : part)
        SW_TRY(hipMemcpyAsync(m + pt[0], meta + pt[0], pt[1], hipMemcpyHostToDevice, s), "H2D sw plan");
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
    SW_TRY(hipMemcpyAsync(P.ustat, m + o_ust, nunk, hipMemcpyDeviceToHost, s), "D2H sw status");
    return 0;  // P.ustat is valid once the stream has completed
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
    uint64_t wmax = 1, prev_fss = 0;
    for (uint64_t t = 0; t < nrep; t++) {
        if (!header_ok(hdr[t], nsrc)) return FECGPU_ERR_INVALID_ARG;
        if (hdr[t].fss < prev_fss) return FECGPU_ERR_INVALID_ARG;  // fss nondecreasing
        prev_fss = hdr[t].fss;
        wmax = std::max<uint64_t>(wmax, hdr[t].nss);
    }
    SwPlan &P = sw_plan_scratch();
    const uint64_t nlost = sw_scan_lost(src_present, nsrc, src_status, P.lost);
    if (nlost == 0 || nrep == 0) return 0;
    const SwLayout L = sw_plan_layout(nlost, nrep);
    void *ph = nullptr;
    RC_TRY(ctx_sw_host(ctx, L.host, &ph));
    uint8_t *meta = static_cast<uint8_t *>(ph);
    P.comps = reinterpret_cast<SwComp *>(meta);
    P.unk = reinterpret_cast<uint64_t *>(meta + L.o_unk);
    P.eqr = reinterpret_cast<uint64_t *>(meta + L.o_eqr);
    P.eqc = reinterpret_cast<uint32_t *>(meta + L.o_eqc);
    P.eqh = reinterpret_cast<fecgpu_sw_repair *>(meta + L.o_eqh);
    P.ustat = meta + L.o_ust;
    sw_build_plan(rep_present, hdr, nrep, wmax, P);
    if (P.ncomp == 0) return 0;
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
    RC_TRY(sw_decode_dev(ctx, dsrc, drep, P, L, sym_len, stride, s));
    if (flags & FECGPU_F_HOST_PTRS)
        SW_TRY(hipMemcpyAsync(src, dsrc, nsrc * stride, hipMemcpyDeviceToHost, s), "D2H sw sources");
    RC_TRY(ctx_sw_end(ctx, s));
    SW_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    ssize_t rec = 0;
    for (uint64_t u = 0; u < P.nunk; u++)
        if (P.ustat[u] == 0) {
            src_status[P.unk[u]] = FECGPU_STATUS_OK;
            rec++;
        }
    return rec;
}

}  // extern "C"
