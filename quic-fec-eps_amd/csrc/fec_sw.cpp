// fec_sw.cpp — sliding-window random linear code entry points (include/fecgpu.h
// fecgpu_sw_encode / fecgpu_sw_decode; RFC 8681 with m = 8; SURVEY.md Appendix
// B q6).  Host side: argument checks, staging, the decode's split of the lost
// sources into linked systems, and the launches of fec_kernels.hip's
// sliding-window kernels.  No CPU fallback: every symbol byte is computed on
// the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
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

// LDS of one combine workgroup's job tables.  Jobs of >= 64 columns (a wave's
// worth) get the smaller budget: fewer jobs per workgroup (3 at S = 1200 B,
// W 32 step 8 groups of 4: one pass at 0.88 lane use) and more workgroups per
// CU.  cfg7 encode 0.249 -> 0.229 ms against 40 KB (7 jobs, 2 passes), 64 KB
// 0.282 ms, 96 KB 0.513 ms (profiles/r02_comb_budget_ab.txt).  Narrow jobs
// keep the larger budget, which packs more of them per pass.
#ifndef FECGPU_COMB_BUDGET_KB
#define FECGPU_COMB_BUDGET_KB 40
#endif
#ifndef FECGPU_COMB_BUDGET_WIDE_KB
#define FECGPU_COMB_BUDGET_WIDE_KB 20
#endif
constexpr uint32_t kCombBudget = FECGPU_COMB_BUDGET_KB << 10;
constexpr uint32_t kCombBudgetWide = FECGPU_COMB_BUDGET_WIDE_KB << 10;
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
    const uint32_t base = a.ncol >= 64 ? kCombBudgetWide : kCombBudget;
    const uint32_t budget = skip && R == 8 ? base * 2 : base;
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
// (comps | unk | eqr | eqc | eqh) are written into the ctx's pinned staging
// block at offsets sized for the worst case (sw_plan_layout), so the plan goes
// up with one copy per array and no host-side repacking; the device block uses
// the same offsets.  The same struct is a sweep's output cursor (SwPart).
struct SwPlan {
    SwComp *comps = nullptr;
    uint64_t *unk = nullptr, *eqr = nullptr;
    uint32_t *eqc = nullptr;
    fecgpu_sw_repair *eqh = nullptr;
    uint8_t *ustat = nullptr;  // statuses of the unknowns, copied back
    uint64_t ncomp = 0, nunk = 0, neq = 0;
    uint64_t amat = 0, nsolve = 0, tcoef = 0;
    int max_nss = 1, max_p = 1;
    std::vector<uint64_t> lost;  // lost sources ascending (per-thread scratch, see sw_plan_scratch)
};

SwPlan &sw_plan_scratch() {
    thread_local SwPlan P;
    std::vector<uint64_t> lost = std::move(P.lost);
    lost.clear();
    P = SwPlan{};
    P.lost = std::move(lost);
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

// Statuses (0 present, 1 lost) of sources [lo, hi) and their lost indices,
// ascending, in one pass over the arrival flags, 8 at a time (lo a multiple of
// 8): bit 7 of byte b of ((v & 0x7f..) + 0x7f..) | v is set iff flag b is
// nonzero (no carries cross bytes), so the status word is its complement
// shifted down.
void sw_scan_lost(const uint8_t *src_present, uint64_t lo, uint64_t hi, uint8_t *src_status,
                  std::vector<uint64_t> &lost) {
    constexpr uint64_t k7f = 0x7f7f7f7f7f7f7f7full, k01 = 0x0101010101010101ull;
    uint64_t i = lo;
    for (; i + 8 <= hi; i += 8) {
        uint64_t v;
        std::memcpy(&v, src_present + i, 8);
        const uint64_t st = ~((((v & k7f) + k7f) | v) >> 7) & k01;
        std::memcpy(src_status + i, &st, 8);
        for (uint64_t m = st; m; m &= m - 1) lost.push_back(i + ((uint64_t)__builtin_ctzll(m) >> 3));
    }
    for (; i < hi; i++) {
        src_status[i] = src_present[i] ? FECGPU_STATUS_OK : FECGPU_STATUS_UNRECOVERABLE;
        if (!src_present[i]) lost.push_back(i);
    }
}

// First repair whose fss >= lo (headers are in fss order).
uint64_t sw_first_repair(const fecgpu_sw_repair *hdr, uint64_t nrep, uint64_t lo) {
    return (uint64_t)(std::partition_point(hdr, hdr + nrep, [lo](const fecgpu_sw_repair &h) { return h.fss < lo; }) -
                      hdr);
}

// lost[x] begins a linked system iff no received repair with fss <= lost[x-1]
// ends past lost[x] (only repairs with fss > lost[x-1] - wmax can).
bool sw_system_start(const uint64_t *lost, size_t x, const uint8_t *rep_present,
                     const fecgpu_sw_repair *hdr, uint64_t nrep, uint64_t wmax) {
    if (x == 0) return true;
    const uint64_t p = lost[x - 1];
    for (uint64_t t = sw_first_repair(hdr, nrep, p >= wmax ? p - wmax + 1 : 0); t < nrep && hdr[t].fss <= p; t++)
        if (rep_present[t] && hdr[t].fss + hdr[t].nss > lost[x]) return false;
    return true;
}

// The sweep over lost[0 .. nl), which begins a system and ends where the next
// one begins (or at the end of the lost sources): consecutive lost sources
// a < b are linked iff a received repair's window holds both, i.e. some
// received repair with fss <= a ends past b (windows are intervals, so this
// links every pair a repair holds).  Each system's equations are the received
// repairs whose windows hold one of its lost sources (the first kSwMaxEq).
// Systems of more than kSwMaxUnknowns lost sources, or with no equation, are
// left out (their sources stay lost).  wmax: an upper bound of the received
// windows' nss (a repair holding source i has fss > i - wmax).  Headers are in
// fss order, so the repairs are walked directly with their arrival flags.
// Offsets in O's systems are relative to O's own arrays.
void sw_sweep(const uint64_t *lost, size_t nl, const uint8_t *rep_present, const fecgpu_sw_repair *hdr,
              uint64_t nrep, uint64_t wmax, SwPlan &O) {
    if (nl == 0) return;
    uint64_t eq[kSwMaxEq];
    const uint64_t first = sw_first_repair(hdr, nrep, lost[0] >= wmax ? lost[0] - wmax + 1 : 0);
    uint64_t ip = first;  // repairs with fss <= the current lost source are folded into max_end
    uint64_t jp = first;  // first repair that can hold the next system's sources
    uint64_t max_end = 0;
    size_t start = 0;
    for (size_t x = 0; x < nl; x++) {
        for (; ip < nrep && hdr[ip].fss <= lost[x]; ip++)
            if (rep_present[ip]) max_end = std::max(max_end, hdr[ip].fss + hdr[ip].nss);
        if (x + 1 < nl && max_end > lost[x + 1]) continue;
        // system = lost[start .. x]
        const uint64_t *U = lost + start;
        const size_t e = x + 1 - start;
        start = x + 1;
        if (e > (size_t)kSwMaxUnknowns) continue;
        // systems come in ascending order, so the first candidate repair only
        // moves forward (a sweep, not a search per system)
        const uint64_t lo = U[0] >= wmax ? U[0] - wmax + 1 : 0;
        while (jp < nrep && hdr[jp].fss < lo) jp++;
        int neq = 0;
        for (uint64_t it = jp; it < nrep && hdr[it].fss <= U[e - 1] && neq < kSwMaxEq; ++it) {
            if (!rep_present[it]) continue;
            const fecgpu_sw_repair &h = hdr[it];
            const uint64_t *u = e == 1 ? U : std::lower_bound(U, U + e, h.fss);
            if (u != U + e && *u >= h.fss && *u < h.fss + h.nss) eq[neq++] = it;
        }
        if (neq == 0) continue;
        SwComp c{};
        c.u_off = O.nunk;
        c.q_off = O.neq;
        c.a_off = O.amat;
        c.j_off = O.nsolve;
        c.t_off = O.tcoef;  // relative; the syndrome coefficients go first
        c.o_off = c.u_off;  // relative; the syndrome outputs go first
        c.e = (uint32_t)e;
        c.p = (uint32_t)neq;
        O.amat += (uint64_t)c.e * c.p;
        O.nsolve += (e + kSwSolveOut - 1) / kSwSolveOut;
        O.tcoef += (uint64_t)((e + kSwSolveOut - 1) / kSwSolveOut * kSwSolveOut) * c.p;
        O.max_p = std::max(O.max_p, (int)c.p);
        const uint32_t ci = (uint32_t)O.ncomp;
        for (size_t j = 0; j < e; j++) O.unk[O.nunk++] = U[j];
        for (int q = 0; q < neq; q++) {
            const uint64_t t = eq[q];
            O.eqr[O.neq] = t;
            O.eqc[O.neq] = ci;
            O.eqh[O.neq++] = hdr[t];
            O.max_nss = std::max(O.max_nss, (int)hdr[t].nss);
        }
        O.comps[O.ncomp++] = c;
    }
}

// Process-wide helper threads for large plans (FECGPU_PLAN_THREADS, default 4
// including the caller; 1 = always serial).  Workers spin briefly between
// runs (a stream of decodes comes every few hundred microseconds), then
// sleep.  One plan holds the pool at a time (acquire); a caller that finds it
// held plans alone.  The pool is never torn down (its threads are detached).
class PlanPool {
  public:
    static PlanPool &get() {
        static PlanPool *pool = new PlanPool();
        return *pool;
    }
    int size() const { return n_; }
    std::unique_lock<std::mutex> acquire() { return std::unique_lock<std::mutex>(run_mu_, std::try_to_lock); }
    // fn(i) for every i in [0, size()), i = 0 on the caller; the caller holds acquire()'s lock
    void run(const std::function<void(int)> &fn) {
        fn_ = &fn;
        pending_.store(n_ - 1, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(mu_);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        fn(0);
        while (pending_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    }

  private:
    PlanPool() {
        int n = 4;
        if (const char *e = std::getenv("FECGPU_PLAN_THREADS")) n = std::atoi(e);
        n = std::max(1, std::min(n, std::max(1, (int)std::thread::hardware_concurrency())));
        n_ = std::min(n, kMaxThreads);
        for (int i = 1; i < n_; i++) std::thread([this, i] { work(i); }).detach();
    }
    void work(int i) {
        uint64_t seen = 0;
        for (;;) {
            for (int spin = 0; gen_.load(std::memory_order_acquire) == seen; spin++) {
                if (spin < (1 << 16)) {
                    __builtin_ia32_pause();
                    continue;
                }
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
                break;
            }
            seen = gen_.load(std::memory_order_acquire);
            (*fn_)(i);
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }

  public:
    static constexpr int kMaxThreads = 16;

  private:
    int n_ = 1;
    std::mutex run_mu_, mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    const std::function<void(int)> *fn_ = nullptr;
};

// One helper's share of a parallel plan: its source chunk's lost list, then
// its systems in its own arrays (capacity kept from call to call).
struct SwPart {
    std::vector<uint64_t> lost;
    std::vector<SwComp> comps;
    std::vector<uint64_t> unk, eqr;
    std::vector<uint32_t> eqc;
    std::vector<fecgpu_sw_repair> eqh;
    SwPlan out;
    size_t lo = 0, hi = 0;  // range of the global lost list whose systems this part plans
};

constexpr uint64_t kSwParallelSources = 1u << 16;  // below this the plan runs on the caller alone

// Statuses, lost list, staging and systems of one decode.  Returns the number
// of lost sources (P.lost), or a negative error; P's arrays point into the
// staging block host(bytes, &p) returns (the ctx's pinned block) at layout L
// (not requested when nothing is lost).  threads: 0 = the pool's size.
template <class HostBlock>
ssize_t sw_plan(HostBlock &&host, const uint8_t *src_present, uint64_t nsrc, uint8_t *src_status,
                const uint8_t *rep_present, const fecgpu_sw_repair *hdr, uint64_t nrep, uint64_t wmax,
                SwPlan &P, SwLayout &L, int threads = 0) {
    auto bind = [&](void *ph) {
        uint8_t *meta = static_cast<uint8_t *>(ph);
        P.comps = reinterpret_cast<SwComp *>(meta);
        P.unk = reinterpret_cast<uint64_t *>(meta + L.o_unk);
        P.eqr = reinterpret_cast<uint64_t *>(meta + L.o_eqr);
        P.eqc = reinterpret_cast<uint32_t *>(meta + L.o_eqc);
        P.eqh = reinterpret_cast<fecgpu_sw_repair *>(meta + L.o_eqh);
        P.ustat = meta + L.o_ust;
    };
    PlanPool &pool = PlanPool::get();
    const int n = threads > 0 ? std::min(threads, pool.size()) : pool.size();
    std::unique_lock<std::mutex> held;
    if (n > 1 && nsrc >= kSwParallelSources) held = pool.acquire();
    const bool par = held.owns_lock();
    static SwPart parts[PlanPool::kMaxThreads];  // used while the pool is held only
    if (par) {
        pool.run([&](int i) {
            if (i >= n) return;  // a smaller share than the pool
            const uint64_t lo = (nsrc * (uint64_t)i / n) & ~7ull;
            const uint64_t hi = i + 1 == n ? nsrc : (nsrc * (uint64_t)(i + 1) / n) & ~7ull;
            parts[i].lost.clear();
            sw_scan_lost(src_present, lo, hi, src_status, parts[i].lost);
        });
        for (int i = 0; i < n; i++) P.lost.insert(P.lost.end(), parts[i].lost.begin(), parts[i].lost.end());
    } else {
        sw_scan_lost(src_present, 0, nsrc, src_status, P.lost);
    }
    const uint64_t nlost = P.lost.size();
    if (nlost == 0 || nrep == 0) return (ssize_t)nlost;
    L = sw_plan_layout(nlost, nrep);
    void *ph = nullptr;
    RC_TRY(host(L.host, &ph));
    bind(ph);
    const uint64_t *lost = P.lost.data();
    if (!par || nlost < 1024) {
        sw_sweep(lost, nlost, rep_present, hdr, nrep, wmax, P);
        return (ssize_t)nlost;
    }
    pool.run([&](int i) {
        if (i >= n) return;  // a smaller share than the pool
        // this part's systems: from the first system start at or after its
        // nominal share of the lost list to the next part's
        auto start_at = [&](int j) {
            if (j >= n) return (size_t)nlost;
            size_t x = (size_t)(nlost * (uint64_t)j / n);
            while (x < nlost && !sw_system_start(lost, x, rep_present, hdr, nrep, wmax)) x++;
            return x;
        };
        SwPart &q = parts[i];
        q.lo = start_at(i);
        q.hi = std::max(q.lo, start_at(i + 1));
        const size_t nl = q.hi - q.lo;
        uint64_t ne = 0;  // bound on equations: repairs with fss in [lost[lo] - wmax + 1, lost[hi - 1]]
        if (nl) {
            const uint64_t a = lost[q.lo], b = lost[q.hi - 1];
            ne = sw_first_repair(hdr, nrep, b + 1) - sw_first_repair(hdr, nrep, a >= wmax ? a - wmax + 1 : 0);
        }
        if (q.comps.size() < nl) q.comps.resize(nl);
        if (q.unk.size() < nl) q.unk.resize(nl);
        if (q.eqr.size() < ne) {
            q.eqr.resize(ne);
            q.eqc.resize(ne);
            q.eqh.resize(ne);
        }
        q.out = SwPlan{};
        q.out.comps = q.comps.data();
        q.out.unk = q.unk.data();
        q.out.eqr = q.eqr.data();
        q.out.eqc = q.eqc.data();
        q.out.eqh = q.eqh.data();
        sw_sweep(lost + q.lo, nl, rep_present, hdr, nrep, wmax, q.out);
    });
    // concatenate the parts in order, rebasing their offsets
    struct Base { uint64_t comp, unk, eq, amat, nsolve, tcoef; };
    Base base[PlanPool::kMaxThreads];
    Base acc{0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        const SwPlan &o = parts[i].out;
        base[i] = acc;
        acc.comp += o.ncomp;
        acc.unk += o.nunk;
        acc.eq += o.neq;
        acc.amat += o.amat;
        acc.nsolve += o.nsolve;
        acc.tcoef += o.tcoef;
        P.max_nss = std::max(P.max_nss, o.max_nss);
        P.max_p = std::max(P.max_p, o.max_p);
    }
    P.ncomp = acc.comp;
    P.nunk = acc.unk;
    P.neq = acc.eq;
    P.amat = acc.amat;
    P.nsolve = acc.nsolve;
    P.tcoef = acc.tcoef;
    pool.run([&](int i) {
        if (i >= n) return;  // a smaller share than the pool
        const SwPlan &o = parts[i].out;
        const Base &b = base[i];
        for (uint64_t j = 0; j < o.ncomp; j++) {
            SwComp c = o.comps[j];
            c.u_off += b.unk;
            c.o_off += b.unk;
            c.q_off += b.eq;
            c.a_off += b.amat;
            c.j_off += b.nsolve;
            c.t_off += b.tcoef;
            P.comps[b.comp + j] = c;
        }
        std::memcpy(P.unk + b.unk, o.unk, o.nunk * 8);
        std::memcpy(P.eqr + b.eq, o.eqr, o.neq * 8);
        std::memcpy(P.eqh + b.eq, o.eqh, o.neq * sizeof(fecgpu_sw_repair));
        for (uint64_t j = 0; j < o.neq; j++) P.eqc[b.eq + j] = o.eqc[j] + (uint32_t)b.comp;
    });
    return (ssize_t)nlost;
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
    SwLayout L{};
    const ssize_t nlost = sw_plan([ctx](size_t bytes, void **p) { return ctx_sw_host(ctx, bytes, p); }, src_present,
                                  nsrc, src_status, rep_present, hdr, nrep, wmax, P, L);
    if (nlost <= 0 || nrep == 0) return nlost < 0 ? nlost : 0;
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
