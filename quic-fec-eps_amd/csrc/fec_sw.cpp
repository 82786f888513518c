// fec_sw.cpp — sliding-window random linear code entry points (include/fecgpu.h
// fecgpu_sw_encode / fecgpu_sw_decode / fecgpu_sw_decode_device; RFC 8681 with
// m = 8).  Host side: argument checks, staging and the
// launches.  The decode is planned on the device (fec_swdec.hip): the host
// copies the receiver's bookkeeping up (or takes it on the device) and reads
// statuses and counters back.  No CPU fallback: every symbol byte is computed
// on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <functional>
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
// (decode syndromes: 16 / 20 / 32 KB gave 0.197 / 0.198 / 0.209 ms per cfg7 call, r04)
constexpr uint32_t kCombBudget = 40u << 10;
constexpr uint32_t kCombBudgetWide = 20u << 10;
// kSwSolveOut (fec_internal.h): recovered sources per solve job
constexpr int kSwSolveIn = 128;              // syndrome rows a small system's solve reads (fec_swdec.hip)
// LDS of a solve workgroup: its jobs' 8-output tables over the widest range of
// syndrome rows (device-sized); more room than the encode's budget keeps
// several jobs per workgroup
// (r03: 32 KB 0.235 vs 64 KB 0.241 ms per cfg7 decode call, 1.62 vs 1.71 at 10 % loss)
constexpr uint32_t kSolveBudget = 32u << 10;
// LDS for one streaming-encode workgroup's multiply tables (segment of up to
// kSwSeg repairs x max_window coefficients x 21 B): 43 KB for 64 repairs at W 32
// (cfg7, r04: 28 / 32 / 36 KB 0.200-0.202 vs 44 KB 0.216 ms: more workgroups per CU)
constexpr uint32_t kStreamBudget = 32u << 10;
constexpr uint64_t kSwStreamSources = 1ull << 32;  // the streaming encode's source positions are 32-bit
// sources and repairs per call: the device plan numbers them in 32 bits
constexpr uint64_t kSwMaxSources = (1ull << 32) - 256;
constexpr int kSwMaxRetries = 4;  // larger-log rounds of a synchronous decode

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
                 const uint8_t *in_base, uint64_t in_bytes, uint8_t *out_base, uint64_t out_bytes, uint32_t S,
                 uint32_t stride, int R, int nin_max, hipStream_t s, const uint32_t *extra = nullptr,
                 uint64_t extra_max = 0, bool skip = false) {
    CombArgs a{};
    a.chk.lo[0] = reinterpret_cast<uint64_t>(in_base);  // FECGPU_CHECK builds: the sources and the repairs
    a.chk.n[0] = in_bytes;
    a.chk.lo[1] = reinterpret_cast<uint64_t>(out_base);
    a.chk.n[1] = out_bytes;
    a.jobs = jobs;
    a.coef = coef;
    a.outs = outs;
    a.in_base = in_base;
    a.out_base = out_base;
    a.xor_base = nullptr;
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

// Dwords per lane of the streaming encode for ctx "sw_stream" value `stream`
// (1..5: that many, or the largest divisor of the row's dwords below it;
// kSwStreamAuto: the fewest lane-slots per row, waves x C, ties to the
// smaller C).  A lane's table reads (the same on every lane) are shared by
// its C dwords, but the VALU work per dword is not, and C > 1 costs
// registers: on cfg7 C = 1 was fastest (fec_internal.h kSwStreamDefault).  The row's dwords D = 4 x 16-B columns; C
// divides D so no lane runs past a row.
int sw_stream_dwords(int stream, uint32_t S) {
    const uint32_t D = ((S + 15u) >> 4) * 4u;
    if (stream != kSwStreamAuto) {
        int C = std::min(std::max(stream, 1), 5);
        while (D % (uint32_t)C) C--;
        return C;
    }
    int best = 1;
    uint64_t best_cost = ~0ull;
    for (int C = 1; C <= 5; C++) {
        if (D % (uint32_t)C) continue;
        const uint64_t units = D / (uint32_t)C, cost = (units + 63) / 64 * (uint32_t)C;
        if (cost < best_cost) {
            best_cost = cost;
            best = C;
        }
    }
    return best;
}

ssize_t sw_encode_core(const uint8_t *src, uint64_t nsrc, uint8_t *rep, const fecgpu_sw_repair *hdr,
                       uint64_t nrep, int max_window, uint32_t S, uint32_t stride, void *pj, void *pc,
                       void *po, hipStream_t s, int group, const fecgpu_sw_repair *hdr_host, int stream,
                       const uint8_t *rlc, ChkRec *chk) {
    if (stream > 0 && nsrc < kSwStreamSources) {
        SwStreamArgs sa{};
        sa.rlc = rlc;
        sa.chk = chk;
        sa.src = src;
        sa.rep = rep;
        sa.hdr = hdr;
        sa.nsrc = nsrc;
        sa.nrep = nrep;
        sa.stride = stride;
        sa.max_window = max_window;
        const int C = sw_stream_dwords(stream, S);
        sa.ncu = ((S + 15u) >> 4) * 4u / (uint32_t)C;
        SW_TRY(launch_sw_stream(sa, C, kStreamBudget, s), "sliding-window streaming encode launch");
        return 0;
    }
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
    ca.rlc = rlc;
    if (ca.group == 1) {
        SW_TRY(launch_sw_enc_coef(ca, s), "sliding-window coefficient launch");
        return run_comb(ca.jobs, nrep, ca.coef, ca.outs, src, nsrc * stride, rep, nrep * stride, S, stride, 1,
                        max_window, s);
    }
    // the tail counter sits after the jobs (sw_enc_jobs leaves room); the host
    // copy of the headers, when given, says whether a tail can occur at all
    const uint64_t ngroups = (nrep + ca.group - 1) / ca.group;
    const bool tail = !hdr_host || !sw_groups_fit(hdr_host, nrep, nsrc, max_window, ca.group, ca.span_max);
    ca.tail = reinterpret_cast<uint32_t *>(ca.jobs + ngroups + nrep);
    SW_TRY(hipMemsetAsync(ca.tail, 0, sizeof(uint32_t), s), "sliding-window tail reset");
    SW_TRY(launch_sw_enc_coef(ca, s), "sliding-window coefficient launch");
    return run_comb(ca.jobs, ngroups, ca.coef, ca.outs, src, nsrc * stride, rep, nrep * stride, S, stride, ca.group,
                    std::max(ca.span_max, max_window), s, tail ? ca.tail : nullptr, nrep, true);
}

}  // namespace fecgpu

namespace {

ssize_t sw_encode_dev(fecgpu_ctx *ctx, const uint8_t *src, uint64_t nsrc, uint8_t *rep,
                      const fecgpu_sw_repair *hdr, uint64_t nrep, int max_window, uint32_t S,
                      uint32_t stride, hipStream_t s, const fecgpu_sw_repair *hdr_host = nullptr) {
    void *pj = nullptr, *pc = nullptr, *po = nullptr;
    const int group = ctx_sw_group(ctx), stream = ctx_sw_stream(ctx);
    const uint8_t *rlc = nullptr;
    RC_TRY(ctx_rlc_table(ctx, s, &rlc));
    ChkRec *chk = nullptr;
    RC_TRY(ctx_chk_record(ctx, &chk));
    if (stream > 0 && nsrc < kSwStreamSources)
        return sw_encode_core(src, nsrc, rep, hdr, nrep, max_window, S, stride, nullptr, nullptr, nullptr, s,
                              group, hdr_host, stream, rlc, chk);
    RC_TRY(ctx_sw_scratch(ctx, 0, sw_enc_jobs(nrep, group) * sizeof(CombJob), &pj));
    RC_TRY(ctx_sw_scratch(ctx, 1, nrep * kSwCoefPitch, &pc));
    RC_TRY(ctx_sw_scratch(ctx, 2, nrep * sizeof(uint64_t), &po));
    return sw_encode_core(src, nsrc, rep, hdr, nrep, max_window, S, stride, pj, pc, po, s, group, hdr_host, 0, rlc,
                          chk);
}

// ---- decode (device plan: fec_swdec.hip) ----------------------------------
size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Device scratch of one decode, carved out of ctx slot 6 (plan arrays, jobs,
// long-system tables), slot 7 (syndrome rows), slot 8 (long systems' pivot
// rows), slot 9 (their operation log) and slot 10 (device copies of host
// bookkeeping).
struct DecBlock {
    size_t o_reach, o_rcnt, o_lost, o_reachL, o_ctr, o_synj, o_syno, o_coef, o_solj, o_solo, o_solc, o_long,
        o_synrow, o_pivc, o_colpiv, o_pivhi, o_pivt, o_lkind, o_starts, total;
    uint64_t long_cap, piv_cap;
};
DecBlock dec_block(uint64_t nsrc, uint64_t nrep) {
    DecBlock L{};
    L.long_cap = nsrc + 1;  // queued long systems: at most one per lost source
    L.piv_cap = std::max<uint64_t>(1, nrep);
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += align256(bytes);
        return at;
    };
    L.o_ctr = take(sizeof(SwDecCtr));
    L.o_reach = take((nsrc + 1) * 4);
    L.o_rcnt = take((nsrc + 1) * 4);
    L.o_lost = take(nsrc * 4);
    L.o_reachL = take(nsrc * 4);
    // syndrome slots: one per repair, and one per lost source for the
    // one-unknown systems the plan solves
    const uint64_t nsyn = nrep + nsrc;
    L.o_synj = take(nsyn * sizeof(CombJob));
    L.o_syno = take(nsyn * 8);
    L.o_coef = take(nsyn * (size_t)kSwCoefPitch);
    // solve jobs / outputs: a slot per unknown
    L.o_solj = take((nsrc + 8) * sizeof(CombJob));
    L.o_solo = take(nsrc * 8);
    L.o_solc = take(nrep * (size_t)kSwSmallE);
    L.o_long = take(L.long_cap * sizeof(SwLong));
    L.o_synrow = take(nrep * 4);
    L.o_pivc = take(L.piv_cap * 256);
    L.o_colpiv = take(nsrc * 4);
    L.o_pivhi = take(L.piv_cap * 4);
    L.o_pivt = take(L.piv_cap * 4);
    L.o_lkind = take(nsrc);
    L.o_starts = take(nsrc * 4);
    L.total = o;
    return L;
}

// One decode on the device.  src / rep / present / rep_present / hdr / stat
// are device pointers; ctr_out (pinned, nullable) receives the counters once
// the stream reaches the end of the call; sticky (nullable, asynchronous
// calls) collects its errors for fecgpu_sw_decode_errors.
ssize_t sw_decode_core(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *present, uint64_t nsrc, const uint8_t *rep,
                       const uint8_t *rep_present, const fecgpu_sw_repair *hdr, uint64_t nrep, uint32_t S,
                       uint32_t stride, uint8_t *stat, hipStream_t s, SwDecCtr *ctr_out, uint64_t log_entries,
                       SwSticky *sticky = nullptr) {
    const int long_min = ctx_sw_long_min(ctx);
    const DecBlock L = dec_block(nsrc, nrep);
    void *pb = nullptr, *psyn = nullptr, *ppiv = nullptr, *plog = nullptr;
    RC_TRY(ctx_sw_scratch(ctx, 6, L.total, &pb));
    RC_TRY(ctx_sw_scratch(ctx, 7, std::max<uint64_t>(1, nrep) * stride, &psyn));
    RC_TRY(ctx_sw_scratch(ctx, 8, L.piv_cap * stride, &ppiv));
    RC_TRY(ctx_sw_scratch(ctx, 9, log_entries * sizeof(SwOp), &plog));
    uint8_t *b = static_cast<uint8_t *>(pb);
    SwDecArgs a{};
    a.src_present = present;
    a.rep_present = rep_present;
    a.hdr = hdr;
    a.stat = stat;
    a.nsrc = nsrc;
    a.nrep = nrep;
    a.stride = stride;
    a.S = S;
    a.long_min = long_min;
    a.reach = reinterpret_cast<uint32_t *>(b + L.o_reach);
    a.rcnt = reinterpret_cast<uint32_t *>(b + L.o_rcnt);
    a.lost = reinterpret_cast<uint32_t *>(b + L.o_lost);
    a.reachL = reinterpret_cast<uint32_t *>(b + L.o_reachL);
    a.ctr = reinterpret_cast<SwDecCtr *>(b + L.o_ctr);
    a.syn_jobs = reinterpret_cast<CombJob *>(b + L.o_synj);
    a.syn_outs = reinterpret_cast<uint64_t *>(b + L.o_syno);
    a.coef = b + L.o_coef;
    a.sol_jobs = reinterpret_cast<CombJob *>(b + L.o_solj);
    a.sol_outs = reinterpret_cast<uint64_t *>(b + L.o_solo);
    a.sol_coef = b + L.o_solc;
    a.longs = reinterpret_cast<SwLong *>(b + L.o_long);
    a.long_cap = L.long_cap;
    a.log = static_cast<SwOp *>(plog);
    a.log_cap = log_entries;
    a.synrow = reinterpret_cast<uint32_t *>(b + L.o_synrow);
    a.pivcoef = b + L.o_pivc;
    a.colpiv = reinterpret_cast<uint32_t *>(b + L.o_colpiv);
    a.pivhi = reinterpret_cast<uint32_t *>(b + L.o_pivhi);
    a.pivt = reinterpret_cast<uint32_t *>(b + L.o_pivt);
    a.lkind = b + L.o_lkind;
    a.starts = reinterpret_cast<uint32_t *>(b + L.o_starts);
    a.pivdata = static_cast<uint8_t *>(ppiv);
    a.piv_cap = L.piv_cap;
    a.src = src;
    a.synd = static_cast<const uint8_t *>(psyn);
    a.sticky = sticky;
    RC_TRY(ctx_chk_record(ctx, &a.chk));
    RC_TRY(ctx_rlc_table(ctx, s, &a.rlc));
    {  // the plan kernel writes the counters itself: nothing to clear
        SwLookback lb{};
        RC_TRY(ctx_sw_lookback(ctx, (nsrc + kSwPlanChunk - 1) / kSwPlanChunk, &lb, &a.epoch));
        a.lb_cap = (nsrc + kSwPlanChunk - 1) / kSwPlanChunk;
        a.lb_flag = lb.flag;
        a.lb_agg = lb.agg;
        a.lb_inc = lb.inc;
        a.lb_ticket = lb.ticket;
    }
    SW_TRY(launch_sw_dec_plan(a, s), "sliding-window decode plan launch");
    // (the one-unknown systems' syndromes on a second stream beside the
    // systems launch, joined at the end, measured 0.209 vs 0.197 ms per cfg7
    // call, r05: removed)
    SW_TRY(launch_sw_dec_sys(a, s), "sliding-window decode systems launch");
    SW_TRY(launch_sw_dec_long(a, s), "sliding-window long-system plan launch");
    const uint32_t ncol = (S + 15u) >> 4;
    // syndromes (one output each, at most the widest window of inputs), then the
    // small systems' solves (<= 8 outputs over <= kSwSmallP syndromes)
    CombArgs sa{};
    sa.jobs = a.syn_jobs;
    sa.coef = a.coef;
    sa.outs = a.syn_outs;
    sa.in_base = src;
    sa.out_base = static_cast<uint8_t *>(psyn);
    sa.xor_base = rep;
    sa.njobs = nrep;  // a slot per repair; the needed ones filled by their systems
    sa.extra = &a.ctr->nlost;  // then a slot per lost source: the plan's one-unknown systems
    sa.extra_max = nsrc;
    sa.interleave = 1;  // those are dense at the end: deal the groups round-robin
    // mostly empty slots: each workgroup gathers its share's non-empty jobs
    // (decode 0.239 -> 0.223 ms per cfg7 call against walking every slot, r04)
    sa.sparse = 1;
    sa.ncol = ncol;
    sa.stride = stride;
    sa.nin_max = kSwMaxWindow;
    sa.nout_max = 1;
    sa.nin_dev = &a.ctr->wmax;
    sa.err = &a.ctr->err;
    // FECGPU_CHECK builds: sources in (and out: the one-unknown systems), repairs
    // xor-ed in, syndrome rows out; less "check_shrink" bytes each
    const uint64_t shrink = ctx_check_shrink(ctx);
    const auto range = [&](CombArgs &c, int i, const void *p, uint64_t n) {
        c.chk.lo[i] = reinterpret_cast<uint64_t>(p);
        c.chk.n[i] = n - std::min(n, shrink);
    };
    range(sa, 0, src, nsrc * stride);
    range(sa, 1, rep, nrep * stride);
    range(sa, 2, psyn, nrep * stride);
    sa.budget = ncol >= 64 ? kCombBudgetWide : kCombBudget;
    SW_TRY(launch_comb(sa, 1, s), "sliding-window syndrome launch");
    CombArgs va = sa;
    va.jobs = a.sol_jobs;
    va.coef = a.sol_coef;
    va.outs = a.sol_outs;
    va.in_base = static_cast<const uint8_t *>(psyn);
    va.out_base = src;
    va.xor_base = nullptr;
    va.chk = ChkRange{};
    range(va, 0, psyn, nrep * stride);
    range(va, 1, src, nsrc * stride);
    va.extra = &a.ctr->nlost;  // a slot per unknown, filled by its small system
    va.extra_max = nsrc;
    va.njobs = 0;
    va.nin_max = kSwSolveIn;
    va.nout_max = kSwSolveOut;
    va.nin_dev = &a.ctr->maxin;
    va.budget = kSolveBudget;
    SW_TRY(launch_comb(va, kSwSolveOut, s), "sliding-window solve launch");
    SW_TRY(launch_sw_dec_replay(a, s), "sliding-window long-system replay launch");
    if (ctr_out) SW_TRY(hipMemcpyAsync(ctr_out, a.ctr, sizeof(SwDecCtr), hipMemcpyDeviceToHost, s), "D2H sw counters");
    return 0;
}

// Synchronous decode with the counters read back.  A long system whose
// operation log overflowed the reservation is decoded again with a log sized
// past what the overflow asked for (a decode is idempotent: it reads only
// received symbols and rewrites the lost ones); kSwMaxRetries such rounds,
// each at least 4x larger, then FECGPU_ERR_DEVICE.  No other condition leaves
// a determined source lost.
ssize_t sw_decode_sync(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *present, uint64_t nsrc, const uint8_t *rep,
                       const uint8_t *rep_present, const fecgpu_sw_repair *hdr, uint64_t nrep, uint32_t S,
                       uint32_t stride, uint8_t *stat, hipStream_t s, const std::function<ssize_t()> &after) {
    void *ph = nullptr;
    RC_TRY(ctx_sw_host(ctx, sizeof(SwDecCtr), &ph));
    SwDecCtr *ctr = static_cast<SwDecCtr *>(ph);
    uint64_t log_entries = ctx_sw_log_entries(ctx, nsrc, nrep);
    for (int attempt = 0;; attempt++) {
        RC_TRY(sw_decode_core(ctx, src, present, nsrc, rep, rep_present, hdr, nrep, S, stride, stat, s, ctr,
                              log_entries));
        RC_TRY(after());
        SW_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
        if (ctr->err & kSwErrHeader) return FECGPU_ERR_INVALID_ARG;
        if (ctr->err & ~(kSwErrHeader | kSwErrCapacity))
            return set_dev_error(hipErrorUnknown, "sliding-window decode: unexpected device error flag");
        if (!(ctr->err & kSwErrCapacity)) break;
        if (attempt == kSwMaxRetries)
            return set_dev_error(hipErrorOutOfMemory, "sliding-window decode: operation log capacity");
        log_entries = std::max<uint64_t>(log_entries * 4, (uint64_t)ctr->nlog + 1);
        ctx_sw_log_grow(ctx, log_entries);
    }
    return (ssize_t)ctr->recovered;
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
        RC_TRY(ctx_chk_finish(ctx, s, "sliding-window encode"));  // FECGPU_CHECK builds (release: nothing)
        RC_TRY(ctx_sw_end(ctx, s));
        SW_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
        return (ssize_t)nrep;
    }
    RC_TRY(ctx_sw_begin(ctx, s));
    RC_TRY(sw_encode_dev(ctx, src, nsrc, rep, hdr, nrep, mw, sym_len, stride, s));
    RC_TRY(ctx_chk_finish(ctx, s, "sliding-window encode"));  // FECGPU_CHECK builds (release: nothing)
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
    if (nsrc >= kSwMaxSources || nrep >= kSwMaxSources) return FECGPU_ERR_UNSUPPORTED;
    RC_TRY(check_geometry(sym_len, stride, src, nrep ? rep : src));
    uint64_t prev_fss = 0;
    for (uint64_t t = 0; t < nrep; t++) {
        if (!header_ok(hdr[t], nsrc)) return FECGPU_ERR_INVALID_ARG;
        if (hdr[t].fss < prev_fss) return FECGPU_ERR_INVALID_ARG;  // fss nondecreasing
        prev_fss = hdr[t].fss;
    }
    if (nrep == 0) {  // nothing to decode with: statuses only
        for (uint64_t i = 0; i < nsrc; i++) src_status[i] = src_present[i] ? FECGPU_STATUS_OK : FECGPU_STATUS_UNRECOVERABLE;
        return 0;
    }
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    RC_TRY(ctx_sw_begin(ctx, s));
    // the bookkeeping (flags, headers, statuses) goes up and comes back down
    void *pm = nullptr;
    const size_t o_rp = align256(nsrc), o_hdr = o_rp + align256(nrep), o_st = o_hdr + align256(nrep * sizeof(fecgpu_sw_repair));
    RC_TRY(ctx_sw_scratch(ctx, 10, o_st + nsrc, &pm));
    uint8_t *m = static_cast<uint8_t *>(pm);
    SW_TRY(hipMemcpyAsync(m, src_present, nsrc, hipMemcpyHostToDevice, s), "H2D sw source flags");
    SW_TRY(hipMemcpyAsync(m + o_rp, rep_present, nrep, hipMemcpyHostToDevice, s), "H2D sw repair flags");
    SW_TRY(hipMemcpyAsync(m + o_hdr, hdr, nrep * sizeof(fecgpu_sw_repair), hipMemcpyHostToDevice, s), "H2D sw headers");
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
    const ssize_t rc = sw_decode_sync(
        ctx, dsrc, m, nsrc, drep, m + o_rp, reinterpret_cast<const fecgpu_sw_repair *>(m + o_hdr), nrep, sym_len,
        stride, m + o_st, s, [&]() -> ssize_t {
            SW_TRY(hipMemcpyAsync(src_status, m + o_st, nsrc, hipMemcpyDeviceToHost, s), "D2H sw statuses");
            if (flags & FECGPU_F_HOST_PTRS)
                SW_TRY(hipMemcpyAsync(src, dsrc, nsrc * stride, hipMemcpyDeviceToHost, s), "D2H sw sources");
            return 0;
        });
    RC_TRY(ctx_chk_finish(ctx, s, "sliding-window decode"));  // FECGPU_CHECK builds (release: nothing)
    RC_TRY(ctx_sw_end(ctx, s));
    return rc;
}

ssize_t fecgpu_sw_decode_device(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *src_present, uint64_t nsrc,
                                const uint8_t *rep, const uint8_t *rep_present, const fecgpu_sw_repair *hdr,
                                uint64_t nrep, uint32_t sym_len, uint32_t stride, uint8_t *src_status,
                                uint32_t flags, void *stream) {
    if (!ctx || !src || !src_present || !src_status || nsrc == 0) return FECGPU_ERR_INVALID_ARG;
    if (nrep && (!rep || !rep_present || !hdr)) return FECGPU_ERR_INVALID_ARG;
    if (flags & FECGPU_F_HOST_PTRS) return FECGPU_ERR_INVALID_ARG;
    if (nsrc >= kSwMaxSources || nrep >= kSwMaxSources) return FECGPU_ERR_UNSUPPORTED;
    RC_TRY(check_geometry(sym_len, stride, src, nrep ? rep : src));
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    RC_TRY(ctx_sw_begin(ctx, s));
    ssize_t rc = 0;
    if (flags & FECGPU_F_SYNC) {
        rc = sw_decode_sync(ctx, src, src_present, nsrc, rep, rep_present, hdr, nrep, sym_len, stride, src_status, s,
                            [] { return (ssize_t)0; });
    } else {
        SwSticky *sticky = nullptr;
        RC_TRY(ctx_sw_sticky(ctx, &sticky));
        rc = sw_decode_core(ctx, src, src_present, nsrc, rep, rep_present, hdr, nrep, sym_len, stride, src_status, s,
                            nullptr, ctx_sw_log_entries(ctx, nsrc, nrep), sticky);
    }
    RC_TRY(ctx_chk_finish(ctx, s, "sliding-window decode"));  // FECGPU_CHECK builds (release: nothing)
    RC_TRY(ctx_sw_end(ctx, s));
    return rc;
}

ssize_t fecgpu_sw_decode_errors(fecgpu_ctx *ctx, uint32_t *flags) {
    if (!ctx || !flags) return FECGPU_ERR_INVALID_ARG;
    *flags = 0;
    SwSticky *d = nullptr;
    RC_TRY(ctx_sw_sticky(ctx, &d));
    RC_TRY(ctx_sw_wait(ctx));  // every sliding-window call issued so far on this device
    SwSticky h{};
    SW_TRY(hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost), "D2H sw error flags");
    // cleared by a synchronous copy, complete on return (a null-stream memset
    // may still be pending when the next asynchronous decode raises a flag)
    const SwSticky z{};
    SW_TRY(hipMemcpy(d, &z, sizeof(z), hipMemcpyHostToDevice), "sw error flags reset");
    // the next asynchronous calls reserve what the overflow asked for, twice over
    if (h.err & kSwErrCapacity) ctx_sw_log_grow(ctx, std::max<uint64_t>(2 * h.need, 1u << 16));
    *flags = h.err;
    return 0;
}

}  // extern "C"
