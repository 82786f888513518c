// fec_wide.hip — GF(2^8) block codes wider than one 64-bit mask: k + r up to
// 256 (the Cauchy construction's limit), r <= 8,
// through fecgpu_encode_batch / fecgpu_decode_batch (include/fecgpu.h: present
// masks of ceil((k + r) / 64) words per window).
//
//  * encode: the runtime-mask bit-sliced kernel (fec_kernels.hip rbs4::, r >= 4)
//    over every window's k sources, or else the sliding-window path's combine
//    kernel (comb_kernel<8>) with a job per window: inputs the k sources,
//    outputs the r repairs, coefficients the code's parity rows P[r][k] (one
//    block whose tables every workgroup builds once);
//  * decode: a wave per window plans it (wide_dec_plan_kernel): the missing
//    sources m_u (e <= r), the system A[t][u] = P[sel_t][m_u] of every present
//    repair reduced by Gauss-Jordan with pivot search (so an RLC window is
//    recovered whenever its present repairs have rank e), the stage-2 block
//    C[u][i] = T[P_u][c] for the repair i of pivot row c.  Stage 1: every
//    repair's syndrome s_i = rep_i + sum_j P[i][j] src_j (the missing rows
//    zeroed by the plan) by one coefficient block [P | I] for all windows;
//    stage 2: x_u = sum_i C[u][i] s_i, a combine job per window.
#include "fec_internal.h"

namespace fecgpu {

namespace {

__constant__ GfTables c_gfw = make_gf_tables();

// (A one-launch decode with a job of all k + r rows per window built
// (k + r + 1) x 161 B of tables per window: 3 (k 120) or 1 (k 248) windows
// per workgroup, 75 of its 256 lanes busy per 1200-B window; k120 decode
// 3.22 ms against 1.71 for the two stages, r04.)
// stage 2: LDS budget of a workgroup's window jobs (k120: 16 KB 1.656 vs 32 KB 1.683 ms, r04)
constexpr uint32_t kWideS2Budget = 16u << 10;

#define WIDE_WAVE_SYNC()                                        \
    do {                                                        \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                        \
    } while (0)

struct WideArgs {
    uint8_t *win;
    const uint64_t *present;  // [nwin][nw]
    uint8_t *status;
    const uint8_t *P;         // parity rows [r][k] on the device
    uint64_t nwin, wpitch;
    uint32_t stride;
    int k, r, nw;
    CombJob *jobs;   // [nwin]
    uint64_t *outs;  // [nwin][8] (encode: [nwin][r])
    uint8_t *coef;   // decode: [nwin][8][8], stage 2
    // two-stage decode: stage-1 jobs [nwin] and outputs [nwin][r] (syndrome
    // rows in syn, [nwin][r][stride])
    CombJob *jobs1;
    uint64_t *outs1;
    ChkRec *chk;  // FECGPU_CHECK builds: the fault record (release: null)
    bool zero_missing;  // stage 1 reads every row: the plan zeroes the missing ones
};

__global__ __launch_bounds__(kBlock) void wide_enc_jobs_kernel(WideArgs a) {
    const uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (w >= a.nwin) return;
    CombJob J;
    J.in_off = w * a.wpitch;
    J.coef_off = 0;
    J.out_list = w * (uint64_t)a.r;
    J.xor_off = kNoXor;
    J.nin = (uint32_t)a.k;
    J.nout = (uint32_t)a.r;
    a.jobs[w] = J;
    for (int i = 0; i < a.r; i++) a.outs[w * a.r + i] = w * a.wpitch + (uint64_t)(a.k + i) * a.stride;
}

__device__ __forceinline__ uint32_t wmul(const uint8_t *ex, const uint8_t *lg, uint32_t x, uint32_t y) {
    return (x && y) ? ex[lg[x] + lg[y]] : 0u;
}

// A wave per window: plan, job, status.
__global__ __launch_bounds__(kBlock) void wide_dec_plan_kernel(WideArgs a) {
    __shared__ uint8_t s_exp[512], s_log[256];
    __shared__ uint8_t s_m[kBlock / 64][kMaxR];  // missing sources, ascending
    for (int i = threadIdx.x; i < 512; i += kBlock) s_exp[i] = c_gfw.exp[i];
    for (int i = threadIdx.x; i < 256; i += kBlock) s_log[i] = c_gfw.log[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * (kBlock / 64) + wave;
    if (w >= a.nwin) return;  // whole waves: no barrier below
    const int k = a.k, r = a.r, n = k + r;
    const uint64_t *pw = a.present + w * (uint64_t)a.nw;
    CombJob J{};
    J.xor_off = kNoXor;
    // missing sources (the first kMaxR kept) and their count
    int e = 0;
    for (int c0 = 0; c0 < k; c0 += 64) {
        const int i = c0 + lane;
        const bool miss = i < k && !((pw[i >> 6] >> (i & 63)) & 1ull);
        const uint64_t b = __ballot(miss);
        const int pos = e + __popcll(b & ((1ull << lane) - 1ull));
        if (miss && pos < kMaxR) s_m[wave][pos] = (uint8_t)i;
        e += __popcll(b);
    }
    const bool rp = lane < r && ((pw[(k + lane) >> 6] >> ((k + lane) & 63)) & 1ull);
    const uint32_t rep = (uint32_t)__ballot(rp);  // present repairs (bit i: repair i)
    const int np = __popcll(rep);
    WIDE_WAVE_SYNC();
    if (e == 0 || e > r || np < e) {
        if (lane == 0) {
            a.status[w] = e == 0 ? FECGPU_STATUS_OK : FECGPU_STATUS_UNRECOVERABLE;
            a.jobs[w] = J;
            a.jobs1[w] = J;
        }
        return;
    }
    // [A | I], lane = t * 8 + u: row t = the t-th present repair, column u
    const int t = lane >> 3, u = lane & 7;
    int sel_t = 0;
    {
        uint32_t rr = rep;
        for (int i = 0; i < t && rr; i++) rr &= rr - 1;
        sel_t = rr ? __ffs(rr) - 1 : 0;
    }
    const bool row = t < np;
    const int m_u = u < e ? (int)s_m[wave][u] : 0;
    uint32_t xl = (row && u < e) ? a.P[(size_t)sel_t * k + m_u] : 0u;
    uint32_t xr = (row && t == u) ? 1u : 0u;
    uint32_t used = 0;  // rows already pivots (wave-uniform)
    int my_piv = 0;     // lane c < e: pivot row of column c
    for (int c = 0; c < e; c++) {
        const uint64_t cand = __ballot(row && u == c && !((used >> t) & 1u) && xl != 0);
        if (!cand) {  // rank < e: the window stays lost
            if (lane == 0) {
                a.status[w] = FECGPU_STATUS_UNRECOVERABLE;
                a.jobs[w] = J;
                a.jobs1[w] = J;
            }
            return;
        }
        const int pr = (int)(__ffsll((unsigned long long)cand) - 1) >> 3;
        used |= 1u << pr;
        if (lane == c) my_piv = pr;
        const uint32_t pv = __shfl(xl, pr * 8 + c, 64);
        const uint32_t ip = s_exp[255 - s_log[pv]];
        if (t == pr) {
            xl = wmul(s_exp, s_log, xl, ip);
            xr = wmul(s_exp, s_log, xr, ip);
        }
        const uint32_t f = __shfl(xl, t * 8 + c, 64);
        const uint32_t rl = __shfl(xl, pr * 8 + u, 64);
        const uint32_t rq = __shfl(xr, pr * 8 + u, 64);
        if (t != pr && row) {
            xl ^= wmul(s_exp, s_log, f, rl);
            xr ^= wmul(s_exp, s_log, f, rq);
        }
    }
    // stage 2's block C[u][i] (8 x 8 per window): T[P_u][c] for the repair i
    // of pivot row c, else 0; the missing rows zeroed for stage 1
    {
        uint8_t *C2 = a.coef + w * (uint64_t)(kMaxR * kMaxR);  // [e][r] used
        const int cu = lane >> 3, ci = lane & 7;                 // lane = output u * 8 + repair i
        const int pu = __shfl(my_piv, min(cu, e - 1), 64);      // every lane takes part in the shuffles
        uint32_t v = 0;
        for (int c = 0; c < e; c++) {
            const int pc = __shfl(my_piv, c, 64);
            const uint32_t tv = __shfl(xr, (pu * 8 + pc) & 63, 64);
            uint32_t rr = rep;
            for (int i2 = 0; i2 < pc && rr; i2++) rr &= rr - 1;
            if (__ffs(rr) - 1 == ci) v = tv;  // repair ci is pivot row pc's
        }
        if (cu < e && ci < r) C2[cu * r + ci] = (uint8_t)v;
        uint8_t *wb = a.win + w * a.wpitch;
        for (int u2 = 0; a.zero_missing && u2 < e && CHK_IDX(a.chk, s_m[wave][u2], k, 1); u2++) {
            uint4 *row = reinterpret_cast<uint4 *>(wb + (uint64_t)s_m[wave][u2] * a.stride);
            for (uint32_t c16 = lane; c16 < a.stride / 16u; c16 += 64) row[c16] = make_uint4(0, 0, 0, 0);
        }
    }
    if (lane < r) a.outs1[w * (uint64_t)r + lane] = (w * (uint64_t)r + lane) * a.stride;
    if (lane < e) a.outs[w * kMaxR + lane] = w * a.wpitch + (uint64_t)s_m[wave][lane] * a.stride;
    if (lane == 0) {
        CombJob J1;
        J1.in_off = w * a.wpitch;
        J1.coef_off = 0;
        J1.out_list = w * (uint64_t)r;
        J1.xor_off = kNoXor;
        J1.nin = (uint32_t)n;
        J1.nout = (uint32_t)r;
        a.jobs1[w] = J1;
        J.in_off = w * (uint64_t)r * a.stride;
        J.coef_off = w * (uint64_t)(kMaxR * kMaxR) + 0;
        J.out_list = w * kMaxR;
        J.nin = (uint32_t)r;
        J.nout = (uint32_t)e;
        a.jobs[w] = J;
        a.status[w] = FECGPU_STATUS_OK;
    }
}

}  // namespace

// Wide batch (k + r > 64): device pointers, uniform stride; scratch from the
// caller (jobs, outs, coef, P already on the device).  The caller orders the
// call against others that share the scratch.
hipError_t launch_wide(uint8_t *win, const uint64_t *present, uint8_t *status, const uint8_t *P_dev,
                       uint64_t nwin, uint32_t stride, uint32_t ncol, int k, int r, bool decode, CombJob *jobs,
                       uint64_t *outs, uint8_t *coef, hipStream_t s, CombJob *jobs1, uint64_t *outs1,
                       uint8_t *syn, const uint32_t *masks_P, const uint32_t *masks_PI, ChkRec *chk,
                       bool mask_rows) {
    WideArgs a{};
    a.chk = chk;
    a.win = win;
    a.present = present;
    a.status = status;
    a.P = P_dev;
    a.nwin = nwin;
    a.stride = stride;
    a.wpitch = (uint64_t)(k + r) * stride;
    a.k = k;
    a.r = r;
    a.nw = (k + r + 63) / 64;
    a.jobs = jobs;
    a.outs = outs;
    a.coef = coef;
    a.jobs1 = jobs1;
    a.outs1 = outs1;
    const int n = k + r;
    // stage 1 by plane picks skips the missing rows itself (absent rows read as
    // zeros through a buffer resource: no zeroing writes, no reads of them);
    // the combine-job stage 1 reads every row, so the plan zeroes them
    const bool masked = decode && masks_PI && mask_rows && rbs_masked_ok(ncol, a.wpitch);
    a.zero_missing = !masked;
    if (!decode && masks_P) {  // every window's k sources times P by plane picks
        return launch_rbs_rows(win, nwin, ncol, stride, a.wpitch, k, r, masks_P, 0, 0, s);
    }
    if (decode)
        hipLaunchKernelGGL(wide_dec_plan_kernel, dim3((unsigned)((nwin + kBlock / 64 - 1) / (kBlock / 64))),
                           dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL(wide_enc_jobs_kernel, dim3((unsigned)((nwin + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                           s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    constexpr uint32_t kBudget = 64u << 10;
    if (decode) {
        // (1) syndromes: every window's k + r rows times [P | I] (at P_dev + r k),
        // outputs the r syndrome rows: by plane picks (output i of window w at
        // syn + (w r + i) stride, i.e. its input row n + i's address plus
        // syn - win - n stride + w (r stride - wpitch)), or combine jobs with the
        // tables shared by the workgroup's jobs
        if (masks_PI) {
            e = launch_rbs_rows(win, nwin, ncol, stride, a.wpitch, n, r, masks_PI,
                                (uint64_t)syn - (uint64_t)win - (uint64_t)n * stride,
                                (uint64_t)r * stride - a.wpitch, s, masked ? present : nullptr,
                                masked ? (uint32_t)a.nw : 0u);
        } else {
        CombArgs c1{};
        c1.jobs = jobs1;
        c1.coef = P_dev + (size_t)r * k;
        c1.outs = outs1;
        c1.in_base = win;
        c1.out_base = syn;
        c1.njobs = nwin;
        c1.ncol = ncol;
        c1.stride = stride;
        c1.nin_max = k + r;
        c1.nout_max = r;
        c1.job_lds = comb_job_lds(c1.nin_max, kMaxR);
        c1.shared_coef = 1;
        c1.chk.lo[0] = reinterpret_cast<uint64_t>(win);  // FECGPU_CHECK builds: windows in, syndromes out
        c1.chk.n[0] = nwin * a.wpitch;
        c1.chk.lo[1] = reinterpret_cast<uint64_t>(syn);
        c1.chk.n[1] = nwin * (uint64_t)r * stride;
        const uint32_t cap = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kMaxWpb, nwin / 1024));
        const uint32_t room =
            std::min<uint32_t>(kBudget - comb_shared_lds(k + r, kMaxR), cap * comb_job_small_lds(kMaxR));
        c1.wpb = std::max(1, std::min(kMaxWpb, choose_wpb_for(ncol, comb_job_small_lds(kMaxR), room)));
        e = launch_comb(c1, kMaxR, s);
        }
        if (e != hipSuccess) return e;
        // (2) x_u = sum_c T[P_u][c] s_c over the window's r syndromes
        CombArgs c2{};
        c2.jobs = jobs;
        c2.coef = coef;
        c2.outs = outs;
        c2.in_base = syn;
        c2.out_base = win;
        c2.njobs = nwin;
        c2.ncol = ncol;
        c2.stride = stride;
        c2.nin_max = r;
        c2.nout_max = kMaxR;
        c2.job_lds = comb_job_lds(r, kMaxR);
        c2.chk.lo[0] = reinterpret_cast<uint64_t>(syn);  // FECGPU_CHECK builds: syndromes in, windows out
        c2.chk.n[0] = nwin * (uint64_t)r * stride;
        c2.chk.lo[1] = reinterpret_cast<uint64_t>(win);
        c2.chk.n[1] = nwin * a.wpitch;
        c2.wpb = std::max(1, std::min(kMaxWpb, choose_wpb_for(ncol, c2.job_lds, kWideS2Budget)));
        return launch_comb(c2, kMaxR, s);
    }
    CombArgs c{};
    c.jobs = jobs;
    c.coef = P_dev;
    c.outs = outs;
    c.in_base = win;
    c.out_base = win;
    c.xor_base = nullptr;
    c.njobs = nwin;
    c.ncol = ncol;
    c.stride = stride;
    c.nin_max = k;
    c.nout_max = r;
    c.job_lds = comb_job_lds(c.nin_max, kMaxR);
    // every encode job multiplies by the same parity rows: one table block per
    // workgroup, so the jobs per workgroup follow lane use alone (1200-B rows
    // are 75 of a workgroup's 256 lanes)
    c.shared_coef = 1;
    c.chk.lo[0] = reinterpret_cast<uint64_t>(win);  // FECGPU_CHECK builds: the windows, in and out
    c.chk.n[0] = nwin * a.wpitch;
    // at most nwin / 1024 jobs each, so the grid keeps >= 4 workgroups per CU
    const uint32_t cap = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kMaxWpb, nwin / 1024));
    const uint32_t room = std::min<uint32_t>(kBudget - comb_shared_lds(k, kMaxR), cap * comb_job_small_lds(kMaxR));
    c.wpb = std::max(1, std::min(kMaxWpb, choose_wpb_for(ncol, comb_job_small_lds(kMaxR), room)));
    return launch_comb(c, kMaxR, s);
}

}  // namespace fecgpu
