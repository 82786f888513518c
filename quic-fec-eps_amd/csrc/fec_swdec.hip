// fec_swdec.hip — sliding-window RLC decode (RFC 8681, m = 8) planned on the
// device: include/fecgpu.h fecgpu_sw_decode / fecgpu_sw_decode_device
// (DESIGN.md §4b).  No CPU work besides argument
// checks: the receiver's arrival flags and repair headers go to the GPU and
// every step below runs there.
//
//  1. plan (sw_dec_plan_kernel, one launch, decoupled look-back over chunks
//     of sources): statuses, the lost list in stream order, and for each lost
//     source the farthest window end of the received repairs that start at or
//     before it (a system ends where that reach stops short of the next lost
//     source).  The reach array is then reused as rank[i] = lost sources
//     before i, which gives any window's unknown range in two loads.  The
//     one-unknown systems are finished here (a combine job each).
//  2. systems (sw_dec_sys_kernel): a wave per larger system's start.  A
//     system of at most 64 unknowns and 96 equations is solved by that wave:
//     Gauss-Jordan with pivot search on [A | I] in LDS, solve jobs x_u =
//     sum_t T[u][t] s_t for the determined unknowns (also when the system is
//     rank deficient), syndrome jobs only for the rows a solve reads.  A
//     longer system is queued for step 3.
//  3. long systems (sw_dec_long_kernel): a wave per system plans a banded
//     elimination (oracle/fec_sw_banded.c is its CPU statement) into an
//     operation log — forward elimination with the pivot whose range ends
//     first (rows never widen, so at most the repairs covering one source are
//     alive at once), a null-space sweep from the last column down that marks
//     the determined unknowns exactly, and back substitution with the free
//     unknowns at 0.  sw_dec_replay_kernel replays the log over the data, a
//     wave per (system, 256-byte column chunk), rows in LDS.
//  4. data (fec_kernels.hip comb_kernel, sized on the device): syndromes
//     s_t = repair_t + sum of the received sources' terms, then the small
//     systems' solves; then the replay.
#include "fec_internal.h"

namespace fecgpu {

namespace {

__constant__ GfTables c_gfs = make_gf_tables();

#define SWD_WAVE_SYNC()                                         \
    do {                                                        \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                        \
    } while (0)

struct GfLds {
    uint8_t exp[512];
    uint8_t log[256];
};
__device__ __forceinline__ void gf_load(GfLds &g) {
    for (int i = threadIdx.x; i < 512; i += blockDim.x) g.exp[i] = c_gfs.exp[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) g.log[i] = c_gfs.log[i];
}
__device__ __forceinline__ uint32_t gmul(const GfLds &g, uint32_t a, uint32_t b) {
    return (a && b) ? g.exp[g.log[a] + g.log[b]] : 0u;
}
__device__ __forceinline__ uint32_t ginv(const GfLds &g, uint32_t a) { return g.exp[255 - g.log[a]]; }

// four packed bytes times the coefficient of table t (a_lo, a_hi, b_lo, b_hi, c)
__device__ __forceinline__ uint32_t tmul(uint32_t x, const uint32_t (&t)[5]) {
    return __builtin_amdgcn_perm(t[1], t[0], x & 0x07070707u) ^
           __builtin_amdgcn_perm(t[3], t[2], (x >> 3) & 0x07070707u) ^
           __builtin_amdgcn_perm(t[4], t[4], (x >> 6) & 0x03030303u);
}
__device__ __forceinline__ void set_tab(uint32_t (&t)[5], uint32_t c) {
    const CoefTab ct = make_coef_tab(c);
    t[0] = ct.a_lo;
    t[1] = ct.a_hi;
    t[2] = ct.b_lo;
    t[3] = ct.b_hi;
    t[4] = ct.c;
}

__device__ __forceinline__ uint64_t lanes_below(int lane) { return (1ull << lane) - 1ull; }

// FECGPU_CHECK builds: every row, job slot, record and log entry an index
// addresses is checked against its allocation (SwDecArgs sizes); a failing
// access is skipped and recorded in a.chk with its site (the host fails the
// call).  Sites:
enum : uint32_t {
    kChkSynJob = 1,    // syn_jobs / syn_outs / coef rows: nrep + nsrc slots
    kChkSolJob = 2,    // sol_jobs / sol_outs: nsrc + 8 slots
    kChkSolCoef = 3,   // sol_coef bytes: nrep * kSwSmallE
    kChkSrcRow = 4,    // sources (stat, arrival flags, src rows): nsrc
    kChkLost = 5,      // lost list / reachL / lkind / starts: nsrc
    kChkRank = 6,      // reach / rcnt: nsrc + 1
    kChkHdr = 7,       // headers / repair flags / synrow: nrep
    kChkLook = 8,      // look-back records and flags: lb_cap chunks
    kChkLong = 9,      // queued long systems: long_cap
    kChkLog = 10,      // operation log entries: log_cap
    kChkPiv = 11,      // pivot rows (pivcoef / pivhi / pivt / pivdata): piv_cap
    kChkSynRow = 12,   // syndrome rows: nrep
    kChkColumn = 13,   // byte offset within a row: stride
};
#define SWC(i, n, site) CHK_IDX(a.chk, (i), (n), (site))

// a header the plan may act on (fec_sw.cpp header_ok's device twin): a window
// of 1..kSwMaxWindow sources inside the stream, dt <= 15
__device__ __forceinline__ bool hdr_ok(const fecgpu_sw_repair &h, uint64_t nsrc) {
    return h.nss >= 1 && h.nss <= kSwMaxWindow && h.dt <= 15 && h.fss <= nsrc && nsrc - h.fss >= h.nss;
}

// An error of this call (kSwErr* bits), also raised in the ctx's sticky word for
// asynchronous calls (need: the log size an overflow asked for)
__device__ __forceinline__ void dec_err(const SwDecArgs &a, uint32_t bits, unsigned long long need = 0) {
    atomicOr(&a.ctr->err, bits);
    if (a.sticky) {
        atomicOr(&a.sticky->err, bits);
        if (need) atomicMax(&a.sticky->need, need);
    }
}

template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = max(v, (uint32_t)__shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = min(v, (uint32_t)__shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = min(v, (uint64_t)__shfl_xor((unsigned long long)v, o));
    return v;
}

// First header t in [lo, hi) with fss >= key (headers in fss order), by the
// whole wave: 64-ary steps, so three rounds of loads for 2^16 headers.
__device__ uint64_t wave_lower_bound(const fecgpu_sw_repair *h, uint64_t lo, uint64_t hi, uint64_t key, int lane) {
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo + 63) / 64;
        const uint64_t pos = min(lo + (uint64_t)(lane + 1) * step, hi) - 1;  // last of segment `lane`
        const uint64_t b = __ballot(h[pos].fss >= key);
        if (!b) return hi;
        const int f = __ffsll((unsigned long long)b) - 1;
        const uint64_t nlo = lo + (uint64_t)f * step;
        hi = min(lo + (uint64_t)(f + 1) * step, hi);
        lo = nlo;
    }
    const uint64_t pos = lo + (uint64_t)lane;
    const uint64_t b = __ballot(pos < hi && h[pos].fss >= key);
    return b ? lo + (uint64_t)(__ffsll((unsigned long long)b) - 1) : hi;
}
// The same answer starting from a guess g (repairs spread evenly over the
// stream put the answer near key * nrep / nsrc): one round of 64 loads around
// g decides it when the answer lies inside, else the 64-ary search over the
// side it lies on.
__device__ uint64_t wave_lower_bound_near(const fecgpu_sw_repair *h, uint64_t hi, uint64_t key, uint64_t g, int lane) {
    const uint64_t lo = g > 32 ? min(g - 32, hi > 64 ? hi - 64 : 0) : 0;
    const uint64_t pos = lo + (uint64_t)lane;
    const bool in = pos < hi;
    const uint64_t b = __ballot(in && h[pos].fss >= key);
    const bool first_below = !(b & 1ull) || lo == 0;  // lane 0's header is below key (or there is none before it)
    if (b && first_below) return lo + (uint64_t)(__ffsll((unsigned long long)b) - 1);
    if (!b) return lo + 64 >= hi ? hi : wave_lower_bound(h, lo + 64, hi, key, lane);
    return wave_lower_bound(h, 0, lo + 1, key, lane);  // the answer is at or before lo
}

// the repair's window holds one of the lost sources lost[x .. x + e) (rank =
// lost sources before i)
__device__ __forceinline__ bool holds(const SwDecArgs &a, const fecgpu_sw_repair &h, uint32_t x, uint32_t e) {
    const uint32_t r0 = a.reach[h.fss], r1 = a.reach[h.fss + h.nss];
    return r1 > r0 && r0 < x + e && r1 > x;
}

// ================================================== coefficient table ===
// RFC 8681 §3.6 at dt 15 draws every coefficient nonzero, so a repair's window
// takes a prefix of one sequence per repair key: the 65536 sequences are drawn
// once per device (ctx_rlc_table, 16 MiB) and the decode reads a row's words
// instead of stepping TinyMT32 once or more per coefficient.  A thread's chain
// of ~300 dependent generator steps (the key's 15 warm-up steps, the pivot's
// coefficient, then its row again) set the plan kernel's critical path: two
// thirds of it on cfg7 (FECGPU_SWD_TRACE, r04).  Other dt values draw as before.
__global__ __launch_bounds__(kBlock) void rlc_table_kernel(uint8_t *tab) {
    const uint32_t key = blockIdx.x * kBlock + threadIdx.x;
    Tinymt32 st;
    tinymt32_init(st, key);
    uint4 *row = reinterpret_cast<uint4 *>(tab + (size_t)key * kRlcRow);
    for (int q = 0; q < (int)(kRlcRow / 16); q++) {
        uint32_t w[4];
        for (int d = 0; d < 4; d++) {
            w[d] = 0;
            for (int b = 0; b < 4; b++) {
                uint32_t c = 0;
                if (q * 16 + d * 4 + b < kSwMaxWindow) {
                    do {
                        c = tinymt32_u32(st) & 0xFFu;
                    } while (c == 0);
                }
                w[d] |= c << (8 * b);
            }
        }
        row[q] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}
static_assert(kRlcRow == 256 && kSwMaxWindow < (int)kRlcRow, "a table row holds a window's coefficients");

__device__ __forceinline__ const uint4 *rlc_row(const SwDecArgs &a, const fecgpu_sw_repair &h) {
    return a.rlc && h.dt == 15 ? reinterpret_cast<const uint4 *>(a.rlc + (size_t)h.key * kRlcRow) : nullptr;
}

// f(q, w) for the words q < ceil(nss / 4) of the window's coefficients, 4 per
// word (bytes past nss zero); from the table 64 coefficients per round trip
template <class F>
__device__ __forceinline__ void rlc_words(const SwDecArgs &a, const fecgpu_sw_repair &h, F f) {
    const uint32_t nss = h.nss, nw = (nss + 3u) >> 2;
    if (const uint4 *row = rlc_row(a, h)) {
        for (uint32_t g = 0; g * 16 < nw; g++) {  // g <= 3: the row's 16 uint4 are in bounds
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = row[g * 4 + k];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                for (int d = 0; d < 4; d++) {
                    const uint32_t q = g * 16 + k * 4 + d;
                    if (q < nw) {
                        uint32_t w = w4[d];
                        if (q == nw - 1 && (nss & 3u)) w &= (1u << (8 * (nss & 3u))) - 1u;
                        f(q, w);
                    }
                }
            }
        }
        return;
    }
    Tinymt32 st;
    tinymt32_init(st, h.key);
    const uint32_t dt = h.dt;
    uint32_t word = 0;
    for (uint32_t j = 0; j < nss; j++) {
        uint32_t c = 0;
        if (dt == 15 || (tinymt32_u32(st) & 0xFu) <= dt) {
            do {
                c = tinymt32_u32(st) & 0xFFu;
            } while (c == 0);
        }
        word |= c << (8 * (j & 3));
        if ((j & 3) == 3) {
            f(j >> 2, word);
            word = 0;
        }
    }
    if (nss & 3u) f(nss >> 2, word);
}

// f(g, v) for the window's coefficients 16 at a time (uint4 g < ceil(nss /
// 16), bytes past nss zero): rows go out as 16-B stores (the 4-B ones of
// rlc_words, 64 lanes on 64 rows, were most of the plan's store time)
// quad g of a coefficient row with bytes past nss zero
__device__ __forceinline__ uint4 quad_tail(uint32_t g, uint4 v, uint32_t nss) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const uint32_t b0 = g * 16 + d * 4;  // first byte of word d
        if (b0 >= nss) w[d] = 0;
        else if (nss - b0 < 4) w[d] &= (1u << (8 * (nss - b0))) - 1u;
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}
template <class F>
__device__ __forceinline__ void rlc_quads(const SwDecArgs &a, const fecgpu_sw_repair &h, F f) {
    const uint32_t nss = h.nss, ng = (nss + 15u) >> 4;
    const auto tail = [&](uint32_t g, uint4 v) { return quad_tail(g, v, nss); };
    if (const uint4 *row = rlc_row(a, h)) {
        for (uint32_t g0 = 0; g0 < ng; g0 += 4) {  // four loads in flight
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = row[min(g0 + k, kRlcRow / 16 - 1)];
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (g0 + k < ng) f(g0 + k, tail(g0 + k, v[k]));
        }
        return;
    }
    uint32_t w[4] = {0, 0, 0, 0};
    rlc_words(a, h, [&](uint32_t q, uint32_t x) {
        w[q & 3] = x;
        if ((q & 3) == 3 || q == ((nss + 3u) >> 2) - 1) {
            f(q >> 2, tail(q >> 2, make_uint4(w[0], w[1], w[2], w[3])));
            w[0] = w[1] = w[2] = w[3] = 0;
        }
    });
}

// The window's coefficients one at a time (next(j) for j = 0, 1, ... in
// order); from the table 16 per load, the next 16 loaded ahead
struct RlcSeq {
    const uint4 *row;
    uint4 cur, nxt;
    Tinymt32 st;
    uint32_t dt;
    __device__ __forceinline__ RlcSeq(const SwDecArgs &a, const fecgpu_sw_repair &h) : row(rlc_row(a, h)), dt(h.dt) {
        if (row) {
            cur = row[0];
            nxt = row[1];
        } else {
            tinymt32_init(st, h.key);
        }
    }
    __device__ __forceinline__ uint32_t next(uint32_t j) {
        if (row) {
            if (j && (j & 15u) == 0) {
                cur = nxt;
                nxt = row[min((j >> 4) + 1u, kRlcRow / 16 - 1)];
            }
            const uint32_t q = (j >> 2) & 3u;
            const uint32_t w = q == 0 ? cur.x : q == 1 ? cur.y : q == 2 ? cur.z : cur.w;
            return (w >> (8 * (j & 3))) & 0xFFu;
        }
        uint32_t c = 0;
        if (dt == 15 || (tinymt32_u32(st) & 0xFu) <= dt) {
            do {
                c = tinymt32_u32(st) & 0xFFu;
            } while (c == 0);
        }
        return c;
    }
};

// ============================================================= systems ===
// Small systems are solved by one wave each with [A | I] in LDS: "tiny" ones
// (e <= 16, p <= 48) in the wave's own 3 KB, larger ones (e <= 64, p <= 96)
// in one of the block's shared mid-size regions, taken under an LDS lock.
// Syndrome job / row of equation t: slot t (the plan empties every slot); a
// system's solve reads its syndrome rows t_first ..
// t_last (the repairs in between that are not its equations get coefficient
// 0: the ranges of two systems never interleave, since a repair between two
// equations of one system that held a lost source of another would link them).
constexpr int kSwTinyE = 16, kSwTinyP = 48;
constexpr int kSwSolveIn = 128;  // widest syndrome range a small system's solve reads

template <int ME, int MP>
struct SysLds {
    static constexpr int kPitch = ME + MP;
    uint8_t M[MP * kPitch];
    uint32_t U[ME];
    uint32_t eq[MP];
    uint64_t efss[MP];  // the equations' windows, kept from the candidate scan
    uint16_t enss[MP];
    int8_t piv[ME];
};

__device__ __forceinline__ int d_of(uint64_t dm, int lane) { return __popcll(dm & lanes_below(lane)); }

// One wave solves the small system lost[x .. x + e) with its p equations
// (repair indices eq[], ascending): the round-2 sw_plan_kernel, fed on the
// device.  Returns the unknowns it determined; *nin the solve's input rows.
template <int ME, int MP>
__device__ int small_solve(const SwDecArgs &a, const GfLds &g, uint32_t x, int e, int p, SysLds<ME, MP> &S,
                           int lane, uint32_t *nin_out) {
    constexpr int kPitch = SysLds<ME, MP>::kPitch;
    uint8_t *M = S.M;
    const uint32_t *U = S.U, *eq = S.eq;
    const int W = e + p, W4 = (W + 3) / 4;  // row bytes, dwords
    for (int q = 0; q < p; q++)
        for (int j = lane; j < 4 * W4; j += 64) M[q * kPitch + j] = (uint8_t)(j >= e && j - e == q);
    SWD_WAVE_SYNC();
    // lane per equation: its coefficients (RFC 8681 §3.6); the lost sources'
    // go into A, the received sources' into its syndrome job
    for (int q = lane; q < p; q += 64) {
        const uint32_t t = eq[q];
        if (!SWC(t, a.nrep, kChkHdr)) continue;
        fecgpu_sw_repair h{};  // (the scan's copy: fss and nss)
        h.fss = S.efss[q];
        h.nss = S.enss[q];
        {
            // the row was drawn by the plan: move the unknowns' entries into A
            // (the unknowns are ascending; the window holds a run of them).
            // (Reading dense rows from the table here instead, with the
            // unknowns zeroed as the row goes out, cost the system pass 23 us
            // on cfg7, r04: serial LDS lookups per coefficient.)
            uint8_t *cb = a.coef + (uint64_t)t * kSwCoefPitch;
            for (int u = 0; u < e; u++) {
                const uint64_t i = U[u];
                if (i < h.fss) continue;
                if (i >= h.fss + h.nss) break;
                if (!SWC(i - h.fss, kSwCoefPitch, kChkSynJob)) break;
                M[q * kPitch + u] = cb[i - h.fss];
                cb[i - h.fss] = 0;
            }
        }
        CombJob J;
        J.in_off = h.fss * a.stride;
        J.coef_off = (uint64_t)t * kSwCoefPitch;
        J.out_list = t;
        J.xor_off = (uint64_t)t * a.stride;
        J.nin = h.nss;
        J.nout = 1;
        a.syn_jobs[t] = J;
        a.syn_outs[t] = (uint64_t)t * a.stride;
    }
    SWD_WAVE_SYNC();
    uint64_t used0 = 0, used1 = 0;  // wave-uniform: rows 0..63, 64..127 already pivots
    for (int col = 0; col < e; col++) {
        const bool c0 = lane < p && !((used0 >> lane) & 1) && M[lane * kPitch + col] != 0;
        const bool c1 = MP > 64 && lane + 64 < p && !((used1 >> lane) & 1) && M[(lane + 64) * kPitch + col] != 0;
        const uint64_t b0 = __ballot(c0), b1 = __ballot(c1);
        int pr = -1;
        if (b0) pr = (int)__ffsll((unsigned long long)b0) - 1;
        else if (b1) pr = 64 + (int)__ffsll((unsigned long long)b1) - 1;
        if (lane == 0) S.piv[col] = (int8_t)pr;
        if (pr < 0) continue;  // free column (uniform)
        if (pr < 64) used0 |= 1ull << pr;
        else used1 |= 1ull << (pr - 64);
        // rows as dwords: a multiply is one split-table product per 4 bytes
        uint8_t *P = M + pr * kPitch;
        uint32_t *Pw = reinterpret_cast<uint32_t *>(P);
        const uint32_t iv = ginv(g, P[col]);
        SWD_WAVE_SYNC();
        {
            uint32_t tab[5];
            set_tab(tab, iv);
            for (int j = lane; j < W4; j += 64) Pw[j] = tmul(Pw[j], tab);
        }
        SWD_WAVE_SYNC();
        for (int q = lane; q < p; q += 64) {
            if (q == pr) continue;
            uint32_t *row = reinterpret_cast<uint32_t *>(M + q * kPitch);
            const uint32_t f = M[q * kPitch + col];
            if (!f) continue;
            uint32_t tab[5];
            set_tab(tab, f);
            for (int j = 0; j < W4; j++) row[j] ^= tmul(Pw[j], tab);
        }
        SWD_WAVE_SYNC();
    }
    SWD_WAVE_SYNC();
    bool det = false;
    int prc = -1;
    if (lane < e) {
        prc = S.piv[lane];
        det = prc >= 0;
        for (int j = 0; j < e && det; j++)
            if (S.piv[j] < 0 && M[prc * kPitch + j]) det = false;
    }
    const uint64_t dm = __ballot(det);
    const int ndet = __popcll(dm);
    // syndromes no solve reads (non-pivot rows, undetermined unknowns' rows)
    // are not computed: only pivot rows can appear in a solve row
    for (int q = lane; q < p; q += 64) {
        bool need = false;
        for (int col = 0; col < e && !need; col++) need = ((dm >> col) & 1) && M[S.piv[col] * kPitch + e + q] != 0;
        if (!need && SWC(eq[q], a.nrep, kChkSynJob)) a.syn_jobs[eq[q]].nout = 0;
    }
    if (ndet == 0) return 0;
    // One unknown (most systems at low loss): x = s_t / c for the pivot
    // equation t, s_t = repair_t + sum of its received sources' terms.  Its
    // syndrome job computes x directly: coefficients times 1/c, the repair row
    // times 1/c (kCombXorScaled), output the lost source's row.  No syndrome
    // row, no solve job.  Nothing else reads that row with a nonzero
    // coefficient: a received repair holding it is an equation of this system.
    if (e == 1) {
        const int pr = S.piv[0];
        const uint32_t t = eq[pr];
        const uint32_t iv = M[pr * kPitch + e + pr];  // T[pr][pr] = 1 / c
        if (!SWC(t, a.nrep, kChkSynJob) || !SWC(U[0], a.nsrc, kChkSrcRow)) return 0;
        const uint32_t nss = S.enss[pr];
        uint32_t *cc = reinterpret_cast<uint32_t *>(a.coef + (uint64_t)t * kSwCoefPitch);
        uint32_t tab[5];
        set_tab(tab, iv);
        for (uint32_t j = lane; j < (nss + 3) / 4; j += 64) cc[j] = tmul(cc[j], tab);
        SWD_WAVE_SYNC();
        if (lane == 0) {
            a.coef[(uint64_t)t * kSwCoefPitch + nss] = (uint8_t)iv;  // nss < kSwCoefPitch
            a.syn_jobs[t].nout = 1u | kCombXorScaled;
            a.syn_outs[t] = (uint64_t)(a.src + (uint64_t)U[0] * a.stride) - (uint64_t)a.synd;
            a.stat[U[0]] = FECGPU_STATUS_OK;
        }
        return 1;
    }
    // solve jobs (ndet <= e): inputs the syndrome rows t_first .. t_last,
    // coefficients at 64 bytes per repair from t_first (ndet <= 64, so
    // ndet * nin fits), kSwSolveOut outputs per job, in the system's unknown
    // slots x .. (outputs at x + d; a compact list of jobs, one atomic per
    // system, measured 24 us slower on cfg7, r04)
    const uint32_t t_first = eq[0], nin = eq[p - 1] - t_first + 1;
    const uint64_t c0 = (uint64_t)t_first * kSwSmallE;
    const uint64_t o0 = x, j0 = x;
    if (det && SWC(c0 + (uint64_t)(d_of(dm, lane) + 1) * nin - 1, (uint64_t)a.nrep * kSwSmallE, kChkSolCoef) &&
        SWC(o0 + d_of(dm, lane), a.nsrc + 8, kChkSolJob) && SWC(U[lane], a.nsrc, kChkSrcRow)) {
        const int d = __popcll(dm & lanes_below(lane));
        uint8_t *cf = a.sol_coef + c0 + (uint64_t)d * nin;
        int q = 0;
        for (uint32_t r = 0; r < nin; r++) {
            uint8_t v = 0;
            if (q < p && eq[q] == t_first + r) v = M[prc * kPitch + e + q++];
            cf[r] = v;
        }
        a.sol_outs[o0 + d] = (uint64_t)U[lane] * a.stride;
        a.stat[U[lane]] = FECGPU_STATUS_OK;
    }
    const int nj = (ndet + kSwSolveOut - 1) / kSwSolveOut;
    if (lane < nj && SWC(j0 + lane, a.nsrc + 8, kChkSolJob)) {
        CombJob J;
        J.in_off = (uint64_t)t_first * a.stride;
        J.coef_off = c0 + (uint64_t)lane * kSwSolveOut * nin;
        J.out_list = o0 + (uint64_t)lane * kSwSolveOut;
        J.xor_off = kNoXor;
        J.nin = nin;
        J.nout = (uint32_t)min(kSwSolveOut, ndet - kSwSolveOut * lane);
        a.sol_jobs[j0 + lane] = J;
    }
    *nin_out = nin;
    return ndet;
}

// The system lost[x .. x + e) with candidate repairs [t_lo, t_hi): solved here
// when its equations fit ME / MP (and the range of syndrome rows kSwSolveIn),
// else queued for the long pass.  LOCAL: a system too large for ME / MP but
// within the mid size (kSwSmallE) is not queued; the call returns true and the
// caller solves it in its workgroup's shared mid region.
template <int ME, int MP, bool LOCAL = false>
__device__ bool sys_one(const SwDecArgs &a, const GfLds &g, SysLds<ME, MP> &S, uint32_t x, uint32_t e,
                        uint64_t t_lo, uint64_t t_hi, int lane, uint32_t &rec, uint32_t &maxin) {
    bool fits = (int)e <= ME && (int)e < a.long_min;
    uint32_t p = 0;
    if (fits) {
        // the unknowns' positions load beside the candidate scan's first loads;
        // a candidate's arrival flag and header in one round trip (clamped index)
        const uint32_t ux = lane < (int)e && SWC(x + lane, a.nsrc, kChkLost) ? a.lost[x + lane] : 0u;
        for (uint64_t t0 = t_lo; t0 < t_hi; t0 += 64) {
            const uint64_t t = t0 + lane, tc = min(t, t_hi - 1);
            const uint8_t rp = a.rep_present[tc];
            const fecgpu_sw_repair h = a.hdr[tc];
            const bool hd = t < t_hi && rp && holds(a, h, x, e);
            const uint64_t b = __ballot(hd);
            const uint32_t n = __popcll(b);
            if (p + n > (uint32_t)MP) {
                fits = false;
                break;
            }
            if (hd) {
                const uint32_t q = p + __popcll(b & lanes_below(lane));
                S.eq[q] = (uint32_t)t;
                S.efss[q] = h.fss;
                S.enss[q] = h.nss;
            }
            p += n;
        }
        if (lane < (int)e) S.U[lane] = ux;
        SWD_WAVE_SYNC();
        if (fits && p && S.eq[p - 1] - S.eq[0] + 1 > (uint32_t)kSwSolveIn) fits = false;
    }
    if (!fits) {
        if (LOCAL && (int)e <= kSwSmallE && (int)e < a.long_min) return true;
        if (lane == 0) {
            const uint32_t k = atomicAdd(&a.ctr->nlong, 1u);
            if (k < a.long_cap) {  // (the capacity test is the check: a full queue is kSwErrCapacity)
                SwLong L{};
                L.x0 = x;
                L.e = e;
                L.t_lo = (uint32_t)t_lo;
                L.t_hi = (uint32_t)t_hi;
                a.longs[k] = L;
            } else {
                dec_err(a, kSwErrCapacity);
            }
        }
        return false;
    }
    if (p == 0) return false;  // no received repair holds it: stays lost
    uint32_t nin = 0;
    const int nd = small_solve<ME, MP>(a, g, x, (int)e, (int)p, S, lane, &nin);
    rec += (uint32_t)nd;
    if (nd) maxin = max(maxin, nin);
    return false;
}

// The block's recovered count and widest solve into the call's counters: one
// atomic each per block (same-address atomics from every wave serialised at
// the L2 and cost more than the systems themselves).
__device__ __forceinline__ void block_counts(const SwDecArgs &a, uint32_t rec, uint32_t maxin, int lane, int wave) {
    __shared__ uint32_t s_rec[kBlock / 64], s_in[kBlock / 64];
    if (lane == 0) {
        s_rec[wave] = rec;
        s_in[wave] = maxin;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t r = 0, m = 0;
        for (int w = 0; w < kBlock / 64; w++) {
            r += s_rec[w];
            m = max(m, s_in[w]);
        }
        if (r) atomicAdd(&a.ctr->recovered, r);
        if (m) atomicMax(&a.ctr->maxin, m);
    }
}

// The RFC 8681 coefficients of a received repair whose window holds a lost
// source, into its syndrome coefficient row (the plan, a thread per repair).
// The system pass then reads them (small_solve moves the unknowns' entries
// into A and zeroes them): every lane of a wave draws one, instead of a wave
// per system drawing its few equations' on as many lanes.  The long-system
// pass draws its own rows again (and overwrites these).
__device__ __forceinline__ void draw_row(const SwDecArgs &a, uint64_t t, const fecgpu_sw_repair &h) {
    if (!SWC(t, a.nrep, kChkSynJob)) return;
    uint4 *cc = reinterpret_cast<uint4 *>(a.coef + t * kSwCoefPitch);
    rlc_quads(a, h, [&](uint32_t g, uint4 v) { cc[g] = v; });
}

// ======================================================= fused plan ===
// One launch for the whole plan: a block per chunk of
// kPlanChunk sources, in ticket order, chained by a decoupled look-back over
// (lost sources, farthest reach, repairs, widest window | error bits) so no
// pass waits for a separate scan.  Per chunk: its repairs' header range (the
// headers are in fss order; every block also checks its share of headers, so a
// bad or unordered list raises kSwErrHeader and the later kernels stand down),
// reach / repair counts in LDS, statuses, the lost list with its prefix-max
// reach, rank / repfirst, empty job slots, and the RFC 8681 coefficient rows of
// the chunk's received repairs that hold a lost source (a 255-source halo of
// arrival flags past the chunk answers that locally).  The last chunk writes
// the call's counters, so nothing is cleared before the launch.
constexpr int kPlanChunk = kSwPlanChunk;
constexpr int kPlanPer = kPlanChunk / kBlock;  // sources per thread
constexpr int kPlanHalo = 256;                 // >= kSwMaxWindow
static_assert(kPlanPer == 8, "the per-thread source loads are 8 bytes");
constexpr uint32_t kLbAgg = 1u, kLbInc = 2u;
constexpr int kPlanHdr = 512;  // headers cached per chunk (cfg7: 288 from tb to t1)

// lost sources, max reach, repairs, widest window | error bits << 16, and the
// reach at the last lost source (prefix max of reach up to it: its reachL)
struct LbRec {
    uint32_t lost, reach, rep, wme, L;
};
__device__ __forceinline__ LbRec lb_join(const LbRec &x, const LbRec &y) {  // x before y
    LbRec r;
    r.lost = x.lost + y.lost;
    r.reach = max(x.reach, y.reach);
    r.rep = x.rep + y.rep;
    r.wme = max(x.wme & 0xFFFFu, y.wme & 0xFFFFu) | ((x.wme | y.wme) & 0xFFFF0000u);
    r.L = y.lost ? max(x.reach, y.L) : x.L;
    return r;
}
__device__ __forceinline__ uint32_t lb_flag_load(const uint32_t *f) {
    return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
// records are two uint4 per chunk (lb_agg / lb_inc [2 * chunk]; kLbRecBytes)
static_assert(kLbRecBytes == 2 * sizeof(uint4), "look-back record size");
__device__ __forceinline__ void lb_publish(const SwDecArgs &a, uint32_t c, const LbRec &r, uint32_t state) {
    if (!SWC(c, a.lb_cap, kChkLook)) return;
    uint32_t *dst = reinterpret_cast<uint32_t *>((state == kLbInc ? a.lb_inc : a.lb_agg) + 2 * (size_t)c);
    const uint32_t v[5] = {r.lost, r.reach, r.rep, r.wme, r.L};
#pragma unroll
    for (int i = 0; i < 5; i++) __hip_atomic_store(dst + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&a.lb_flag[c], (a.epoch << 2) | state, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ LbRec lb_read(const uint4 *src2) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(src2);
    uint32_t v[5];
#pragma unroll
    for (int i = 0; i < 5; i++) v[i] = __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return LbRec{v[0], v[1], v[2], v[3], v[4]};
}

// One-unknown systems (most of them at low loss) are finished here too: the
// lost source x at position i is alone in its system iff the reach of the
// sources up to the previous lost source stops at or before i and its own
// reach stops at or before the next lost source (the halo shows whether there
// is one within 255 sources).  Its pivot is the first received repair t
// holding it with a nonzero coefficient there (the small solver's choice), and
// x = s_t / c: a combine job in syndrome slot nrep + (x's lost index) over t's
// window with the coefficients times 1/c and t's row times 1/c (as
// small_solve's one-unknown case).  lkind[x] tells the system pass what is left: 0 a member
// of a larger system, 1 recovered here, 2 a larger system's first unknown,
// 3 alone but undetermined.
__device__ __forceinline__ uint8_t coef_at(const SwDecArgs &a, const fecgpu_sw_repair &h, uint32_t j) {
    // RFC 8681 coefficient j
    if (const uint4 *row = rlc_row(a, h)) return reinterpret_cast<const uint8_t *>(row)[j];
    Tinymt32 st;
    tinymt32_init(st, h.key);
    const uint32_t dt = h.dt;
    uint32_t c = 0;
    for (uint32_t q = 0; q <= j; q++) {
        c = 0;
        if (dt == 15 || (tinymt32_u32(st) & 0xFu) <= dt) {
            do {
                c = tinymt32_u32(st) & 0xFFu;
            } while (c == 0);
        }
    }
    return (uint8_t)c;
}

#ifndef FECGPU_SWD_TRACE
#define FECGPU_SWD_TRACE 0  // measurement aid: the plan kernel prints its phases' times (3 blocks)
#endif
#if FECGPU_SWD_TRACE
#define SWD_TRACE(n)                                   \
    do {                                               \
        if (threadIdx.x == 0) s_tr[n] = wall_clock64(); \
    } while (0)
#else
#define SWD_TRACE(n) \
    do {             \
    } while (0)
#endif
__global__ __launch_bounds__(kBlock) void sw_dec_plan_kernel(SwDecArgs a) {
#if FECGPU_SWD_TRACE
    __shared__ unsigned long long s_tr[16];
    if (threadIdx.x == 0) s_tr[0] = wall_clock64();
#endif
    __shared__ uint32_t s_reach[kPlanChunk], s_rcnt[kPlanChunk];
    __shared__ uint32_t s_lpos[kPlanChunk], s_rl[kPlanChunk];  // per local lost source: position, reachL
    // per local lost source that may be alone: its pivot repair (~0: none), key | nss << 16 | j << 24,
    // coefficient | dt << 8
    __shared__ uint2 s_pv[kPlanChunk];
    __shared__ uint16_t s_pcd[kPlanChunk];
    __shared__ uint32_t s_rf[kPlanChunk + 1];                  // repfirst of the chunk's sources (and of i1)
    __shared__ uint32_t s_rcb[kPlanHalo], s_rfb[kPlanHalo];    // repairs starting in [i0 - 256, i0), repfirst there
    __shared__ uint32_t s_bits[(kPlanChunk + kPlanHalo) / 32];      // lost flags, chunk + halo
    __shared__ uint32_t s_wpfx[(kPlanChunk + kPlanHalo) / 32 + 1];  // lost before each word
    __shared__ uint32_t s_c[kBlock / 64], s_m[kBlock / 64], s_r[kBlock / 64], s_w[kBlock / 64];
    __shared__ uint32_t s_lh[kBlock / 64], s_lv[kBlock / 64];
    // the headers [tb, tb + kPlanHdr) and their arrival flags, cached by the
    // reach pass for the row draws and pivot searches (one global round trip
    // less each; later headers are read from global memory)
    __shared__ fecgpu_sw_repair s_hc[kPlanHdr];
    __shared__ uint8_t s_hp[kPlanHdr];
    __shared__ uint32_t s_chunk, s_bad, s_wmb;
    __shared__ uint32_t s_nst, s_nsg, s_stbase;  // the chunk's larger-system starts, singles recovered
    __shared__ uint64_t s_t0, s_t1, s_tb;
    __shared__ LbRec s_excl, s_agg;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nch = (uint32_t)((a.nsrc + kPlanChunk - 1) / kPlanChunk);
    if (!SWC(nch - 1, a.lb_cap, kChkLook)) return;  // (uniform: the look-back state must hold every chunk)
    if (tid == 0) {
        // chunks in dispatch order, so the look-back never waits on a block not
        // yet running (the counter starts every launch at 0; modulo: a counter
        // left behind by an aborted launch still hands out each chunk once)
        s_chunk = atomicAdd(&a.lb_ticket[0], 1u) % nch;
        s_bad = 0;
        s_wmb = 0;
        s_nst = 0;
        s_nsg = 0;
    }
    for (int i = tid; i < kPlanChunk; i += kBlock) {
        s_reach[i] = 0;
        s_rcnt[i] = 0;
    }
    s_rcb[tid] = 0;
    __syncthreads();
    SWD_TRACE(1);
    const uint32_t c = s_chunk;
    const uint64_t i0 = (uint64_t)c * kPlanChunk, i1 = min(i0 + kPlanChunk, a.nsrc);
    const uint64_t ib = i0 >= (uint64_t)kPlanHalo ? i0 - kPlanHalo : 0;  // back region [ib, i0)
    // the arrival flags' loads first (no dependence on the headers, so they are
    // in flight with the searches' first round): 8 sources per thread, and the
    // halo past the chunk (8 flags per lane of wave 0's lanes 0-31, full chunks only)
    const uint32_t n = (uint32_t)(i1 - i0), my0 = (uint32_t)tid * kPlanPer;
    // 8-byte flag loads / status stores where both arrays allow (caller pointers)
    const bool vec = ((reinterpret_cast<uintptr_t>(a.src_present) | reinterpret_cast<uintptr_t>(a.stat)) & 7u) == 0;
    const bool fast = vec && my0 + kPlanPer <= n;
    const bool hl = wave == 0 && lane < kPlanHalo / 8 && n == (uint32_t)kPlanChunk;
    const uint64_t hh0 = i1 + (uint64_t)lane * 8;
    const bool hfast = hl && vec && hh0 + 8 <= a.nsrc;  // one 8-byte load (the chunk is 8-aligned)
    uint2 pv = make_uint2(0, 0), hpv = make_uint2(0, 0);
    if (fast) pv = *reinterpret_cast<const uint2 *>(a.src_present + i0 + my0);
    if (hfast) hpv = *reinterpret_cast<const uint2 *>(a.src_present + hh0);
    // the chunk's repairs (fss in [i0, i1)) and those of the back region: three
    // searches, a wave each, from the even-spread guess (one round of loads when
    // the repairs are spread evenly).  Chunk c's range ends where chunk c + 1's
    // begins (the same search), so the ranges cover every header whatever the
    // list holds (t1 = max(t0, search(i1)): the first chunk at or before a
    // header whose range starts at or before it holds it)
    if (wave < 3) {
        const uint64_t key = wave == 0 ? i0 : wave == 1 ? i1 : ib;
        const uint64_t g = (uint64_t)(((unsigned __int128)key * a.nrep) / max<uint64_t>(a.nsrc, 1));
        const uint64_t t = (wave == 1 && i1 == a.nsrc) ? a.nrep : wave_lower_bound_near(a.hdr, a.nrep, key, g, lane);
        if (lane == 0) (wave == 0 ? s_t0 : wave == 1 ? s_t1 : s_tb) = t;
    }
    uint32_t lostm = 0;  // bit j: source i0 + my0 + j lost
    if (fast) {
        uint2 st;
        for (int j = 0; j < 8; j++) {
            const uint32_t byte = ((j < 4 ? pv.x : pv.y) >> (8 * (j & 3))) & 0xFFu;
            lostm |= (byte == 0 ? 1u : 0u) << j;
        }
        st.x = ((lostm & 1u) ? 1u : 0u) | ((lostm & 2u) ? 1u << 8 : 0u) | ((lostm & 4u) ? 1u << 16 : 0u) |
               ((lostm & 8u) ? 1u << 24 : 0u);
        st.y = ((lostm & 16u) ? 1u : 0u) | ((lostm & 32u) ? 1u << 8 : 0u) | ((lostm & 64u) ? 1u << 16 : 0u) |
               ((lostm & 128u) ? 1u << 24 : 0u);
        *reinterpret_cast<uint2 *>(a.stat + i0 + my0) = st;  // FECGPU_STATUS_UNRECOVERABLE = 1 when lost
    } else {
        for (uint32_t j = 0; my0 + j < n && j < kPlanPer; j++) {
            const bool lost = a.src_present[i0 + my0 + j] == 0;
            lostm |= (lost ? 1u : 0u) << j;
            a.stat[i0 + my0 + j] = lost ? FECGPU_STATUS_UNRECOVERABLE : FECGPU_STATUS_OK;
        }
    }
    {  // the chunk's bits: 4 threads per word
        const uint32_t sh = (uint32_t)(tid & 3) * 8u;
        uint32_t wv = lostm << sh;
        wv |= __shfl_xor(wv, 1);
        wv |= __shfl_xor(wv, 2);
        if ((tid & 3) == 0) s_bits[tid >> 2] = wv;
    }
    if (wave == 0) {  // halo words, 4 lanes per word
        uint32_t hw = 0;
        if (hl) {
            uint32_t m8 = 0;
            if (hfast) {
                for (int j = 0; j < 8; j++) m8 |= ((((j < 4 ? hpv.x : hpv.y) >> (8 * (j & 3))) & 0xFFu) == 0 ? 1u : 0u) << j;
            } else {
                for (int j = 0; j < 8; j++) m8 |= (hh0 + j < a.nsrc && a.src_present[hh0 + j] == 0 ? 1u : 0u) << j;
            }
            hw = m8 << ((lane & 3) * 8);
        }
        hw |= __shfl_xor(hw, 1);  // the whole wave takes part in the shuffles
        hw |= __shfl_xor(hw, 2);
        if (hl && (lane & 3) == 0) s_bits[kPlanChunk / 32 + (lane >> 2)] = hw;
    }
    if (n < (uint32_t)kPlanChunk) {  // last chunk (nothing past nsrc): clear the tail words
        for (uint32_t w = tid; w < (kPlanChunk + kPlanHalo) / 32; w += kBlock)
            if (w * 32 >= ((n + 31) & ~31u)) s_bits[w] = 0;
    }
    __syncthreads();
    SWD_TRACE(2);
    const uint64_t t0 = s_t0, t1 = max(s_t0, s_t1), tb = min(s_tb, t0);
    // reach / repair counts of the chunk's sources and the back region's
    // repair counts; the widest received window among them (pivot searches);
    // and, for the chunk's own range [t0, t1), the header checks (a bad or
    // unordered list raises kSwErrHeader) and emptying the syndrome job slots
    // (every slot, whatever the headers hold: the syndrome pass walks them all)
    uint32_t wm = 0, wmb = 0;
    bool bad = false;
    CombJob E0{};
    E0.xor_off = kNoXor;
    for (uint64_t t = tb + tid; t < t1; t += kBlock) {
        if (!SWC(t, a.nrep, kChkSynJob)) break;
        const fecgpu_sw_repair h = a.hdr[t];
        const uint8_t rpb = a.rep_present[t];
        const bool rp = rpb != 0;
        if (t - tb < (uint64_t)kPlanHdr) {
            s_hc[t - tb] = h;
            s_hp[t - tb] = rpb;
        }
        if (t >= t0) {
            a.syn_jobs[t] = E0;
            bad |= !hdr_ok(h, a.nsrc);
            if (t > 0 && a.hdr[t - 1].fss > h.fss) bad = true;
        }
        if (h.nss < 1 || h.nss > kSwMaxWindow) continue;
        if (h.fss >= i0 && h.fss < i1) {
            atomicAdd(&s_rcnt[h.fss - i0], 1u);
            if (rp) {
                wm = max(wm, (uint32_t)h.nss);
                atomicMax(&s_reach[h.fss - i0], (uint32_t)(h.fss + h.nss));
            }
        } else if (h.fss >= ib && h.fss < i0) {
            atomicAdd(&s_rcb[h.fss - (i0 - kPlanHalo)], 1u);
        }
        if (rp) wmb = max(wmb, (uint32_t)h.nss);
    }
    if (__ballot(bad) && lane == 0) s_bad = 1;
    wmb = wave_max(wmb);
    if (lane == 0 && wmb) atomicMax(&s_wmb, wmb);
    __syncthreads();
    SWD_TRACE(3);
    // per thread: its 8 sources' lost count, max reach, repair count
    uint32_t cnt = __popc(lostm), tm = 0, tr = 0;
    for (int j = 0; j < kPlanPer; j++)
        if (my0 + j < n) {
            tm = max(tm, s_reach[my0 + j]);
            tr += s_rcnt[my0 + j];
        }
    uint32_t ic = cnt, im = tm, ir = tr;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(ic, o), ym = __shfl_up(im, o), yr = __shfl_up(ir, o);
        if (lane >= o) {
            ic += y;
            im = max(im, ym);
            ir += yr;
        }
    }
    uint32_t em = __shfl_up(im, 1);
    if (lane == 0) em = 0;
    wm = wave_max(wm);
    if (lane == 63) {
        s_c[wave] = ic;
        s_m[wave] = im;
        s_r[wave] = ir;
    }
    if (lane == 0) s_w[wave] = wm;
    // lost before each word of the chunk + halo (the coefficient pass's window test)
    if (wave == 0) {
        constexpr int NW = (kPlanChunk + kPlanHalo) / 32;
        uint32_t carry = 0;
        for (int w0 = 0; w0 < NW; w0 += 64) {
            const uint32_t v = w0 + lane < NW ? __popc(s_bits[w0 + lane]) : 0u;
            uint32_t x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o);
                if (lane >= o) x += y;
            }
            if (w0 + lane < NW) s_wpfx[w0 + lane] = carry + x - v;
            carry += __shfl(x, 63);
        }
        if (lane == 0) s_wpfx[NW] = carry;
    } else if (wave == 1) {  // repfirst over the back region: tb + repairs starting before each source
        uint32_t carry = (uint32_t)tb;
        for (int q0 = 0; q0 < kPlanHalo; q0 += 64) {
            const uint32_t v = s_rcb[q0 + lane];
            uint32_t x = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o);
                if (lane >= o) x += y;
            }
            s_rfb[q0 + lane] = carry + x - v;
            carry += __shfl(x, 63);
        }
    }
    __syncthreads();
    SWD_TRACE(4);
    uint32_t wc = 0, wmx = 0, wr = 0;
    for (int w = 0; w < wave; w++) {
        wc += s_c[w];
        wmx = max(wmx, s_m[w]);
        wr += s_r[w];
    }
    {  // the chunk-local reachL of the last lost source (the look-back's L)
        uint32_t run = max(wmx, em), myl = 0;
        bool has = false;
        for (int j = 0; j < kPlanPer; j++)
            if (my0 + j < n) {
                run = max(run, s_reach[my0 + j]);
                if ((lostm >> j) & 1u) {
                    myl = run;
                    has = true;
                }
            }
        const uint64_t hb = __ballot(has);  // uniform: the last lane holding a lost source
        const uint32_t lv = hb ? (uint32_t)__builtin_amdgcn_readlane((int)myl, 63 - __builtin_clzll(hb)) : 0u;
        if (lane == 0) {
            s_lh[wave] = hb != 0;
            s_lv[wave] = lv;
        }
    }
    __syncthreads();
    SWD_TRACE(5);
    if (tid == 0) {
        LbRec agg{0, 0, 0, 0, 0};
        for (int w = 0; w < kBlock / 64; w++) {
            agg.lost += s_c[w];
            agg.reach = max(agg.reach, s_m[w]);
            agg.rep += s_r[w];
            agg.wme = max(agg.wme, s_w[w]);
            if (s_lh[w]) agg.L = s_lv[w];
        }
        if (s_bad) agg.wme |= kSwErrHeader << 16;
        s_agg = agg;
        lb_publish(a, c, agg, c == 0 ? kLbInc : kLbAgg);
    }
    // the chunk's lost sources in LDS (nothing here needs the look-back):
    // positions, reachL within the chunk (the look-back's reach is joined in
    // later), and repfirst of the chunk's sources counted from t0 (the
    // repairs before i0: the same count as the look-back's, headers being in
    // fss order; bad headers stop the call anyway)
    {
        uint32_t loff = wc + ic - cnt, lrun = max(wmx, em), lrep = (uint32_t)t0 + wr + ir - tr;
#pragma unroll
        for (int j = 0; j < kPlanPer; j++)
            if (my0 + j < n) {
                s_rf[my0 + j] = lrep;
                lrun = max(lrun, s_reach[my0 + j]);
                lrep += s_rcnt[my0 + j];
                if ((lostm >> j) & 1u) {
                    s_lpos[loff] = my0 + j;
                    s_rl[loff] = lrun;
                    loff++;
                }
            }
        if (my0 <= n && n <= my0 + kPlanPer) s_rf[n] = lrep;  // repfirst at i1
    }
    __syncthreads();
    SWD_TRACE(6);
    const uint32_t nl = s_agg.lost, wmb_all = s_wmb;
    if (wave == 0) {
        // decoupled look-back, 256 predecessors per round: lane l polls chunks
        // base - 4l - k (k < 4); once all have published, the records back to
        // the nearest inclusive prefix are joined (a lane's four in chunk
        // order, then across lanes) and the window moves back 256 chunks if
        // there was none.  Two round trips a round (flags, records): waiting
        // on 256 predecessors 64 at a time took ~11 us at chunk 255 (r04 trace).
        LbRec ex{0, 0, 0, 0, 0};
        uint32_t spins = 0;
        int64_t wait_q = (int64_t)c - 1;  // a chunk polled alone before the window is read
        for (int64_t base = (int64_t)c - 1; base >= 0;) {
            // one flag by one lane until it has published: every waiting block
            // polling its whole window (1 KB of flags from 255 blocks) made the
            // flags' memory channel a hot spot that slowed every other access
            while (wait_q >= 0) {
                uint32_t f = 0;
                if (lane == 0) f = lb_flag_load(&a.lb_flag[wait_q]);
                f = __shfl(f, 0);
                if ((f >> 2) == a.epoch && (f & 3u) != 0) break;
                if (++spins == (1u << 22)) break;
                __builtin_amdgcn_s_sleep(2);
            }
            wait_q = -1;
            bool ready = true;
            uint32_t incb = 0, nrd = ~0u;  // nrd: nearest unpublished d
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t q = base - 4 * lane - k;
                if (q >= 0) {
                    const uint32_t f = lb_flag_load(&a.lb_flag[q]);
                    const bool pub = (f >> 2) == a.epoch && (f & 3u) != 0;
                    ready &= pub;
                    if (!pub) nrd = min(nrd, (uint32_t)(4 * lane + k));
                    if ((f & 3u) == kLbInc) incb |= 1u << k;
                }
            }
            if (__ballot(!ready)) {
                // bounded: a predecessor that never publishes (which the
                // dispatch order rules out) ends as an error, not a hang
                if (spins >= (1u << 22)) {
                    ex.wme |= kSwErrInternal << 16;
                    break;
                }
                wait_q = base - (int64_t)wave_min(nrd);  // poll the nearest unpublished one alone
                continue;
            }
            // nearest inclusive prefix: d = base - chunk (~0: none in this round)
            const uint32_t dinc = wave_min(incb ? 4u * lane + (uint32_t)(__ffs(incb) - 1) : ~0u);
            const int64_t nd = dinc != ~0u ? (int64_t)dinc + 1 : min<int64_t>(256, base + 1);
            LbRec r{0, 0, 0, 0, 0};
            LbRec v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int64_t d = 4 * lane + k;
                v[k] = d < nd ? lb_read(((uint32_t)d == dinc ? a.lb_inc : a.lb_agg) + 2 * (size_t)(base - d))
                              : LbRec{0, 0, 0, 0, 0};
            }
#pragma unroll
            for (int k = 3; k >= 0; k--) r = lb_join(r, v[k]);  // k = 3 is the lane's earliest
            // ordered join: a higher lane holds earlier chunks
#pragma unroll
            for (int dd = 1; dd < 64; dd <<= 1) {
                LbRec o;
                o.lost = __shfl_down(r.lost, dd);
                o.reach = __shfl_down(r.reach, dd);
                o.rep = __shfl_down(r.rep, dd);
                o.wme = __shfl_down(r.wme, dd);
                o.L = __shfl_down(r.L, dd);
                if (lane + dd < 64 && (lane & (2 * dd - 1)) == 0) r = lb_join(o, r);
            }
            r.lost = __shfl(r.lost, 0);
            r.reach = __shfl(r.reach, 0);
            r.rep = __shfl(r.rep, 0);
            r.wme = __shfl(r.wme, 0);
            r.L = __shfl(r.L, 0);
            ex = lb_join(r, ex);
            if (dinc != ~0u) break;
            base -= 256;
        }
        if (lane == 0) {
            if (c > 0) lb_publish(a, c, lb_join(ex, s_agg), kLbInc);
            s_excl = ex;
        }
    } else {
        // meanwhile (waves 1-3): the coefficient rows of the chunk's received
        // repairs whose window holds a lost source, and the pivots of the lost
        // sources that may be alone in their system
        const auto before = [&](uint32_t j) {  // lost sources in [i0, i0 + j), j <= chunk + halo
            return s_wpfx[j >> 5] + __popc(s_bits[j >> 5] & ((1u << (j & 31)) - 1u));
        };
        // the cached header / arrival flag of repair t (tb <= t < t1)
        const auto hdr_at = [&](uint64_t t) -> fecgpu_sw_repair {
            return t - tb < (uint64_t)kPlanHdr ? s_hc[t - tb] : a.hdr[t];
        };
        const auto rp_at = [&](uint64_t t) -> uint8_t {
            return t - tb < (uint64_t)kPlanHdr ? s_hp[t - tb] : a.rep_present[t];
        };
        // A lost source of the chunk that will be alone in its system (a
        // one-unknown system: the plan writes its pivot's scaled row itself)
        // needs no drawn rows: no repair holding it holds another lost source.
        // Decided here without the look-back, conservatively: not the chunk's
        // first or last lost source, beyond the reach of earlier chunks'
        // windows (pos >= wmb_all), the reach before it stops at it and its
        // own stops before the next.  (At 2 % loss most rows drawn were such
        // systems' and went unused; their scattered dword stores cost the
        // plan ~15 us on cfg7, r05 trace.)
        const auto alone = [&](uint32_t k) {
            return a.long_min > 1 && k > 0 && k + 1 < nl && s_lpos[k] >= wmb_all &&
                   s_rl[k - 1] <= i0 + s_lpos[k] && s_rl[k] <= i0 + s_lpos[k + 1];
        };
        // pivots first: loads only (behind the draws' stores, their loads
        // waited for those to complete: the memory counter is in order)
        for (uint32_t k = tid - 64; k < nl; k += kBlock - 64) {
            uint32_t pt = ~0u, pw = 0, pc = 0;
            const uint32_t pos = s_lpos[k];
            const uint64_t i = i0 + pos;
            if (a.long_min > 1 && (k + 1 >= nl || s_rl[k] <= i0 + s_lpos[k + 1])) {
                // candidates: received repairs with fss in [i - wmb + 1, i] (repair
                // order); the first whose coefficient at i is nonzero (the small
                // solver's choice)
                const uint64_t lo = i + 1 > (uint64_t)wmb_all ? max(i + 1 - wmb_all, ib) : ib;
                const auto rfirst = [&](uint64_t p) -> uint64_t {
                    return p < i0 ? s_rfb[p - (i0 - kPlanHalo)] : s_rf[p - i0];
                };
                // (clamped to the headers this block searched: with a bad or
                // unordered list the counts need not add up, and the call is
                // void anyway, but no read may leave the arrays)
                const uint64_t ta = max(rfirst(lo), tb), te = min(rfirst(i + 1), t1);
                for (uint64_t t = ta; t < te; t++) {
                    const uint8_t rpt = rp_at(t);  // (ta >= tb)
                    const fecgpu_sw_repair h = hdr_at(t);
                    if (!rpt || !hdr_ok(h, a.nsrc)) continue;
                    if (h.fss > i || h.fss + h.nss <= i) continue;
                    const uint32_t j = (uint32_t)(i - h.fss);
                    const uint8_t cj = coef_at(a, h, j);
                    if (!cj) continue;
                    pt = (uint32_t)t;
                    pw = (uint32_t)h.key | (uint32_t)h.nss << 16 | j << 24;
                    pc = cj | (uint32_t)h.dt << 8;
                    break;
                }
            }
            s_pv[k] = make_uint2(pt, pw);
            s_pcd[k] = (uint16_t)pc;
        }
#if FECGPU_SWD_TRACE
        if (tid == 64) s_tr[13] = wall_clock64();  // wave 1: its pivots found
#endif
        for (uint64_t t = t0 + (tid - 64); t < t1; t += kBlock - 64) {
            if (!rp_at(t)) continue;
            const fecgpu_sw_repair h = hdr_at(t);
            if (h.fss < i0 || h.fss >= i1 || !hdr_ok(h, a.nsrc)) continue;
            const uint32_t lo = (uint32_t)(h.fss - i0), hi = lo + h.nss;  // hi <= chunk + halo
            const uint32_t bl = before(lo), bh = before(hi);
            if (bh > bl && !(bh == bl + 1 && alone(bl))) draw_row(a, t, h);
        }
#if FECGPU_SWD_TRACE
        if (tid == 64) s_tr[12] = wall_clock64();  // wave 1: its row draws issued
#endif
    }
    __syncthreads();
    SWD_TRACE(7);
    // this thread's first lost source, if alone with a dense pivot row of <= 32
    // coefficients: the row's two quads load now, beside the lost-list stores
    // below (loads issued after those stores would wait for them)
    uint4 pre[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    bool pre_ok = false;
    if ((uint32_t)tid < nl && a.rlc) {
        const uint2 pv = s_pv[tid];
        const uint32_t nssp = (pv.y >> 16) & 0xFFu;
        pre_ok = pv.x != ~0u && (s_pcd[tid] >> 8) == 15u && nssp <= 32u;
        if (pre_ok) {
            const uint4 *row = reinterpret_cast<const uint4 *>(a.rlc + (size_t)(pv.y & 0xFFFFu) * kRlcRow);
            pre[0] = row[0];
            pre[1] = row[1];
        }
    }
    const LbRec ex = s_excl;
    // lost list, rank / repfirst (as sw_dec_lost_kernel)
    uint32_t off = ex.lost + wc + ic - cnt;
    uint32_t run = max(max(ex.reach, wmx), em);
    uint32_t repc = ex.rep + wr + ir - tr;
    CombJob E{};
    E.xor_off = kNoXor;
    uint32_t rk[kPlanPer], rf[kPlanPer];
#pragma unroll
    for (int j = 0; j < kPlanPer; j++) {
        rk[j] = off;
        rf[j] = repc;
        if (my0 + j < n) {
            const uint64_t i = i0 + my0 + j;
            run = max(run, s_reach[my0 + j]);
            repc += s_rcnt[my0 + j];
            if (((lostm >> j) & 1u) && SWC(off, a.nsrc, kChkLost)) {
                a.lost[off] = (uint32_t)i;
                a.reachL[off] = run;
                a.sol_jobs[off] = E;  // solve jobs in the unknowns' slots: empty unless filled
                off++;
            }
        }
    }
    if (my0 + kPlanPer <= n) {
        uint4 *rkp = reinterpret_cast<uint4 *>(a.reach + i0 + my0), *rfp = reinterpret_cast<uint4 *>(a.rcnt + i0 + my0);
        rkp[0] = make_uint4(rk[0], rk[1], rk[2], rk[3]);
        rkp[1] = make_uint4(rk[4], rk[5], rk[6], rk[7]);
        rfp[0] = make_uint4(rf[0], rf[1], rf[2], rf[3]);
        rfp[1] = make_uint4(rf[4], rf[5], rf[6], rf[7]);
    } else {
        for (uint32_t j = 0; my0 + j < n && j < kPlanPer; j++) {
            a.reach[i0 + my0 + j] = rk[j];
            a.rcnt[i0 + my0 + j] = rf[j];
        }
    }
    if (my0 <= n && n <= my0 + kPlanPer && i1 == a.nsrc) {  // the thread holding the end (reach / rcnt: nsrc + 1)
        a.reach[a.nsrc] = off;
        a.rcnt[a.nsrc] = repc;
    }
    // (no barrier: the starts list below goes to s_rf, free since the pivot
    // searches, so the lost-list stores above and the one-unknown jobs below
    // complete together, r05)
    SWD_TRACE(8);
    // the chunk's lost sources: one-unknown systems solved, the rest classified
    for (uint32_t k = tid; k < nl; k += kBlock) {
        const uint32_t u = ex.lost + k, pos = s_lpos[k], rl = max(ex.reach, s_rl[k]);
        if (!SWC(u, a.nsrc, kChkLost)) break;
        const uint64_t i = i0 + pos;
        const uint32_t prl = k > 0 ? max(ex.reach, s_rl[k - 1]) : (ex.lost ? ex.L : 0u);
        const bool start = u == 0 || prl <= i;
        // the next lost source: in the chunk, else in the halo (a window reaches
        // at most 255 sources past i, so none there means none in reach)
        uint64_t nxt = ~0ull;
        if (k + 1 < nl) {
            nxt = i0 + s_lpos[k + 1];
        } else {
            for (uint32_t w = (pos + 1) >> 5; w < (kPlanChunk + kPlanHalo) / 32 && nxt == ~0ull; w++) {
                uint32_t bits = s_bits[w];
                if (w == (pos + 1) >> 5) bits &= ~((1u << ((pos + 1) & 31)) - 1u);
                if (bits) nxt = i0 + w * 32 + __ffs(bits) - 1;
            }
        }
        // (tuning "sw_long_min" 1 sends every system, these too, down the long path)
        const bool single = start && (nxt == ~0ull || rl <= nxt) && a.long_min > 1;
        uint8_t kind = start ? 2 : 0;
        CombJob J = E;  // syndrome slot nrep + u: empty unless x is solved here
        if (single) {
            kind = 3;
            const uint2 pv = s_pv[k];  // the pivot found during the look-back
            if (pv.x != ~0u && SWC(pv.x, a.nrep, kChkHdr)) {
                const uint64_t t = pv.x;
                const uint32_t cd = s_pcd[k], j = pv.y >> 24;
                fecgpu_sw_repair h{};
                h.fss = i - j;
                h.nss = (uint16_t)((pv.y >> 16) & 0xFFu);
                h.key = (uint16_t)(pv.y & 0xFFFFu);
                h.dt = (uint8_t)(cd >> 8);
                // the job: t's coefficients times 1/c (0 at x), t's row times 1/c;
                // the row scaled 4 bytes at a time as it goes out
                const uint64_t slot = a.nrep + u;
                uint8_t *row = a.coef + slot * kSwCoefPitch;
                const uint32_t iv = c_gfs.exp[255 - c_gfs.log[cd & 0xFFu]];
                uint32_t tab[5];
                set_tab(tab, iv);
                // the xor row's multiplier follows the coefficients (nss < kSwCoefPitch):
                // in the last partial quad, or a quad of its own
                const uint32_t nq = h.nss >> 2, ivw = iv << (8 * (h.nss & 3));
                const auto scale = [&](uint32_t q, uint32_t w) {
                    if (q == (j >> 2)) w &= ~(0xFFu << (8 * (j & 3)));
                    return tmul(w, tab) | (q == nq ? ivw : 0u);
                };
                const auto put = [&](uint32_t g, uint4 v) {
                    reinterpret_cast<uint4 *>(row)[g] =
                        make_uint4(scale(4 * g, v.x), scale(4 * g + 1, v.y), scale(4 * g + 2, v.z), scale(4 * g + 3, v.w));
                };
                if (k == (uint32_t)tid && pre_ok) {  // the prefetched quads
                    put(0, quad_tail(0, pre[0], h.nss));
                    if (h.nss > 16) put(1, quad_tail(1, pre[1], h.nss));
                } else {
                    rlc_quads(a, h, put);
                }
                if (!(h.nss & 15)) reinterpret_cast<uint4 *>(row)[h.nss >> 4] = make_uint4(ivw, 0, 0, 0);
                J.in_off = h.fss * a.stride;
                J.coef_off = slot * kSwCoefPitch;
                J.out_list = slot;
                J.xor_off = t * a.stride;
                J.nin = h.nss;
                J.nout = 1u | kCombXorScaled;
                a.syn_outs[slot] = (uint64_t)(a.src + i * a.stride) - (uint64_t)a.synd;
                a.stat[i] = FECGPU_STATUS_OK;
                kind = 1;
            }
        }
        a.syn_jobs[a.nrep + u] = J;
        a.lkind[u] = kind;
        if (kind == 1) atomicAdd(&s_nsg, 1u);
        if (kind == 2) s_rf[atomicAdd(&s_nst, 1u)] = u;  // s_rf (the pivot searches') is free now
    }
    // the chunk's larger-system starts onto the call's list (one atomic per block;
    // ticket[2] / [3] count starts / singles and are cleared by the last block out)
    __syncthreads();
    SWD_TRACE(9);
    if (tid == 0) {
        s_stbase = s_nst ? atomicAdd(&a.lb_ticket[2], s_nst) : 0u;
        if (s_nsg) atomicAdd(&a.lb_ticket[3], s_nsg);
    }
    __syncthreads();
    // (a count left behind by an aborted launch: raise an error instead of writing past the list)
    if ((uint64_t)s_stbase + s_nst > a.nsrc) {
        if (tid == 0) atomicOr(&a.lb_ticket[4], kSwErrInternal);  // into the counters by the last block out
    } else {
        for (uint32_t k = tid; k < s_nst; k += kBlock) a.starts[s_stbase + k] = s_rf[k];
    }
    // the last block out writes the call's counters (nothing was cleared before
    // the launch) and resets the tickets for the next launch
    __syncthreads();
    SWD_TRACE(10);
    if (tid == 0) {
        __threadfence();
        if (atomicAdd(&a.lb_ticket[1], 1u) == nch - 1) {
            __threadfence();
            const LbRec tot = lb_read(a.lb_inc + 2 * (size_t)(nch - 1));
            SwDecCtr z{};
            z.nlost = tot.lost;
            z.wmax = tot.wme & 0xFFFFu;
            z.err = (tot.wme >> 16) | atomicExch(&a.lb_ticket[4], 0u);
            z.nstart = min(atomicExch(&a.lb_ticket[2], 0u), (uint32_t)tot.lost);
            z.recovered = atomicExch(&a.lb_ticket[3], 0u);
            *a.ctr = z;
            if (z.err && a.sticky) atomicOr(&a.sticky->err, z.err);
            atomicExch(&a.lb_ticket[0], 0u);
            atomicExch(&a.lb_ticket[1], 0u);
        }
    }
#if FECGPU_SWD_TRACE
    if (threadIdx.x == 0 && (s_chunk == 0 || s_chunk == nch / 2 || s_chunk == nch - 1)) {
        const unsigned long long t11 = wall_clock64();
        printf("swd plan chunk %u: %llu %llu %llu %llu %llu %llu %llu %llu %llu %llu end %llu (start %llu)\n", s_chunk,
               s_tr[1] - s_tr[0], s_tr[2] - s_tr[0], s_tr[3] - s_tr[0], s_tr[4] - s_tr[0], s_tr[5] - s_tr[0],
               s_tr[6] - s_tr[0], s_tr[7] - s_tr[0], s_tr[8] - s_tr[0], s_tr[9] - s_tr[0], s_tr[10] - s_tr[0],
               t11 - s_tr[0], s_tr[0]);
        printf("swd plan chunk %u: wave 1 draws %llu pivots %llu\n", s_chunk, s_tr[12] - s_tr[0], s_tr[13] - s_tr[0]);
    }
#endif
}

// A wave per listed start of a larger system (the plan's start list): its
// extent, then solved (tiny or mid) or queued (long).  LDS: 3 KB tiny regions
// per wave and kSysMid mid-size regions per block under LDS locks (cfg7, r04:
// a 16 KB mid region per wave, 2 blocks per CU, measured 0.214 vs 0.207 ms
// per call at 2 % loss, 1.73 vs 1.75 at 10 %, against 3 blocks per CU here).
constexpr int kSysMid = 2;
__global__ __launch_bounds__(kBlock) void sw_dec_sys_kernel(SwDecArgs a) {
    __shared__ GfLds g;
    __shared__ SysLds<kSwTinyE, kSwTinyP> s_sys[kBlock / 64];
    __shared__ SysLds<kSwSmallE, kSwSmallP> s_mid[kSysMid];
    __shared__ int s_lock[kSysMid];
    if (threadIdx.x < kSysMid) s_lock[threadIdx.x] = 0;
    gf_load(g);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (a.ctr->err & kSwErrStop) {
        // a bad or unordered header list (or a failed look-back): the call
        // recovers nothing and the statuses are the arrival flags.  The plan's blocks finished the
        // one-unknown systems of their chunks before every chunk's headers were
        // checked, so their statuses are undone here (the combine launches
        // stand down on the same flag, and write nothing).
        for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < a.nsrc; i += (uint64_t)gridDim.x * kBlock)
            a.stat[i] = a.src_present[i] ? FECGPU_STATUS_OK : FECGPU_STATUS_UNRECOVERABLE;
        return;
    }
    const uint32_t nlost = a.ctr->nlost, wmax = max(1u, a.ctr->wmax);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
    uint32_t rec = 0, maxin = 0;  // this wave's recovered count, widest solve
    // the plan solved the one-unknown systems and listed the larger ones' starts
    const uint32_t nstart = a.ctr->nstart;
    for (uint64_t k = (uint64_t)blockIdx.x * (kBlock / 64) + wave; k < nstart; k += nwaves) {
        const uint64_t x = a.starts[k];
        if (!SWC(x, a.nsrc, kChkLost)) continue;
        const uint32_t lx = a.lost[x];
        // extent: up to the next start
        uint32_t e = 1;
        for (;;) {
            const uint64_t y = x + e + lane;
            const bool stop = y >= nlost || a.reachL[y - 1] <= a.lost[y];
            const uint64_t b = __ballot(stop);
            if (b) {
                e += __ffsll((unsigned long long)b) - 1;
                break;
            }
            e += 64;
        }
        if (!SWC(x + e - 1, a.nsrc, kChkLost)) continue;
        const uint32_t last = a.lost[x + e - 1];
        // candidate repairs: fss in [lx - wmax + 1, last]
        const uint64_t t_lo = a.rcnt[lx >= wmax ? lx - wmax + 1 : 0], t_hi = a.rcnt[(uint64_t)last + 1];
        // tiny systems in the wave's own 3 KB; a mid-size one takes the block's
        // shared region (lane 0 spins on an LDS lock, the wave waits with it);
        // longer ones go to the long pass
        if (sys_one<kSwTinyE, kSwTinyP, true>(a, g, s_sys[wave], (uint32_t)x, e, t_lo, t_hi, lane, rec, maxin)) {
            const int m = wave % kSysMid;  // waves m, m + kSysMid, ... share region m
            if (lane == 0)
                while (atomicCAS(&s_lock[m], 0, 1) != 0) __builtin_amdgcn_s_sleep(2);
            SWD_WAVE_SYNC();
            sys_one<kSwSmallE, kSwSmallP>(a, g, s_mid[m], (uint32_t)x, e, t_lo, t_hi, lane, rec, maxin);
            SWD_WAVE_SYNC();
            __threadfence_block();  // the region's LDS traffic done before the next holder
            if (lane == 0) atomicExch(&s_lock[m], 0);
        }
    }
    block_counts(a, rec, maxin, lane, wave);
}

// ========================================================= long systems ===
constexpr int kStg = 64;  // generated rows waiting for admission

struct LongLds {
    GfLds g;
    uint8_t rowc[kSwRows][256];  // forward: row coefficients (unknown u at [u & 255]); backward: VT
    uint8_t stg[kStg][256];      // generated rows
    uint32_t stg_t[kStg], stg_lo[kStg], stg_hi[kStg];
    uint32_t act[kSwRows];       // alive rows (slots), in admission order
    uint32_t row_hi[kSwRows], row_t[kSwRows];
    uint8_t freel[kSwRows];      // free slots (stack)
    uint8_t fq[kSwRows];         // elimination factor per alive position
    uint8_t lead[kSwRows];       // compaction: alive position holds a leading row
    uint8_t prow[256];           // backward: the pivot row
};

__device__ __forceinline__ void emit(SwOp *op, uint32_t kind, uint32_t sa, uint32_t sb, uint32_t aux, uint32_t aux2,
                                     const uint32_t (&tab)[5]) {
    SwOp o;
    o.op = kind | (sa << 8) | (sb << 16);
    o.aux = aux;
#pragma unroll
    for (int i = 0; i < 5; i++) o.tab[i] = tab[i];
    o.aux2 = aux2;
    *op = o;
}

// emit into log entry pos (checked against log_cap in FECGPU_CHECK builds)
__device__ __forceinline__ void emit_at(const SwDecArgs &a, uint64_t pos, uint32_t kind, uint32_t sa, uint32_t sb,
                                        uint32_t aux, uint32_t aux2, const uint32_t (&tab)[5]) {
    if (SWC(pos, a.log_cap, kChkLog)) emit(a.log + pos, kind, sa, sb, aux, aux2, tab);
}

// Generate the next batch of rows (up to 64 equations from repair *next on)
// into the staging area; returns the number staged (0: no more repairs).
__device__ int long_refill(const SwDecArgs &a, LongLds &L, const SwLong &S, uint64_t &next, int lane) {
    int n = 0;
    while (n == 0 && next < S.t_hi) {
        const uint64_t t = next + lane;
        bool hd = false;
        fecgpu_sw_repair h{};
        if (t < S.t_hi && a.rep_present[t]) {
            h = a.hdr[t];
            hd = holds(a, h, S.x0, S.e);
        }
        const uint64_t b = __ballot(hd);
        n = __popcll(b);
        if (hd) {
            const int k = __popcll(b & lanes_below(lane));
            const uint32_t lo = a.reach[h.fss] - S.x0, hi = a.reach[h.fss + h.nss] - 1 - S.x0;
            L.stg_t[k] = (uint32_t)t;
            L.stg_lo[k] = lo;
            L.stg_hi[k] = hi;
            uint8_t *row = L.stg[k];
            for (uint32_t u = lo; u <= hi; u++) row[u & 255] = 0;
            uint32_t *cc = reinterpret_cast<uint32_t *>(a.coef + (uint64_t)t * kSwCoefPitch);
            (void)SWC(t, a.nrep, kChkSynJob);  // (t < S.t_hi <= nrep: recorded if not)
            RlcSeq sq(a, h);
            uint32_t word = 0;
            for (int j = 0; j < (int)h.nss; j++) {
                uint32_t c = sq.next((uint32_t)j);
                const uint64_t i = h.fss + (uint64_t)j;
                if (!a.src_present[i]) {
                    row[(a.reach[i] - S.x0) & 255] = (uint8_t)c;
                    c = 0;
                }
                word |= c << (8 * (j & 3));
                if ((j & 3) == 3) {
                    cc[j >> 2] = word;
                    word = 0;
                }
            }
            if (h.nss & 3) cc[h.nss >> 2] = word;
        }
        next += 64;
    }
    SWD_WAVE_SYNC();
    return n;
}

// Forward log writer of one long system (wave-uniform): entries go to
// a.log[pos ..); a chunk that runs out is linked to a new one, taken from the
// call's log counter, by a kOpJump entry (the replay follows it).
constexpr uint64_t kLogChunk = 4096;
struct LogW {
    uint64_t pos, end;  // next entry; chunk end (its last entry kept for a jump)
    uint32_t count;     // entries written, jumps included (the replay's trip count)
};

// Room for n more entries at w.pos; false when the log is full (the caller
// gives the system up with kSwErrCapacity).
__device__ bool log_room(const SwDecArgs &a, LogW &w, uint32_t n, int lane) {
    if (w.pos + n < w.end) return true;
    const unsigned long long size = max<unsigned long long>((unsigned long long)n + 1, kLogChunk);
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(&a.ctr->nlog, size);
    base = __shfl(base, 0);
    if (base + size > a.log_cap) {
        if (lane == 0) dec_err(a, kSwErrCapacity, base + size);
        return false;
    }
    if (lane == 0) {
        const uint32_t notab[5] = {0, 0, 0, 0, 0};
        emit_at(a, w.pos, kOpJump, 0, 0, (uint32_t)base, (uint32_t)(base >> 32), notab);
    }
    w.pos = base;
    w.end = base + size;
    w.count++;
    return true;
}

// All kSwRows slots are taken at column c and another row is due.  The alive
// rows are zero before c and end by c + 254 (a window holds at most 255
// sources), so at most 255 of them are independent.  Reduce them to echelon
// form over columns c .. c + 254 — per column, the row with a nonzero there
// that ends first leads, as in the forward pass, so no row widens — and free
// the rows left zero: they were combinations of the others, so dropping them
// changes neither the row space nor any unknown the system determines.  The
// eliminations are logged like the forward ones (the replay applies them to the
// rows' data).  Frees at least one slot; false if the log is full.
__device__ bool long_compact(const SwDecArgs &a, LongLds &L, uint32_t c, int &nact, int &nfree, LogW &fw,
                             int lane) {
    for (int i = lane; i < nact; i += 64) L.lead[i] = 0;
    SWD_WAVE_SYNC();
    int nlead = 0;
    for (uint32_t jj = 0; jj < (uint32_t)kSwRows - 1 && nlead < nact; jj++) {
        const uint32_t j = (c + jj) & 255;
        uint64_t best = ~0ull;
        for (int i = lane; i < nact; i += 64) {
            const uint32_t s = L.act[i];
            // a row's ring bytes past its hi were never written (staging writes
            // [lo, hi] only): look at column c + jj only inside the row's range
            if (!L.lead[i] && c + jj <= L.row_hi[s] && L.rowc[s][j])
                best = min(best, ((uint64_t)L.row_hi[s] << 9) | (uint64_t)i);
        }
        best = wave_min64(best);
        if (best == ~0ull) continue;  // no unled row has column j (uniform)
        const int ppos = (int)(best & 511);
        const uint32_t P = L.act[ppos], hiP = L.row_hi[P];
        const uint32_t ip = ginv(L.g, L.rowc[P][j]);
        for (int i0 = 0; i0 < nact; i0 += 64) {
            if (!log_room(a, fw, 64, lane)) return false;
            const int i = i0 + lane;
            uint32_t f = 0;
            if (i < nact && i != ppos && !L.lead[i] && c + jj <= L.row_hi[L.act[i]])
                f = gmul(L.g, L.rowc[L.act[i]][j], ip);
            if (i < nact) L.fq[i] = (uint8_t)f;
            const uint64_t b = __ballot(f != 0);
            if (f) {
                uint32_t tab[5];
                set_tab(tab, f);
                emit_at(a, fw.pos + __popcll(b & lanes_below(lane)), kOpElim, L.act[i], P, 0, 0, tab);
            }
            fw.pos += __popcll(b);
            fw.count += __popcll(b);
        }
        SWD_WAVE_SYNC();
        if (lane == 0) L.lead[ppos] = 1;
        // the unled rows are zero on [c, c + jj) (eliminated or empty there): update [c + jj, hiP]
        const uint32_t wP = hiP - (c + jj) + 1;
        const uint32_t total = (uint32_t)nact * wP;
        for (uint32_t w0 = 0; w0 < total; w0 += 64) {
            const uint32_t wi = w0 + lane;
            if (wi < total) {
                const uint32_t i = wi / wP, col = (c + jj + wi % wP) & 255;
                const uint32_t f = L.fq[i];
                if (f) L.rowc[L.act[i]][col] ^= (uint8_t)gmul(L.g, f, L.rowc[P][col]);
            }
        }
        SWD_WAVE_SYNC();
        nlead++;
    }
    // keep the leading rows (in admission order), free the rest
    int keep = 0;
    for (int i0 = 0; i0 < nact; i0 += 64) {
        const int i = i0 + lane;
        const uint32_t s = i < nact ? L.act[i] : 0u;
        const bool live = i < nact && L.lead[i];
        const bool dead = i < nact && !live;
        const uint64_t bl = __ballot(live), bd = __ballot(dead);
        SWD_WAVE_SYNC();
        if (live) L.act[keep + __popcll(bl & lanes_below(lane))] = s;
        if (dead) L.freel[nfree + __popcll(bd & lanes_below(lane))] = (uint8_t)s;
        keep += __popcll(bl);
        nfree += __popcll(bd);
        SWD_WAVE_SYNC();
    }
    nact = keep;
    return true;
}

// A wave per long system: forward elimination, null-space sweep, logs.
__global__ __launch_bounds__(64) void sw_dec_long_kernel(SwDecArgs a) {
    extern __shared__ uint4 dyn_long[];
    LongLds &L = *reinterpret_cast<LongLds *>(dyn_long);
    if ((a.ctr->err & kSwErrStop) || blockIdx.x >= min(a.ctr->nlong, (uint32_t)a.long_cap)) return;  // nothing for this block
    gf_load(L.g);
    __syncthreads();
    const int lane = threadIdx.x;
    if (a.ctr->err & kSwErrStop) return;
    const uint32_t nlong = min(a.ctr->nlong, (uint32_t)a.long_cap);
    uint32_t notab[5] = {0, 0, 0, 0, 0};
    for (uint32_t k = blockIdx.x; k < nlong; k += gridDim.x) {
        SwLong S = a.longs[k];
        const uint32_t e = S.e, x0 = S.x0;
        // pass 0: equations and their total width, for the log's reservation
        uint32_t p = 0;
        unsigned long long wsum = 0;
        for (uint64_t t0 = S.t_lo; t0 < S.t_hi; t0 += 64) {
            const uint64_t t = t0 + lane;
            bool hd = false;
            uint32_t w = 0;
            if (t < S.t_hi && a.rep_present[t]) {
                const fecgpu_sw_repair h = a.hdr[t];
                hd = holds(a, h, x0, e);
                if (hd) w = a.reach[h.fss + h.nss] - a.reach[h.fss];
            }
            p += __popcll(__ballot(hd));
            wsum += wave_sum((unsigned long long)w);
        }
        S.ok = 0;
        S.nfwd = S.nbwd = 0;
        if (p == 0) {
            if (lane == 0) a.longs[k] = S;
            continue;
        }
        // forward: loads p, stores <= p, eliminations <= wsum (more after a
        // compaction: chained chunks), one entry kept for a jump; backward:
        // per column a free mark, or begin + end + the pivot row's terms (<= wsum)
        const unsigned long long nfw0 = 2ull * p + wsum + 1, need = nfw0 + wsum + 2ull * e;
        const uint32_t npmax = min(p, e);
        unsigned long long base = 0;
        uint32_t piv0 = 0;
        if (lane == 0) {
            base = atomicAdd(&a.ctr->nlog, need);
            piv0 = atomicAdd(&a.ctr->npiv, npmax);
        }
        base = __shfl(base, 0);
        piv0 = __shfl(piv0, 0);
        if (base + need > a.log_cap || (uint64_t)piv0 + npmax > a.piv_cap) {
            if (lane == 0) {
                dec_err(a, kSwErrCapacity, base + need);
                a.longs[k] = S;
            }
            continue;
        }
        LogW fw{base, base + nfw0, 0};
        const uint64_t bwd0 = base + nfw0;  // the backward log's first entry
        // ---- forward elimination ----
        for (int i = lane; i < kSwRows; i += 64) L.freel[i] = (uint8_t)(kSwRows - 1 - i);
        int nfree = kSwRows, nact = 0, sh = 0, sn = 0;
        uint32_t npiv = 0, B = 1;
        uint64_t next = S.t_lo;
        bool fail = false;
        SWD_WAVE_SYNC();
        for (uint32_t c = 0; c < e && !fail; c++) {
            // admit the rows whose range starts here
            for (;;) {
                if (sh == sn) {
                    if (next >= S.t_hi) break;
                    sn = long_refill(a, L, S, next, lane);
                    sh = 0;
                    if (sn == 0) break;
                }
                if (L.stg_lo[sh] > c) break;  // rows arrive in order of lo, and every lo <= c is admitted by now
                if (nfree == 0 && !long_compact(a, L, c, nact, nfree, fw, lane)) {
                    fail = true;  // log full
                    break;
                }
                if (!log_room(a, fw, 1, lane)) {
                    fail = true;
                    break;
                }
                const uint32_t slot = L.freel[--nfree];
                reinterpret_cast<uint32_t *>(L.rowc[slot])[lane] = reinterpret_cast<const uint32_t *>(L.stg[sh])[lane];
                if (lane == 0) {
                    L.row_hi[slot] = L.stg_hi[sh];
                    L.row_t[slot] = L.stg_t[sh];
                    L.act[nact] = slot;
                    if (SWC(L.stg_t[sh], a.nrep, kChkHdr)) a.synrow[L.stg_t[sh]] = ~0u;
                    emit_at(a, fw.pos, kOpLoad, slot, 0, L.stg_t[sh], 0, notab);
                }
                nact++;
                fw.pos++;
                fw.count++;
                sh++;
                SWD_WAVE_SYNC();
            }
            if (fail) break;
            // pivot: the alive row with a nonzero at c whose range ends first
            const uint32_t cs = c & 255;
            uint64_t best = ~0ull;
            for (int i = lane; i < nact; i += 64) {
                const uint32_t s = L.act[i];
                if (L.rowc[s][cs]) best = min(best, ((uint64_t)L.row_hi[s] << 9) | (uint64_t)i);
            }
            best = wave_min64(best);
            if (best == ~0ull) {
                if (lane == 0 && SWC(x0 + c, a.nsrc, kChkLost)) a.colpiv[x0 + c] = ~0u;
            } else {
                const int ppos = (int)(best & 511);
                const uint32_t P = L.act[ppos];
                const uint32_t hiP = L.row_hi[P];
                const uint32_t ip = ginv(L.g, L.rowc[P][cs]);
                // factors and ELIM entries
                for (int i0 = 0; i0 < nact && !fail; i0 += 64) {
                    if (!log_room(a, fw, 64, lane)) {
                        fail = true;
                        break;
                    }
                    const int i = i0 + lane;
                    uint32_t f = 0;
                    if (i < nact && i != ppos) f = gmul(L.g, L.rowc[L.act[i]][cs], ip);
                    if (i < nact) L.fq[i] = (uint8_t)f;
                    const uint64_t b = __ballot(f != 0);
                    if (f) {
                        uint32_t tab[5];
                        set_tab(tab, f);
                        emit_at(a, fw.pos + __popcll(b & lanes_below(lane)), kOpElim, L.act[i], P, 0, 0, tab);
                    }
                    fw.pos += __popcll(b);
                    fw.count += __popcll(b);
                }
                if (fail || !log_room(a, fw, 1, lane)) {
                    fail = true;
                    break;
                }
                SWD_WAVE_SYNC();
                // row updates over [c, hiP]: lanes over (alive position, column) pairs
                const uint32_t wP = hiP - c + 1;
                const uint32_t total = (uint32_t)nact * wP;
                for (uint32_t w0 = 0; w0 < total; w0 += 64) {
                    const uint32_t wi = w0 + lane;
                    if (wi < total) {
                        const uint32_t i = wi / wP, j = c + wi % wP;
                        const uint32_t f = L.fq[i];
                        if (f) {
                            uint8_t *r = &L.rowc[L.act[i]][j & 255];
                            *r ^= (uint8_t)gmul(L.g, f, L.rowc[P][j & 255]);
                        }
                    }
                }
                SWD_WAVE_SYNC();
                // the pivot row: coefficients to the pivot area, STORE
                const uint32_t pv = piv0 + npiv;
                if (SWC(pv, a.piv_cap, kChkPiv))
                    reinterpret_cast<uint32_t *>(a.pivcoef + (uint64_t)pv * 256)[lane] =
                        reinterpret_cast<const uint32_t *>(L.rowc[P])[lane];
                if (lane == 0 && SWC(pv, a.piv_cap, kChkPiv) && SWC(x0 + c, a.nsrc, kChkLost)) {
                    a.pivhi[pv] = hiP;
                    a.pivt[pv] = L.row_t[P];
                    a.colpiv[x0 + c] = pv;
                    emit_at(a, fw.pos, kOpStore, P, 0, pv, 0, notab);
                }
                fw.pos++;
                fw.count++;
                npiv++;
                B = max(B, wP);
            }
            // retire the pivot and the rows whose range ends at c (now zero)
            const uint32_t P = best == ~0ull ? ~0u : L.act[best & 511];
            int keep = 0;
            for (int i0 = 0; i0 < nact; i0 += 64) {
                const int i = i0 + lane;
                const uint32_t s = i < nact ? L.act[i] : 0u;
                const bool live = i < nact && s != P && L.row_hi[s] > c;
                const bool dead = i < nact && !live;
                const uint64_t bl = __ballot(live), bd = __ballot(dead);
                SWD_WAVE_SYNC();
                if (live) L.act[keep + __popcll(bl & lanes_below(lane))] = s;
                if (dead) L.freel[nfree + __popcll(bd & lanes_below(lane))] = (uint8_t)s;
                keep += __popcll(bl);
                nfree += __popcll(bd);
                SWD_WAVE_SYNC();
            }
            nact = keep;
        }
        if (fail) {  // the log is full (kSwErrCapacity raised): the system stays lost
            if (lane == 0) a.longs[k] = S;
            continue;
        }
        // syndrome jobs for the pivot rows (the only rows whose data is used), in
        // their repairs' slots; the other slots stay empty
        for (uint32_t q = lane; q < npiv; q += 64) {
            if (!SWC(piv0 + q, a.piv_cap, kChkPiv)) break;
            const uint32_t t = a.pivt[piv0 + q];
            if (!SWC(t, a.nrep, kChkSynJob)) continue;
            const uint32_t gq = t;
            const fecgpu_sw_repair h = a.hdr[t];
            CombJob J;
            J.in_off = h.fss * a.stride;
            J.coef_off = (uint64_t)t * kSwCoefPitch;
            J.out_list = gq;
            J.xor_off = (uint64_t)t * a.stride;
            J.nin = h.nss;
            J.nout = 1;
            a.syn_jobs[gq] = J;
            a.syn_outs[gq] = (uint64_t)gq * a.stride;
            a.synrow[t] = gq;
        }
        // ---- null-space sweep and back substitution log ----
        // VT[coordinate & 255][vector] bytes (LDS rowc), nv vectors
        uint8_t(*VT)[256] = L.rowc;
        uint32_t nv = 0, nb = 0, ndet = 0;
        for (int c = (int)e - 1; c >= 0; c--) {
            const uint32_t cs = (uint32_t)c & 255;
            const uint32_t pv = SWC(x0 + c, a.nsrc, kChkLost) ? a.colpiv[x0 + c] : ~0u;
            if (pv == ~0u) {
                if (nv == (uint32_t)kSwRows) {
                    // reduce to a basis of the projection on [c + 1, c + B)
                    uint32_t rank = 0;
                    for (uint32_t jj = 1; jj < B && rank < nv; jj++) {
                        const uint32_t s = (uint32_t)(c + jj) & 255;
                        uint32_t first = ~0u;
                        for (uint32_t v = rank + lane; v < nv; v += 64)
                            if (VT[s][v]) first = min(first, v);
                        first = wave_min(first);
                        if (first == ~0u) continue;
                        if (first != rank)
                            for (int cc2 = lane; cc2 < 256; cc2 += 64) {
                                const uint8_t t0 = VT[cc2][first];
                                VT[cc2][first] = VT[cc2][rank];
                                VT[cc2][rank] = t0;
                            }
                        SWD_WAVE_SYNC();
                        const uint32_t iv = ginv(L.g, VT[s][rank]);
                        // eliminate coordinate s from the vectors after `rank`
                        const uint32_t nvv = nv - rank - 1;
                        for (uint32_t w0 = 0; w0 < nvv * B; w0 += 64) {
                            const uint32_t wi = w0 + lane;
                            if (wi < nvv * B) {
                                const uint32_t v = rank + 1 + wi / B, s2 = (uint32_t)(c + wi % B) & 255;
                                const uint32_t f = gmul(L.g, VT[s][v], iv);
                                if (f && s2 != s) VT[s2][v] ^= (uint8_t)gmul(L.g, f, VT[s2][rank]);
                            }
                        }
                        SWD_WAVE_SYNC();
                        for (uint32_t v = rank + 1 + lane; v < nv; v += 64) VT[s][v] = 0;
                        SWD_WAVE_SYNC();
                        rank++;
                    }
                    nv = rank;
                }
                // coordinate c of every vector is 0; the new vector is e_c
                reinterpret_cast<uint32_t *>(VT[cs])[lane] = 0;
                SWD_WAVE_SYNC();
                for (int cc2 = lane; cc2 < 256; cc2 += 64) VT[cc2][nv] = (uint8_t)(cc2 == (int)cs);
                nv++;
                if (lane == 0) emit_at(a, bwd0 + nb, kOpXFree, cs, 0, 0, 0, notab);
                nb++;
                SWD_WAVE_SYNC();
                continue;
            }
            if (!SWC(pv, a.piv_cap, kChkPiv)) break;
            reinterpret_cast<uint32_t *>(L.prow)[lane] = reinterpret_cast<const uint32_t *>(a.pivcoef + (uint64_t)pv * 256)[lane];
            const uint32_t hi = a.pivhi[pv];
            SWD_WAVE_SYNC();
            const uint32_t ip = ginv(L.g, L.prow[cs]);
            uint32_t det = 1;
            if (nv) {
                uint32_t acc = 0;
                for (uint32_t j = (uint32_t)c + 1; j <= hi; j++) {
                    const uint32_t cj = L.prow[j & 255];
                    if (!cj) continue;
                    uint32_t tab[5];
                    set_tab(tab, cj);
                    acc ^= tmul(reinterpret_cast<const uint32_t *>(VT[j & 255])[lane], tab);
                }
                uint32_t tip[5];
                set_tab(tip, ip);
                acc = tmul(acc, tip);
                // bytes of vectors >= nv are not vectors
                const uint32_t v0 = 4u * lane;
                const uint32_t keepm = v0 + 4 <= nv ? 0xFFFFFFFFu : v0 >= nv ? 0u : (0xFFFFFFFFu >> (8 * (v0 + 4 - nv)));
                acc &= keepm;
                reinterpret_cast<uint32_t *>(VT[cs])[lane] = acc;
                det = __ballot(acc != 0) ? 0u : 1u;
            }
            const uint32_t src_i = a.lost[x0 + c];  // (x0 + c < nsrc: checked with colpiv above)
            // back substitution entries: x_c = ip * y_P + sum (ip * a_Pj) x_j
            {
                uint32_t tip[5];
                set_tab(tip, ip);
                if (lane == 0) emit_at(a, bwd0 + nb, kOpXBegin, cs, 0, pv, 0, tip);
                nb++;
                const uint32_t w = hi >= (uint32_t)c ? hi - (uint32_t)c : 0u;  // a pivot row ends at or after its column
                for (uint32_t j0 = 0; j0 < w; j0 += 64) {
                    const uint32_t j = (uint32_t)c + 1 + j0 + lane;
                    const uint32_t cj = j0 + lane < w ? L.prow[j & 255] : 0u;
                    const uint64_t b = __ballot(cj != 0);
                    if (cj) {
                        uint32_t tab[5];
                        set_tab(tab, gmul(L.g, cj, ip));
                        emit_at(a, bwd0 + nb + __popcll(b & lanes_below(lane)), kOpXTerm, j & 255, 0, 0, 0, tab);
                    }
                    nb += __popcll(b);
                }
                if (lane == 0) emit_at(a, bwd0 + nb, kOpXEnd, 0, cs, det ? src_i : ~0u, 0, notab);
                nb++;
            }
            if (det) {
                if (lane == 0 && SWC(src_i, a.nsrc, kChkSrcRow)) a.stat[src_i] = FECGPU_STATUS_OK;
                ndet++;
            }
            SWD_WAVE_SYNC();
        }
        if (lane == 0) {
            S.ok = 1;
            S.fwd = base;
            S.nfwd = fw.count;
            S.bwd = base + nfw0;
            S.nbwd = nb;
            S.piv0 = piv0;
            a.longs[k] = S;
            if (ndet) atomicAdd(&a.ctr->recovered, ndet);
        }
    }
}

// A wave per (long system, 64-dword column chunk): replay the log.
__global__ __launch_bounds__(64) void sw_dec_replay_kernel(SwDecArgs a) {
    __shared__ uint32_t slots[kSwRows][64];
    const int lane = threadIdx.x;
    if (a.ctr->err & kSwErrStop) return;
    const uint32_t nlong = min(a.ctr->nlong, (uint32_t)a.long_cap);
    const uint32_t ndw = ((a.S + 15u) >> 4) * 4u;  // whole 16-B columns, as the combine passes
    const uint32_t nch = (ndw + 63) / 64;
    const uint64_t units = (uint64_t)nlong * nch;
    for (uint64_t u = blockIdx.x; u < units; u += gridDim.x) {
        const uint32_t s = (uint32_t)(u / nch), ch = (uint32_t)(u % nch);
        const SwLong S = a.longs[s];
        if (!S.ok) continue;
        const uint32_t dw = ch * 64 + lane;
        const bool live = dw < ndw;
        const uint64_t boff = (uint64_t)dw * 4;
        uint64_t at = S.fwd;
        for (uint32_t i = 0; i < S.nfwd; i++) {
            if (!SWC(at, a.log_cap, kChkLog)) break;
            const SwOp o = a.log[at++];
            const uint32_t kind = o.op & 0xFFu, sa = (o.op >> 8) & 0xFFu, sb = (o.op >> 16) & 0xFFu;
            if (kind == kOpJump) {
                at = (uint64_t)o.aux | ((uint64_t)o.aux2 << 32);
            } else if (kind == kOpElim) {
                const uint32_t t[5] = {o.tab[0], o.tab[1], o.tab[2], o.tab[3], o.tab[4]};
                slots[sa][lane] ^= tmul(slots[sb][lane], t);
            } else if (kind == kOpLoad) {
                const uint32_t g = SWC(o.aux, a.nrep, kChkHdr) ? a.synrow[o.aux] : ~0u;
                uint32_t v = 0;
                if (g != ~0u && live && SWC(g, a.nrep, kChkSynRow) && SWC(boff + 3, a.stride, kChkColumn))
                    v = *reinterpret_cast<const uint32_t *>(a.synd + (uint64_t)g * a.stride + boff);
                slots[sa][lane] = v;
            } else if (kind == kOpStore) {
                if (live && SWC(o.aux, a.piv_cap, kChkPiv) && SWC(boff + 3, a.stride, kChkColumn))
                    *reinterpret_cast<uint32_t *>(a.pivdata + (uint64_t)o.aux * a.stride + boff) = slots[sa][lane];
            }
        }
        const SwOp *op = a.log + S.bwd;
        uint32_t x = 0;
        for (uint32_t i = 0; i < S.nbwd; i++) {
            if (!SWC(S.bwd + i, a.log_cap, kChkLog)) break;
            const SwOp o = op[i];
            const uint32_t kind = o.op & 0xFFu, sa = (o.op >> 8) & 0xFFu, sb = (o.op >> 16) & 0xFFu;
            const uint32_t t[5] = {o.tab[0], o.tab[1], o.tab[2], o.tab[3], o.tab[4]};
            if (kind == kOpXTerm) {
                x ^= tmul(slots[sa][lane], t);
            } else if (kind == kOpXBegin) {
                x = live && SWC(o.aux, a.piv_cap, kChkPiv)
                        ? tmul(*reinterpret_cast<const uint32_t *>(a.pivdata + (uint64_t)o.aux * a.stride + boff), t)
                        : 0u;
            } else if (kind == kOpXEnd) {
                slots[sb][lane] = x;
                if (o.aux != ~0u && live && SWC(o.aux, a.nsrc, kChkSrcRow) && SWC(boff + 3, a.stride, kChkColumn))
                    *reinterpret_cast<uint32_t *>(a.src + (uint64_t)o.aux * a.stride + boff) = x;
            } else if (kind == kOpXFree) {
                slots[sa][lane] = 0;
            }
        }
    }
}

int cu_count() {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
    return cus;
}

}  // namespace

hipError_t launch_rlc_table(uint8_t *tab, hipStream_t s) {
    hipLaunchKernelGGL(rlc_table_kernel, dim3(65536 / kBlock), dim3(kBlock), 0, s, tab);
    return hipGetLastError();
}

hipError_t launch_sw_dec_plan(const SwDecArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(sw_dec_plan_kernel, dim3((unsigned)((a.nsrc + kPlanChunk - 1) / kPlanChunk)), dim3(kBlock), 0, s,
                       a);
    return hipGetLastError();
}

hipError_t launch_sw_dec_sys(const SwDecArgs &a, hipStream_t s) {
    if (a.nrep) {
        // a wave per lost source at most; persistent beyond what fits the chip
        // (two shared mid regions, ~30 KB per block with the tiny ones: 3 per CU)
        const uint64_t want = (a.nsrc + kBlock / 64 - 1) / (kBlock / 64);
        const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(want, (uint64_t)cu_count() * 3));
        hipLaunchKernelGGL(sw_dec_sys_kernel, dim3(grid), dim3(kBlock), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_sw_dec_long(const SwDecArgs &a, hipStream_t s) {
    if (a.nrep == 0) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(sw_dec_long_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(LongLds));
    if (e != hipSuccess) return e;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(a.long_cap, (uint64_t)cu_count()));
    hipLaunchKernelGGL(sw_dec_long_kernel, dim3(grid), dim3(64), sizeof(LongLds), s, a);
    return hipGetLastError();
}

hipError_t launch_sw_dec_replay(const SwDecArgs &a, hipStream_t s) {
    if (a.nrep == 0) return hipSuccess;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(a.long_cap * 64, (uint64_t)cu_count() * 4));
    hipLaunchKernelGGL(sw_dec_replay_kernel, dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError();
}

}  // namespace fecgpu
