// fec_swenc.hip — streaming sliding-window RLC encode (RFC 8681, m = 8):
// include/fecgpu.h fecgpu_sw_encode and the per-connection encoder's batches
// (DESIGN.md §4a).
//
// The combine-job encode (fec_kernels.hip comb_kernel) reads every source once
// per group of repairs whose windows hold it: W + 3 steps of rows for 4
// repairs at W / step = 4, 1.7x the algorithmic bytes.  Here a workgroup takes
// a segment of up to kSwSeg consecutive repairs and streams the union of their
// windows ONCE: lane = C dwords of a symbol column, one accumulator per slot,
// and slot m holds the repairs m, m + A, m + 2A, ... of the segment in turn
// (fec_internal.h SwStreamArgs).  Only the A - 1 steps of rows before a
// segment's first window are read again (by the workgroup's previous segment,
// from L2).  Multiply tables (make_coef_tab, 20 B per coefficient) for the
// whole segment are built in LDS from the RFC 8682 PRNG by the workgroup; the
// window bookkeeping is wave-uniform (scalar registers and branches).
//
// Work per source and dword: one split (a, b, c index words) and, per window
// holding it, 3 v_perm + 2 xor (5 VALU) with its table read from LDS
// (ds_read_b128 + ds_read_b32, same address on every lane).
#include <mutex>
#include <vector>

#include "fec_internal.h"

namespace fecgpu {

namespace {

constexpr int kSwsU = kSwStreamU;
// multiply-table LDS per wave of a workgroup (capped by the budget)
constexpr uint32_t kSwsWaveLds = 12u << 10;
// accumulator slots compiled (a segment needing more takes P > 1 passes)
constexpr int kSwsAmax = 4 < kSwSlots ? 4 : kSwSlots;
// Measured and removed (r05): tables read one source ahead (0.35 vs 0.24 ms on
// cfg7, registers), a source pair's tables for every slot loaded before any
// product (108 VGPRs instead of 73: 0.287 vs 0.213 ms), 4-entry tables in
// global memory read by scalar loads (0.45 vs 0.214 ms: four v_perm per
// product and a scalar-load wait per (source, slot)).

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define SWS_WAVE_SYNC()                                         \
    do {                                                        \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                        \
    } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) uint32_t *g32;
typedef __attribute__((address_space(1))) u32x2 *g64;

// C dwords of a lane: one store for C = 1, 2, 4 (4: 16-B aligned, the rows
// are), dword by dword for 3 and 5 (4-B aligned)
typedef __attribute__((address_space(1))) u32x4 *g128;
// Source rows by buffer loads: the resource (a batch's first row, scalar) plus
// a scalar row offset plus this lane's column offset, no per-load address
// arithmetic on the vector ALU (global loads measured 3 % slower, r03).  Word
// 3 of the resource: raw 32-bit data on gfx9.
constexpr int kRsrcWord3 = 0x00020000;
template <int C>
__device__ __forceinline__ void ldc_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, uint32_t (&x)[C]) {
    if constexpr (C == 1) {
        x[0] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0);
    } else if constexpr (C == 2) {
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0);
        x[0] = v.x;
        x[1] = v.y;
    } else if constexpr (C == 4) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
        x[3] = v.w;
    } else {
#pragma unroll
        for (int d = 0; d < C; d++) x[d] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)voff + 4 * d, (int)soff, 0);
    }
}
template <int C>
__device__ __forceinline__ void stc(uint8_t *p, const uint32_t (&x)[C]) {
    if constexpr (C == 1) {
        *(g32)(p) = x[0];
    } else if constexpr (C == 2) {
        const u32x2 v = {x[0], x[1]};
        *(g64)(p) = v;
    } else if constexpr (C == 4) {
        const u32x4 v = {x[0], x[1], x[2], x[3]};
        *(g128)(p) = v;
    } else {
#pragma unroll
        for (int d = 0; d < C; d++) ((g32)(p))[d] = x[d];
    }
}

__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    return (uint64_t)rfl((uint32_t)x) | ((uint64_t)rfl((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
    for (int o = 32; o; o >>= 1) v = min(v, (uint64_t)__shfl_xor((unsigned long long)v, o));
    return v;
}

// a ^ b ^ c in one gfx950 VALU op (truth table 0x96)
__device__ __forceinline__ uint32_t xor3s(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// The plan of one segment (wave 0): its non-empty repairs in order (window
// [f, e) in sources, offset in the segment), the passes' source ranges and
// the slot shape; repairs whose clipped window is empty get zero rows.
struct SwsPlan {
    uint2 fe[kSwSeg];                   // windows [f, e), relative to lo (the call has < 2^32 sources)
    uint32_t plo[kSwSeg], phi[kSwSeg];
    uint16_t out[kSwSeg], empty[kSwSeg];
    uint64_t lo;
    int nn, nempty, P, A;
};

__device__ __forceinline__ void sws_plan(const SwStreamArgs &a, SwsPlan &pl, uint8_t *CB, uint64_t j0, int n, int lane) {
    const int W = a.max_window;
    uint64_t fss = 0, end = 0;
    bool ne = false;
    fecgpu_sw_repair h{};
    if (lane < n) {
        h = a.hdr[j0 + lane];
        fss = min(h.fss, a.nsrc);
        const uint64_t nss = min((uint64_t)min((int)h.nss, W), a.nsrc - fss);
        end = fss + nss;
        ne = nss > 0;
    }
    const uint64_t below = (1ull << lane) - 1ull;
    const uint64_t bne = __ballot(ne), bem = __ballot(lane < n && !ne);
    const int nn = __popcll(bne);
    const uint64_t lo = wave_min64(ne ? fss : ~0ull);
    if (ne) {
        const int v = __popcll(bne & below);
        pl.fe[v] = make_uint2((uint32_t)(fss - lo), (uint32_t)(end - lo));
        pl.out[v] = (uint16_t)lane;
        rlc_coefs_tab(a.rlc, h.key, (int)(end - fss), min((uint32_t)h.dt, 15u), CB + (size_t)v * W);
    }
    if (lane < n && !ne) pl.empty[__popcll(bem & below)] = (uint16_t)lane;
    SWS_WAVE_SYNC();
    const uint32_t fv = lane < nn ? pl.fe[lane].x : 0, ev = lane < nn ? pl.fe[lane].y : 0;
    // smallest P, then A, with every window starting at or after the end of
    // the one A P repairs before it (P > nn / kSwsAmax always qualifies)
    int P = 1, A = 0;
    for (int pp = 1; pp <= kSwSeg && !A; pp++) {
        for (int aa = 1; aa <= kSwsAmax; aa++) {
            const int d = pp * aa;
            const uint32_t fn = (uint32_t)__shfl((int)fv, min(lane + d, 63));
            if (!__ballot(lane + d < nn && fn < ev)) {
                P = pp;
                A = aa;
                break;
            }
        }
    }
    if (lane < P) {
        pl.plo[lane] = ~0u;
        pl.phi[lane] = 0;
    }
    SWS_WAVE_SYNC();
    if (lane < nn) {
        atomicMin(&pl.plo[lane % P], fv);
        atomicMax(&pl.phi[lane % P], ev);
    }
    if (lane == 0) {
        pl.lo = lo;
        pl.nn = nn;
        pl.nempty = __popcll(bem);
        pl.P = P;
        pl.A = A;
    }
}

template <int C>
struct SplitC {
    uint32_t a[C], b[C], c[C];
};
template <int C>
__device__ __forceinline__ SplitC<C> split_c(const uint32_t (&x)[C]) {
    SplitC<C> s;
#pragma unroll
    for (int d = 0; d < C; d++) {
        s.a[d] = x[d] & 0x07070707u;
        s.b[d] = (x[d] >> 3) & 0x07070707u;
        s.c[d] = (x[d] >> 6) & 0x03030303u;
    }
    return s;
}
template <int C>
__device__ __forceinline__ void gmac_c(uint32_t (&acc)[C], const SplitC<C> &s, uint4 ab, uint32_t tc) {
#pragma unroll
    for (int d = 0; d < C; d++)
        acc[d] = xor3s(acc[d], __builtin_amdgcn_perm(ab.y, ab.x, s.a[d]), __builtin_amdgcn_perm(ab.w, ab.z, s.b[d])) ^
                 __builtin_amdgcn_perm(tc, tc, s.c[d]);
}

// Pass p of a segment over this lane's column (byte offset loff in a row):
// A slots, repairs p, p + P, ... in slot order; every window is met in source
// order, a slot's repair is stored when its last source is in.  Sources go in
// batches of L <= U that end at or before the next window end (so stores and
// slot changes happen between batches only); the next batch's rows are
// loaded while this one is multiplied.  Within a batch a slot's table entries are
// consecutive: its repair's zero run (U entries before its coefficients)
// covers the sources before its window opens, so the batch body is straight
// line code with LDS addresses as immediate offsets from one base per slot.
// window [f, e) of plan repair v (scalar), or none past the last
__device__ __forceinline__ void sws_window(const SwsPlan &pl, uint32_t v, uint32_t nn, uint32_t &f, uint32_t &e) {
    if (v < nn) {
        const uint2 w = pl.fe[v];
        f = rfl(w.x);
        e = rfl(w.y);
    } else {
        f = e = ~0u;
    }
}

template <int A, int C>
__device__ __forceinline__ void sws_pass(const SwStreamArgs &a, const SwsPlan &pl, const uint4 *AB,
                                         const uint32_t *TC, uint64_t j0, int p, int P, uint32_t loff,
                                         bool live) {
    constexpr int U = kSwsU;
    static_assert(U % 2 == 0, "sources go in pairs");
    const uint32_t RW = (uint32_t)a.max_window + U, nn = rfl((uint32_t)pl.nn), stepv = (uint32_t)(A * P);
    const bool dense = rfl((uint32_t)pl.nempty) == 0;  // plan order = segment order
    const uint64_t stride = a.stride;
    uint32_t acc[A][C];
    uint32_t v[A], f[A], e[A];  // slot's repair (plan order), its window [f, e)
#pragma unroll
    for (int m = 0; m < A; m++) {
#pragma unroll
        for (int d = 0; d < C; d++) acc[m][d] = 0;
        v[m] = (uint32_t)(p + m * P);
        sws_window(pl, v[m], nn, f[m], e[m]);
    }
    const uint32_t hi = rfl(pl.phi[p]);
    uint32_t s = rfl(pl.plo[p]);
    if (s >= hi) return;  // an empty pass (hi >= 1 below)
    // FECGPU_CHECK builds: the pass's rows lie in the sources, its column in a row
    if (!CHK_IDX(a.chk, rfl64(pl.lo) + hi - 1, a.nsrc, 1) || !CHK_IDX(a.chk, loff + 4 * C - 1, stride, 2)) return;
    const uint8_t *base = a.src + rfl64(pl.lo) * stride;
    // rows s0 .. s0 + U - 1, clamped to hi - 1 (valid rows only).  Every batch
    // issues its loads unconditionally: with a load under a branch the
    // compiler's wait counts merge to the stricter path, and the batch waited
    // for the rows it had just prefetched (s_waitcnt vmcnt(7..0) in its body).
    auto load = [&](uint32_t s0, uint32_t (&x)[U][C]) __attribute__((always_inline)) {
        s0 = rfl(min(s0, hi - 1));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(base + (uint64_t)s0 * stride), 0, (int)(U * stride), kRsrcWord3);
        const uint32_t last = rfl(hi - 1 - s0);  // scalar: rows past it reload row hi - 1
#pragma unroll
        for (int i = 0; i < U; i++) ldc_buf<C>(r, loff, min((uint32_t)i, last) * (uint32_t)stride, x[i]);
    };
    // one batch: multiply the rows in X, while the next batch's rows load into Y
    auto batch = [&](uint32_t (&X)[U][C], uint32_t (&Y)[U][C]) __attribute__((always_inline)) -> bool {
        if (s >= hi) return false;
        uint32_t ev = e[0];
#pragma unroll
        for (int m = 1; m < A; m++) ev = min(ev, e[m]);
        const uint32_t L = min((uint32_t)U, min(ev, hi) - s);  // >= 1
        const uint32_t sn = s + L;
        load(sn, Y);  // past the end: a harmless reload of row hi - 1
        // slot m's entry for source s + i: tb[m] + i (its repair's zero run
        // before the window; repair 0's zero run while the window is ahead)
        const uint4 *tab[A];
        const uint32_t *tcb[A];
#pragma unroll
        for (int m = 0; m < A; m++) {
            const uint32_t tb = f[m] < sn ? v[m] * RW + U + s - f[m] : 0u;
            tab[m] = AB + tb;
            tcb[m] = TC + tb;
        }
        // a batch cut short by a window end multiplies zero rows past it (their
        // table reads stay inside the LDS tables: kSwsU spare entries at the end)
        if (L < (uint32_t)U) {
#pragma unroll
            for (int i = 1; i < U; i++)
#pragma unroll
                for (int d = 0; d < C; d++) X[i][d] = (uint32_t)i < L ? X[i][d] : 0u;
        }
        // sources in pairs: the six table lookups of two products fold into
        // the accumulator with three 3-input XORs
#pragma unroll
        for (int i = 0; i < U; i += 2) {
            const SplitC<C> s0 = split_c<C>(X[i]), s1 = split_c<C>(X[i + 1]);
#pragma unroll
            for (int m = 0; m < A; m++) {
                uint4 a0 = tab[m][i], a1 = tab[m][i + 1];
                uint32_t c0 = tcb[m][i], c1 = tcb[m][i + 1];
                // tables stay in vector registers (uniform values would be
                // moved to scalar ones with a readfirstlane each)
                asm("" : "+v"(a0.x), "+v"(a0.y), "+v"(a0.z), "+v"(a0.w), "+v"(c0));
                asm("" : "+v"(a1.x), "+v"(a1.y), "+v"(a1.z), "+v"(a1.w), "+v"(c1));
#pragma unroll
                for (int d = 0; d < C; d++) {
                    uint32_t t = xor3s(acc[m][d], __builtin_amdgcn_perm(a0.y, a0.x, s0.a[d]),
                                       __builtin_amdgcn_perm(a0.w, a0.z, s0.b[d]));
                    t = xor3s(t, __builtin_amdgcn_perm(c0, c0, s0.c[d]), __builtin_amdgcn_perm(a1.y, a1.x, s1.a[d]));
                    acc[m][d] = xor3s(t, __builtin_amdgcn_perm(a1.w, a1.z, s1.b[d]), __builtin_amdgcn_perm(c1, c1, s1.c[d]));
                    // pin the products here: left alone the compiler defers slots'
                    // products past later sources and keeps their tables live (spills)
                    asm volatile("" : "+v"(acc[m][d]));
                }
            }
        }
        // windows ending at sn: store, next repair of the slot
#pragma unroll
        for (int m = 0; m < A; m++) {
            if (e[m] == sn) {
                const uint32_t o = dense ? v[m] : rfl(pl.out[v[m]]);
                if (live && CHK_IDX(a.chk, j0 + o, a.nrep, 3)) stc<C>(a.rep + (j0 + o) * stride + loff, acc[m]);
#pragma unroll
                for (int d = 0; d < C; d++) acc[m][d] = 0;
                v[m] += stepv;
                sws_window(pl, v[m], nn, f[m], e[m]);
            }
        }
        uint32_t fmin = f[0];
#pragma unroll
        for (int m = 1; m < A; m++) fmin = min(fmin, f[m]);
        if (fmin > sn) {  // no window open at sn: skip to the next one's start
            s = fmin;
            load(s, Y);
        } else {
            s = sn;
        }
        return true;
    };
    uint32_t XA[U][C], XB[U][C];
    load(s, XA);
    // two batches per trip, the row buffers trading roles (no copies); one
    // exit on a flag (a loop with two exits loses the bookkeeping's
    // uniformity: vector registers and readfirstlane loops around the loads)
    bool go = true;
    while (go) {
        go = batch(XA, XB);
        if (go) go = batch(XB, XA);
    }
}

template <int C>
__global__ __launch_bounds__(512) void sw_stream_kernel(SwStreamArgs a) {
    extern __shared__ uint4 sws_dyn[];
    __shared__ SwsPlan pl;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int W = a.max_window;
    const int RW = W + kSwsU;  // table entries per repair: kSwsU zeros, then its coefficients
    uint4 *AB = sws_dyn;
    // each table array ends with kSwsU spare entries (read by cut-short batches)
    uint32_t *TC = reinterpret_cast<uint32_t *>(AB + (size_t)a.segcap * RW + kSwsU);
    uint8_t *CB = reinterpret_cast<uint8_t *>(TC + (size_t)a.segcap * RW + kSwsU);
    const uint64_t sb = (uint64_t)blockIdx.x * a.nseg / gridDim.x;
    const uint64_t se = (uint64_t)(blockIdx.x + 1) * a.nseg / gridDim.x;
    for (uint64_t sg = sb; sg < se; sg++) {
        const uint64_t j0 = sg * (uint64_t)a.segcap;
        const int n = (int)min((uint64_t)a.segcap, a.nrep - j0);
        if (wave == 0) sws_plan(a, pl, CB, j0, n, lane);
        __syncthreads();
        const int nn = (int)rfl((uint32_t)pl.nn);
        // every entry a batch may read is a table: zero runs, coefficients,
        // zeros past a window (a cut-short batch reads up to kSwsU - 1 entries
        // on, and multiplies them by zero rows: the zero table gives 0)
        for (int i = tid; i < nn * RW + kSwsU; i += blockDim.x) {
            const int v = i / RW, q = i - v * RW - kSwsU;
            CoefTab ct{0u, 0u, 0u, 0u, 0u};
            if (q >= 0 && v < nn && (uint32_t)q < pl.fe[v].y - pl.fe[v].x) ct = make_coef_tab(CB[v * W + q]);
            AB[i] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
            TC[i] = ct.c;
        }
        for (int k = 0; k < (int)rfl((uint32_t)pl.nempty); k++)
            for (uint32_t cu = tid; cu < a.ncu && CHK_IDX(a.chk, j0 + pl.empty[k], a.nrep, 3); cu += blockDim.x) {
                const uint32_t z[C] = {};
                stc<C>(a.rep + (j0 + pl.empty[k]) * a.stride + cu * 4u * C, z);
            }
        __syncthreads();
        const int A = (int)rfl((uint32_t)pl.A), P = (int)rfl((uint32_t)pl.P);
        for (uint32_t c0 = 0; c0 < a.ncu; c0 += a.cpass) {
            const uint32_t cu = c0 + tid;
            const bool live = cu < a.ncu;
            const uint32_t loff = min(cu, a.ncu - 1) * 4u * C;
            for (int p = 0; p < P; p++) {
                switch (A) {
                case 1: sws_pass<1, C>(a, pl, AB, TC, j0, p, P, loff, live); break;
                case 2: sws_pass<2, C>(a, pl, AB, TC, j0, p, P, loff, live); break;
                case 3: sws_pass<3, C>(a, pl, AB, TC, j0, p, P, loff, live); break;
                default: sws_pass<kSwsAmax, C>(a, pl, AB, TC, j0, p, P, loff, live); break;
                }
            }
        }
        __syncthreads();  // the next segment's plan and tables reuse the LDS
    }
}

}  // namespace

namespace {
// Resident workgroups of the streaming kernel on the current device (the
// occupancy query costs microseconds per call; per-connection encoders launch
// small batches often): cached per (device, C, block, LDS).
uint64_t resident(const void *fn, int C, uint32_t block, uint32_t lds) {
    struct Entry {
        int dev, C;
        uint32_t block, lds;
        uint64_t r;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    {
        std::lock_guard<std::mutex> g(mu);
        for (const Entry &x : cache)
            if (x.dev == dev && x.C == C && x.block == block && x.lds == lds) return x.r;
    }
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, (int)block, lds) != hipSuccess || per < 1) per = 1;
    const uint64_t r = (uint64_t)cus * per;
    std::lock_guard<std::mutex> g(mu);
    if (cache.size() < 64) cache.push_back({dev, C, block, lds, r});
    return r;
}
}  // namespace

template <int C>
const void *sws_fn() {
    return reinterpret_cast<const void *>(sw_stream_kernel<C>);
}

hipError_t launch_sw_stream(SwStreamArgs a, int C, uint32_t budget, hipStream_t s) {
    if (a.nrep == 0) return hipSuccess;
    const void *fn = nullptr;
    switch (C) {
        case 1: fn = sws_fn<1>(); break;
        case 2: fn = sws_fn<2>(); break;
        case 3: fn = sws_fn<3>(); break;
        case 4: fn = sws_fn<4>(); break;
        case 5: fn = sws_fn<5>(); break;
        default: return hipErrorInvalidValue;
    }
    const int W = std::max(1, a.max_window);
    a.max_window = W;
    // column passes of at most 512 lanes, as even as 64-lane waves allow
    const uint32_t passes = (a.ncu + 511) / 512;
    a.cpass = ((a.ncu + passes - 1) / passes + 63) / 64 * 64;
    // LDS per workgroup in proportion to its waves (kSwsWaveLds each, at most
    // `budget`): a one-wave workgroup (C = 5 over a 1200-B row) with the whole
    // budget would leave 3 waves on a CU
    budget = std::min<uint32_t>(budget, std::max<uint32_t>(1, a.cpass / 64) * kSwsWaveLds);
    a.segcap = (int)std::max<uint32_t>(1, std::min<uint32_t>(kSwSeg, budget / sw_stream_rep_lds(W)));
    a.lds = sw_stream_lds(a.segcap, W);
    hipError_t e = hipSuccess;
    if (a.lds > 64u * 1024u) {
        e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)a.lds);
        if (e != hipSuccess) return e;
    }
    // one round of segments per resident workgroup, sized so the rounds are whole
    const uint64_t R = resident(fn, C, a.cpass, a.lds);
    const uint64_t nseg0 = (a.nrep + a.segcap - 1) / a.segcap;
    const uint64_t rounds = (nseg0 + R - 1) / R;
    a.segcap = (int)std::max<uint64_t>(1, (a.nrep + R * rounds - 1) / (R * rounds));
    a.nseg = (a.nrep + a.segcap - 1) / a.segcap;
    const uint64_t grid = std::min<uint64_t>(a.nseg, R);
    const dim3 gd((unsigned)grid), bd(a.cpass);
    const uint32_t lds = a.lds;
    switch (C) {
        case 1: hipLaunchKernelGGL((sw_stream_kernel<1>), gd, bd, lds, s, a); break;
        case 2: hipLaunchKernelGGL((sw_stream_kernel<2>), gd, bd, lds, s, a); break;
        case 3: hipLaunchKernelGGL((sw_stream_kernel<3>), gd, bd, lds, s, a); break;
        case 4: hipLaunchKernelGGL((sw_stream_kernel<4>), gd, bd, lds, s, a); break;
        default: hipLaunchKernelGGL((sw_stream_kernel<5>), gd, bd, lds, s, a); break;
    }
    return hipGetLastError();
}

}  // namespace fecgpu
