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
#ifndef FECGPU_SWS_WAVE_LDS_KB
#define FECGPU_SWS_WAVE_LDS_KB 12  // multiply-table LDS per wave of a workgroup (capped by the budget)
#endif
constexpr uint32_t kSwsWaveLds = FECGPU_SWS_WAVE_LDS_KB << 10;
#ifndef FECGPU_SWS_AMAX
#define FECGPU_SWS_AMAX 4  // accumulator slots compiled (a segment needing more takes P > 1 passes)
#endif
constexpr int kSwsAmax = FECGPU_SWS_AMAX < kSwSlots ? FECGPU_SWS_AMAX : kSwSlots;
#ifndef FECGPU_SWS_TPF
#define FECGPU_SWS_TPF 0  // multiply tables read one source ahead (A/B: 0.35 vs 0.24 ms cfg7, registers)
#endif
#ifndef FECGPU_SWS_PINGPONG
#define FECGPU_SWS_PINGPONG 1  // row buffers trade roles between batches (else copied)
#endif
#ifndef FECGPU_SWS_LDSBATCH
#define FECGPU_SWS_LDSBATCH 0  // a source pair's tables for every slot loaded before any product
                               // (108 VGPRs instead of 73: cfg7 encode 0.287 vs 0.213 ms, r04: off)
#endif
#ifndef FECGPU_SWS_BUF
#define FECGPU_SWS_BUF 1  // source rows by buffer loads (scalar row offsets)
#endif

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const u32x4 *k4p;  // uniform loads: s_load_dwordx4

#define SWS_WAVE_SYNC()                                         \
    do {                                                        \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                        \
    } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const uint32_t *g32c;
typedef __attribute__((address_space(1))) uint32_t *g32;
typedef __attribute__((address_space(1))) const u32x2 *g64c;
typedef __attribute__((address_space(1))) u32x2 *g64;

// C dwords of a lane: one load / store for C = 1, 2, 4 (4: 16-B aligned, the
// rows are), dword by dword for 3 and 5 (4-B aligned)
typedef __attribute__((address_space(1))) const u32x4 *g128c;
typedef __attribute__((address_space(1))) u32x4 *g128;
template <int C>
__device__ __forceinline__ void ldc(const uint8_t *p, uint32_t (&x)[C]) {
    if constexpr (C == 1) {
        x[0] = *(g32c)(p);
    } else if constexpr (C == 2) {
        const u32x2 v = *(g64c)(p);
        x[0] = v.x;
        x[1] = v.y;
    } else if constexpr (C == 4) {
        const u32x4 v = *(g128c)(p);
        x[0] = v.x;
        x[1] = v.y;
        x[2] = v.z;
        x[3] = v.w;
    } else {
#pragma unroll
        for (int d = 0; d < C; d++) x[d] = ((g32c)(p))[d];
    }
}
// Buffer loads: the resource (a batch's first row, scalar) plus a scalar row
// offset plus this lane's column offset, no per-load address arithmetic on
// the vector ALU.  Word 3 of the resource: raw 32-bit data on gfx9.
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
    // CB null: the tables are in global memory (FECGPU_SWS_SGPR), no coefficients here
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
        if (CB) rlc_coefs_tab(a.rlc, h.key, (int)(end - fss), min((uint32_t)h.dt, 15u), CB + (size_t)v * W);
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

// 4-entry tables: c*x = Q0[x & 3] ^ Q1[(x >> 2) & 3] ^ Q2[(x >> 4) & 3] ^ Q3[x >> 6]
// with Qk[b] = c * (b << 2k): Q0 = TA's low dword, Q3 = TC (make_coef_tab)
template <int C>
struct Split4 {
    uint32_t i[4][C];
};
template <int C>
__device__ __forceinline__ Split4<C> split4(const uint32_t (&x)[C]) {
    Split4<C> s;
#pragma unroll
    for (int d = 0; d < C; d++) {
        s.i[0][d] = x[d] & 0x03030303u;
        s.i[1][d] = (x[d] >> 2) & 0x03030303u;
        s.i[2][d] = (x[d] >> 4) & 0x03030303u;
        s.i[3][d] = (x[d] >> 6) & 0x03030303u;
    }
    return s;
}
__device__ __forceinline__ u32x4 quad_tab(uint32_t c) {
    uint32_t p[8];
    p[0] = c & 0xFFu;
    for (int b = 1; b < 8; b++) p[b] = gf_xtime(p[b - 1]);
    u32x4 q;
    q.x = (p[0] << 8) ^ (p[1] << 16) ^ ((p[0] ^ p[1]) << 24);
    q.y = (p[2] << 8) ^ (p[3] << 16) ^ ((p[2] ^ p[3]) << 24);
    q.z = (p[4] << 8) ^ (p[5] << 16) ^ ((p[4] ^ p[5]) << 24);
    q.w = (p[6] << 8) ^ (p[7] << 16) ^ ((p[6] ^ p[7]) << 24);
    return q;
}

// The global tables (FECGPU_SWS_SGPR): a thread per repair draws its clipped
// window's coefficients and writes their 4-entry tables after a run of
// kSwStreamU zero tables; entries past its window are zero; the array starts
// and ends with kSwStreamU zero tables (sw_stream_gtab_bytes).
__global__ __launch_bounds__(kBlock) void sws_tab_kernel(SwStreamArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    u32x4 *G = reinterpret_cast<u32x4 *>(a.gtab);
    const int W = a.max_window, RW = W + kSwsU;
    const u32x4 z = {0u, 0u, 0u, 0u};
    if (t == 0)
        for (int i = 0; i < kSwsU; i++) {
            G[i] = z;
            G[kSwsU + a.nrep * (uint64_t)RW + i] = z;
        }
    if (t >= a.nrep) return;
    const fecgpu_sw_repair h = a.hdr[t];
    const uint64_t fss = min(h.fss, a.nsrc);
    const int nss = (int)min((uint64_t)min((int)h.nss, W), a.nsrc - fss);
    u32x4 *row = G + kSwsU + t * (uint64_t)RW;
    for (int i = 0; i < kSwsU; i++) row[i] = z;
    Tinymt32 st;
    tinymt32_init(st, h.key & 0xFFFFu);
    const uint32_t dt = min((uint32_t)h.dt, 15u);
    for (int q = 0; q < W; q++) {
        uint32_t c = 0;
        if (q < nss && (dt == 15 || (tinymt32_u32(st) & 0xFu) <= dt)) {
            do {
                c = tinymt32_u32(st) & 0xFFu;
            } while (c == 0);
        }
        row[kSwsU + q] = c ? quad_tab(c) : z;
    }
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

template <int A, int C, bool G>
__device__ __forceinline__ void sws_pass(const SwStreamArgs &a, const SwsPlan &pl, const uint4 *AB,
                                         const uint32_t *TC, uint64_t j0, int p, int P, uint32_t loff,
                                         bool live) {
    const k4p GT = (k4p)a.gtab;  // G: the global tables
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
    const uint8_t *base = a.src + rfl64(pl.lo) * stride;
    // rows s0 .. s0 + U - 1, clamped to hi - 1 (valid rows only).  Every batch
    // issues its loads unconditionally: with a load under a branch the
    // compiler's wait counts merge to the stricter path, and the batch waited
    // for the rows it had just prefetched (s_waitcnt vmcnt(7..0) in its body).
    auto load = [&](uint32_t s0, uint32_t (&x)[U][C]) __attribute__((always_inline)) {
        s0 = rfl(min(s0, hi - 1));
#if FECGPU_SWS_BUF
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(base + (uint64_t)s0 * stride), 0, (int)(U * stride), kRsrcWord3);
        const uint32_t last = rfl(hi - 1 - s0);  // scalar: rows past it reload row hi - 1
#pragma unroll
        for (int i = 0; i < U; i++) ldc_buf<C>(r, loff, min((uint32_t)i, last) * (uint32_t)stride, x[i]);
#else
#pragma unroll
        for (int i = 0; i < U; i++) ldc<C>(base + (uint64_t)min(s0 + (uint32_t)i, hi - 1) * stride + loff, x[i]);
#endif
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
        uint64_t gb[A];  // G: entry of source s of slot m's repair (0: the leading zero run)
#pragma unroll
        for (int m = 0; m < A; m++) {
            if constexpr (G) {
                const uint64_t t = j0 + (dense ? v[m] : rfl(pl.out[min(v[m], (uint32_t)kSwSeg - 1)]));
                gb[m] = f[m] < sn ? (uint64_t)kSwsU + t * RW + U + s - f[m] : 0ull;
            } else {
                const uint32_t tb = f[m] < sn ? v[m] * RW + U + s - f[m] : 0u;
                tab[m] = AB + tb;
                tcb[m] = TC + tb;
            }
        }
        // a batch cut short by a window end multiplies zero rows past it (their
        // table reads stay inside the LDS tables: kSwsU spare entries at the end)
        if (L < (uint32_t)U) {
#pragma unroll
            for (int i = 1; i < U; i++)
#pragma unroll
                for (int d = 0; d < C; d++) X[i][d] = (uint32_t)i < L ? X[i][d] : 0u;
        }
        if constexpr (G) {
            // per source and slot: one s_load_dwordx4 of 4 tables, 4 v_perm
            // with an SGPR table each, two 3-input XORs
#pragma unroll
            for (int i = 0; i < U; i++) {
                const Split4<C> q = split4<C>(X[i]);
#pragma unroll
                for (int m = 0; m < A; m++) {
                    const u32x4 tq = GT[gb[m] + i];
#pragma unroll
                    for (int d = 0; d < C; d++) {
                        uint32_t t = xor3s(acc[m][d], __builtin_amdgcn_perm(tq.x, tq.x, q.i[0][d]),
                                           __builtin_amdgcn_perm(tq.y, tq.y, q.i[1][d]));
                        acc[m][d] = xor3s(t, __builtin_amdgcn_perm(tq.z, tq.z, q.i[2][d]),
                                          __builtin_amdgcn_perm(tq.w, tq.w, q.i[3][d]));
                        asm volatile("" : "+v"(acc[m][d]));
                    }
                }
            }
        } else
        // sources in pairs: the six table lookups of two products fold into
        // the accumulator with three 3-input XORs
#pragma unroll
        for (int i = 0; i < U; i += 2) {
            const SplitC<C> s0 = split_c<C>(X[i]), s1 = split_c<C>(X[i + 1]);
#if FECGPU_SWS_LDSBATCH
            // every slot's tables for the pair in flight at once (one LDS wait,
            // not one per slot)
            uint4 A0[A], A1[A];
            uint32_t C0[A], C1[A];
#pragma unroll
            for (int m = 0; m < A; m++) {
                A0[m] = tab[m][i];
                A1[m] = tab[m][i + 1];
                C0[m] = tcb[m][i];
                C1[m] = tcb[m][i + 1];
            }
#pragma unroll
            for (int m = 0; m < A; m++) {
                asm("" : "+v"(A0[m].x), "+v"(A0[m].y), "+v"(A0[m].z), "+v"(A0[m].w), "+v"(C0[m]));
                asm("" : "+v"(A1[m].x), "+v"(A1[m].y), "+v"(A1[m].z), "+v"(A1[m].w), "+v"(C1[m]));
            }
#endif
#pragma unroll
            for (int m = 0; m < A; m++) {
#if FECGPU_SWS_LDSBATCH
                const uint4 a0 = A0[m], a1 = A1[m];
                const uint32_t c0 = C0[m], c1 = C1[m];
#else
                uint4 a0 = tab[m][i], a1 = tab[m][i + 1];
                uint32_t c0 = tcb[m][i], c1 = tcb[m][i + 1];
                // tables stay in vector registers (uniform values would be
                // moved to scalar ones with a readfirstlane each)
                asm("" : "+v"(a0.x), "+v"(a0.y), "+v"(a0.z), "+v"(a0.w), "+v"(c0));
                asm("" : "+v"(a1.x), "+v"(a1.y), "+v"(a1.z), "+v"(a1.w), "+v"(c1));
#endif
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
                if (live) stc<C>(a.rep + (j0 + o) * stride + loff, acc[m]);
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
#if FECGPU_SWS_PINGPONG
    // two batches per trip, the row buffers trading roles (no copies); one
    // exit on a flag (a loop with two exits loses the bookkeeping's
    // uniformity: vector registers and readfirstlane loops around the loads)
    bool go = true;
    while (go) {
        go = batch(XA, XB);
        if (go) go = batch(XB, XA);
    }
#else
    while (batch(XA, XB)) {
#pragma unroll
        for (int i = 0; i < U; i++)
#pragma unroll
            for (int d = 0; d < C; d++) XA[i][d] = XB[i][d];
    }
#endif
}

template <int C, bool G>
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
        if (wave == 0) sws_plan(a, pl, G ? nullptr : CB, j0, n, lane);
        __syncthreads();
        const int nn = (int)rfl((uint32_t)pl.nn);
        // every entry a batch may read is a table: zero runs, coefficients,
        // zeros past a window (a cut-short batch reads up to kSwsU - 1 entries
        // on, and multiplies them by zero rows: the zero table gives 0)
        for (int i = tid; !G && i < nn * RW + kSwsU; i += blockDim.x) {
            const int v = i / RW, q = i - v * RW - kSwsU;
            CoefTab ct{0u, 0u, 0u, 0u, 0u};
            if (q >= 0 && v < nn && (uint32_t)q < pl.fe[v].y - pl.fe[v].x) ct = make_coef_tab(CB[v * W + q]);
            AB[i] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
            TC[i] = ct.c;
        }
        for (int k = 0; k < (int)rfl((uint32_t)pl.nempty); k++)
            for (uint32_t cu = tid; cu < a.ncu; cu += blockDim.x) {
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
                case 1: sws_pass<1, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
                case 2: sws_pass<2, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
                case 3: sws_pass<3, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
#if FECGPU_SWS_AMAX > 4
                case 4: sws_pass<4, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
                case 5: sws_pass<5, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
                case 6: sws_pass<6, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
                case 7: sws_pass<7, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
                default: sws_pass<8, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
#else
                default: sws_pass<4, C, G>(a, pl, AB, TC, j0, p, P, loff, live); break;
#endif
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

template <int C, bool G>
const void *sws_fn() {
    return reinterpret_cast<const void *>(sw_stream_kernel<C, G>);
}

hipError_t launch_sw_stream(SwStreamArgs a, int C, uint32_t budget, hipStream_t s) {
    if (a.nrep == 0) return hipSuccess;
    const bool G = FECGPU_SWS_SGPR && a.gtab && C <= 2;
    const void *fn = nullptr;
    switch (C) {
        case 1: fn = G ? sws_fn<1, true>() : sws_fn<1, false>(); break;
        case 2: fn = G ? sws_fn<2, true>() : sws_fn<2, false>(); break;
        case 3: fn = sws_fn<3, false>(); break;
        case 4: fn = sws_fn<4, false>(); break;
        case 5: fn = sws_fn<5, false>(); break;
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
    a.segcap = G ? kSwSeg : (int)std::max<uint32_t>(1, std::min<uint32_t>(kSwSeg, budget / sw_stream_rep_lds(W)));
    a.lds = G ? 0u : sw_stream_lds(a.segcap, W);
    if (G) {
        hipLaunchKernelGGL(sws_tab_kernel, dim3((unsigned)((a.nrep + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
        const hipError_t e0 = hipGetLastError();
        if (e0 != hipSuccess) return e0;
    }
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
    const uint32_t lds = G ? 0u : a.lds;
    switch (C) {
        case 1:
            if (G) hipLaunchKernelGGL((sw_stream_kernel<1, true>), gd, bd, lds, s, a);
            else hipLaunchKernelGGL((sw_stream_kernel<1, false>), gd, bd, lds, s, a);
            break;
        case 2:
            if (G) hipLaunchKernelGGL((sw_stream_kernel<2, true>), gd, bd, lds, s, a);
            else hipLaunchKernelGGL((sw_stream_kernel<2, false>), gd, bd, lds, s, a);
            break;
        case 3: hipLaunchKernelGGL((sw_stream_kernel<3, false>), gd, bd, lds, s, a); break;
        case 4: hipLaunchKernelGGL((sw_stream_kernel<4, false>), gd, bd, lds, s, a); break;
        default: hipLaunchKernelGGL((sw_stream_kernel<5, false>), gd, bd, lds, s, a); break;
    }
    return hipGetLastError();
}

}  // namespace fecgpu
