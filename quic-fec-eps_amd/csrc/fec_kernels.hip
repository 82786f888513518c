// fec_kernels.hip — gfx950 kernels of the FEC hot path.
//
// Work decomposition.  The unit of work is a *slot*: one
// 16-byte column of one window.  A lane owns a slot and walks the window's
// input symbols with coalesced 16-B loads (consecutive lanes = consecutive
// columns of one symbol row), accumulates up to r outputs in registers and
// stores them.  All kernels are persistent: the grid is sized to the blocks
// that fit the chip at once and loops, so no partial last wave of blocks.
//   flat mode  — every window has the same S and stride: slot s -> window
//                s / ncol, column s % ncol, advanced incrementally.
//   group mode — per-window S or ragged offsets, and every GF decode: a
//                workgroup takes `wpb` windows at a time, plans them in LDS
//                (geometry, and for GF decode the per-window decode tables),
//                then streams the flattened column range of those windows.
//
// GF(2^8) multiply (DESIGN.md §GF multiply): a coefficient c becomes three
// byte tables over 3+3+2 bits of the data byte, so c*x for four packed bytes
// is 3 v_perm_b32, accumulated with gfx950's 3-input v_bitop3_b32 (1.5-2 ops
// per product); the bit-field split of the data (5 VALU per dword) is shared
// by every output.
#include "fec_internal.h"

#include <utility>

// Tuning constants (measured on the box; the A/B knobs that lost were removed in r05)
// XOR encode: input rows loaded per batch (rounded up to r); 4 beat 2 and 8 at
// 2 workgroups/CU (scripts/sweep.py, r01)
constexpr int kXorLoads = 4;
// GF bodies: input rows loaded per batch.  r <= 4 runs best with 2 rows in
// flight per lane (fewer bytes in flight keep HBM efficient), r = 8 with 8
// (its long VALU phase needs more loads queued; scripts/sweep.py)
#define GF_ENC_U(R) ((R) <= 4 ? 2 : 8)
// GF decode: input rows loaded per batch.  Decode's input rows come through an
// LDS index (received sources, chosen repairs), so a deeper batch hides that
// extra latency: 8 rows at r <= 4 (cfg3 decode -1.7% vs 2, scripts/ab.py r01);
// at r > 4, 4 rows, which with the paired-row products below leave the
// registers for 3 waves per SIMD (cfg4 decode 4.55 vs 4.59 ms, r06)
#define GF_DEC_U(R) ((R) > 4 ? 4 : 8)
// GF encode at r > 4 (VALU-bound, paired rows): at least 3 waves per SIMD, a
// few spilled registers for occupancy: 7% faster than 2 waves on cfg4 (r01)
#define GFE_WAVES __attribute__((amdgpu_waves_per_eu(R > 4 ? 3 : 1, 8)))

namespace fecgpu {

__constant__ GfTables c_gf = make_gf_tables();

// ------------------------------------------------------------ helpers ---
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Symbol data is always in global memory.  Pointers that pass through LDS
// (group-mode window bases) are generic to the compiler and would become
// flat_load/flat_store, which count against lgkmcnt as well as vmcnt and force
// conservative waits on LDS traffic; the explicit address space keeps them
// global_load_dwordx4 / global_store_dwordx4.
typedef __attribute__((address_space(1))) const u32x4 *gptr_c;
typedef __attribute__((address_space(1))) u32x4 *gptr;

#if FECGPU_CHECK
__shared__ ChkRange s_chk;                   // the launch's ranges (copied by CHK_PROLOGUE)
__device__ unsigned long long g_chk_bad[2];  // faulting accesses, first address

__device__ __forceinline__ bool chk_ok(const uint8_t *p) {
    const uint64_t x = reinterpret_cast<uint64_t>(p);
    bool ok = false;
#pragma unroll
    for (int i = 0; i < kChkRanges; i++) ok |= s_chk.n[i] >= 16 && x - s_chk.lo[i] <= s_chk.n[i] - 16;
    if (!ok) {
        atomicAdd(&g_chk_bad[0], 1ull);
        atomicCAS(&g_chk_bad[1], 0ull, (unsigned long long)x);
    }
    return ok;
}
#define CHK_PROLOGUE(a)                      \
    do {                                     \
        if (threadIdx.x == 0) s_chk = (a).chk; \
        __syncthreads();                     \
    } while (0)
#else
#define CHK_PROLOGUE(a) \
    do {                \
    } while (0)
#endif

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
#if FECGPU_CHECK
    if (!chk_ok(p)) return make_uint4(0, 0, 0, 0);
#endif
    const u32x4 v = *(gptr_c)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) {
#if FECGPU_CHECK
    if (!chk_ok(p)) return;
#endif
    // nontemporal: repairs and recovered symbols are written once and not read
    // back by the kernel (+2.8% on cfg2, neutral on cfg3 / cfg4; r01)
    const u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (gptr)(p));
}
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
    return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ uint4 and4(uint4 a, uint32_t m) { return make_uint4(a.x & m, a.y & m, a.z & m, a.w & m); }
__device__ __forceinline__ uint4 zero4() { return make_uint4(0, 0, 0, 0); }

struct Split {
    uint32_t a[4], b[4], c[4];
};

__device__ __forceinline__ Split split(uint4 v) {
    Split s;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s.a[i] = d[i] & 0x07070707u;
        s.b[i] = (d[i] >> 3) & 0x07070707u;
        s.c[i] = (d[i] >> 6) & 0x03030303u;
    }
    return s;
}

// a ^ b ^ c in one gfx950 VALU op (truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc ^= c*x for the 4 dwords of a column: 3 perm + 2 VALU per dword
__device__ __forceinline__ uint32_t gmac1(uint32_t acc, const Split &s, int i, uint4 ab, uint32_t tc) {
    return xor3(acc, __builtin_amdgcn_perm(ab.y, ab.x, s.a[i]), __builtin_amdgcn_perm(ab.w, ab.z, s.b[i])) ^
           __builtin_amdgcn_perm(tc, tc, s.c[i]);
}
__device__ __forceinline__ void gmac(uint4 &acc, const Split &s, uint4 ab, uint32_t tc) {
    acc.x = gmac1(acc.x, s, 0, ab, tc);
    acc.y = gmac1(acc.y, s, 1, ab, tc);
    acc.z = gmac1(acc.z, s, 2, ab, tc);
    acc.w = gmac1(acc.w, s, 3, ab, tc);
}

// acc ^= c0*x0 ^ c1*x1 (two input rows): 6 perm + 3 xor3 per dword
__device__ __forceinline__ uint32_t gmac2_1(uint32_t acc, const Split &s0, const Split &s1, int i,
                                            uint4 ab0, uint32_t tc0, uint4 ab1, uint32_t tc1) {
    uint32_t t = xor3(acc, __builtin_amdgcn_perm(ab0.y, ab0.x, s0.a[i]),
                      __builtin_amdgcn_perm(ab0.w, ab0.z, s0.b[i]));
    t = xor3(t, __builtin_amdgcn_perm(tc0, tc0, s0.c[i]), __builtin_amdgcn_perm(ab1.y, ab1.x, s1.a[i]));
    return xor3(t, __builtin_amdgcn_perm(ab1.w, ab1.z, s1.b[i]), __builtin_amdgcn_perm(tc1, tc1, s1.c[i]));
}
__device__ __forceinline__ void gmac2(uint4 &acc, const Split &s0, const Split &s1, uint4 ab0,
                                      uint32_t tc0, uint4 ab1, uint32_t tc1) {
    acc.x = gmac2_1(acc.x, s0, s1, 0, ab0, tc0, ab1, tc1);
    acc.y = gmac2_1(acc.y, s0, s1, 1, ab0, tc0, ab1, tc1);
    acc.z = gmac2_1(acc.z, s0, s1, 2, ab0, tc0, ab1, tc1);
    acc.w = gmac2_1(acc.w, s0, s1, 3, ab0, tc0, ab1, tc1);
}

__device__ __forceinline__ void win_geom(const BatchArgs &a, uint64_t w, uint64_t &base,
                                         uint32_t &stride, uint32_t &S) {
    S = a.sym_len ? a.sym_len[w] : a.S_all;
    if (a.win_off) {
        // 64-bit wrap-around add: offsets may point below `win` (pooled windows)
        base = reinterpret_cast<uint64_t>(a.win) + a.win_off[w];
        if (a.off_stride) {
            stride = a.off_stride;
            S = min(S, stride);  // a symbol never spills into the next row
        } else {
            S = min(S, (uint32_t)FECGPU_MAX_SYMBOL);  // keeps group prefix sums in 32 bits
            stride = (S + 15u) & ~15u;
        }
    } else {
        base = reinterpret_cast<uint64_t>(a.win) + w * a.wpitch;
        stride = a.stride;
        S = min(S, stride);  // a bad sym_len[w] (device data, unchecked) stays in its rows
    }
}

// Inclusive scan of per-window column counts by wave 0 (nb <= 64).
__device__ __forceinline__ void block_prefix(uint32_t *pfx, uint32_t v, int lane) {
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    pfx[lane + 1] = x;
    if (lane == 0) pfx[0] = 0;
}

#define WAVE_SYNC()                                             \
    do {                                                        \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
        __builtin_amdgcn_wave_barrier();                        \
    } while (0)

// ------------------------------------------------------ slot iterators ---
// XCD-aware work split (speed only, never correctness): the dispatcher deals
// workgroups round-robin over the 8 XCDs, so b, b + 8, b + 16, ... share an
// L2.  Work units (256-slot chunks, or window groups) are cut into `nx`
// contiguous regions and region b % nx is walked by workgroups b / nx, so
// neighbouring units — which share the 128-B lines straddling 1200-B symbol
// rows and window edges — are fetched through one L2 instead of two.
struct XcdRange {
    uint64_t cur, hi, step;
};

__device__ __forceinline__ XcdRange xcd_range(uint64_t nunits, uint32_t nx) {
    const uint32_t bx = blockIdx.x % nx, bi = blockIdx.x / nx, nbx = gridDim.x / nx;
    const uint64_t lo = nunits * bx / nx, hi = nunits * (bx + 1) / nx;
    return {lo + bi, hi, nbx};
}

// Flat mode: the lane's slots are chunk*256 + tid for its region's chunks;
// (window, column) advance incrementally by the per-iteration slot step
// (step / ncol and step % ncol precomputed on host).
template <class Body>
__device__ __forceinline__ void for_flat_slots(const BatchArgs &a, Body &&body) {
    const uint32_t ncol = a.ncol;
    const uint64_t total = a.nwin * ncol;
    XcdRange xr = xcd_range((total + kBlock - 1) / kBlock, a.nx);
    if (xr.cur >= xr.hi) return;
    uint64_t s = xr.cur * kBlock + threadIdx.x;
    uint64_t w = s / ncol;
    uint32_t col = (uint32_t)(s - w * ncol);
    const uint64_t wbytes = a.wpitch;
    for (; xr.cur < xr.hi; xr.cur += xr.step) {
        // lanes past the end skip the body (measured faster than running a
        // clamped dummy slot to keep control flow uniform: scripts/ab.py, r01)
        if (s < total) body(a.win + w * wbytes + col * 16u, a.stride, w, col, true);
        s += xr.step * kBlock;
        col += a.step_col;
        w += a.step_win;
        if (col >= ncol) {
            col -= ncol;
            w++;
        }
    }
}

// Group mode header: geometry of windows [w0, w0 + nb) into LDS; `ncol_eff`
// lets a plan drop windows with nothing to do (decode).
struct GroupLds {
    uint32_t pfx[kMaxWpb + 1];
    uint64_t base[kMaxWpb];
    uint32_t stride[kMaxWpb];
    uint32_t ncol[kMaxWpb];
};

// Streams the flattened columns of the current group:
// body(base_of_column, stride, wl, valid = true).
template <class Body>
__device__ __forceinline__ void for_group_slots(const GroupLds &g, int nb, Body &&body) {
    const uint32_t total = g.pfx[nb];
    int wl = 0;
    for (uint32_t s = threadIdx.x; s < total; s += kBlock) {
        while (s >= g.pfx[wl + 1]) wl++;
        const uint32_t col = s - g.pfx[wl];
        body(reinterpret_cast<uint8_t *>(g.base[wl]) + col * 16u, g.stride[wl], wl, true);
    }
}

__device__ __forceinline__ void group_geometry(const BatchArgs &a, GroupLds &g, uint64_t w0, int nb) {
    const int tid = threadIdx.x;
    if (tid < nb) {
        uint64_t base; uint32_t stride, S;
        win_geom(a, w0 + tid, base, stride, S);
        g.base[tid] = base;
        g.stride[tid] = stride;
        g.ncol[tid] = (S + 15u) >> 4;
    }
}

// ============================================================== bodies ===
// XOR encode (a4): R_g = xor of S_j, j = g (mod r).  All loads of a slot are
// issued before the xors (8 x 16 B in flight per lane at k = 8).
template <int R>
__device__ __forceinline__ void xor_encode_slot(uint8_t *base, uint32_t stride, int k, bool valid,
                                                uint64_t od) {
    constexpr int STEP = R * ((kXorLoads + R - 1) / R);
    uint4 acc[R];
#pragma unroll
    for (int g = 0; g < R; g++) acc[g] = zero4();
    for (int j0 = 0; j0 < k; j0 += STEP) {
        // branch-free: rows past k re-read row k-1 (cache hit) and are not accumulated
        uint4 v[STEP];
#pragma unroll
        for (int t = 0; t < STEP; t++) v[t] = ld16(base + (uint32_t)min(j0 + t, k - 1) * stride);
#pragma unroll
        for (int t = 0; t < STEP; t++)
            if (j0 + t < k) acc[t % R] = xor4(acc[t % R], v[t]);
    }
    if (valid) {
#pragma unroll
        for (int g = 0; g < R; g++) st16(base + od + (size_t)(k + g) * stride, acc[g]);
    }
}

// GF multiply-accumulate over k inputs of one slot: acc[m] ^= D[q][m] * in_q
// for q < k, m < min(ne, R), U inputs loaded per batch (register double
// buffering measured no gain and cost occupancy, r01).  `addr(q)` gives input
// q's column address, tables are [q][m] in LDS.  PAIR: rows in pairs, one
// xor3 chain folds both rows' lookups (1.5 instead of 2 ops per product:
// encode, cfg4 -14 %; in decode the register pressure cost 12 % on cfg3, r01).
template <int R, int U, bool PAIR, class Addr, class TabP, class TcP>
__device__ __forceinline__ void gf_mac_batched(uint4 (&acc)[R], int k, int ne, Addr &&addr,
                                               TabP tab, TcP tc) {
    uint4 va[U];
    auto load = [&](uint4(&v)[U], int q0) {
#pragma unroll
        for (int t = 0; t < U; t++) v[t] = ld16(addr(min(q0 + t, k - 1)));  // past k: unused re-read
    };
    auto mul = [&](const uint4(&v)[U], int q0) {
        int t0 = 0;
        // PAIR: rows in pairs, one xor3 chain folds both rows' lookups
#pragma unroll
        for (int t = 0; t + 1 < U; t += 2) {
            if (PAIR && q0 + t + 1 < k) {
                const Split s0 = split(v[t]), s1 = split(v[t + 1]);
                const int row = __builtin_amdgcn_readfirstlane((q0 + t) * R);
#pragma unroll
                for (int m = 0; m < R; m++)
                    if (m < ne) gmac2(acc[m], s0, s1, tab[row + m], tc[row + m], tab[row + R + m], tc[row + R + m]);
                t0 = t + 2;
            }
        }
#pragma unroll
        for (int t = 0; t < U; t++) {
            if (t >= t0 && q0 + t < k) {
                const Split sp = split(v[t]);
                // wave-uniform row index (lets uniform table reads become scalar loads)
                const int row = __builtin_amdgcn_readfirstlane((q0 + t) * R);
#pragma unroll
                for (int m = 0; m < R; m++)
                    if (m < ne) gmac(acc[m], sp, tab[row + m], tc[row + m]);
            }
        }
    };
    for (int q0 = 0; q0 < k; q0 += U) {
        load(va, q0);
        mul(va, q0);
    }
}

// GF encode (a5): R_i = sum_j C[i][j] * S_j, tables [j][i] in LDS (broadcast reads).
template <int R, int UO, class TabP, class TcP>
__device__ __forceinline__ void gf_encode_slot(uint8_t *base, uint32_t stride, int k, TabP tab,
                                               TcP tc, bool valid, uint64_t od) {
    constexpr int U = UO ? UO : GF_ENC_U(R);
    uint4 acc[R];
#pragma unroll
    for (int m = 0; m < R; m++) acc[m] = zero4();
    gf_mac_batched<R, U, true>(acc, k, R, [&](int q) { return base + (uint32_t)q * stride; }, tab, tc);
    if (valid) {
#pragma unroll
        for (int m = 0; m < R; m++) st16(base + od + (size_t)(k + m) * stride, acc[m]);
    }
}

// XOR decode (a6/a8), planned inline from the window's present mask: every
// group with exactly one missing source and its repair present is rebuilt as
// repair ^ (other members).  Loads of all recoverable groups are issued first.
// Returns the window status (1 if some source stays missing).
template <int R>
__device__ __forceinline__ uint32_t xor_decode_slot(const BatchArgs &a, uint8_t *base,
                                                    uint32_t stride, uint64_t pres, bool valid) {
    const int k = a.k;
    const uint64_t kmask = (k >= 64) ? ~0ull : ((1ull << k) - 1);
    const uint64_t miss = ~pres & kmask;
    uint32_t bad = 0;
#pragma unroll
    for (int g = 0; g < R; g++) {
        const uint64_t gm = a.gmask[g];
        const uint64_t mg = miss & gm;
        if (!mg) continue;
        const bool rec = ((mg & (mg - 1)) == 0) && ((pres >> (k + g)) & 1);
        if (!rec) {
            bad = 1;
            continue;
        }
        const int m = __ffsll((unsigned long long)mg) - 1;
        uint4 acc = ld16(base + (size_t)(k + g) * stride);
        for (int j0 = g; j0 < k; j0 += 8 * R) {
            uint4 v[8];
#pragma unroll
            for (int t = 0; t < 8; t++) {
                const int j = j0 + t * R;
                v[t] = (j < k && j != m) ? ld16(base + (size_t)j * stride) : zero4();
            }
#pragma unroll
            for (int t = 0; t < 8; t++) acc = xor4(acc, v[t]);
        }
        if (valid) st16(base + a.out_delta + (size_t)m * stride, acc);
    }
    return bad;
}

// ============================================================ encode ===
template <int R, bool FLAT>
__global__ __launch_bounds__(kBlock) void xor_encode_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    if constexpr (FLAT) {
        for_flat_slots(a, [&](uint8_t *p, uint32_t stride, uint64_t w, uint32_t, bool valid) {
            xor_encode_slot<R>(p, stride, a.k, valid, a.out_delta + w * a.out_wdelta);
        });
    } else {
        __shared__ GroupLds g;
        for (XcdRange xr = xcd_range((a.nwin + a.wpb - 1) / a.wpb, a.nx); xr.cur < xr.hi;
             xr.cur += xr.step) {
            const uint64_t w0 = xr.cur * a.wpb;
            const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
            group_geometry(a, g, w0, nb);
            __syncthreads();
            if (threadIdx.x < 64) block_prefix(g.pfx, (int)threadIdx.x < nb ? g.ncol[threadIdx.x] : 0u, threadIdx.x);
            __syncthreads();
            for_group_slots(g, nb, [&](uint8_t *p, uint32_t stride, int wl, bool valid) {
                xor_encode_slot<R>(p, stride, a.k, valid, a.out_delta + (w0 + wl) * a.out_wdelta);
            });
            __syncthreads();
        }
    }
}

// UO: input rows per load batch (0 = GF_ENC_U(R)); 8 for windows in mapped
// host memory, where each batch of loads is a PCIe round trip.
template <int R, bool FLAT, int UO = 0>
__global__ __launch_bounds__(kBlock) GFE_WAVES void gf_encode_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    const int k = a.k;
    extern __shared__ uint4 dyn[];
    uint4 *tab = dyn;
    uint32_t *tc = reinterpret_cast<uint32_t *>(dyn + k * R);
    for (int i = threadIdx.x; i < k * R; i += kBlock) {
        tab[i] = a.enc_ab[i];
        tc[i] = a.enc_c[i];
    }
    __syncthreads();
    if constexpr (FLAT) {
        for_flat_slots(a, [&](uint8_t *p, uint32_t stride, uint64_t w, uint32_t, bool valid) {
            gf_encode_slot<R, UO>(p, stride, k, tab, tc, valid, a.out_delta + w * a.out_wdelta);
        });
    } else {
        __shared__ GroupLds g;
        for (XcdRange xr = xcd_range((a.nwin + a.wpb - 1) / a.wpb, a.nx); xr.cur < xr.hi;
             xr.cur += xr.step) {
            const uint64_t w0 = xr.cur * a.wpb;
            const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
            group_geometry(a, g, w0, nb);
            __syncthreads();
            if (threadIdx.x < 64) block_prefix(g.pfx, (int)threadIdx.x < nb ? g.ncol[threadIdx.x] : 0u, threadIdx.x);
            __syncthreads();
            for_group_slots(g, nb, [&](uint8_t *p, uint32_t stride, int wl, bool valid) {
                gf_encode_slot<R, UO>(p, stride, k, tab, tc, valid, a.out_delta + (w0 + wl) * a.out_wdelta);
            });
            __syncthreads();
        }
    }
}

// ================================== gathered-store encode (round 6) ===
// Uniform windows of short symbols (a row of at most kBlock 16-B columns).
// A 1200-B row is 9.4 128-B lines, and the flat kernels' wave of 64 slots
// stores a repair row in one or two pieces that straddle windows, so most of
// a row's lines are completed by two different waves at different times.
// The same HBM bytes then move at 4.8 TB/s on cfg3's mix against 5.25-5.4
// when every repair row is stored as one contiguous run
// (scripts/win_probe.hip, profiles/r06_store_pattern_probe.json).  Here a
// workgroup takes a.wpb whole windows per step with the flat kernels' lanes
// (lane = window, 16-B column; rows loaded from HBM as before), writes the
// repairs to LDS, and after one barrier stores each window's r repair rows
// front to back, consecutive lanes on consecutive 16-B chunks.  Two LDS
// images alternate, so the next step's writes never meet this step's reads
// and one barrier per step suffices.
struct FastDiv {
    uint32_t d, m;  // q / d = umulhi(q, m) for q * d < 2^32 (m = ceil(2^32 / d))
};
__device__ __forceinline__ FastDiv fdiv_make(uint32_t d) { return {d, d > 1 ? 0xFFFFFFFFu / d + 1u : 0u}; }
__device__ __forceinline__ uint32_t fdiv(uint32_t q, FastDiv f) { return f.d > 1 ? __umulhi(q, f.m) : q; }

// ================================================ bit-sliced GF encode ===
// GF encode for codes whose matrix is known at compile time (DESIGN.md §GF
// bit-slicing).  Multiplying by a constant c is linear over GF(2): output bit
// p of c*x is the XOR of the input bits q for which bit p of c*2^q is set.  A
// lane takes 32 byte positions of a window (two 16-B columns, A = u and
// B = u + half the columns, so loads stay coalesced), transposes each source's
// 8 dwords into 8 bit planes (plane q = bit q of the 32 bytes, in a fixed
// lane order), and every output plane becomes a compile-time XOR of input
// planes.  Per source the 15 XOR combinations of planes 0-3 and of planes
// 4-7 are formed once (those used), so an output plane costs one 3-input XOR.
// No v_perm, no tables: ~150 VALU ops per source and 32 bytes at r = 8
// against ~450 v_perm-weighted cycles for the table multiply.  Bytes are the
// same as the table multiply's (tests/test_gpu_parity.py).
namespace bs {

constexpr GfTables kGf = make_gf_tables();

constexpr uint8_t gmul(uint8_t a, uint8_t b) {
    return (a && b) ? kGf.exp[kGf.log[a] + kGf.log[b]] : 0;
}

// masks[j][i][p]: input planes of source j feeding output plane p of repair i
// (M: the code's matrix, fecgpu_matrix)
template <int K, int R, int M>
struct Masks {
    uint8_t m[K][R][8];
    constexpr Masks() : m{} {
        constexpr ParityRows<K, R, M> P{};
        for (int j = 0; j < K; j++)
            for (int i = 0; i < R; i++) {
                const uint8_t c = P.p[i][j];
                for (int q = 0; q < 8; q++) {
                    const uint8_t col = gmul(c, (uint8_t)(1u << q));
                    for (int p = 0; p < 8; p++)
                        if ((col >> p) & 1) m[j][i][p] |= (uint8_t)(1u << q);
                }
            }
    }
};

// (m & x) | (~m & y) as one v_bitop3_b32 (truth table of S0 ? S1 : S2 over
// S0 = 0xF0, S1 = 0xCC, S2 = 0xAA).  The intrinsic keeps the optimiser from
// distributing the planes' XORs through the selects, which multiplies live
// values (masked halves of every plane) and spills.
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t x, uint32_t y) {
    return __builtin_amdgcn_bitop3_b32(m, x, y, 0xCA);
}

// 8 x 8 bit transpose in every byte lane of d[0..7] (rows = dwords, columns =
// bits of the byte): three block-swap stages, 2 shifts + 2 selects per pair.
// An involution, so the same call turns output planes back into bytes.
__device__ __forceinline__ void tr8(uint32_t (&d)[8]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t x = d[i], y = d[i + 4];
        d[i] = bsel(0xF0F0F0F0u, y << 4, x);
        d[i + 4] = bsel(0x0F0F0F0Fu, x >> 4, y);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
        if (i & 2) continue;
        const uint32_t x = d[i], y = d[i + 2];
        d[i] = bsel(0xCCCCCCCCu, y << 2, x);
        d[i + 2] = bsel(0x33333333u, x >> 2, y);
    }
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        const uint32_t x = d[i], y = d[i + 1];
        d[i] = bsel(0xAAAAAAAAu, y << 1, x);
        d[i + 1] = bsel(0x55555555u, x >> 1, y);
    }
}

template <int K, int R, int M>
inline constexpr Masks<K, R, M> kMasks{};

// a ^ b through the bitop3 intrinsic (S0 ^ S1 = 0xF0 ^ 0xCC): opaque to the
// reassociation pass, which otherwise flattens every output plane into one
// XOR over all sources' planes, undoes the shared combinations and keeps
// planes of many sources live at once
__device__ __forceinline__ uint32_t oxor(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_bitop3_b32(a, b, b, 0x3C);
}

// output plane IP % 8 of repair IP / 8 takes source J's planes (compile time)
template <int K, int R, int M, int J, int IP>
__device__ __forceinline__ void plane(uint32_t (&acc)[R][8], const uint32_t (&lo)[16], const uint32_t (&hi)[16]) {
    constexpr int m = kMasks<K, R, M>.m[J][IP / 8][IP % 8], l = m & 15, h = m >> 4;
    uint32_t &v = acc[IP / 8][IP % 8];
    if constexpr (J == 0) v = l && h ? oxor(lo[l], hi[h]) : (l ? lo[l] : hi[h]);
    else if constexpr (l && h) v = xor3(v, lo[l], hi[h]);
    else if constexpr (l) v = oxor(v, lo[l]);
    else if constexpr (h) v = oxor(v, hi[h]);
}

// acc ^= source J's contribution to every repair, from its planes x
template <int K, int R, int M, int J, int... IP>
__device__ __forceinline__ void source(const uint32_t (&x)[8], uint32_t (&acc)[R][8],
                                       std::integer_sequence<int, IP...>) {
    uint32_t lo[16], hi[16];
    lo[0] = hi[0] = 0;
#pragma unroll
    for (int s = 1; s < 16; s++) {
        const int b = __builtin_ctz(s), rest = s & (s - 1);
        lo[s] = rest ? oxor(lo[rest], x[b]) : x[b];
        hi[s] = rest ? oxor(hi[rest], x[4 + b]) : x[4 + b];
    }
    (plane<K, R, M, J, IP>(acc, lo, hi), ...);
    // pin the accumulators here: otherwise IR sinking moves every repair's XOR
    // chain down to its store, past all later sources, and keeps their planes live
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int p = 0; p < 8; p++) asm volatile("" : "+v"(acc[i][p]));
}

// MASKED (the syndrome decode): source J0 + T is loaded only when bit J0 + T of
// pm is set, and is zero otherwise (a missing row is never read)
template <int T, bool MASKED = false>
__device__ __forceinline__ void load_src(const uint8_t *pa, const uint8_t *pb, uint32_t stride,
                                         uint32_t (&x)[8], uint32_t pm = 0) {
    uint4 va = zero4(), vb = zero4();
    if (!MASKED || ((pm >> T) & 1u)) {
        va = ld16(pa + T * stride);
        vb = ld16(pb + T * stride);
    }
    x[0] = va.x; x[1] = va.y; x[2] = va.z; x[3] = va.w;
    x[4] = vb.x; x[5] = vb.y; x[6] = vb.z; x[7] = vb.w;
}

// one batch of sources J0 + T (pa / pb point at source J0): all loads first,
// then transposes and XORs
template <int K, int R, int M, int J0, bool MASKED, int... T>
__device__ __forceinline__ void batch(const uint8_t *pa, const uint8_t *pb, uint32_t stride,
                                      uint32_t (&acc)[R][8], uint32_t pm, std::integer_sequence<int, T...>) {
    uint32_t x[sizeof...(T)][8];
    (load_src<T, MASKED>(pa, pb, stride, x[T], pm >> J0), ...);
    ((tr8(x[T]), source<K, R, M, J0 + T>(x[T], acc, std::make_integer_sequence<int, R * 8>{}),
      __builtin_amdgcn_sched_barrier(0)), ...);
}

template <int K, int R, int M, int U, int J0, bool MASKED = false>
__device__ __forceinline__ void sources(const uint8_t *pa, const uint8_t *pb, uint32_t stride,
                                        uint32_t (&acc)[R][8], uint32_t pm = 0) {
    if constexpr (J0 < K) {
        batch<K, R, M, J0, MASKED>(pa, pb, stride, acc, pm,
                                   std::make_integer_sequence<int, ((K - J0) < U ? (K - J0) : U)>{});
        // (no workgroup barrier per batch: the r01 knob for one was defined after
        // its use and so never compiled in; every measurement ran without it)
        // advance opaquely, so the compiler does not keep K addresses live at once
        pa += U * stride;
        pb += U * stride;
        asm volatile("" : "+v"(pa), "+v"(pb));
        sources<K, R, M, U, J0 + U, MASKED>(pa, pb, stride, acc, pm);
    }
}

// The syndrome decode's masked sources through a raw buffer resource over the
// workgroup's windows: a row not to be read gets offset kOob, past the
// resource's records, and the load returns zeros without a memory access
// (straight-line code where ld16 under a mask branches per row).  oa / ob:
// the unit's column offsets from the resource base (< 2^31, fec_capi.cpp).
[[maybe_unused]] constexpr uint32_t kOob = 0x80000000u;
[[maybe_unused]] constexpr int kRsrcRaw = 0x00020000;  // buffer resource word 3: raw 32-bit data (gfx9)

__device__ __forceinline__ void load_rs(__amdgpu_buffer_rsrc_t rs, uint32_t oa, uint32_t ob, uint32_t d,
                                        uint32_t (&x)[8]) {
    const u32x4 va = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(oa + d), 0, 0);
    const u32x4 vb = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(ob + d), 0, 0);
    x[0] = va.x; x[1] = va.y; x[2] = va.z; x[3] = va.w;
    x[4] = vb.x; x[5] = vb.y; x[6] = vb.z; x[7] = vb.w;
}

template <int K, int R, int M, int J0, int... T>
__device__ __forceinline__ void batch_rs(__amdgpu_buffer_rsrc_t rs, uint32_t oa, uint32_t ob, uint32_t stride,
                                         uint32_t (&acc)[R][8], uint32_t pm, std::integer_sequence<int, T...>) {
    uint32_t x[sizeof...(T)][8];
    (load_rs(rs, oa, ob, ((pm >> (J0 + T)) & 1u) ? (uint32_t)(J0 + T) * stride : kOob, x[T]), ...);
    ((tr8(x[T]), source<K, R, M, J0 + T>(x[T], acc, std::make_integer_sequence<int, R * 8>{}),
      __builtin_amdgcn_sched_barrier(0)), ...);
}

template <int K, int R, int M, int U, int J0>
__device__ __forceinline__ void sources_rs(__amdgpu_buffer_rsrc_t rs, uint32_t oa, uint32_t ob, uint32_t stride,
                                           uint32_t (&acc)[R][8], uint32_t pm) {
    if constexpr (J0 < K) {
        batch_rs<K, R, M, J0>(rs, oa, ob, stride, acc, pm,
                              std::make_integer_sequence<int, ((K - J0) < U ? (K - J0) : U)>{});
        sources_rs<K, R, M, U, J0 + U>(rs, oa, ob, stride, acc, pm);
    }
}

}  // namespace bs

// bit-sliced encode: sources loaded per batch.  Group mode 8 (> 4 > 2 by
// 1-3 % on cfg4, r01); flat mode 2 (> 4 > 8: k32 r8 4.72 / 4.60 / 4.59 TB/s at
// S = 1200, profiles/r01_bs_layout.txt).  Flat mode, one unit space over all
// uniform windows, beat group mode there: S = 1200 k32 r8 3.84 -> 4.60 TB/s.
constexpr int kBsU = 8, kBsUFlat = 2;

namespace bs {

// The two 16-B columns of unit u of a window with ncol columns (h = ceil(ncol / 2)
// units): u and u + h, so each load instruction stays coalesced (two adjacent
// columns per unit were 10-25 % slower, profiles/r01_bs_layout.txt).  Without
// a second column B repeats A: same inputs, same outputs, so its stores
// rewrite A's bytes with equal values (no branch).
__device__ __forceinline__ void unit_cols(uint8_t *base, uint32_t u, uint32_t h, uint32_t ncol,
                                          uint8_t *&pa, uint8_t *&pb) {
    pa = base + u * 16u;
    pb = u + h < ncol ? pa + h * 16u : pa;
}

// one unit: every source's planes into the R x 8 output planes (U sources
// loaded per batch), then stores
template <int K, int R, int M, int U>
__device__ __forceinline__ void unit(uint8_t *pa, uint8_t *pb, uint32_t stride, bool live, uint64_t od) {
    uint32_t acc[R][8];
    sources<K, R, M, U, 0>(pa, pb, stride, acc);
#pragma unroll
    for (int i = 0; i < R; i++) {
        tr8(acc[i]);
        if (live) {
            st16(pa + od + (size_t)(K + i) * stride, make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
            st16(pb + od + (size_t)(K + i) * stride, make_uint4(acc[i][4], acc[i][5], acc[i][6], acc[i][7]));
        }
    }
}

}  // namespace bs

// Units of h = ceil(ncol / 2) per window, each two 16-B columns (bs::unit_cols).
//   FLAT : uniform windows; units numbered over the whole batch, 256-unit chunks
//          split over the XCDs and walked by a persistent grid.
//   group: per-window S / ragged windows; a workgroup streams the units of
//          `wpb` windows at a time (prefix sums in LDS).
// Trip counts are workgroup-uniform (lanes past the end redo the last unit
// without storing), so the barriers inside a unit are safe.
template <int K, int R, int M, bool FLAT>
__global__ __launch_bounds__(kBlock) void gf_encode_bs_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    if constexpr (FLAT) {
        const uint32_t ncol = a.ncol, h = (ncol + 1) >> 1;
        const uint64_t total = a.nwin * h;
        for (XcdRange xr = xcd_range((total + kBlock - 1) / kBlock, a.nx); xr.cur < xr.hi; xr.cur += xr.step) {
            uint64_t s = xr.cur * kBlock + threadIdx.x;
            const bool live = s < total;
            if (!live) s = total - 1;
            const uint64_t w = s / h;
            const uint32_t u = (uint32_t)(s - w * h);
            uint8_t *pa, *pb;
            bs::unit_cols(a.win + w * a.wpitch, u, h, ncol, pa, pb);
            bs::unit<K, R, M, kBsUFlat>(pa, pb, a.stride, live, a.out_delta + w * a.out_wdelta);
        }
        return;
    } else {
        __shared__ GroupLds g;
        for (XcdRange xr = xcd_range((a.nwin + a.wpb - 1) / a.wpb, a.nx); xr.cur < xr.hi; xr.cur += xr.step) {
            const uint64_t w0 = xr.cur * a.wpb;
            const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
            group_geometry(a, g, w0, nb);
            __syncthreads();
            if (threadIdx.x < 64)
                block_prefix(g.pfx, (int)threadIdx.x < nb ? (g.ncol[threadIdx.x] + 1u) >> 1 : 0u, threadIdx.x);
            __syncthreads();
            const uint32_t total = g.pfx[nb];
            int wl = 0;
            for (uint32_t s0 = 0; s0 < total; s0 += kBlock) {
                const bool live = s0 + threadIdx.x < total;
                const uint32_t s = live ? s0 + threadIdx.x : total - 1;
                while (s >= g.pfx[wl + 1]) wl++;
                uint8_t *pa, *pb;
                bs::unit_cols(reinterpret_cast<uint8_t *>(g.base[wl]), s - g.pfx[wl], g.pfx[wl + 1] - g.pfx[wl],
                              g.ncol[wl], pa, pb);
                bs::unit<K, R, M, kBsU>(pa, pb, g.stride[wl], live, a.out_delta + (w0 + wl) * a.out_wdelta);
            }
            __syncthreads();
        }
    }
}

// gathered-store encode: sources loaded per batch (3: 1.196 vs 1.202 ms at 2, r06)
#ifndef GSE_U
#define GSE_U 3
#endif
// Bit-sliced encode of uniform windows with short rows, stores gathered
// (DESIGN.md §4g): a.wpb whole windows per step (a.wpb * ceil(ncol / 2) <=
// kBlock units, one pass), a lane per unit with the flat kernel's column pair
// (u, u + h).  The repair planes, back in bytes, go to an LDS image
// [window][repair][column]; after one barrier every window's r repair rows
// are stored front to back, consecutive lanes on consecutive 16-B chunks.
// Two images alternate, so the next step's writes never meet these reads.
template <int K, int R, int M>
__global__ __launch_bounds__(kBlock) void gf_encode_bs_gs_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    extern __shared__ uint4 dyn[];
    const uint32_t ncol = a.ncol, h = (ncol + 1) >> 1, G = (uint32_t)a.wpb, per = G * R * ncol;
    const FastDiv dh = fdiv_make(h), dn = fdiv_make(ncol), drn = fdiv_make(R * ncol);
    int buf = 0;
    for (XcdRange xr = xcd_range((a.nwin + G - 1) / G, a.nx); xr.cur < xr.hi; xr.cur += xr.step, buf ^= 1) {
        const uint64_t w0 = xr.cur * G;
        const uint32_t nb = (uint32_t)min((uint64_t)G, a.nwin - w0);
        uint4 *im = dyn + buf * per;
        const uint32_t nu = nb * h;
        {
            // lanes past the last unit redo it and write nothing (uniform trip count)
            // the network at priority 1, the stores below at 0 (1.203 vs
            // 1.211 ms on cfg3, r06)
            __builtin_amdgcn_s_setprio(1);
            const bool live = threadIdx.x < nu;
            const uint32_t s = live ? threadIdx.x : nu - 1;
            const uint32_t wl = fdiv(s, dh), u = s - wl * h;
            uint8_t *pa, *pb;
            bs::unit_cols(a.win + (w0 + wl) * a.wpitch, u, h, ncol, pa, pb);
            uint32_t acc[R][8];
            bs::sources<K, R, M, GSE_U, 0>(pa, pb, a.stride, acc);
#pragma unroll
            for (int i = 0; i < R; i++) {
                bs::tr8(acc[i]);
                if (live) {
                    im[(wl * R + i) * ncol + u] = make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
                    if (u + h < ncol)
                        im[(wl * R + i) * ncol + u + h] = make_uint4(acc[i][4], acc[i][5], acc[i][6], acc[i][7]);
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb * R * ncol; q += kBlock) {
            const uint32_t wl = fdiv(q, drn), o = q - wl * R * ncol, i = fdiv(o, dn), c = o - i * ncol;
            const uint64_t w = w0 + wl;
            st16(a.win + w * a.wpitch + a.out_delta + w * a.out_wdelta + (size_t)(K + i) * a.stride + c * 16u, im[q]);
        }
    }
}

// ==================================== runtime-mask bit-sliced GF encode ===
// The bit-sliced encode for a matrix known only at run time (RLC rows, and
// every (k, r) without a compiled kernel): the same planes, combinations and
// 3-input XORs as bs::, with each output plane's pick of lo[] / hi[] read from
// a per-code index table (a.enc_bs, fec_capi.cpp rbs_masks) through scalar
// loads.  The wave-uniform index selects a combination by relative VGPR
// addressing (s_set_gpr_idx_on / _idx / _off, M0[7:0] = index), so an output
// plane costs 2 VALU ops and a few SALU ops where the table multiply spends
// 3 v_perm + XOR per dword and repair.  Bytes equal the table multiply's
// (tests/test_gpu_parity.py).
namespace rbs {

#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(4))) const uint32_t *cmask;
#else
typedef const uint32_t *cmask;
#endif

}  // namespace rbs

// Four-column units: a lane takes 64 byte positions, so each output plane is
// a dword pair and one pair of index sets serves 64 bytes (two-column units,
// 32 bytes per index pair, measured 16 % slower on cfg4 RLC, r02; removed r05)
// at ~240 VGPRs: 2 waves per SIMD.  lo / hi entries are pairs pinned at
// v32-v63 / v64-v95 (entry s at v[32 + 2s : 33 + 2s]), so the table holds
// 2 x index, a byte per index, two planes per dword (k48 r8 0.497 -> 0.321 ms
// against a dword per plane: the table stays in the scalar cache, r02).  The
// compiler's own lowering of lo[i] hoists every pick of a source ahead of the
// XORs (251 VGPRs), so one asm block holds the picks and XORs; M0 is declared
// clobbered, which puts an implicit def of M0 on the asm so no M0 def / use
// pair of the compiler's is scheduled across it.
namespace rbs4 {

using rbs::cmask;

#define R4_IN(A, N, R0) "{v" #R0 "}"(A[N])
// planes QA, QB of one repair half from the index dword D (a byte per index:
// QA's hi, lo at bits 8, 0; QB's at 24, 16): (a[q], b[q]) ^= lo[l] ^ hi[h]
#define R4_B(D, QA, QB, TA, TB)                                                 \
    "s_lshr_b32 %[t], %[" D "], 8\n\ts_set_gpr_idx_idx %[t]\n\t"               \
    "v_mov_b64 v[" #TA ":" #TB "], v[64:65]\n\t"                               \
    "s_set_gpr_idx_idx %[" D "]\n\t"                                           \
    "v_bitop3_b32 %[a" #QA "], v32, %[a" #QA "], v" #TA " bitop3:0x96\n\t"      \
    "v_bitop3_b32 %[b" #QA "], v33, %[b" #QA "], v" #TB " bitop3:0x96\n\t"      \
    "s_lshr_b32 %[t], %[" D "], 24\n\ts_set_gpr_idx_idx %[t]\n\t"              \
    "v_mov_b64 v[" #TA ":" #TB "], v[64:65]\n\t"                               \
    "s_lshr_b32 %[t], %[" D "], 16\n\ts_set_gpr_idx_idx %[t]\n\t"              \
    "v_bitop3_b32 %[a" #QB "], v32, %[a" #QB "], v" #TA " bitop3:0x96\n\t"      \
    "v_bitop3_b32 %[b" #QB "], v33, %[b" #QB "], v" #TB " bitop3:0x96\n\t"

// planes q = 0..3 of one repair half: (a[q], b[q]) ^= lo[.] ^ hi[.], indices l[0..1]
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void pick4(uint32_t (&a)[4], uint32_t (&b)[4], const uint32_t (&l)[2],
                                      const uint32_t (&lo)[32], const uint32_t (&hi)[32]) {
    uint32_t t;  // an index shifted down
    asm("s_set_gpr_idx_on %[l0], gpr_idx(SRC0)\n\t"  // any index: the first set below replaces it
        R4_B("l0", 0, 1, 96, 97) R4_B("l1", 2, 3, 98, 99)
        "s_set_gpr_idx_off"
        : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]),
          [b0] "+v"(b[0]), [b1] "+v"(b[1]), [b2] "+v"(b[2]), [b3] "+v"(b[3]), [t] "=&s"(t)
        : [l0] "s"(l[0]), [l1] "s"(l[1]),
          R4_IN(lo, 0, 32), R4_IN(lo, 1, 33), R4_IN(lo, 2, 34), R4_IN(lo, 3, 35),
          R4_IN(lo, 4, 36), R4_IN(lo, 5, 37), R4_IN(lo, 6, 38), R4_IN(lo, 7, 39),
          R4_IN(lo, 8, 40), R4_IN(lo, 9, 41), R4_IN(lo, 10, 42), R4_IN(lo, 11, 43),
          R4_IN(lo, 12, 44), R4_IN(lo, 13, 45), R4_IN(lo, 14, 46), R4_IN(lo, 15, 47),
          R4_IN(lo, 16, 48), R4_IN(lo, 17, 49), R4_IN(lo, 18, 50), R4_IN(lo, 19, 51),
          R4_IN(lo, 20, 52), R4_IN(lo, 21, 53), R4_IN(lo, 22, 54), R4_IN(lo, 23, 55),
          R4_IN(lo, 24, 56), R4_IN(lo, 25, 57), R4_IN(lo, 26, 58), R4_IN(lo, 27, 59),
          R4_IN(lo, 28, 60), R4_IN(lo, 29, 61), R4_IN(lo, 30, 62), R4_IN(lo, 31, 63),
          R4_IN(hi, 0, 64), R4_IN(hi, 1, 65), R4_IN(hi, 2, 66), R4_IN(hi, 3, 67),
          R4_IN(hi, 4, 68), R4_IN(hi, 5, 69), R4_IN(hi, 6, 70), R4_IN(hi, 7, 71),
          R4_IN(hi, 8, 72), R4_IN(hi, 9, 73), R4_IN(hi, 10, 74), R4_IN(hi, 11, 75),
          R4_IN(hi, 12, 76), R4_IN(hi, 13, 77), R4_IN(hi, 14, 78), R4_IN(hi, 15, 79),
          R4_IN(hi, 16, 80), R4_IN(hi, 17, 81), R4_IN(hi, 18, 82), R4_IN(hi, 19, 83),
          R4_IN(hi, 20, 84), R4_IN(hi, 21, 85), R4_IN(hi, 22, 86), R4_IN(hi, 23, 87),
          R4_IN(hi, 24, 88), R4_IN(hi, 25, 89), R4_IN(hi, 26, 90), R4_IN(hi, 27, 91),
          R4_IN(hi, 28, 92), R4_IN(hi, 29, 93), R4_IN(hi, 30, 94), R4_IN(hi, 31, 95)
        : "v96", "v97", "v98", "v99", "m0", "scc");  // index mode writes M0, s_lshr SCC
}
#pragma clang diagnostic pop
#undef R4_IN
#undef R4_B

// acc ^= one source (planes xa of columns 0-1, xb of columns 2-3) times its
// index row mk ([R][2][kRbsDw4] dwords)
template <int R>
__device__ __forceinline__ void source(const uint32_t (&xa)[8], const uint32_t (&xb)[8], uint32_t (&aa)[R][8],
                                       uint32_t (&ab)[R][8], cmask mk) {
    uint32_t lo[32], hi[32];
    lo[0] = lo[1] = hi[0] = hi[1] = 0;
    // opaque zeros: a constant is re-materialised into its pinned register
    // before every asm block (4 v_mov per block)
    asm volatile("" : "+v"(lo[0]), "+v"(lo[1]), "+v"(hi[0]), "+v"(hi[1]));
#pragma unroll
    for (int s = 1; s < 16; s++) {
        const int b = __builtin_ctz(s), rest = s & (s - 1);
        lo[2 * s] = rest ? bs::oxor(lo[2 * rest], xa[b]) : xa[b];
        lo[2 * s + 1] = rest ? bs::oxor(lo[2 * rest + 1], xb[b]) : xb[b];
        hi[2 * s] = rest ? bs::oxor(hi[2 * rest], xa[4 + b]) : xa[4 + b];
        hi[2 * s + 1] = rest ? bs::oxor(hi[2 * rest + 1], xb[4 + b]) : xb[4 + b];
    }
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int w = 0; w < 2; w++) {
            const cmask m = mk + (i * 2 + w) * kRbsDw4;
            const uint32_t l[2] = {m[0], m[1]};  // two dwords for the 4 planes
            uint32_t(&ca)[4] = *reinterpret_cast<uint32_t(*)[4]>(&aa[i][w * 4]);
            uint32_t(&cb)[4] = *reinterpret_cast<uint32_t(*)[4]>(&ab[i][w * 4]);
            pick4(ca, cb, l, lo, hi);
        }
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int p = 0; p < 8; p++) asm volatile("" : "+v"(aa[i][p]), "+v"(ab[i][p]));
}

__device__ __forceinline__ void load(uint8_t *const (&pc)[4], uint32_t off, uint32_t (&xa)[8], uint32_t (&xb)[8]) {
    const uint4 v0 = ld16(pc[0] + off), v1 = ld16(pc[1] + off), v2 = ld16(pc[2] + off), v3 = ld16(pc[3] + off);
    xa[0] = v0.x; xa[1] = v0.y; xa[2] = v0.z; xa[3] = v0.w;
    xa[4] = v1.x; xa[5] = v1.y; xa[6] = v1.z; xa[7] = v1.w;
    xb[0] = v2.x; xb[1] = v2.y; xb[2] = v2.z; xb[3] = v2.w;
    xb[4] = v3.x; xb[5] = v3.y; xb[6] = v3.z; xb[7] = v3.w;
}

// one unit: columns pc[0..3]; the next source's loads are issued before the
// current one's XOR work
template <int R>
__device__ __forceinline__ void unit(uint8_t *const (&pc)[4], uint32_t stride, int k, cmask mk, bool live,
                                     uint64_t od) {
    uint32_t aa[R][8], ab[R][8];
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int p = 0; p < 8; p++) aa[i][p] = ab[i][p] = 0;
    uint32_t xa[8], xb[8];
    load(pc, 0, xa, xb);
    for (int j = 0; j < k; j++) {
        uint32_t na[8], nb[8];
        load(pc, (uint32_t)min(j + 1, k - 1) * stride, na, nb);
        bs::tr8(xa);
        bs::tr8(xb);
        source<R>(xa, xb, aa, ab, mk + (size_t)j * (R * 2 * kRbsDw4));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            xa[q] = na[q];
            xb[q] = nb[q];
        }
    }
#pragma unroll
    for (int i = 0; i < R; i++) {
        bs::tr8(aa[i]);
        bs::tr8(ab[i]);
        if (live) {
            const size_t o = od + (size_t)(k + i) * stride;
            st16(pc[0] + o, make_uint4(aa[i][0], aa[i][1], aa[i][2], aa[i][3]));
            st16(pc[1] + o, make_uint4(aa[i][4], aa[i][5], aa[i][6], aa[i][7]));
            st16(pc[2] + o, make_uint4(ab[i][0], ab[i][1], ab[i][2], ab[i][3]));
            st16(pc[3] + o, make_uint4(ab[i][4], ab[i][5], ab[i][6], ab[i][7]));
        }
    }
}

// columns u + c * h (c < 4) of a window with ncol columns, h = ceil(ncol / 4);
// a column past the end repeats column u (same inputs and outputs)
__device__ __forceinline__ void unit_cols(uint8_t *base, uint32_t u, uint32_t h, uint32_t ncol, uint8_t *(&pc)[4]) {
    pc[0] = base + u * 16u;
#pragma unroll
    for (int c = 1; c < 4; c++) pc[c] = u + c * h < ncol ? pc[0] + c * h * 16u : pc[0];
}

// unit() over the rows present in the window (pw: its presence words, row j =
// bit j % 64 of word j / 64); an absent row reads as zeros.  Release builds
// load through the wave's buffer resource rs over gb (co: the unit's column
// offsets from gb, row j at scalar offset j * stride; 4 VGPRs instead of the
// columns' 8 pointer words), an absent row's offset
// pushed past the records (bs::kOob): no branch, no memory access (exec-masked
// ld16 loads measured 1.87 vs 1.67 ms at k 120, r05).  Checked builds use ld16
// under the mask.
template <int R>
__device__ __forceinline__ void unit_m(__amdgpu_buffer_rsrc_t rs, uint8_t *gb, const uint32_t (&co)[4],
                                       uint32_t stride, int k, cmask mk, bool live, uint64_t od,
                                       const uint64_t *pw) {
    uint32_t aa[R][8], ab[R][8];
#pragma unroll
    for (int i = 0; i < R; i++)
#pragma unroll
        for (int p = 0; p < 8; p++) aa[i][p] = ab[i][p] = 0;
    uint64_t cur = pw[0];
    auto ldm = [&](int j, uint32_t (&xa)[8], uint32_t (&xb)[8]) {
        const bool on = (cur >> (j & 63)) & 1ull;
#if FECGPU_CHECK
        (void)rs;
        (void)co;
        uint4 v[4];
#pragma unroll
        for (int c = 0; c < 4; c++) v[c] = on ? ld16(gb + co[c] + (size_t)j * stride) : zero4();
        xa[0] = v[0].x; xa[1] = v[0].y; xa[2] = v[0].z; xa[3] = v[0].w;
        xa[4] = v[1].x; xa[5] = v[1].y; xa[6] = v[1].z; xa[7] = v[1].w;
        xb[0] = v[2].x; xb[1] = v[2].y; xb[2] = v[2].z; xb[3] = v[2].w;
        xb[4] = v[3].x; xb[5] = v[3].y; xb[6] = v[3].z; xb[7] = v[3].w;
#else
        const uint32_t d = on ? 0u : bs::kOob;
        const int so = (int)((uint32_t)j * stride);
        const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(co[0] + d), so, 0);
        const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(co[1] + d), so, 0);
        const u32x4 v2 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(co[2] + d), so, 0);
        const u32x4 v3 = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(co[3] + d), so, 0);
        xa[0] = v0.x; xa[1] = v0.y; xa[2] = v0.z; xa[3] = v0.w;
        xa[4] = v1.x; xa[5] = v1.y; xa[6] = v1.z; xa[7] = v1.w;
        xb[0] = v2.x; xb[1] = v2.y; xb[2] = v2.z; xb[3] = v2.w;
        xb[4] = v3.x; xb[5] = v3.y; xb[6] = v3.z; xb[7] = v3.w;
#endif
    };
    uint32_t xa[8], xb[8];
    ldm(0, xa, xb);
    for (int j = 0; j < k; j++) {
        const int jn = min(j + 1, k - 1);
        if (jn != j && (jn & 63) == 0) cur = pw[jn >> 6];  // wave-uniform: once per 64 rows
        uint32_t na[8], nb[8];
        ldm(jn, na, nb);
        bs::tr8(xa);
        bs::tr8(xb);
        source<R>(xa, xb, aa, ab, mk + (size_t)j * (R * 2 * kRbsDw4));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            xa[q] = na[q];
            xb[q] = nb[q];
        }
    }
#pragma unroll
    for (int i = 0; i < R; i++) {
        bs::tr8(aa[i]);
        bs::tr8(ab[i]);
        if (live) {
            uint8_t *o = gb + od + (size_t)(k + i) * stride;
            st16(o + co[0], make_uint4(aa[i][0], aa[i][1], aa[i][2], aa[i][3]));
            st16(o + co[1], make_uint4(aa[i][4], aa[i][5], aa[i][6], aa[i][7]));
            st16(o + co[2], make_uint4(ab[i][0], ab[i][1], ab[i][2], ab[i][3]));
            st16(o + co[3], make_uint4(ab[i][4], ab[i][5], ab[i][6], ab[i][7]));
        }
    }
}

}  // namespace rbs4

// Unit spaces as gf_encode_bs_kernel (flat over uniform windows, group mode
// otherwise); the masks are the code's, R = its r.
// MASKED (flat only, launch_rbs_rows with present masks): rows absent from a
// window read as zeros (rbs4::unit_m).
template <int R, bool FLAT, bool MASKED = false>
__global__ __launch_bounds__(kBlock) void gf_encode_rbs_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    const rbs::cmask mk = (rbs::cmask)a.enc_bs;
    const int k = a.k;
    constexpr uint32_t C = kRbsCols;  // columns per unit
    // one unit of window base (units h, columns ncol)
    auto run = [&](uint8_t *base, uint32_t u, uint32_t h, uint32_t ncol, uint32_t stride, bool live, uint64_t od) {
        uint8_t *pc[4];
        rbs4::unit_cols(base, u, h, ncol, pc);
        rbs4::unit<R>(pc, stride, k, mk, live, od);
    };
    if constexpr (FLAT) {
        const uint32_t ncol = a.ncol, h = (ncol + C - 1) / C;
        const uint64_t total = a.nwin * h;
        for (XcdRange xr = xcd_range((total + kBlock - 1) / kBlock, a.nx); xr.cur < xr.hi; xr.cur += xr.step) {
            uint64_t s = xr.cur * kBlock + threadIdx.x;
            const bool live = s < total;
            if (!live) s = total - 1;
            const uint64_t w = s / h;
            if constexpr (MASKED) {
                // the wave's resource: from its first lane's window over the
                // windows to the batch's end (capped; the host keeps a wave's
                // span below 2^31 B, rbs_masked_ok)
                const uint64_t wf = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)w) |
                                    ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(w >> 32)) << 32);
                uint8_t *gb = a.win + wf * a.wpitch;
                const uint64_t span = (a.nwin - wf) * a.wpitch;
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    gb, 0, (int)(uint32_t)min(span, (uint64_t)0x7FFFFFFFu), bs::kRsrcRaw);
                uint8_t *pc[4];
                rbs4::unit_cols(a.win + w * a.wpitch, (uint32_t)(s - w * h), h, ncol, pc);
                uint32_t co[4];
#pragma unroll
                for (int c = 0; c < 4; c++) co[c] = (uint32_t)(pc[c] - gb);
                rbs4::unit_m<R>(rs, gb, co, a.stride, k, mk, live, a.out_delta + w * a.out_wdelta,
                                a.present + w * a.pres_nw);
            } else {
                run(a.win + w * a.wpitch, (uint32_t)(s - w * h), h, ncol, a.stride, live,
                    a.out_delta + w * a.out_wdelta);
            }
        }
    } else {
        __shared__ GroupLds g;
        for (XcdRange xr = xcd_range((a.nwin + a.wpb - 1) / a.wpb, a.nx); xr.cur < xr.hi; xr.cur += xr.step) {
            const uint64_t w0 = xr.cur * a.wpb;
            const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
            group_geometry(a, g, w0, nb);
            __syncthreads();
            if (threadIdx.x < 64)
                block_prefix(g.pfx, (int)threadIdx.x < nb ? (g.ncol[threadIdx.x] + C - 1) / C : 0u, threadIdx.x);
            __syncthreads();
            const uint32_t total = g.pfx[nb];
            int wl = 0;
            for (uint32_t s0 = 0; s0 < total; s0 += kBlock) {
                const bool live = s0 + threadIdx.x < total;
                const uint32_t s = live ? s0 + threadIdx.x : total - 1;
                while (s >= g.pfx[wl + 1]) wl++;
                run(reinterpret_cast<uint8_t *>(g.base[wl]), s - g.pfx[wl], g.pfx[wl + 1] - g.pfx[wl], g.ncol[wl],
                    g.stride[wl], live, a.out_delta + (w0 + wl) * a.out_wdelta);
            }
            __syncthreads();
        }
    }
}

// ============================================================ decode ===
template <int R, bool FLAT>
__global__ __launch_bounds__(kBlock) void xor_decode_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    if constexpr (FLAT) {
        // for_flat_slots with the next slot's present mask loaded one iteration
        // ahead: the plan (and so the data loads) never waits on that load.
        const uint32_t ncol = a.ncol;
        const uint64_t total = a.nwin * ncol;
        XcdRange xr = xcd_range((total + kBlock - 1) / kBlock, a.nx);
        if (xr.cur >= xr.hi) return;
        uint64_t s = xr.cur * kBlock + threadIdx.x;
        uint64_t w = s / ncol;
        uint32_t col = (uint32_t)(s - w * ncol);
        const uint64_t wbytes = a.wpitch;
        uint64_t pres = a.present[min(w, a.nwin - 1)];
        for (; xr.cur < xr.hi; xr.cur += xr.step) {
            const uint64_t s_now = s, w_now = w, p_now = pres;
            const uint32_t col_now = col;
            s += xr.step * kBlock;
            col += a.step_col;
            w += a.step_win;
            if (col >= ncol) {
                col -= ncol;
                w++;
            }
            pres = a.present[min(w, a.nwin - 1)];  // prefetch for the next iteration
            if (s_now < total) {
                const uint32_t bad = xor_decode_slot<R>(a, a.win + w_now * wbytes + col_now * 16u,
                                                        a.stride, p_now, true);
                if (col_now == 0) a.status[w_now] = (uint8_t)bad;
            }
        }
    } else {
        __shared__ GroupLds g;
        __shared__ uint64_t s_pres[kMaxWpb];
        for (XcdRange xr = xcd_range((a.nwin + a.wpb - 1) / a.wpb, a.nx); xr.cur < xr.hi;
             xr.cur += xr.step) {
            const uint64_t w0 = xr.cur * a.wpb;
            const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
            group_geometry(a, g, w0, nb);
            if ((int)threadIdx.x < nb) s_pres[threadIdx.x] = a.present[w0 + threadIdx.x];
            __syncthreads();
            if (threadIdx.x < 64) {
                uint32_t n = 0;
                const int t = threadIdx.x;
                if (t < nb) {
                    // status from the mask alone; drop windows with nothing to rebuild
                    const uint64_t kmask = (a.k >= 64) ? ~0ull : ((1ull << a.k) - 1);
                    const uint64_t miss = ~s_pres[t] & kmask;
                    uint32_t bad = 0, any = 0;
                    for (int gi = 0; gi < a.r; gi++) {
                        const uint64_t mg = miss & a.gmask[gi];
                        if (!mg) continue;
                        if ((mg & (mg - 1)) == 0 && ((s_pres[t] >> (a.k + gi)) & 1)) any = 1;
                        else bad = 1;
                    }
                    a.status[w0 + t] = (uint8_t)bad;
                    n = any ? g.ncol[t] : 0u;
                }
                block_prefix(g.pfx, n, t);
            }
            __syncthreads();
            for_group_slots(g, nb, [&](uint8_t *p, uint32_t stride, int wl, bool valid) {
                (void)xor_decode_slot<R>(a, p, stride, s_pres[wl], valid);
            });
            __syncthreads();
        }
    }
}

// Per-window LDS region of the GF decode (size: gf_dec_win_lds).  The decode
// matrix D (e x k, entry [u][q] = coefficient of input q in missing source u)
// as multiply tables: ab[q][u] (TA/TB, one ds_read_b128) and tc[q][u] (TC,
// rows padded to 4 so a row's TC entries are one ds_read_b128).  roff[q] is
// input q's row offset in the window (received sources ascending, then the
// chosen repairs; padded with row 0, so a load batch never clamps), ooff[u]
// the output row of missing source u.  Entries for u >= e are stale: they
// feed only accumulators that are never stored.
template <int R>
struct DecRegion {
    static constexpr int R4 = (R + 3) & ~3;
    uint4 *ab;
    uint32_t *tc, *roff, *ooff;
    uint8_t *insym, *outsym;
    __device__ __forceinline__ DecRegion(uint8_t *region, int k) {
        ab = reinterpret_cast<uint4 *>(region);
        tc = reinterpret_cast<uint32_t *>(region + k * R * 16);
        roff = tc + k * R4;
        ooff = roff + ((k + 7) & ~7);
        insym = reinterpret_cast<uint8_t *>(ooff + 8);
        outsym = insym + 64;
    }
};

// Row offsets of a planned window from its symbol lists (every lane of the
// wave; the lists were written before the plan's last wave sync).
template <int R>
__device__ __forceinline__ void plan_offsets(const BatchArgs &a, uint64_t w, int lane,
                                             const DecRegion<R> &rg, int e) {
    uint64_t base;
    uint32_t stride, S;
    win_geom(a, w, base, stride, S);
    const int k = a.k;
    if (lane < ((k + 7) & ~7)) rg.roff[lane] = lane < k ? (uint32_t)rg.insym[lane] * stride : 0u;
    if (lane < 8) rg.ooff[lane] = lane < e ? (uint32_t)rg.outsym[lane] * stride : 0u;
}

// GF plan (a6/a7) by one wave, closed form.  Missing sources m_0..m_{e-1},
// the first e present repairs with points x_t = k + sel_t; the system is the
// Cauchy matrix A[t][u] = 1/(x_t ^ m_u).  Its inverse folded
// into the decode matrix D (e x k inputs z_q: received sources, then the
// chosen repairs) has a closed form — with
//   A_u = sum_t log(x_t ^ m_u) - sum_{v != u} log(m_u ^ m_v)      (lane u)
//   K_q = sum_v log(z_q ^ m_v) - sum_{t: x_t != z_q} log(x_t ^ z_q) (lane q)
// every entry is  log D[u][q] = A_u + K_q - log(z_q ^ m_u)  (mod 255).
// (g(z) = sum_t Ainv[u][t] / (x_t ^ z) is the rational function that is 1 at
// m_u, 0 at the other m_v and has poles at the x_t; D[u][j] = g(j) for a
// received source j and D[u][t] = its residue at x_t.)  All lookups are
// independent: two LDS round trips instead of an e-step elimination chain.
template <int R>
__device__ void plan_gf(const BatchArgs &a, uint64_t w, uint64_t pres, int lane, uint8_t *region,
                        const uint8_t *ex, const uint8_t *lg, uint8_t &ne_out) {
    const int k = a.k, r = a.r;
    const DecRegion<R> rg(region, k);
    uint8_t *insym = rg.insym, *outsym = rg.outsym;
    const uint64_t kmask = (k >= 64) ? ~0ull : ((1ull << k) - 1);
    const uint64_t miss = ~pres & kmask;
    const uint64_t rep = (pres >> k) & ((1ull << r) - 1);
    const int e = __popcll(miss);
    if (e == 0 || __popcll(rep) < e || e > R) {
        if (lane == 0) {
            ne_out = 0;
            a.status[w] = (e == 0) ? 0 : 1;
        }
        return;
    }
    // wave-uniform m_v and x_t (pres is uniform: SGPR bit scans)
    int mv[R], xt[R];
    {
        uint64_t mm = miss, rr = rep;
#pragma unroll
        for (int v = 0; v < R; v++) {
            mv[v] = (int)__ffsll((unsigned long long)mm) - 1;
            xt[v] = k + (int)__ffsll((unsigned long long)rr) - 1;
            mm &= mm - 1;
            rr &= rr - 1;
        }
    }
    const int kr = k - e;
    // input list: received sources ascending, then the chosen repairs
    if (lane < k && ((pres >> lane) & 1)) insym[__popcll(pres & kmask & ((1ull << lane) - 1))] = (uint8_t)lane;
    int my_m = 0, my_x = 0;
#pragma unroll
    for (int v = 0; v < R; v++) {
        if (lane == v) { my_m = mv[v]; my_x = xt[v]; }
    }
    if (lane < e) {
        insym[kr + lane] = (uint8_t)my_x;
        outsym[lane] = (uint8_t)my_m;
    }
    WAVE_SYNC();
    const int zq = (lane < k) ? (int)insym[lane] : 0;
    int K = 0, A = 0;
#pragma unroll
    for (int v = 0; v < R; v++) {
        if (v < e) {
            const uint32_t dz = (uint32_t)(zq ^ mv[v]), dx = (uint32_t)(xt[v] ^ zq);
            const uint32_t ax = (uint32_t)(xt[v] ^ my_m), am = (uint32_t)(my_m ^ mv[v]);
            K += (int)lg[dz & 255] - (dx ? (int)lg[dx & 255] : 0);
            A += (int)lg[ax & 255] - (am ? (int)lg[am & 255] : 0);
        }
    }
    // D[u][q] for idx = u*k + q; every __shfl with the whole wave active
    for (int base = 0; base < e * k; base += 64) {
        const int idx = base + lane;
        // idx = dq * e + du: consecutive lanes write consecutive table entries
        // (lanes along dq put 4 lanes of every 8 on the same LDS banks:
        // SQ_LDS_BANK_CONFLICT 7.3e6 -> 0.52e6 on cfg3, r03)
        const int dq = idx / e, du = idx - dq * e;
        const int Au = __shfl(A, du & 63, 64);
        const int Kq = __shfl(K, dq & 63, 64);
        const int z = __shfl(zq, dq & 63, 64);
        const int mu = __shfl(my_m, du & 63, 64);
        if (idx < e * k) {
            const int lgd = Au + Kq - (int)lg[(z ^ mu) & 255] + 255 * 4 * kMaxR;
            const CoefTab ct = make_coef_tab(ex[lgd % 255]);
            rg.ab[dq * R + du] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
            rg.tc[dq * DecRegion<R>::R4 + du] = ct.c;
        }
    }
    plan_offsets<R>(a, w, lane, rg, e);
    if (lane == 0) {
        ne_out = (uint8_t)e;
        a.status[w] = 0;
    }
}

// GF(2^8) multiply / inverse through the LDS copies of the exp / log tables
__device__ __forceinline__ uint32_t gf_mul_lds(const uint8_t *ex, const uint8_t *lg, uint32_t x,
                                               uint32_t y) {
    return (x && y) ? ex[lg[x] + lg[y]] : 0u;
}
__device__ __forceinline__ uint32_t gf_inv_lds(const uint8_t *ex, const uint8_t *lg, uint32_t x) {
    return ex[255 - lg[x]];
}

// General-matrix plan (FECGPU_MATRIX_VANDERMONDE, FECGPU_MATRIX_RLC, any
// systematic generator): the parity rows P[r][k] sit in LDS.  The system of
// EVERY present repair, A[t][u] = P[sel_t][m_u] (t < np <= 8 rows, u < e
// columns), is reduced by wave-parallel Gauss-Jordan with pivot search: the
// pivot of column c is the first row not yet used whose entry is nonzero, so
// a random linear code (not MDS) recovers whenever its present repairs have
// rank e, and is unrecoverable otherwise.  Row operations only ever add pivot
// rows, so pivot row P_u of column u ends as x_u = sum_c T[P_u][P_c] * s_{P_c}
// over the chosen repairs (T: the identity columns carried along), which is
// folded into the decode matrix D like the Cauchy plans.
template <int R>
__device__ void plan_gf_mat(const BatchArgs &a, uint64_t w, uint64_t pres, int lane, uint8_t *region,
                            const uint8_t *ex, const uint8_t *lg, const uint8_t *P, uint8_t &ne_out) {
    const int k = a.k, r = a.r;
    const DecRegion<R> rg(region, k);
    uint8_t *insym = rg.insym, *outsym = rg.outsym;
    const uint64_t kmask = (k >= 64) ? ~0ull : ((1ull << k) - 1);
    const uint64_t miss = ~pres & kmask;
    const uint64_t rep = (pres >> k) & ((1ull << r) - 1);
    const int e = __popcll(miss), np = __popcll(rep);
    if (e == 0 || np < e || e > R) {
        if (lane == 0) {
            ne_out = 0;
            a.status[w] = (e == 0) ? 0 : 1;
        }
        return;
    }
    uint64_t mm = miss, rr = rep;
    for (int i = 0; i < lane && i < 8; i++) { mm &= mm - 1; rr &= rr - 1; }
    const int my_m = (int)__ffsll((unsigned long long)mm) - 1;    // lane u < e: u-th missing source
    const int my_sel = (int)__ffsll((unsigned long long)rr) - 1;  // lane t < np: t-th present repair
    if (lane < k && ((pres >> lane) & 1)) insym[__popcll(pres & kmask & ((1ull << lane) - 1))] = (uint8_t)lane;
    if (lane < e) outsym[lane] = (uint8_t)my_m;
    // [A | I], lane = t*8 + u; every __shfl and ballot with the whole wave active
    const int t = lane >> 3, u = lane & 7;
    const int sel_t = __shfl(my_sel, t, 64);
    const int m_u = __shfl(my_m, u, 64);
    const bool row = t < np;
    uint32_t xl = (row && u < e) ? P[sel_t * k + m_u] : 0u;
    uint32_t xr = (row && t == u) ? 1u : 0u;
    uint32_t used = 0;  // wave-uniform: rows already pivots
    int my_piv = 0;     // lane c < e: pivot row of column c
    bool singular = false;
    for (int c = 0; c < e; c++) {
        const uint64_t cand = __ballot(row && u == c && !((used >> t) & 1) && xl != 0);
        if (!cand) { singular = true; break; }
        const int pr = (int)(__ffsll((unsigned long long)cand) - 1) >> 3;
        used |= 1u << pr;
        if (lane == c) my_piv = pr;
        const uint32_t ip = gf_inv_lds(ex, lg, __shfl(xl, pr * 8 + c, 64));
        if (t == pr) {
            xl = gf_mul_lds(ex, lg, xl, ip);
            xr = gf_mul_lds(ex, lg, xr, ip);
        }
        const uint32_t f = __shfl(xl, t * 8 + c, 64);
        const uint32_t rl = __shfl(xl, pr * 8 + u, 64);
        const uint32_t rq = __shfl(xr, pr * 8 + u, 64);
        if (t != pr && row) {
            xl ^= gf_mul_lds(ex, lg, f, rl);
            xr ^= gf_mul_lds(ex, lg, f, rq);
        }
    }
    if (singular) {
        if (lane == 0) { ne_out = 0; a.status[w] = 1; }
        return;
    }
    const int kr = k - e;
    {
        const int sel_piv = __shfl(my_sel, my_piv & 7, 64);  // lane c: repair chosen for column c
        if (lane < e) insym[kr + lane] = (uint8_t)(k + sel_piv);
    }
    WAVE_SYNC();
    // D[u][q] for idx = u*k + q; Ainv'[u][c] = T[P_u][P_c] = xr of lane P_u*8 + P_c
    for (int base = 0; base < e * k; base += 64) {
        const int idx = base + lane;
        // idx = dq * e + du: consecutive lanes write consecutive table entries
        // (lanes along dq put 4 lanes of every 8 on the same LDS banks:
        // SQ_LDS_BANK_CONFLICT 7.3e6 -> 0.52e6 on cfg3, r03)
        const int dq = idx / e, du = idx - dq * e;
        const bool live = idx < e * k;
        const bool is_src = dq < kr;
        const uint32_t j = (live && is_src) ? insym[dq] : 0u;
        const int pu = __shfl(my_piv, du & 7, 64);
        uint32_t csrc = 0;
        for (int tt = 0; tt < e; tt++) {
            const int pt = __shfl(my_piv, tt, 64);
            const uint32_t ai = __shfl(xr, (pu * 8 + pt) & 63, 64);
            const int st = __shfl(my_sel, pt & 7, 64);
            if (is_src) csrc ^= gf_mul_lds(ex, lg, ai, P[st * k + j]);
        }
        const int pc = __shfl(my_piv, (is_src ? 0 : dq - kr) & 7, 64);
        const uint32_t crep = __shfl(xr, (pu * 8 + pc) & 63, 64);
        const uint32_t c = is_src ? csrc : crep;
        if (live) {
            const CoefTab ct = make_coef_tab(c);
            rg.ab[dq * R + du] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
            rg.tc[dq * DecRegion<R>::R4 + du] = ct.c;
        }
    }
    plan_offsets<R>(a, w, lane, rg, e);
    if (lane == 0) {
        ne_out = (uint8_t)e;
        a.status[w] = 0;
    }
}

// GF decode of one slot for NE outputs (wave-uniform): acc[u] = sum_q D[u][q]
// * in_q over the k inputs, U rows loaded per batch; output u is stored when
// u < ne (this lane's window).  OFF: the first output (the outputs OFF ..
// OFF + NE - 1 of the window's plan; a multiple of 4).
template <int R, int NE, int OFF = 0>
__device__ __forceinline__ void dec_slot(uint8_t *base, int k, int ne, uint64_t out_delta,
                                         const DecRegion<R> &rg) {
    static_assert(OFF % 4 == 0 && OFF + NE <= R, "output range");
    constexpr int U = GF_DEC_U(R), R4 = DecRegion<R>::R4;
    static_assert(U == 2 || U == 4 || U == 8, "row offsets are padded to 8 rows");
    uint4 acc[NE];
#pragma unroll
    for (int m = 0; m < NE; m++) acc[m] = zero4();
    for (int q0 = 0; q0 < k; q0 += U) {
        uint4 v[U];
        uint32_t ro[U];
        if constexpr (U >= 4) {
#pragma unroll
            for (int t = 0; t < U; t += 4) {  // roff is padded to a multiple of 8 rows
                const uint4 o = *reinterpret_cast<const uint4 *>(rg.roff + q0 + t);
                ro[t] = o.x; ro[t + 1] = o.y; ro[t + 2] = o.z; ro[t + 3] = o.w;
            }
        } else {
            const uint2 o = *reinterpret_cast<const uint2 *>(rg.roff + q0);
            ro[0] = o.x; ro[1] = o.y;
        }
#pragma unroll
        for (int t = 0; t < U; t++) v[t] = ld16(base + ro[t]);
        // rows in pairs: one xor3 chain folds both rows' lookups (1.5 instead of
        // 2 ops per product; cfg3 1.360 vs 1.372 ms, cfg4 4.55 vs 4.59 at 4-row
        // batches, r06 — in r01, before the LDS index and 8-row batches, the
        // pairs' registers cost more than they saved)
        int t0 = 0;
#pragma unroll
        for (int t = 0; t + 1 < U; t += 2) {
            if (q0 + t + 1 < k) {
                const int q = q0 + t;
                const Split s0 = split(v[t]), s1 = split(v[t + 1]);
                uint32_t c0[R4], c1[R4];
#pragma unroll
                for (int j = 0; j < (NE + 3) / 4; j++) {
                    const uint4 x = *reinterpret_cast<const uint4 *>(rg.tc + q * R4 + OFF + 4 * j);
                    const uint4 y = *reinterpret_cast<const uint4 *>(rg.tc + (q + 1) * R4 + OFF + 4 * j);
                    c0[4 * j] = x.x; c0[4 * j + 1] = x.y; c0[4 * j + 2] = x.z; c0[4 * j + 3] = x.w;
                    c1[4 * j] = y.x; c1[4 * j + 1] = y.y; c1[4 * j + 2] = y.z; c1[4 * j + 3] = y.w;
                }
#pragma unroll
                for (int m = 0; m < NE; m++)
                    gmac2(acc[m], s0, s1, rg.ab[q * R + OFF + m], c0[m], rg.ab[(q + 1) * R + OFF + m], c1[m]);
                t0 = t + 2;
            }
        }
#pragma unroll
        for (int t = 0; t < U; t++) {
            if (t >= t0 && q0 + t < k) {
                const int q = q0 + t;
                const Split sp = split(v[t]);
                uint32_t c[R4];
#pragma unroll
                for (int j = 0; j < (NE + 3) / 4; j++) {
                    const uint4 x = *reinterpret_cast<const uint4 *>(rg.tc + q * R4 + OFF + 4 * j);
                    c[4 * j] = x.x; c[4 * j + 1] = x.y; c[4 * j + 2] = x.z; c[4 * j + 3] = x.w;
                }
#pragma unroll
                for (int m = 0; m < NE; m++) gmac(acc[m], sp, rg.ab[q * R + OFF + m], c[m]);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < NE; m++)
        if (OFF + m < ne) st16(base + out_delta + rg.ooff[OFF + m], acc[m]);
}


template <int R, int NE = R>
__device__ __forceinline__ void dec_dispatch(int nw, uint8_t *base, int k, int ne, uint64_t out_delta,
                                             const DecRegion<R> &rg) {
    // (two passes of 4 outputs at R = 8, for 4 waves per SIMD instead of 3:
    // the second pass's reads cost more than the wave gained, r03)
    if constexpr (NE >= 1) {
        if (nw == NE) dec_slot<R, NE>(base, k, ne, out_delta, rg);
        else dec_dispatch<R, NE - 1>(nw, base, k, ne, out_delta, rg);
    }
}

// (5 or 6 waves per SIMD at r <= 4 spill 284+ B per lane: 2.39 / 2.62 vs 1.36 ms, r06)
template <int R>
__global__ __launch_bounds__(kBlock) void gf_decode_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    extern __shared__ uint4 dyn[];
    __shared__ uint8_t s_exp[512];
    __shared__ uint8_t s_log[256];
    __shared__ GroupLds g;
    __shared__ uint8_t s_ne[kMaxWpb];
    __shared__ uint8_t s_perm[kMaxWpb];        // group windows, descending e
    __shared__ uint8_t s_coef[kMaxR * kMaxK];  // general-matrix codes: parity rows P[r][k]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, k = a.k;
    uint8_t *regions = reinterpret_cast<uint8_t *>(dyn);
    for (int i = tid; i < 512; i += kBlock) s_exp[i] = c_gf.exp[i];
    for (int i = tid; i < 256; i += kBlock) s_log[i] = c_gf.log[i];
    if (a.coef)
        for (int i = tid; i < a.r * k; i += kBlock) s_coef[i] = a.coef[i];
    __syncthreads();
    for (XcdRange xr = xcd_range((a.nwin + a.wpb - 1) / a.wpb, a.nx); xr.cur < xr.hi;
         xr.cur += xr.step) {
        const uint64_t w0 = xr.cur * a.wpb;
        const int nb = (int)min((uint64_t)a.wpb, a.nwin - w0);
        group_geometry(a, g, w0, nb);
        {
            // this wave plans windows wave, wave + 4, ...: their masks in one load
            // (prefetching the next group's masks in persistent workgroups did
            // not pay: the default one-group-per-workgroup grid was faster, r02)
            constexpr int NW = kBlock / 64;
            const int wl_l = wave + NW * lane;
            const uint64_t pl = (wl_l < nb) ? a.present[w0 + wl_l] : 0ull;
            for (int i = 0, wl = wave; wl < nb; i++, wl += NW) {
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pl, i);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pl >> 32), i);
                const uint64_t pw = ((uint64_t)hi << 32) | lo;
                if (a.coef)  // wave-uniform: one code per launch
                    plan_gf_mat<R>(a, w0 + wl, pw, lane, regions + (size_t)wl * a.win_lds, s_exp, s_log,
                                   s_coef, s_ne[wl]);
                else
                    plan_gf<R>(a, w0 + wl, pw, lane, regions + (size_t)wl * a.win_lds, s_exp, s_log,
                               s_ne[wl]);
            }
        }
        __syncthreads();
        if (tid < 64) {
            // Windows in descending order of e (ties by index): a wave's first
            // active lane then holds the largest e among its lanes, so the
            // multiply runs for that many outputs, wave-uniform (no per-product
            // exec masking); lanes of windows with smaller e accumulate extra
            // outputs from stale table rows and do not store them.
            const int t = tid;
            const int ne_t = t < nb ? (int)s_ne[t] : -1;
            const uint64_t below = (1ull << t) - 1;
            int rank = 0;
#pragma unroll
            for (int v = R; v >= 0; v--) {
                const uint64_t b = __ballot(ne_t == v);  // whole wave active
                if (v > ne_t) rank += __popcll(b);
                else if (v == ne_t) rank += __popcll(b & below);
            }
            if (t < nb) s_perm[rank] = (uint8_t)t;
            WAVE_SYNC();
            const int wl = t < nb ? (int)s_perm[t] : 0;
            block_prefix(g.pfx, (t < nb && s_ne[wl]) ? g.ncol[wl] : 0u, t);
        }
        __syncthreads();
        const uint32_t total = g.pfx[nb];
        int i = 0;
        for (uint32_t s = tid; s < total; s += kBlock) {
            while (s >= g.pfx[i + 1]) i++;
            const int wl = s_perm[i];
            const int ne = s_ne[wl];
            const int nw = __builtin_amdgcn_readfirstlane(ne);  // max e over the wave's lanes
            uint8_t *base = reinterpret_cast<uint8_t *>(g.base[wl]) + (s - g.pfx[i]) * 16u;
            const DecRegion<R> rg(regions + (size_t)wl * a.win_lds, k);
            dec_dispatch<R>(nw, base, k, ne, a.out_delta, rg);
        }
        __syncthreads();
    }
}

// ====================================== bit-sliced syndrome GF decode ===
// Cauchy codes with a compiled network (k 16 r 4: cfg3) on uniform short rows
// (DESIGN.md §4h).  With missing sources m_u (u < e) and the first e present
// repairs i_t, the received sources' part of every repair comes from the
// encode's bit-sliced network (missing rows are not loaded: zero planes), so
// the syndromes s_i = R_i ^ sum_{j received} P[i][j] S_j need no per-window
// tables; then S_{m_u} = sum_t Ainv[u][t] s_{i_t} is an e x e table multiply
// (16 products per column at e = 4 instead of the product decode's 64).
// Ainv of the Cauchy block A[t][u] = 1 / (x_t ^ m_u), x_t = k + i_t, in closed
// form (the repair entries of plan_gf's D): log Ainv[u][t] = A_u + K_t -
// log(x_t ^ m_u), one lane per entry.  A workgroup takes G whole windows per
// step (G * ceil(ncol / 2) <= NT units of two 16-B columns, as the
// gathered-store encode) in three phases: (A) syndromes by the network, a lane
// per unit, to an LDS image [window][repair][column] in bytes; (B) the solve
// per 16-B column, in place; (C) the recovered rows stored front to back.
// cfg3: 1.26-1.27 ms against 1.36 for the table decode in-process (512
// threads, 13 windows a step; 256 threads, 6 windows, 4 workgroups per CU:
// 1.29-1.30).  Measured and removed (r06): the solve in registers right after
// the network (199-225 VGPRs, 2 waves per SIMD: 1.47 ms with per-lane stores,
// 1.53 gathered) and (B) storing its columns directly (1.61 ms).
// Sources loaded per batch in (A): 3 (1.259 vs 1.271 ms at 2, r06).
#ifndef BSD_U
#define BSD_U 3
#endif
namespace bsd {

// Per-step LDS after the image (fec_internal.h bsd_lds_bytes), two buffers:
// ab / tc [buf][window][i * R + u] the solve's tables, syndrome of repair i ->
// output u (0 unless chosen; one pad entry per window, so two windows' tables
// read by one wave start on different LDS banks); pm the rows to load
// (received sources: bits < k, chosen repairs: k + i; 0: no work); rows byte
// u: missing source m_u; ne: sources recovered
template <int R>
struct Lds {
    static constexpr uint32_t E = R * R + 1;
    uint4 *ab_;
    uint32_t *tc_, *pm_, *rows_, *ne_;
    uint32_t G;
    const uint8_t *ex, *lg;
    __device__ __forceinline__ Lds(uint4 *im, uint32_t G_, uint32_t ncol, const uint8_t *ex_, const uint8_t *lg_)
        : G(G_), ex(ex_), lg(lg_) {
        ab_ = im + (size_t)G * R * ncol;
        tc_ = reinterpret_cast<uint32_t *>(ab_ + 2 * G * E);
        pm_ = tc_ + 2 * G * E;
        rows_ = pm_ + 2 * G;
        ne_ = rows_ + 2 * G;
    }
    __device__ __forceinline__ uint4 *ab(int buf, uint32_t wl) const { return ab_ + (buf * G + wl) * E; }
    __device__ __forceinline__ uint32_t *tc(int buf, uint32_t wl) const { return tc_ + (buf * G + wl) * E; }
    __device__ __forceinline__ uint32_t &pm(int buf, uint32_t wl) const { return pm_[buf * G + wl]; }
    __device__ __forceinline__ uint32_t &rows(int buf, uint32_t wl) const { return rows_[buf * G + wl]; }
    __device__ __forceinline__ uint32_t &ne(int buf, uint32_t wl) const { return ne_[buf * G + wl]; }
};

template <int K, int R>
__device__ __forceinline__ void plan(const BatchArgs &a, const Lds<R> &L, int buf, uint64_t w0, uint32_t nb) {
    const uint32_t tid = threadIdx.x;
    if (tid >= nb * R * R) return;
    const uint32_t wl = tid / (R * R), idx = tid - wl * (R * R), i = idx / R, u = idx - i * R;
    const uint64_t pres = a.present[w0 + wl];
    const uint32_t kmask = (1u << K) - 1u;
    const uint32_t miss = ~(uint32_t)pres & kmask, rep = (uint32_t)(pres >> K) & ((1u << R) - 1u);
    const int e = __popc(miss), np = __popc(rep);
    const bool ok = e > 0 && np >= e;
    int mv[R], xv[R];
    uint32_t chosen = 0;
    {
        uint32_t mm = miss, rr = rep;
#pragma unroll
        for (int v = 0; v < R; v++) {
            mv[v] = mm ? __ffs(mm) - 1 : 0;
            xv[v] = K + (rr ? __ffs(rr) - 1 : 0);
            if (v < e) chosen |= rr & (0u - rr);
            mm &= mm - 1;
            rr &= rr - 1;
        }
    }
    uint32_t c = 0;
    if (ok && (int)u < e && ((chosen >> i) & 1u)) {
        int mu = 0;
#pragma unroll
        for (int v = 0; v < R; v++)
            if (v == (int)u) mu = mv[v];
        const int x = K + (int)i;
        int s = 255 * 4 * R - (int)L.lg[x ^ mu];
#pragma unroll
        for (int v = 0; v < R; v++) {
            if (v < e) {
                s += (int)L.lg[xv[v] ^ mu] + (int)L.lg[x ^ mv[v]];
                if (v != (int)u) s -= (int)L.lg[mu ^ mv[v]];
                if (xv[v] != x) s -= (int)L.lg[xv[v] ^ x];
            }
        }
        c = L.ex[s % 255];
    }
    const CoefTab ct = make_coef_tab(c);
    L.ab(buf, wl)[idx] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
    L.tc(buf, wl)[idx] = ct.c;
    if (idx == 0) {
        a.status[w0 + wl] = (e == 0 || ok) ? 0 : 1;
        L.pm(buf, wl) = ok ? ((~miss & kmask) | (chosen << K)) : 0u;
        uint32_t rows = 0;
#pragma unroll
        for (int v = 0; v < R; v++) rows |= (uint32_t)mv[v] << (8 * v);
        L.rows(buf, wl) = rows;
        L.ne(buf, wl) = ok ? (uint32_t)e : 0u;
    }
}

// out[u] = sum_i D[i][u] * s_i over one 16-B column (s: the R syndromes)
template <int R>
__device__ __forceinline__ void solve_col(const uint4 (&s)[R], uint4 (&out)[R], const uint4 *ab, const uint32_t *tc) {
#pragma unroll
    for (int u = 0; u < R; u++) out[u] = zero4();
#pragma unroll
    for (int i = 0; i + 1 < R; i += 2) {
        const Split s0 = split(s[i]), s1 = split(s[i + 1]);
#pragma unroll
        for (int u = 0; u < R; u++) gmac2(out[u], s0, s1, ab[i * R + u], tc[i * R + u], ab[(i + 1) * R + u], tc[(i + 1) * R + u]);
        __builtin_amdgcn_sched_barrier(0);  // one pair's tables live at a time (neutral vs none, r06)
    }
    if constexpr (R & 1) {
        const Split sp = split(s[R - 1]);
#pragma unroll
        for (int u = 0; u < R; u++) gmac(out[u], sp, ab[(R - 1) * R + u], tc[(R - 1) * R + u]);
    }
}

}  // namespace bsd

template <int K, int R, int M, int NT>
__global__ __launch_bounds__(NT) void gf_decode_bs_gs_kernel(BatchArgs a) {
    CHK_PROLOGUE(a);
    static_assert(M == FECGPU_MATRIX_CAUCHY, "closed-form plan: Cauchy rows");
    extern __shared__ uint4 im[];  // [window][syndrome, then output][column], then bsd::Lds
    __shared__ uint8_t s_ex[512], s_lg[256];
    const uint32_t ncol = a.ncol, h = (ncol + 1) >> 1, G = (uint32_t)a.wpb;
    const bsd::Lds<R> L(im, G, ncol, s_ex, s_lg);
    const FastDiv dh = fdiv_make(h), dn = fdiv_make(ncol), drn = fdiv_make(R * ncol);
    for (uint32_t i = threadIdx.x; i < 512; i += NT) s_ex[i] = c_gf.exp[i];
    for (uint32_t i = threadIdx.x; i < 256; i += NT) s_lg[i] = c_gf.log[i];
    __syncthreads();
    XcdRange xr = xcd_range((a.nwin + G - 1) / G, a.nx);
    // the next step's plan is made before each step's last barrier (its LDS
    // round trips overlap the other waves' tails); tables and headers alternate
    if (xr.cur < xr.hi) bsd::plan<K, R>(a, L, 0, xr.cur * G, (uint32_t)min((uint64_t)G, a.nwin - xr.cur * G));
    __syncthreads();
    for (int buf = 0; xr.cur < xr.hi; xr.cur += xr.step, buf ^= 1) {
        const uint64_t w0 = xr.cur * G;
        const uint32_t nb = (uint32_t)min((uint64_t)G, a.nwin - w0);
        const uint32_t nu = nb * h;
        {
            // (A) syndromes: lane = unit; lanes past the last unit redo it and
            // write nothing (uniform trip count)
            // waves issuing loads win issue arbitration over the other
            // workgroup's solve (s_setprio 1: 1.277 vs 1.310 ms on cfg3; 2,
            // and 1 for the stores of (C) as well, the same, r06)
            __builtin_amdgcn_s_setprio(1);
            const bool live = threadIdx.x < nu;
            const uint32_t s = live ? threadIdx.x : nu - 1;
            const uint32_t wl = fdiv(s, dh), u = s - wl * h;
            const uint32_t pm = L.pm(buf, wl);
            uint8_t *pa, *pb;
            bs::unit_cols(a.win + (w0 + wl) * a.wpitch, u, h, ncol, pa, pb);
            uint32_t acc[R][8];
            uint32_t rep[R][8];
#if FECGPU_CHECK
            // checked loads (ld16), each row under its mask
            bs::sources<K, R, M, kBsUFlat, 0, true>(pa, pb, a.stride, acc, pm);
#pragma unroll
            for (int i = 0; i < R; i++) {
                uint4 va = zero4(), vb = zero4();
                if ((pm >> (K + i)) & 1u) {
                    va = ld16(pa + (size_t)(K + i) * a.stride);
                    vb = ld16(pb + (size_t)(K + i) * a.stride);
                }
                rep[i][0] = va.x; rep[i][1] = va.y; rep[i][2] = va.z; rep[i][3] = va.w;
                rep[i][4] = vb.x; rep[i][5] = vb.y; rep[i][6] = vb.z; rep[i][7] = vb.w;
            }
#else
            {
                uint8_t *gb = a.win + w0 * a.wpitch;
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(gb, 0, (int)(uint32_t)((uint64_t)nb * a.wpitch), bs::kRsrcRaw);
                const uint32_t oa = (uint32_t)(pa - gb), ob = (uint32_t)(pb - gb);
                bs::sources_rs<K, R, M, BSD_U, 0>(rs, oa, ob, a.stride, acc, pm);
#pragma unroll
                for (int i = 0; i < R; i++)
                    bs::load_rs(rs, oa, ob, ((pm >> (K + i)) & 1u) ? (uint32_t)(K + i) * a.stride : bs::kOob, rep[i]);
            }
#endif
#pragma unroll
            for (int i = 0; i < R; i++) {
                bs::tr8(acc[i]);
                if (live) {
                    im[(wl * R + i) * ncol + u] = make_uint4(acc[i][0] ^ rep[i][0], acc[i][1] ^ rep[i][1],
                                                             acc[i][2] ^ rep[i][2], acc[i][3] ^ rep[i][3]);
                    if (u + h < ncol)
                        im[(wl * R + i) * ncol + u + h] = make_uint4(acc[i][4] ^ rep[i][4], acc[i][5] ^ rep[i][5],
                                                                     acc[i][6] ^ rep[i][6], acc[i][7] ^ rep[i][7]);
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
        __syncthreads();
        // (B) the e x e solve per 16-B column, in place
        for (uint32_t q = threadIdx.x; q < nb * ncol; q += NT) {
            const uint32_t wl = fdiv(q, dn), c = q - wl * ncol;
            uint4 sg[R], out[R];
#pragma unroll
            for (int i = 0; i < R; i++) sg[i] = im[(wl * R + i) * ncol + c];
            bsd::solve_col<R>(sg, out, L.ab(buf, wl), L.tc(buf, wl));
#pragma unroll
            for (int v = 0; v < R; v++) im[(wl * R + v) * ncol + c] = out[v];
        }
        __syncthreads();
        // (C) recovered rows front to back: consecutive lanes on consecutive
        // 16-B chunks, a whole step's rows in one burst (storing from (B)
        // instead, where a row's lines are finished by two waves at different
        // times, measured 1.61 vs 1.31 ms on cfg3, r06)
        for (uint32_t q = threadIdx.x; q < nb * R * ncol; q += NT) {
            const uint32_t wl = fdiv(q, drn), o = q - wl * R * ncol, v = fdiv(o, dn), c = o - v * ncol;
            if (v < L.ne(buf, wl)) {
                const uint32_t row = (L.rows(buf, wl) >> (8 * v)) & 0xFFu;
                st16(a.win + (w0 + wl) * a.wpitch + a.out_delta + (size_t)row * a.stride + c * 16u, im[q]);
            }
        }
        const uint64_t nx = xr.cur + xr.step;
        if (nx < xr.hi) bsd::plan<K, R>(a, L, buf ^ 1, nx * G, (uint32_t)min((uint64_t)G, a.nwin - nx * G));
        __syncthreads();
    }
}

// ========================================================= workloads ===
__global__ __launch_bounds__(kBlock) void synth_kernel(SynthArgs a) {
    __shared__ uint32_t s_len[kMaxK];
    __shared__ uint32_t s_S;
    const uint64_t w = a.w0 + blockIdx.x;
    const int tid = threadIdx.x, k = a.k;
    const uint64_t smtu = sm64(a.seed ^ TAG_MTU), slen = sm64(a.seed ^ TAG_LEN);
    const uint64_t spay = sm64(a.seed ^ TAG_PAY);
    if (tid == 0) s_S = 0;
    __syncthreads();
    if (tid < k) {
        s_len[tid] = pkt_len(a.workload, smtu, slen, w, tid, a.L);
        atomicMax(&s_S, s_len[tid]);
    }
    __syncthreads();
    const uint32_t hdr = a.workload == 0 ? 0u : 2u;
    const uint32_t S = hdr + s_S;
    if (tid == 0 && a.sym_len) a.sym_len[blockIdx.x] = S;
    uint8_t *win = a.win + (uint64_t)blockIdx.x * (uint64_t)(k + a.r) * a.stride;
    const uint32_t ncol = a.stride >> 4;
    for (uint32_t idx = tid; idx < (uint32_t)k * ncol; idx += kBlock) {
        const int j = (int)(idx / ncol);
        const uint32_t c = idx - (uint32_t)j * ncol;
        const uint32_t len = s_len[j];
        uint32_t out[4] = {0, 0, 0, 0};
        uint64_t cw = ~0ull, word = 0;
        for (int b = 0; b < 16; b++) {
            const uint32_t o = c * 16 + b;
            uint32_t byte = 0;
            if (hdr && o == 0) byte = len >> 8;
            else if (hdr && o == 1) byte = len & 0xFF;
            else if (o >= hdr && o < hdr + len) {
                const uint32_t po = o - hdr;
                const uint64_t wi = po >> 3;
                if (wi != cw) {
                    cw = wi;
                    word = sm64(spay + ((w << 24) | ((uint64_t)j << 16) | wi));
                }
                byte = (uint32_t)(word >> (8 * (po & 7))) & 0xFF;
            }
            out[b >> 2] |= byte << (8 * (b & 3));
        }
        *reinterpret_cast<uint4 *>(win + (size_t)j * a.stride + c * 16) =
            make_uint4(out[0], out[1], out[2], out[3]);
    }
}

__global__ __launch_bounds__(kBlock) void erasure_kernel(EraseArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= a.nwin) return;
    const uint64_t w = a.w0 + i;
    const int k = a.k, r = a.r;
    const uint64_t all = (k + r >= 64) ? ~0ull : ((1ull << (k + r)) - 1);
    const uint64_t sera = sm64(a.seed ^ TAG_ERA);
    uint64_t p = all;
    if (a.erasure == 2) {
        for (int s = 0; s < k + r; s++)
            if ((uint32_t)sm64(sera + ((w << 8) | (uint64_t)s)) < P10) p &= ~(1ull << s);
    } else if (a.erasure == 1) {
        if (a.scheme == 1) {
            uint8_t perm[kMaxK];
            for (int j = 0; j < k; j++) perm[j] = (uint8_t)j;
            const int e = r < k ? r : k;
            for (int t = 0; t < e; t++) {
                const uint64_t h = sm64(sera + ((w << 8) | (uint64_t)t));
                const int u = t + (int)(h % (uint64_t)(k - t));
                const uint8_t tmp = perm[t]; perm[t] = perm[u]; perm[u] = tmp;
                p &= ~(1ull << perm[t]);
            }
        } else {
            for (int g = 0; g < r; g++) {
                const int n = (k - g + r - 1) / r;
                if (n <= 0) continue;
                const int idx = (int)(sm64(sera + ((w << 8) | (uint64_t)g)) % (uint64_t)n);
                p &= ~(1ull << (g + idx * r));
            }
        }
    }
    a.present[i] = p;
}

// Digest: one workgroup per window.
__global__ __launch_bounds__(kBlock) void digest_kernel(DigestArgs a) {
    __shared__ uint64_t s_red[kBlock / 64];
    const uint64_t wi = blockIdx.x;
    const int tid = threadIdx.x, n = a.k + a.r;
    const uint32_t S = min(a.sym_len ? a.sym_len[wi] : a.S_all, a.stride);
    const uint32_t nw = (S + 7u) >> 3;
    const uint8_t *win = a.win + wi * (uint64_t)n * a.stride;
    uint64_t d = 0;
    for (uint32_t idx = tid; idx < (uint32_t)n * nw; idx += kBlock) {
        const uint32_t i = idx / nw, t = idx - i * nw;
        uint64_t word = *reinterpret_cast<const uint64_t *>(win + (size_t)i * a.stride + t * 8u);
        const uint32_t valid = S - t * 8u;
        if (valid < 8) word &= (1ull << (8 * valid)) - 1;
        d ^= sm64(word ^ (((uint64_t)i << 16) | t));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d ^= __shfl_xor(d, o, 64);
    if ((tid & 63) == 0) s_red[tid >> 6] = d;
    __syncthreads();
    if (tid == 0) {
        uint64_t x = 0;
        for (int i = 0; i < kBlock / 64; i++) x ^= s_red[i];
        atomicXor(reinterpret_cast<unsigned long long *>(a.digest),
                  (unsigned long long)sm64(x + a.w0 + wi));
    }
}

// ================================================ sliding-window RLC ===
// RFC 8681 sliding-window random linear code (include/fecgpu.h fecgpu_sw_*).
// Every data pass is a combine job (fec_internal.h CombJob): nout <= R outputs
// over nin contiguous input rows, multiply tables built per job in LDS from
// its coefficient bytes, the job's 16-B columns streamed by the workgroup like
// the block kernels' group mode.  Coefficients come from the RFC 8682 PRNG on
// the device (one lane per repair), the decode's linked systems are reduced
// by one wave each (Gauss-Jordan with pivot search).

// combine kernel: input rows loaded per batch.  One output (repairs,
// syndromes): 16 (sliding-window encode k 8 W 32: 0.370 vs 0.387 ms at 8,
// 0.466 at 4; profiles/r02_sw_ab.txt); solves (8 outputs, register-bound) and
// grouped encode jobs (2, 4 outputs): 8.
#define COMB_U(R) ((R) == 1 ? 16 : 8)

// Per-job LDS region of comb_kernel<R>: tables [nin_max][R] uint4 (TA/TB),
// [nin_max][RT] u32 (TC), output column-0 pointers [R], xor pointer, and per
// input row the mask of outputs with a nonzero coefficient [nin_max] u8
// (fec_internal.h comb_job_lds).
template <int R>
struct CombRegion {
    static constexpr int RT = R == 1 ? 1 : ((R + 3) & ~3);
    uint4 *ab;       // [nin_max + 1][R]: row nin_max = the xor row's multiplier (1 unless scaled)
    uint32_t *tc;    // [nin_max + 1][RT]
    uint4 *xab;
    uint32_t *xtc;
    uint64_t *optr;  // [R] + xor pointer at optr[R]
    uint8_t *nz;
    __device__ __forceinline__ CombRegion(uint8_t *region, int nin_max) {
        const size_t n = (size_t)nin_max + 1;
        ab = reinterpret_cast<uint4 *>(region);
        tc = reinterpret_cast<uint32_t *>(region + n * R * 16);
        xab = ab + (size_t)nin_max * R;
        xtc = tc + (size_t)nin_max * RT;
        optr = reinterpret_cast<uint64_t *>(region + n * (16 * R + 4 * RT));
        nz = reinterpret_cast<uint8_t *>(optr + R + 1);
    }
    // CombArgs::shared_coef: tables and nonzero masks shared (comb_shared_lds),
    // the xor row's tables and the output pointers per job (comb_job_small_lds)
    __device__ __forceinline__ CombRegion(uint8_t *tabs, uint8_t *job, int nin_max) {
        ab = reinterpret_cast<uint4 *>(tabs);
        tc = reinterpret_cast<uint32_t *>(tabs + (size_t)nin_max * R * 16);
        nz = tabs + (size_t)nin_max * (16 * R + 4 * RT);
        xab = reinterpret_cast<uint4 *>(job);
        xtc = reinterpret_cast<uint32_t *>(job + R * 16);
        optr = reinterpret_cast<uint64_t *>(job + R * 16 + RT * 4);
    }
};

// Input row q of a combine slot (row 0 at `in`, this lane's column); a row
// past the lane's job (its wave runs to the widest job's row count) re-reads
// the job's last row and is never multiplied.  (Buffer loads with scalar row
// offsets measured 7 % slower on the cfg7 decode, r04; removed r05.)
__device__ __forceinline__ uint4 row_ld(const uint8_t *in, int q, int nin, uint32_t stride) {
    return ld16(in + (uint32_t)min(q, nin - 1) * stride);
}

// One slot (job, 16-B column) for NE outputs (wave-uniform): acc[u] = sum_q
// T[q][u] * in_q over the job's nin rows (8 loads in flight), optional xor
// row, stores for u < ne (this lane's job).
template <int R, int NE>
__device__ __forceinline__ void comb_slot(const uint8_t *rs, uint32_t stride, int nin, int ne, uint32_t col,
                                          const CombRegion<R> &rg, bool skip) {
    constexpr int U = COMB_U(R), RT = CombRegion<R>::RT;
    uint4 acc[NE];
#pragma unroll
    for (int m = 0; m < NE; m++) acc[m] = zero4();
    for (int q0 = 0; q0 < nin; q0 += U) {
        uint4 v[U];
#pragma unroll
        for (int t = 0; t < U; t++) v[t] = row_ld(rs, q0 + t, nin, stride);
#pragma unroll
        for (int t = 0; t < U; t++) {
            if (q0 + t < nin) {
                const int q = q0 + t;
                // the wave's lanes may belong to different jobs: skip what no
                // active lane needs.  With >= 64 columns per job a wave spans at
                // most two jobs, its first and last active lanes'; otherwise no skip.
                uint32_t nzm = 0xffu;
                // only grouped encode launches (CombArgs::skip) have zero runs;
                // single repairs, syndromes and solves are dense (+5 % time with the test)
                if (R > 1 && skip) {
                    const uint32_t z = rg.nz[q];
                    const int last = 63 - __builtin_clzll(__builtin_amdgcn_read_exec());
                    nzm = __builtin_amdgcn_readfirstlane(z) | __builtin_amdgcn_readlane(z, last);
                }
                if (!nzm) continue;
                const Split sp = split(v[t]);
#pragma unroll
                for (int m = 0; m < NE; m++)
                    if ((nzm >> m) & 1u) gmac(acc[m], sp, rg.ab[q * R + m], rg.tc[q * RT + m]);
            }
        }
    }
    const uint64_t xp = rg.optr[R];
    if (xp) gmac(acc[0], split(ld16(reinterpret_cast<const uint8_t *>(xp) + col * 16u)), rg.xab[0], rg.xtc[0]);
#pragma unroll
    for (int m = 0; m < NE; m++)
        if (m < ne) st16(reinterpret_cast<uint8_t *>(rg.optr[m]) + col * 16u, acc[m]);
}

// rows per prefetched batch of the one-output slots (cfg7 decode: 4 rows 0.214
// vs 8 rows 0.223 ms per call, r04: 107 VGPRs, 4 waves per SIMD; 5 and 6 rows,
// 115 / 123 VGPRs, within 1 % of 4, r05).  The 8-output slots do not prefetch
// (221 VGPRs instead of 128: cfg7 decode 0.246 vs 0.238 ms, r04).
constexpr int kCombPfU = 4;
// comb_slot with the rows of batch i + 1 in flight while batch i multiplies
// (two 8-row buffers) and the xor row loaded with the first batch.  A
// workgroup streams its jobs' slots pass after pass, so without the prefetch
// every batch is a dependent round trip to HBM (the syndrome pass of a
// sliding-window decode: 3 per slot).  The trip count is the wave's largest
// nin (its lanes may belong to two jobs), so the loop and every load are
// wave-uniform: no load sits under a lane-dependent branch, where the
// compiler's wait counts would merge to the stricter path.  Rows past a
// lane's nin reload its last row and are not multiplied.
template <int R, int NE>
__device__ __forceinline__ void comb_slot_pf(const uint8_t *rs, uint32_t stride, int nin, int ne, uint32_t col,
                                             const CombRegion<R> &rg, bool skip) {
    constexpr int U = kCombPfU, RT = CombRegion<R>::RT;
    uint4 acc[NE];
#pragma unroll
    for (int m = 0; m < NE; m++) acc[m] = zero4();
    int nw = nin;
#pragma unroll
    for (int o = 32; o; o >>= 1) nw = max(nw, __shfl_xor(nw, o));
    nw = __builtin_amdgcn_readfirstlane(nw);
    const uint64_t xp = rg.optr[R];
    // without an xor row: a load of row 0 (a valid address), discarded
    const uint4 xv = ld16(xp ? reinterpret_cast<const uint8_t *>(xp) + col * 16u : rs);
    auto load = [&](uint4 (&v)[U], int q0) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < U; t++) v[t] = row_ld(rs, q0 + t, nin, stride);
    };
    auto mac = [&](const uint4 (&v)[U], int q0) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < U; t++) {
            const int q = q0 + t;
            if (q < nin) {
                uint32_t nzm = 0xffu;
                if (R > 1 && skip) {
                    const uint32_t z = rg.nz[q];
                    const int last = 63 - __builtin_clzll(__builtin_amdgcn_read_exec());
                    nzm = __builtin_amdgcn_readfirstlane(z) | __builtin_amdgcn_readlane(z, last);
                }
                if (!nzm) continue;
                const Split sp = split(v[t]);
#pragma unroll
                for (int m = 0; m < NE; m++)
                    if ((nzm >> m) & 1u) gmac(acc[m], sp, rg.ab[q * R + m], rg.tc[q * RT + m]);
            }
        }
    };
    uint4 va[U], vb[U];
    load(va, 0);
    for (int q0 = 0;; q0 += 2 * U) {
        if (q0 + U >= nw) {  // uniform
            mac(va, q0);
            break;
        }
        load(vb, q0 + U);
        mac(va, q0);
        if (q0 + 2 * U >= nw) {
            mac(vb, q0 + U);
            break;
        }
        load(va, q0 + 2 * U);
        mac(vb, q0 + U);
    }
    if (xp) gmac(acc[0], split(xv), rg.xab[0], rg.xtc[0]);  // the xor row times its multiplier
#pragma unroll
    for (int m = 0; m < NE; m++)
        if (m < ne) st16(reinterpret_cast<uint8_t *>(rg.optr[m]) + col * 16u, acc[m]);
}

template <int R, int NE = R>
__device__ __forceinline__ void comb_dispatch(int nw, const uint8_t *rs, uint32_t stride, int nin, int ne,
                                              uint32_t col, const CombRegion<R> &rg, bool skip) {
    if constexpr (NE >= 1) {
        if constexpr (R == 1) {
            if (nw == NE) {
                comb_slot_pf<R, NE>(rs, stride, nin, ne, col, rg, skip);
                return;
            }
        } else if (nw == NE) {
            comb_slot<R, NE>(rs, stride, nin, ne, col, rg, skip);
            return;
        }
        comb_dispatch<R, NE - 1>(nw, rs, stride, nin, ne, col, rg, skip);
    }
}

// Device twin of the host's choose_wpb (fec_capi.cpp): jobs per workgroup that
// fit `budget` bytes at job_lds each, picked for lane use over ncol columns.
__device__ __forceinline__ int choose_wpb_dev(uint32_t ncol, uint32_t job_lds, uint32_t budget) {
    int maxw = kMaxWpb;
    if (job_lds) maxw = max(1, min(maxw, (int)(budget / job_lds)));
    if (ncol == 0) return maxw;
    int best = 1;
    float best_u = -1.f;
    for (int w = 1; w <= maxw; w++) {
        const uint32_t slots = (uint32_t)w * ncol, passes = (slots + kBlock - 1) / kBlock;
        const float u = (float)slots / (float)(passes * kBlock) - (passes < 2 ? 0.05f : 0.f);
        if (u > best_u + 1e-6f) {
            best_u = u;
            best = w;
        }
    }
    return best;
}

template <int R>
__global__ __launch_bounds__(kBlock) void comb_kernel(CombArgs a) {
    extern __shared__ uint4 dyn[];
    __shared__ uint32_t s_pfx[kMaxWpb + 1];
    __shared__ uint64_t s_in[kMaxWpb];
    __shared__ uint32_t s_nin[kMaxWpb];
    __shared__ uint8_t s_ne[kMaxWpb], s_perm[kMaxWpb];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // sparse launches: the gathered jobs' headers first (kCombListLds)
    uint8_t *regions = reinterpret_cast<uint8_t *>(dyn) + (a.sparse ? kCombListLds : 0u);
    constexpr int RT = CombRegion<R>::RT;
    // checked builds: every row a job reads or writes lies in the launch's
    // arrays (CombArgs::chk: inputs, xor rows, outputs)
    CHK_PROLOGUE(a);
    if (a.err && (*a.err & kSwErrStop)) return;  // the whole grid stands down (device-sized decode launches)
    const uint64_t njobs = a.njobs + (a.extra ? (uint64_t)(*a.extra >> a.extra_shift) : 0ull);
    int nin_max = a.nin_max, wpb = a.wpb;
    uint32_t job_lds = a.job_lds;
    if (a.nin_dev) {  // device-sized: the widest job is known on the device only
        nin_max = max(1, min((int)*a.nin_dev, a.nin_max));
        job_lds = comb_job_lds(nin_max, R);
        wpb = choose_wpb_dev(a.ncol, job_lds, a.budget);
        if (a.sparse) wpb = max(1, min(kMaxWpb, (int)(a.budget / job_lds)));  // as many gathered jobs as fit
    }
    // shared coefficient block: its tables once per workgroup, before any group
    const bool shared = a.shared_coef != 0;
    const uint32_t tab_lds = shared ? comb_shared_lds(nin_max, R) : 0u;
    if (shared) {
        job_lds = comb_job_small_lds(R);
        const int nout = min(a.nout_max, R);
        const CombRegion<R> rg(regions, regions + tab_lds, nin_max);
        for (int i = tid; i < nout * nin_max; i += kBlock) {
            const int u = i / nin_max, q = i - u * nin_max;
            const CoefTab ct = make_coef_tab(a.coef[i]);
            rg.ab[q * R + u] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
            rg.tc[q * RT + u] = ct.c;
        }
        for (int q = tid; q < nin_max; q += kBlock) {
            uint32_t m = 0;
            for (int u = 0; u < nout; u++) m |= (a.coef[u * nin_max + q] != 0 ? 1u : 0u) << u;
            rg.nz[q] = (uint8_t)m;
        }
        __syncthreads();
    }
    const auto region = [&](int jl) __attribute__((always_inline)) {
        return shared ? CombRegion<R>(regions, regions + tab_lds + (size_t)jl * job_lds, nin_max)
                      : CombRegion<R>(regions + (size_t)jl * job_lds, nin_max);
    };
    // one group of nb jobs (jobAt(jl): job jl of the group): tables, then its
    // (job, column) slots over the workgroup
    constexpr int NW = kBlock / 64;
    const auto run_group = [&](int nb, auto &&jobAt) __attribute__((always_inline)) {
        // plan: wave w builds the tables of jobs w, w + 4, ...  Their headers
        // come in one round of loads, a lane each (the decode passes walk a
        // slot per repair or unknown, most of them empty: one dependent load
        // per job was most of those passes' time)
        CombJob Jl{};
        Jl.xor_off = kNoXor;
        if (wave + NW * lane < nb) Jl = jobAt(wave + NW * lane);
        for (int ji = 0, jl = wave; jl < nb; ji++, jl += NW) {
            const auto rl64 = [&](uint64_t v) __attribute__((always_inline)) {
                return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, ji) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), ji) << 32);
            };
            CombJob J;
            J.in_off = rl64(Jl.in_off);
            J.coef_off = rl64(Jl.coef_off);
            J.out_list = rl64(Jl.out_list);
            J.xor_off = rl64(Jl.xor_off);
            J.nin = (uint32_t)__builtin_amdgcn_readlane((int)Jl.nin, ji);
            J.nout = (uint32_t)__builtin_amdgcn_readlane((int)Jl.nout, ji);
            const int nin = min((int)J.nin, nin_max), nout = min((int)(J.nout & ~kCombXorScaled), R);
            const CombRegion<R> rg = region(jl);
            const uint8_t *cf = a.coef + J.coef_off;
            if (!shared) {
                for (int i = lane; i < nout * nin; i += 64) {
                    const int u = i / nin, q = i - u * nin;
                    const CoefTab ct = make_coef_tab(cf[i]);
                    rg.ab[q * R + u] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
                    rg.tc[q * RT + u] = ct.c;
                }
                for (int q = lane; q < nin; q += 64) {
                    uint32_t m = 0;
                    for (int u = 0; u < nout; u++) m |= (cf[u * nin + q] != 0 ? 1u : 0u) << u;
                    rg.nz[q] = (uint8_t)m;
                }
            }
            if (lane < nout) {
                rg.optr[lane] = reinterpret_cast<uint64_t>(a.out_base) + a.outs[J.out_list + lane];
                const CoefTab ct = make_coef_tab((J.nout & kCombXorScaled) ? cf[nout * nin + lane] : 1u);
                rg.xab[lane] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
                rg.xtc[lane] = ct.c;
            }
            if (lane == 0) {
                rg.optr[R] = J.xor_off == kNoXor ? 0ull : reinterpret_cast<uint64_t>(a.xor_base) + J.xor_off;
                s_in[jl] = reinterpret_cast<uint64_t>(a.in_base) + J.in_off;
                s_nin[jl] = (uint32_t)nin;
                s_ne[jl] = (uint8_t)nout;
            }
        }
        __syncthreads();
        if (tid < 64) {
            // jobs in descending order of outputs (comb_slot runs the wave's largest)
            const int t = tid;
            const int ne_t = t < nb ? (int)s_ne[t] : -1;
            const uint64_t below = (1ull << t) - 1;
            int rank = 0;
#pragma unroll
            for (int v = R; v >= 0; v--) {
                const uint64_t b = __ballot(ne_t == v);
                if (v > ne_t) rank += __popcll(b);
                else if (v == ne_t) rank += __popcll(b & below);
            }
            if (t < nb) s_perm[rank] = (uint8_t)t;
            WAVE_SYNC();
            const int jl = t < nb ? (int)s_perm[t] : 0;
            block_prefix(s_pfx, (t < nb && s_ne[jl]) ? a.ncol : 0u, t);
        }
        __syncthreads();
        const uint32_t total = s_pfx[nb];
        int i = 0;
        for (uint32_t s = tid; s < total; s += kBlock) {
            while (s >= s_pfx[i + 1]) i++;
            const int jl = s_perm[i];
            const uint32_t col = s - s_pfx[i];
            const int ne = s_ne[jl];
            const int nw = __builtin_amdgcn_readfirstlane(ne);
            const CombRegion<R> rg = region(jl);
            const uint8_t *rs = reinterpret_cast<const uint8_t *>(s_in[jl]) + col * 16u;
            comb_dispatch<R>(nw, rs, a.stride, (int)s_nin[jl], ne, col, rg, a.skip && a.ncol >= 64);
        }
        __syncthreads();
    };
    if (a.sparse) {
        // mostly empty job slots (a decode's slot per repair / per unknown): the
        // workgroup gathers the non-empty jobs of 256 slots at a time into LDS,
        // then runs them in groups as large as its LDS holds.  Slots are dealt
        // in runs of kCombRun consecutive ones, round-robin over the
        // workgroups: every workgroup gets a like share of a dense region (the
        // one-unknown systems' slots), and consecutive repairs (overlapping
        // windows) stay together.
        CombJob *s_list = reinterpret_cast<CombJob *>(dyn);
        __shared__ uint32_t s_wc[NW + 1];
        const int cap = max(1, min(kMaxWpb, wpb));
        constexpr uint32_t kRuns = kBlock / kCombRun;  // runs per round
        const uint64_t nrun = (njobs + kCombRun - 1) / kCombRun;
        for (uint64_t r0 = blockIdx.x; r0 < nrun; r0 += (uint64_t)gridDim.x * kRuns) {
            const uint64_t run = r0 + (uint64_t)gridDim.x * (tid / kCombRun);
            const uint64_t slot = run * kCombRun + tid % kCombRun;
            const CombJob J = a.jobs[min(slot, njobs - 1)];  // (njobs > 0 here)
            const bool live = run < nrun && slot < njobs && (J.nout & ~kCombXorScaled) != 0;
            const uint64_t b = __ballot(live);
            if (lane == 0) s_wc[wave] = (uint32_t)__popcll(b);
            __syncthreads();
            uint32_t off = 0, k = 0;
            for (int w = 0; w < NW; w++) {
                off += w < wave ? s_wc[w] : 0u;
                k += s_wc[w];
            }
            if (live) {
                CombJob &L = s_list[off + __popcll(b & ((1ull << lane) - 1ull))];
                L.in_off = J.in_off;
                L.coef_off = J.coef_off;
                L.out_list = J.out_list;
                L.xor_off = J.xor_off;
                L.nin = J.nin;
                L.nout = J.nout;
            }
            __syncthreads();
            for (uint32_t g0 = 0; g0 < k; g0 += (uint32_t)cap)
                run_group((int)min<uint32_t>((uint32_t)cap, k - g0),
                          [&](int jl) __attribute__((always_inline)) {
                              const CombJob &L = s_list[g0 + jl];
                              CombJob J;
                              J.in_off = L.in_off;
                              J.coef_off = L.coef_off;
                              J.out_list = L.out_list;
                              J.xor_off = L.xor_off;
                              J.nin = L.nin;
                              J.nout = L.nout;
                              return J;
                          });
        }
        return;
    }
    for (XcdRange xr = xcd_range((njobs + wpb - 1) / wpb, a.nx); xr.cur < xr.hi; xr.cur += xr.step) {
        const uint64_t j0 = xr.cur * wpb;
        const int nb = (int)min((uint64_t)wpb, njobs - j0);
        run_group(nb, [&](int jl) __attribute__((always_inline)) { return a.jobs[j0 + jl]; });
    }
}

// Encode: lane per repair — clip the window to the batch, draw its RFC 8681
// coefficients, write its job (output: repair row t).
__device__ __forceinline__ void sw_enc_single(const SwEncCoefArgs &a, uint64_t t, uint64_t jt);

// Grouped encode jobs (SwEncCoefArgs::group), lane per repair t of group
// g = t / group: every lane of the group finds the union of its windows; its
// row of the group's coefficients, or (group too wide) its own job in the tail.
__device__ __forceinline__ void sw_enc_grouped(const SwEncCoefArgs &a, uint64_t t) {
    const uint64_t g = t / (uint64_t)a.group, t0 = g * (uint64_t)a.group;
    const uint64_t ngroups = (a.nrep + a.group - 1) / a.group;
    const int n = (int)min((uint64_t)a.group, a.nrep - t0), u = (int)(t - t0);
    uint64_t lo = ~0ull, hi = 0;
    for (int v = 0; v < n; v++) {
        const fecgpu_sw_repair h = a.hdr[t0 + v];
        const uint64_t fss = min(h.fss, a.nsrc);
        const uint64_t nss = min((uint64_t)min((int)h.nss, a.max_window), a.nsrc - fss);
        lo = min(lo, fss);
        hi = max(hi, fss + nss);
    }
    const uint64_t span = hi - lo;
    if (span > (uint64_t)a.span_max || span * (uint64_t)n > (uint64_t)a.group * kSwCoefPitch) {
        if (u == 0) {
            CombJob E{};
            E.xor_off = kNoXor;  // empty: nout = 0
            a.jobs[g] = E;
        }
        sw_enc_single(a, t, ngroups + atomicAdd(a.tail, 1u));
        return;
    }
    const fecgpu_sw_repair h = a.hdr[t];
    const uint64_t fss = min(h.fss, a.nsrc);
    const int nss = (int)min((uint64_t)min((int)h.nss, a.max_window), a.nsrc - fss);
    uint8_t *row = a.coef + t0 * kSwCoefPitch + (uint64_t)u * span;
    const int b = (int)(fss - lo);
    for (int q = 0; q < b; q++) row[q] = 0;
    rlc_coefs_tab(a.rlc, h.key, nss, min((uint32_t)h.dt, 15u), row + b);
    for (int q = b + nss; q < (int)span; q++) row[q] = 0;
    a.outs[t] = t * a.stride;
    if (u == 0) {
        CombJob J;
        J.in_off = lo * a.stride;
        J.coef_off = t0 * kSwCoefPitch;
        J.out_list = t0;
        J.xor_off = kNoXor;
        J.nin = (uint32_t)span;
        J.nout = (uint32_t)n;
        a.jobs[g] = J;
    }
}

__global__ __launch_bounds__(kBlock) void sw_enc_coef_kernel(SwEncCoefArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= a.nrep) return;
    if (a.group > 1) sw_enc_grouped(a, t);
    else sw_enc_single(a, t, t);
}

__device__ __forceinline__ void sw_enc_single(const SwEncCoefArgs &a, uint64_t t, uint64_t jt) {
    const fecgpu_sw_repair h = a.hdr[t];
    const uint64_t fss = min(h.fss, a.nsrc);
    const int nss = (int)min((uint64_t)min((int)h.nss, a.max_window), a.nsrc - fss);
    uint8_t *cc = a.coef + t * kSwCoefPitch;
    rlc_coefs_tab(a.rlc, h.key, nss, min((uint32_t)h.dt, 15u), cc);
    CombJob J;
    J.in_off = fss * a.stride;
    J.coef_off = t * kSwCoefPitch;
    J.out_list = t;
    J.xor_off = kNoXor;
    J.nin = (uint32_t)nss;
    J.nout = 1;
    a.jobs[jt] = J;
    a.outs[t] = t * a.stride;
}

// ========================================================== launchers ===
namespace {

// Persistent grid: blocks resident on the whole chip for this kernel and LDS size.
int resident_blocks(const void *fn, uint32_t lds, int nt = kBlock) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 1024;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, nt, lds) != hipSuccess || per < 1) per = 1;
    return cus * per;
}

// chunks != 0: the kernel walks that many work units of its own (a flat unit
// space other than 16-B slots) on a persistent grid, like flat mode.
template <class K>
hipError_t launch(K kernel, BatchArgs a, const LaunchPlan &p, hipStream_t s, bool flat,
                  uint64_t chunks = 0, int nt = kBlock) {
    const void *fn = reinterpret_cast<const void *>(kernel);
    // work units: 256-slot chunks (flat) or window groups
    const uint64_t want = chunks ? chunks
                          : flat ? (a.nwin * a.ncol + kBlock - 1) / kBlock
                                 : (a.nwin + a.wpb - 1) / a.wpb;
    // Flat mode: persistent, 2 x resident workgroups (measured best on cfg2/cfg3).
    // Group mode: one workgroup per group unless a multiplier is forced — the
    // dispatcher's dynamic assignment balances uneven windows better than a
    // static round-robin over persistent workgroups (cfg4 mixed MTU).
    uint64_t grid = want;
    if (p.blocks_per_cu > 0) {
        int dev = 0, cus = 256;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        grid = std::min<uint64_t>(want, (uint64_t)cus * (uint64_t)p.blocks_per_cu);
    } else if (flat || chunks || p.grid_mult > 0) {
        const int mult = p.grid_mult > 0 ? p.grid_mult : 2;
        grid = std::min<uint64_t>(want, (uint64_t)resident_blocks(fn, p.lds_bytes, nt) * (uint64_t)mult);
    }
    // XCD regions: grid a multiple of 8 so every region has the same walkers
    a.nx = 8;
    if (a.nx == 1) {
        grid = std::max<uint64_t>(1, std::min(grid, want));
    } else if (want < 8) {
        a.nx = 1;
        grid = std::max<uint64_t>(1, want);
    } else if (grid >= want) {
        grid = (want + 7) / 8 * 8;  // one unit per workgroup
    } else {
        grid = std::max<uint64_t>(8, grid / 8 * 8);
    }
    grid = std::min<uint64_t>(grid, 0x7FFFFFF8ull);
    if (flat) {
        const uint64_t step = grid / a.nx * kBlock;  // slots per iteration
        a.step_win = step / a.ncol;
        a.step_col = (uint32_t)(step % a.ncol);
    }
    hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(nt), p.lds_bytes, s, a);
    return hipGetLastError();
}

}  // namespace

#define DISPATCH_R(R_, EXPR)                    \
    switch (R_) {                               \
        case 1: { constexpr int RR = 1; return EXPR; } \
        case 2: { constexpr int RR = 2; return EXPR; } \
        case 3: { constexpr int RR = 3; return EXPR; } \
        case 4: { constexpr int RR = 4; return EXPR; } \
        case 5: { constexpr int RR = 5; return EXPR; } \
        case 6: { constexpr int RR = 6; return EXPR; } \
        case 7: { constexpr int RR = 7; return EXPR; } \
        case 8: { constexpr int RR = 8; return EXPR; } \
        default: return hipErrorInvalidValue;   \
    }

// Codes with a bit-sliced encode (Cauchy and Vandermonde rows, compiled in).
// r = 8, k >= 16: the table multiply is VALU-bound and the bit-sliced kernel
// 1.1-1.4x faster.  k 16 r 4 (cfg3): with its stores gathered (uniform short
// rows, gf_encode_bs_gs_kernel) it runs at 2 workgroups per CU, where HBM
// moves the mix fastest, and beats the table multiply that needs 4-5 waves
// per SIMD for its VALU work (profiles/r06_*); other r <= 4
// codes stay on the table multiply (profiles/r01_bs_r4_and_alternation.txt).
#define BS_CODES(X) X(16, 4) X(16, 8) X(24, 8) X(32, 8)

bool bitslice_supported(int k, int r, int matrix) {
    if (matrix != FECGPU_MATRIX_CAUCHY && matrix != FECGPU_MATRIX_VANDERMONDE) return false;
#define BS_HAS(K_, R_) if (k == K_ && r == R_) return true;
    BS_CODES(BS_HAS)
#undef BS_HAS
    return false;
}

hipError_t launch_encode(int scheme, const BatchArgs &a, const LaunchPlan &p, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    if (p.bitslice) {
#define BS_LAUNCH_M(K_, R_, M_)                                                            \
        if (a.k == K_ && a.r == R_ && p.matrix == M_)                                             \
            return p.bsgs ? launch(gf_encode_bs_gs_kernel<K_, R_, M_>, a, p, s, false,           \
                                   (a.nwin + a.wpb - 1) / a.wpb)                                   \
                 : p.flat ? launch(gf_encode_bs_kernel<K_, R_, M_, true>, a, p, s, false,         \
                                   (a.nwin * ((a.ncol + 1) / 2) + kBlock - 1) / kBlock)             \
                          : launch(gf_encode_bs_kernel<K_, R_, M_, false>, a, p, s, false);
#define BS_LAUNCH(K_, R_)                                 \
        BS_LAUNCH_M(K_, R_, FECGPU_MATRIX_CAUCHY)         \
        BS_LAUNCH_M(K_, R_, FECGPU_MATRIX_VANDERMONDE)
        BS_CODES(BS_LAUNCH)
#undef BS_LAUNCH
#undef BS_LAUNCH_M
        return hipErrorInvalidValue;
    }
    if (p.rbitslice) {
        const uint64_t want = (a.nwin * ((a.ncol + kRbsCols - 1) / kRbsCols) + kBlock - 1) / kBlock;
        switch (a.r) {
#define RBS_CASE(R_)                                                                        \
            case R_:                                                                               \
                return a.pres_nw ? launch(gf_encode_rbs_kernel<R_, true, true>, a, p, s, false, want)  \
                     : p.flat ? launch(gf_encode_rbs_kernel<R_, true>, a, p, s, false, want)       \
                              : launch(gf_encode_rbs_kernel<R_, false>, a, p, s, false);
            RBS_CASE(4) RBS_CASE(5) RBS_CASE(6) RBS_CASE(7) RBS_CASE(8)
#undef RBS_CASE
            default: return hipErrorInvalidValue;
        }
    }
    const bool flat = p.flat;
    if (scheme == 0) {
        if (flat) DISPATCH_R(a.r, launch(xor_encode_kernel<RR, true>, a, p, s, true))
        else DISPATCH_R(a.r, launch(xor_encode_kernel<RR, false>, a, p, s, false))
    }
    if (flat) DISPATCH_R(a.r, launch(gf_encode_kernel<RR, true>, a, p, s, true))
    else if (p.remote) DISPATCH_R(a.r, launch(gf_encode_kernel<RR, false, 8>, a, p, s, false))
    else DISPATCH_R(a.r, launch(gf_encode_kernel<RR, false>, a, p, s, false))
}

// The runtime-mask bit-sliced encode over uniform windows of any k (fec_wide.hip:
// the wide encode, and the two-stage wide decode's syndromes): window w at
// win + w * wpitch, its k input rows first, output i at
// (input row k + i's address) + out_delta + w * out_wdelta.  Flat unit space.
bool rbs_masked_ok(uint32_t ncol, uint64_t wpitch) {
    const uint32_t h = (ncol + kRbsCols - 1) / kRbsCols;
    return h > 0 && (uint64_t)(64 / h + 2) * wpitch < (1ull << 31);
}

hipError_t launch_rbs_rows(uint8_t *win, uint64_t nwin, uint32_t ncol, uint32_t stride, uint64_t wpitch, int k,
                           int r, const uint32_t *masks, uint64_t out_delta, uint64_t out_wdelta, hipStream_t s,
                           const uint64_t *present, uint32_t pres_nw) {
    if (nwin == 0) return hipSuccess;
    if (r < 4 || r > 8) return hipErrorInvalidValue;
    if (present && (pres_nw == 0 || !rbs_masked_ok(ncol, wpitch))) return hipErrorInvalidValue;
    BatchArgs a{};
    a.win = win;
    a.nwin = nwin;
    a.ncol = ncol;
    a.stride = stride;
    a.wpitch = wpitch;
    a.k = k;
    a.r = r;
    a.enc_bs = masks;
    a.out_delta = out_delta;
    a.out_wdelta = out_wdelta;
    a.present = present;
    a.pres_nw = present ? pres_nw : 0u;
    // FECGPU_CHECK builds: the input rows, and the outputs (out_delta /
    // out_wdelta may send them to another array: the wide decode's syndromes)
    a.chk.lo[0] = reinterpret_cast<uint64_t>(win);
    a.chk.n[0] = nwin * wpitch;
    a.chk.lo[1] = reinterpret_cast<uint64_t>(win) + (uint64_t)k * stride + out_delta;
    a.chk.n[1] = (nwin - 1) * (wpitch + out_wdelta) + (uint64_t)r * stride;
    LaunchPlan p{};
    p.flat = true;
    p.rbitslice = true;
    return launch_encode(FECGPU_SCHEME_GF256, a, p, s);
}

namespace {
hipError_t launch_gf_decode_table(const BatchArgs &a, const LaunchPlan &p, hipStream_t s) {
    DISPATCH_R(a.r, launch(gf_decode_kernel<RR>, a, p, s, false))
}
}  // namespace

// Codes with a bit-sliced syndrome decode (Cauchy rows, compiled network)
bool bsdec_supported(int k, int r, int matrix) { return matrix == FECGPU_MATRIX_CAUCHY && k == 16 && r == 4; }

hipError_t launch_decode(int scheme, const BatchArgs &a, const LaunchPlan &p, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    if (p.bsdec) {
        if (a.k != 16 || a.r != 4 || a.wpb < 1 || a.wpb * 16 > kBsdBlock) return hipErrorInvalidValue;
        const uint64_t chunks = (a.nwin + a.wpb - 1) / a.wpb;
        auto go = [&](auto kernel, int nt) {
            if (p.lds_bytes > (64u << 10)) {  // past the default dynamic LDS cap
                const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds_bytes);
                if (e != hipSuccess) return e;
            }
            return launch(kernel, a, p, s, false, chunks, nt);
        };
        return go(gf_decode_bs_gs_kernel<16, 4, FECGPU_MATRIX_CAUCHY, kBsdBlock>, kBsdBlock);
    }
    if (scheme == 0) {
        if (p.flat) DISPATCH_R(a.r, launch(xor_decode_kernel<RR, true>, a, p, s, true))
        else DISPATCH_R(a.r, launch(xor_decode_kernel<RR, false>, a, p, s, false))
    }
    return launch_gf_decode_table(a, p, s);
}

hipError_t take_bounds_faults(uint64_t *count, uint64_t *first) {
    *count = *first = 0;
#if FECGPU_CHECK
    unsigned long long v[2] = {0, 0};
    hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_chk_bad), sizeof(v));
    if (e != hipSuccess) return e;
    *count = v[0];
    *first = v[1];
    if (v[0]) {
        const unsigned long long z[2] = {0, 0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_chk_bad), z, sizeof(z));
    }
    return e;
#else
    return hipSuccess;
#endif
}

hipError_t launch_synth(const SynthArgs &a, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)a.nwin), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_erasure(const EraseArgs &a, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(erasure_kernel, dim3((unsigned)((a.nwin + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, s, a);
    return hipGetLastError();
}

hipError_t launch_comb(CombArgs a, int R, hipStream_t s) {
    const uint64_t nmax = a.njobs + (a.extra ? a.extra_max : 0);
    if (nmax == 0) return hipSuccess;
    uint64_t grid;
    uint32_t lds;
    if (a.nin_dev) {
        // device-sized: persistent, 2 x the workgroups resident at the budget
        // (the job count and widths are device data; surplus workgroups exit)
        lds = a.budget + (a.sparse ? kCombListLds : 0u);
        const void *fn = R == 1 ? (const void *)comb_kernel<1> : R == 2 ? (const void *)comb_kernel<2>
                       : R == 4 ? (const void *)comb_kernel<4> : (const void *)comb_kernel<8>;
        const uint64_t groups_max = nmax;  // at least one job per group
        grid = std::min<uint64_t>(groups_max, (uint64_t)resident_blocks(fn, lds) * 2);
        a.nx = grid >= 8 && !a.interleave ? 8 : 1;
        grid = std::max<uint64_t>(a.nx, grid / a.nx * a.nx);
    } else {
        const uint64_t groups = (nmax + a.wpb - 1) / a.wpb;
        a.nx = groups >= 8 ? 8 : 1;
        grid = (groups + a.nx - 1) / a.nx * a.nx;  // one group per workgroup
        lds = a.shared_coef ? comb_shared_lds(a.nin_max, R) + comb_job_small_lds(R) * (uint32_t)a.wpb
                            : a.job_lds * (uint32_t)a.wpb;
    }
    switch (R) {
        case 1: hipLaunchKernelGGL(comb_kernel<1>, dim3((unsigned)grid), dim3(kBlock), lds, s, a); break;
        case 2: hipLaunchKernelGGL(comb_kernel<2>, dim3((unsigned)grid), dim3(kBlock), lds, s, a); break;
        case 4: hipLaunchKernelGGL(comb_kernel<4>, dim3((unsigned)grid), dim3(kBlock), lds, s, a); break;
        case 8: hipLaunchKernelGGL(comb_kernel<8>, dim3((unsigned)grid), dim3(kBlock), lds, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_sw_enc_coef(const SwEncCoefArgs &a, hipStream_t s) {
    if (a.nrep == 0) return hipSuccess;
    hipLaunchKernelGGL(sw_enc_coef_kernel, dim3((unsigned)((a.nrep + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_digest(const DigestArgs &a, hipStream_t s) {
    if (a.nwin == 0) return hipSuccess;
    hipLaunchKernelGGL(digest_kernel, dim3((unsigned)a.nwin), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace fecgpu
