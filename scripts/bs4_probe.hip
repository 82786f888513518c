// bs4_probe.hip — cfg3 GF(2^8) k16 r4 encode: bit-sliced XOR network
// (compile-time Cauchy masks, the product's bs:: code) against the table
// multiply, with the repairs stored per lane or gathered in LDS and stored row
// by row (whole windows per workgroup step), at several occupancies.
// Outputs compared with the table kernel's.  Tuning aid, not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I quic-fec-eps_amd/csrc -o scripts/bs4_probe scripts/bs4_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "fec_spec.h"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

namespace fecgpu {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 *gptr_c;
typedef __attribute__((address_space(1))) u32x4 *gptr;
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    const u32x4 v = *(gptr_c)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) {
    const u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, (gptr)(p));
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
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

template <int T>
__device__ __forceinline__ void load_src(const uint8_t *pa, const uint8_t *pb, uint32_t stride,
                                         uint32_t (&x)[8]) {
    const uint4 va = ld16(pa + T * stride), vb = ld16(pb + T * stride);
    x[0] = va.x; x[1] = va.y; x[2] = va.z; x[3] = va.w;
    x[4] = vb.x; x[5] = vb.y; x[6] = vb.z; x[7] = vb.w;
}

// one batch of sources J0 + T (pa / pb point at source J0): all loads first,
// then transposes and XORs
template <int K, int R, int M, int J0, int... T>
__device__ __forceinline__ void batch(const uint8_t *pa, const uint8_t *pb, uint32_t stride,
                                      uint32_t (&acc)[R][8], std::integer_sequence<int, T...>) {
    uint32_t x[sizeof...(T)][8];
    (load_src<T>(pa, pb, stride, x[T]), ...);
    ((tr8(x[T]), source<K, R, M, J0 + T>(x[T], acc, std::make_integer_sequence<int, R * 8>{}),
      __builtin_amdgcn_sched_barrier(0)), ...);
}

template <int K, int R, int M, int U, int J0>
__device__ __forceinline__ void sources(const uint8_t *pa, const uint8_t *pb, uint32_t stride,
                                        uint32_t (&acc)[R][8]) {
    if constexpr (J0 < K) {
        batch<K, R, M, J0>(pa, pb, stride, acc, std::make_integer_sequence<int, ((K - J0) < U ? (K - J0) : U)>{});
        // (no workgroup barrier per batch: the r01 knob for one was defined after
        // its use and so never compiled in; every measurement ran without it)
        // advance opaquely, so the compiler does not keep K addresses live at once
        pa += U * stride;
        pb += U * stride;
        asm volatile("" : "+v"(pa), "+v"(pb));
        sources<K, R, M, U, J0 + U>(pa, pb, stride, acc);
    }
}

}  // namespace bs

// ------------------------------------------------------------ geometry ---
constexpr int K = 16, R = 4, M = 0;
constexpr uint32_t S = 1200, NCOL = S / 16, H = (NCOL + 1) / 2, WB = (K + R) * S;

struct XR {
    size_t cur, hi, step;
};
__device__ __forceinline__ XR xr_make(size_t nunits) {
    const uint32_t nx = 8, bx = blockIdx.x % nx, bi = blockIdx.x / nx, nbx = gridDim.x / nx;
    const size_t lo = nunits * bx / nx, hi = nunits * (bx + 1) / nx;
    return {lo + bi, hi, nbx};
}

// ------------------------------------------------- table reference (flat) ---
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
__device__ __forceinline__ uint32_t gm2(uint32_t acc, const Split &s0, const Split &s1, int i, uint4 ab0, uint32_t tc0,
                                        uint4 ab1, uint32_t tc1) {
    uint32_t t = xor3(acc, __builtin_amdgcn_perm(ab0.y, ab0.x, s0.a[i]), __builtin_amdgcn_perm(ab0.w, ab0.z, s0.b[i]));
    t = xor3(t, __builtin_amdgcn_perm(tc0, tc0, s0.c[i]), __builtin_amdgcn_perm(ab1.y, ab1.x, s1.a[i]));
    return xor3(t, __builtin_amdgcn_perm(ab1.w, ab1.z, s1.b[i]), __builtin_amdgcn_perm(tc1, tc1, s1.c[i]));
}
__global__ __launch_bounds__(256) void tab_flat(uint8_t *win, size_t nwin, const uint4 *gab, const uint32_t *gc) {
    __shared__ uint4 tab[K * R];
    __shared__ uint32_t tc[K * R];
    if (threadIdx.x < K * R) { tab[threadIdx.x] = gab[threadIdx.x]; tc[threadIdx.x] = gc[threadIdx.x]; }
    __syncthreads();
    const size_t total = nwin * NCOL;
    for (XR xr = xr_make((total + 255) / 256); xr.cur < xr.hi; xr.cur += xr.step) {
        const size_t s = xr.cur * 256 + threadIdx.x;
        if (s >= total) continue;
        const size_t w = s / NCOL, c = s - w * NCOL;
        uint8_t *b = win + w * WB + c * 16;
        uint4 acc[R] = {};
#pragma unroll 1
        for (int j = 0; j < K; j += 2) {
            const uint4 v0 = ld16(b + (size_t)j * S), v1 = ld16(b + (size_t)(j + 1) * S);
            const Split s0 = split(v0), s1 = split(v1);
            const int row = __builtin_amdgcn_readfirstlane(j * R);
#pragma unroll
            for (int m = 0; m < R; m++) {
                const uint4 a0 = tab[row + m], a1 = tab[row + R + m];
                const uint32_t c0 = tc[row + m], c1 = tc[row + R + m];
                acc[m].x = gm2(acc[m].x, s0, s1, 0, a0, c0, a1, c1);
                acc[m].y = gm2(acc[m].y, s0, s1, 1, a0, c0, a1, c1);
                acc[m].z = gm2(acc[m].z, s0, s1, 2, a0, c0, a1, c1);
                acc[m].w = gm2(acc[m].w, s0, s1, 3, a0, c0, a1, c1);
            }
        }
#pragma unroll
        for (int m = 0; m < R; m++) st16(b + (size_t)(K + m) * S, acc[m]);
    }
}

// ------------------------------------------------------ bit-sliced, flat ---
// unit (w, u < H): columns u and u + H (B = A past the row: same bytes)
template <int U>
__global__ __launch_bounds__(256) void bs_flat(uint8_t *win, size_t nwin) {
    const size_t total = nwin * H;
    for (XR xr = xr_make((total + 255) / 256); xr.cur < xr.hi; xr.cur += xr.step) {
        size_t s = xr.cur * 256 + threadIdx.x;
        const bool live = s < total;
        if (!live) s = total - 1;
        const size_t w = s / H;
        const uint32_t u = (uint32_t)(s - w * H);
        uint8_t *pa = win + w * WB + u * 16u;
        uint8_t *pb = u + H < NCOL ? pa + H * 16u : pa;
        uint32_t acc[R][8];
        bs::sources<K, R, M, U, 0>(pa, pb, S, acc);
#pragma unroll
        for (int i = 0; i < R; i++) {
            bs::tr8(acc[i]);
            if (live) {
                st16(pa + (size_t)(K + i) * S, make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]));
                if (pb != pa) st16(pb + (size_t)(K + i) * S, make_uint4(acc[i][4], acc[i][5], acc[i][6], acc[i][7]));
            }
        }
    }
}

// ------------------------------------------- bit-sliced, gathered stores ---
// G whole windows per step, NT threads; unit (wl, u < H) per lane; repairs to
// an LDS image [wl][m][col] (two images), rows stored front to back
template <int G, int NT, int U>
__global__ __launch_bounds__(NT) void bs_gs(uint8_t *win, size_t nwin) {
    __shared__ uint4 img[2][G * R * NCOL];
    int buf = 0;
    for (XR xr = xr_make((nwin + G - 1) / G); xr.cur < xr.hi; xr.cur += xr.step, buf ^= 1) {
        const size_t w0 = xr.cur * G;
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        for (uint32_t s0 = 0; s0 < nb * H; s0 += NT) {
            const bool live = s0 + threadIdx.x < nb * H;
            const uint32_t s = live ? s0 + threadIdx.x : nb * H - 1;
            const uint32_t wl = s / H, u = s - wl * H;
            uint8_t *pa = win + (w0 + wl) * WB + u * 16u;
            uint8_t *pb = u + H < NCOL ? pa + H * 16u : pa;
            uint32_t acc[R][8];
            bs::sources<K, R, M, U, 0>(pa, pb, S, acc);
#pragma unroll
            for (int i = 0; i < R; i++) {
                bs::tr8(acc[i]);
                if (live) {
                    img[buf][(wl * R + i) * NCOL + u] = make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
                    if (u + H < NCOL)
                        img[buf][(wl * R + i) * NCOL + u + H] = make_uint4(acc[i][4], acc[i][5], acc[i][6], acc[i][7]);
                }
            }
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb * R * NCOL; q += NT) {
            const uint32_t wl = q / (R * NCOL), o = q - wl * (R * NCOL);
            st16(win + (w0 + wl) * WB + (size_t)K * S + o * 16u, img[buf][q]);
        }
    }
}


// ------------------------------------------- bit-sliced syndrome decode ---
// cfg3 decode shape: 4 of the 16 sources missing per window (miss[w]: rows,
// packed 4 x 8 bits), all 4 repairs present.  Syndromes of the received
// sources by the compile-time network (missing rows loaded as zeros), back
// to bytes, plus the repair rows; then the 4 x 4 solve S_m = sum_t D[u][t] s_t
// by the table multiply (D per window: host-computed here, sd/sc [w][t][u]).
__device__ __forceinline__ int mrow(uint32_t m, int u) { return (m >> (8 * u)) & 0xFF; }

template <int J, int... T>
__device__ __forceinline__ void dsrc_batch(const uint8_t *pa, const uint8_t *pb, uint32_t pm, uint32_t (&acc)[R][8],
                                           std::integer_sequence<int, T...>) {
    uint32_t x[sizeof...(T)][8];
    auto ld = [&](int t, uint32_t (&d)[8]) {
        uint4 va = make_uint4(0, 0, 0, 0), vb = va;
        if ((pm >> (J + t)) & 1) {
            va = ld16(pa + (J + t) * S);
            vb = ld16(pb + (J + t) * S);
        }
        d[0] = va.x; d[1] = va.y; d[2] = va.z; d[3] = va.w;
        d[4] = vb.x; d[5] = vb.y; d[6] = vb.z; d[7] = vb.w;
    };
    (ld(T, x[T]), ...);
    ((bs::tr8(x[T]), bs::source<K, R, M, J + T>(x[T], acc, std::make_integer_sequence<int, R * 8>{}),
      __builtin_amdgcn_sched_barrier(0)), ...);
}
template <int U, int J>
__device__ __forceinline__ void dsources(const uint8_t *pa, const uint8_t *pb, uint32_t pm, uint32_t (&acc)[R][8]) {
    if constexpr (J < K) {
        dsrc_batch<J>(pa, pb, pm, acc, std::make_integer_sequence<int, U>{});
        dsources<U, J + U>(pa, pb, pm, acc);
    }
}

template <int G, int NT, int U>
__global__ __launch_bounds__(NT) void bs_dec_gs(uint8_t *win, size_t nwin, const uint32_t *miss, const uint4 *sd,
                                                const uint32_t *sc) {
    __shared__ uint4 img[2][G * R * NCOL];
    __shared__ uint4 tab[2][G][R * R];
    __shared__ uint32_t tcs[2][G][R * R];
    __shared__ uint32_t sm[2][G];
    int buf = 0;
    for (XR xr = xr_make((nwin + G - 1) / G); xr.cur < xr.hi; xr.cur += xr.step, buf ^= 1) {
        const size_t w0 = xr.cur * G;
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        for (uint32_t i = threadIdx.x; i < nb * R * R; i += NT) {
            const uint32_t wl = i / (R * R), e = i - wl * R * R;
            tab[buf][wl][e] = sd[(w0 + wl) * R * R + e];
            tcs[buf][wl][e] = sc[(w0 + wl) * R * R + e];
        }
        if (threadIdx.x < nb) sm[buf][threadIdx.x] = miss[w0 + threadIdx.x];
        __syncthreads();
        for (uint32_t s0 = 0; s0 < nb * H; s0 += NT) {
            const bool live = s0 + threadIdx.x < nb * H;
            const uint32_t s = live ? s0 + threadIdx.x : nb * H - 1;
            const uint32_t wl = s / H, u = s - wl * H;
            const uint32_t m = sm[buf][wl];
            uint32_t pm = 0xFFFFu;
#pragma unroll
            for (int t = 0; t < R; t++) pm &= ~(1u << mrow(m, t));
            uint8_t *pa = win + (w0 + wl) * WB + u * 16u;
            uint8_t *pb = u + H < NCOL ? pa + H * 16u : pa;
            uint32_t acc[R][8];
            dsources<U, 0>(pa, pb, pm, acc);
            // syndromes in bytes, plus the repair rows
            uint4 ra[R], rb[R];
#pragma unroll
            for (int i = 0; i < R; i++) {
                ra[i] = ld16(pa + (size_t)(K + i) * S);
                rb[i] = ld16(pb + (size_t)(K + i) * S);
            }
#pragma unroll
            for (int i = 0; i < R; i++) {
                bs::tr8(acc[i]);
                acc[i][0] ^= ra[i].x; acc[i][1] ^= ra[i].y; acc[i][2] ^= ra[i].z; acc[i][3] ^= ra[i].w;
                acc[i][4] ^= rb[i].x; acc[i][5] ^= rb[i].y; acc[i][6] ^= rb[i].z; acc[i][7] ^= rb[i].w;
            }
            // solve, half by half: out[v] = sum_t D[v][t] * s_t (4 dwords each)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                uint32_t out[R][4];
#pragma unroll
                for (int v = 0; v < R; v++)
#pragma unroll
                    for (int d = 0; d < 4; d++) out[v][d] = 0;
#pragma unroll
                for (int t = 0; t < R; t += 2) {
                    const Split s0 = split(make_uint4(acc[t][4 * h], acc[t][4 * h + 1], acc[t][4 * h + 2], acc[t][4 * h + 3]));
                    const Split s1 = split(make_uint4(acc[t + 1][4 * h], acc[t + 1][4 * h + 1], acc[t + 1][4 * h + 2],
                                                      acc[t + 1][4 * h + 3]));
#pragma unroll
                    for (int v = 0; v < R; v++) {
                        const uint4 a0 = tab[buf][wl][t * R + v], a1 = tab[buf][wl][(t + 1) * R + v];
                        const uint32_t c0 = tcs[buf][wl][t * R + v], c1 = tcs[buf][wl][(t + 1) * R + v];
#pragma unroll
                        for (int d = 0; d < 4; d++) out[v][d] = gm2(out[v][d], s0, s1, d, a0, c0, a1, c1);
                    }
                }
                if (live && (h == 0 || u + H < NCOL)) {
#pragma unroll
                    for (int v = 0; v < R; v++)
                        img[buf][(wl * R + v) * NCOL + u + h * H] = make_uint4(out[v][0], out[v][1], out[v][2], out[v][3]);
                }
            }
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb * R * NCOL; q += NT) {
            const uint32_t wl = q / (R * NCOL), o = q - wl * (R * NCOL), v = o / NCOL, c = o - v * NCOL;
            st16(win + (w0 + wl) * WB + (size_t)mrow(sm[buf][wl], v) * S + c * 16u, img[buf][q]);
        }
    }
}

// table decode reference shape (the product's gf_decode_kernel without its
// plan): 12 sources + 4 repairs through per-window 16 x 4 tables (host-made),
// rowwise, direct stores
__global__ __launch_bounds__(256) void tab_dec(uint8_t *win, size_t nwin, const uint32_t *miss, const uint4 *fd,
                                               const uint32_t *fc) {
    const size_t total = nwin * NCOL;
    for (XR xr = xr_make((total + 255) / 256); xr.cur < xr.hi; xr.cur += xr.step) {
        const size_t s = xr.cur * 256 + threadIdx.x;
        if (s >= total) continue;
        const size_t w = s / NCOL, c = s - w * NCOL;
        const uint32_t m = miss[w];
        uint32_t pm = 0xFFFFFu;
#pragma unroll
        for (int t = 0; t < R; t++) pm &= ~(1u << mrow(m, t));
        uint8_t *b = win + w * WB + c * 16;
        uint4 acc[R] = {};
#pragma unroll 1
        for (int q = 0; q < K; q += 2) {
            const int r0 = __builtin_ctz(pm);
            pm &= pm - 1;
            const int r1 = __builtin_ctz(pm);
            pm &= pm - 1;
            const uint4 v0 = ld16(b + (size_t)r0 * S), v1 = ld16(b + (size_t)r1 * S);
            const Split s0 = split(v0), s1 = split(v1);
#pragma unroll
            for (int v = 0; v < R; v++) {
                const uint4 a0 = fd[(w * K + q) * R + v], a1 = fd[(w * K + q + 1) * R + v];
                const uint32_t c0 = fc[(w * K + q) * R + v], c1 = fc[(w * K + q + 1) * R + v];
                acc[v].x = gm2(acc[v].x, s0, s1, 0, a0, c0, a1, c1);
                acc[v].y = gm2(acc[v].y, s0, s1, 1, a0, c0, a1, c1);
                acc[v].z = gm2(acc[v].z, s0, s1, 2, a0, c0, a1, c1);
                acc[v].w = gm2(acc[v].w, s0, s1, 3, a0, c0, a1, c1);
            }
        }
#pragma unroll
        for (int v = 0; v < R; v++) st16(b + (size_t)mrow(m, v) * S, acc[v]);
    }
}

// software-pipelined sources: batch J + U's loads issued before batch J's
// transposes and XORs (16 more VGPRs, the next batch's latency hidden by this
// batch's work instead of by other waves)
template <int U, int J>
__device__ __forceinline__ void dload(const uint8_t *pa, const uint8_t *pb, uint32_t pm, uint32_t (&x)[U][8]) {
#pragma unroll
    for (int t = 0; t < U; t++) {
        uint4 va = make_uint4(0, 0, 0, 0), vb = va;
        if ((pm >> (J + t)) & 1) {
            va = ld16(pa + (J + t) * S);
            vb = ld16(pb + (J + t) * S);
        }
        x[t][0] = va.x; x[t][1] = va.y; x[t][2] = va.z; x[t][3] = va.w;
        x[t][4] = vb.x; x[t][5] = vb.y; x[t][6] = vb.z; x[t][7] = vb.w;
    }
}
template <int J, int... T>
__device__ __forceinline__ void dcompute(uint32_t (&x)[sizeof...(T)][8], uint32_t (&acc)[R][8], std::integer_sequence<int, T...>) {
    ((bs::tr8(x[T]), bs::source<K, R, M, J + T>(x[T], acc, std::make_integer_sequence<int, R * 8>{}),
      __builtin_amdgcn_sched_barrier(0)), ...);
}
template <int U, int J>
__device__ __forceinline__ void dsources_pf(const uint8_t *pa, const uint8_t *pb, uint32_t pm, uint32_t (&cur)[U][8],
                                            uint32_t (&acc)[R][8]) {
    if constexpr (J < K) {
        uint32_t nxt[U][8];
        if constexpr (J + U < K) dload<U, J + U>(pa, pb, pm, nxt);
        dcompute<J>(cur, acc, std::make_integer_sequence<int, U>{});
        if constexpr (J + U < K) dsources_pf<U, J + U>(pa, pb, pm, nxt, acc);
    }
}

template <int G, int NT, int U, bool PF, bool GS, int W = 1>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(W, 8))) void bs_dec2(uint8_t *win, size_t nwin, const uint32_t *miss, const uint4 *sd,
                                              const uint32_t *sc) {
    __shared__ uint4 img[GS ? 2 : 1][GS ? G * R * NCOL : 1];
    __shared__ uint4 tab[2][G][R * R];
    __shared__ uint32_t tcs[2][G][R * R];
    __shared__ uint32_t sm[2][G];
    int buf = 0;
    for (XR xr = xr_make((nwin + G - 1) / G); xr.cur < xr.hi; xr.cur += xr.step, buf ^= 1) {
        const size_t w0 = xr.cur * G;
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        for (uint32_t i = threadIdx.x; i < nb * R * R; i += NT) {
            const uint32_t wl = i / (R * R), e = i - wl * R * R;
            tab[buf][wl][e] = sd[(w0 + wl) * R * R + e];
            tcs[buf][wl][e] = sc[(w0 + wl) * R * R + e];
        }
        if (threadIdx.x < nb) sm[buf][threadIdx.x] = miss[w0 + threadIdx.x];
        __syncthreads();
        {
            const bool live = threadIdx.x < nb * H;
            const uint32_t s = live ? threadIdx.x : nb * H - 1;
            const uint32_t wl = s / H, u = s - wl * H;
            const uint32_t m = sm[buf][wl];
            uint32_t pm = 0xFFFFu;
#pragma unroll
            for (int t = 0; t < R; t++) pm &= ~(1u << mrow(m, t));
            uint8_t *pa = win + (w0 + wl) * WB + u * 16u;
            uint8_t *pb = u + H < NCOL ? pa + H * 16u : pa;
            uint32_t acc[R][8];
            if constexpr (PF) {
                uint32_t x0[U][8];
                dload<U, 0>(pa, pb, pm, x0);
                dsources_pf<U, 0>(pa, pb, pm, x0, acc);
            } else {
                dsources<U, 0>(pa, pb, pm, acc);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < R; i++) {
                const uint4 ra = ld16(pa + (size_t)(K + i) * S), rb = ld16(pb + (size_t)(K + i) * S);
                bs::tr8(acc[i]);
                acc[i][0] ^= ra.x; acc[i][1] ^= ra.y; acc[i][2] ^= ra.z; acc[i][3] ^= ra.w;
                acc[i][4] ^= rb.x; acc[i][5] ^= rb.y; acc[i][6] ^= rb.z; acc[i][7] ^= rb.w;
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                uint32_t out[R][4];
#pragma unroll
                for (int v = 0; v < R; v++)
#pragma unroll
                    for (int d = 0; d < 4; d++) out[v][d] = 0;
#pragma unroll
                for (int t = 0; t < R; t += 2) {
                    const Split s0 = split(make_uint4(acc[t][4 * h], acc[t][4 * h + 1], acc[t][4 * h + 2], acc[t][4 * h + 3]));
                    const Split s1 = split(make_uint4(acc[t + 1][4 * h], acc[t + 1][4 * h + 1], acc[t + 1][4 * h + 2],
                                                      acc[t + 1][4 * h + 3]));
#pragma unroll
                    for (int v = 0; v < R; v++) {
                        const uint4 a0 = tab[buf][wl][t * R + v], a1 = tab[buf][wl][(t + 1) * R + v];
                        const uint32_t c0 = tcs[buf][wl][t * R + v], c1 = tcs[buf][wl][(t + 1) * R + v];
#pragma unroll
                        for (int d = 0; d < 4; d++) out[v][d] = gm2(out[v][d], s0, s1, d, a0, c0, a1, c1);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (live && (h == 0 || u + H < NCOL)) {
#pragma unroll
                    for (int v = 0; v < R; v++) {
                        const uint4 o = make_uint4(out[v][0], out[v][1], out[v][2], out[v][3]);
                        if constexpr (GS) img[buf][(wl * R + v) * NCOL + u + h * H] = o;
                        else st16(win + (w0 + wl) * WB + (size_t)mrow(m, v) * S + (u + h * H) * 16u, o);
                    }
                }
            }
        }
        if constexpr (GS) {
            __syncthreads();
            for (uint32_t q = threadIdx.x; q < nb * R * NCOL; q += NT) {
                const uint32_t wl = q / (R * NCOL), o = q - wl * (R * NCOL), v = o / NCOL, c = o - v * NCOL;
                st16(win + (w0 + wl) * WB + (size_t)mrow(sm[buf][wl], v) * S + c * 16u, img[buf][q]);
            }
        }
    }
}

// three phases per step of G windows: (A) syndromes by the network, one
// 32-B unit per lane, written to LDS in bytes; (B) the 4 x 4 solve, one 16-B
// column per lane, in place in LDS; (C) the recovered rows stored front to back
template <int G, int U, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8))) void bs_dec3(
    uint8_t *win, size_t nwin, const uint32_t *miss, const uint4 *sd, const uint32_t *sc) {
    __shared__ uint4 img[G * R * NCOL];
    __shared__ uint4 tab[G][R * R];
    __shared__ uint32_t tcs[G][R * R];
    __shared__ uint32_t sm[G];
    for (XR xr = xr_make((nwin + G - 1) / G); xr.cur < xr.hi; xr.cur += xr.step) {
        const size_t w0 = xr.cur * G;
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        for (uint32_t i = threadIdx.x; i < nb * R * R; i += 256) {
            const uint32_t wl = i / (R * R), e = i - wl * R * R;
            tab[wl][e] = sd[(w0 + wl) * R * R + e];
            tcs[wl][e] = sc[(w0 + wl) * R * R + e];
        }
        if (threadIdx.x < nb) sm[threadIdx.x] = miss[w0 + threadIdx.x];
        __syncthreads();
        {   // (A)
            const bool live = threadIdx.x < nb * H;
            const uint32_t s = live ? threadIdx.x : nb * H - 1;
            const uint32_t wl = s / H, u = s - wl * H;
            const uint32_t m = sm[wl];
            uint32_t pm = 0xFFFFu;
#pragma unroll
            for (int t = 0; t < R; t++) pm &= ~(1u << mrow(m, t));
            uint8_t *pa = win + (w0 + wl) * WB + u * 16u;
            uint8_t *pb = u + H < NCOL ? pa + H * 16u : pa;
            uint32_t acc[R][8];
            uint32_t x0[U][8];
            dload<U, 0>(pa, pb, pm, x0);
            dsources_pf<U, 0>(pa, pb, pm, x0, acc);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < R; i++) {
                const uint4 ra = ld16(pa + (size_t)(K + i) * S), rb = ld16(pb + (size_t)(K + i) * S);
                bs::tr8(acc[i]);
                if (live) {
                    img[(wl * R + i) * NCOL + u] =
                        make_uint4(acc[i][0] ^ ra.x, acc[i][1] ^ ra.y, acc[i][2] ^ ra.z, acc[i][3] ^ ra.w);
                    if (u + H < NCOL)
                        img[(wl * R + i) * NCOL + u + H] =
                            make_uint4(acc[i][4] ^ rb.x, acc[i][5] ^ rb.y, acc[i][6] ^ rb.z, acc[i][7] ^ rb.w);
                }
            }
        }
        __syncthreads();
        // (B)
        for (uint32_t s = threadIdx.x; s < nb * NCOL; s += 256) {
            const uint32_t wl = s / NCOL, c = s - wl * NCOL;
            uint4 sg[R];
#pragma unroll
            for (int i = 0; i < R; i++) sg[i] = img[(wl * R + i) * NCOL + c];
            uint4 out[R];
#pragma unroll
            for (int v = 0; v < R; v++) out[v] = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int t = 0; t < R; t += 2) {
                const Split s0 = split(sg[t]), s1 = split(sg[t + 1]);
#pragma unroll
                for (int v = 0; v < R; v++) {
                    const uint4 a0 = tab[wl][t * R + v], a1 = tab[wl][(t + 1) * R + v];
                    const uint32_t c0 = tcs[wl][t * R + v], c1 = tcs[wl][(t + 1) * R + v];
                    out[v].x = gm2(out[v].x, s0, s1, 0, a0, c0, a1, c1);
                    out[v].y = gm2(out[v].y, s0, s1, 1, a0, c0, a1, c1);
                    out[v].z = gm2(out[v].z, s0, s1, 2, a0, c0, a1, c1);
                    out[v].w = gm2(out[v].w, s0, s1, 3, a0, c0, a1, c1);
                }
            }
#pragma unroll
            for (int v = 0; v < R; v++) img[(wl * R + v) * NCOL + c] = out[v];
        }
        __syncthreads();
        // (C)
        for (uint32_t q = threadIdx.x; q < nb * R * NCOL; q += 256) {
            const uint32_t wl = q / (R * NCOL), o = q - wl * (R * NCOL), v = o / NCOL, c = o - v * NCOL;
            st16(win + (w0 + wl) * WB + (size_t)mrow(sm[wl], v) * S + c * 16u, img[q]);
        }
        __syncthreads();
    }
}

}  // namespace fecgpu

using namespace fecgpu;

__global__ void cmp(const uint4 *a, const uint4 *b, size_t n, unsigned long long *bad) {
    unsigned long long nb = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const uint4 x = a[i], y = b[i];
        nb += (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
    }
    if (nb) atomicAdd(bad, nb);
}

template <class F>
static double time_ms(F launch, int reps = 7) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    std::vector<float> ts;
    for (int i = 0; i < reps; i++) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    CK(hipGetLastError());
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t nwin = 262144, bytes = nwin * WB;
    uint8_t *win, *ref;
    CK(hipMalloc(&win, bytes));
    CK(hipMalloc(&ref, bytes));
    {
        std::vector<uint32_t> h(1 << 24);
        uint32_t x = 0x12345678u;
        for (auto &v : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = x; }
        for (size_t off = 0; off < bytes; off += h.size() * 4)
            CK(hipMemcpy(win + off, h.data(), std::min(h.size() * 4, bytes - off), hipMemcpyHostToDevice));
    }
    constexpr ParityRows<K, R, 0> P{};
    std::vector<uint4> hab(K * R);
    std::vector<uint32_t> hc(K * R);
    for (int j = 0; j < K; j++)
        for (int i = 0; i < R; i++) {
            const CoefTab t = make_coef_tab(P.p[i][j]);
            hab[j * R + i] = make_uint4(t.a_lo, t.a_hi, t.b_lo, t.b_hi);
            hc[j * R + i] = t.c;
        }
    uint4 *gab;
    uint32_t *gc;
    unsigned long long *bad;
    CK(hipMalloc(&gab, K * R * 16));
    CK(hipMalloc(&gc, K * R * 4));
    CK(hipMalloc(&bad, 8));
    CK(hipMemcpy(gab, hab.data(), K * R * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(gc, hc.data(), K * R * 4, hipMemcpyHostToDevice));
    const double alg = (double)bytes;
    printf("{\"nwin\": %zu, \"alg_bytes\": %.0f, \"runs\": [\n", nwin, alg);
    auto report = [&](const char *name, int gm, double ms) {
        CK(hipMemset(bad, 0, 8));
        hipLaunchKernelGGL(cmp, 4096, 256, 0, 0, (const uint4 *)win, (const uint4 *)ref, bytes / 16, bad);
        unsigned long long hb = 0;
        CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        printf("  {\"kernel\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"TBps\": %.3f, \"mismatch_chunks\": %llu},\n",
               name, gm, ms, alg / (ms * 1e-3) / 1e12, hb);
        fflush(stdout);
    };
    hipLaunchKernelGGL(tab_flat, cus * 2, 256, 0, 0, win, nwin, gab, gc);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref, win, bytes, hipMemcpyDeviceToDevice));
    for (int round = 0; round < 1; round++) {
        for (int gm : {2, 4}) {
            const double ms = time_ms([&] { hipLaunchKernelGGL(tab_flat, cus * gm, 256, 0, 0, win, nwin, gab, gc); });
            report("tab_flat", gm, ms);
        }
        for (int gm : {2}) {
            double ms = time_ms([&] { hipLaunchKernelGGL((bs_flat<2>), cus * gm, 256, 0, 0, win, nwin); });
            report("bs_flat_U2", gm, ms);
        }
        for (int gm : {1, 2, 3, 4}) {
            double ms = time_ms([&] { hipLaunchKernelGGL((bs_gs<6, 256, 2>), cus * gm, 256, 0, 0, win, nwin); });
            report("bs_gs_G6_256", gm, ms);
        }
        for (int gm : {2, 4, 6, 8}) {
            double ms = time_ms([&] { hipLaunchKernelGGL((bs_gs<3, 128, 2>), cus * gm, 128, 0, 0, win, nwin); });
            report("bs_gs_G3_128", gm, ms);
        }
        for (int gm : {1, 2, 3}) {
            double ms = time_ms([&] { hipLaunchKernelGGL((bs_gs<10, 384, 2>), cus * gm, 384, 0, 0, win, nwin); });
            report("bs_gs_G10_384", gm, ms);
        }
    }

    // ---- decode: 4 missing sources per window, host-made plans
    {
        constexpr GfTables T = make_gf_tables();
        auto mul = [&](uint8_t a, uint8_t b) -> uint8_t { return (a && b) ? T.exp[T.log[a] + T.log[b]] : 0; };
        auto inv = [&](uint8_t a) -> uint8_t { return T.exp[255 - T.log[a]]; };
        std::vector<uint32_t> hm(nwin);
        std::vector<uint4> hsd(nwin * R * R), hfd(nwin * K * R);
        std::vector<uint32_t> hsc(nwin * R * R), hfc(nwin * K * R);
        uint32_t x = 0x9e3779b9u;
        for (size_t w = 0; w < nwin; w++) {
            uint32_t used = 0;
            int n = 0;
            while (n < 4) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; const int r = x & 15; if (!((used >> r) & 1)) { used |= 1u << r; n++; } }
            int mv[4], u = 0;
            uint32_t mm = 0;
            for (int r = 0; r < 16; r++) if ((used >> r) & 1) { mm |= (uint32_t)r << (8 * u); mv[u++] = r; }
            hm[w] = mm;
            // A[t][u] = P[t][m_u]; Ainv by Gauss-Jordan
            uint8_t a[4][8] = {};
            for (int t = 0; t < 4; t++) { for (int v = 0; v < 4; v++) a[t][v] = P.p[t][mv[v]]; a[t][4 + t] = 1; }
            for (int c = 0; c < 4; c++) {
                int pv = c; while (!a[pv][c]) pv++;
                for (int j = 0; j < 8; j++) std::swap(a[pv][j], a[c][j]);
                const uint8_t iv = inv(a[c][c]);
                for (int j = 0; j < 8; j++) a[c][j] = mul(a[c][j], iv);
                for (int i = 0; i < 4; i++) if (i != c && a[i][c]) { const uint8_t f = a[i][c]; for (int j = 0; j < 8; j++) a[i][j] ^= mul(f, a[c][j]); }
            }
            // D[v][t] = Ainv[v][t] (rows of Ainv: unknown v; columns: syndrome t)
            for (int t = 0; t < 4; t++) for (int v = 0; v < 4; v++) {
                const CoefTab ct = make_coef_tab(a[v][4 + t]);
                hsd[(w * R + t) * R + v] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
                hsc[(w * R + t) * R + v] = ct.c;
            }
            // full decode matrix over the 16 inputs (received sources ascending, then repairs 0..3)
            int q = 0;
            for (int j = 0; j < 16 + 4; j++) {
                if (j < 16 && ((used >> j) & 1)) continue;
                for (int v = 0; v < 4; v++) {
                    uint8_t d = 0;
                    if (j < 16) { for (int t = 0; t < 4; t++) d ^= mul(a[v][4 + t], P.p[t][j]); }
                    else d = a[v][4 + (j - 16)];
                    const CoefTab ct = make_coef_tab(d);
                    hfd[(w * K + q) * R + v] = make_uint4(ct.a_lo, ct.a_hi, ct.b_lo, ct.b_hi);
                    hfc[(w * K + q) * R + v] = ct.c;
                }
                q++;
            }
        }
        uint32_t *dm, *dsc, *dfc;
        uint4 *dsd, *dfd;
        CK(hipMalloc(&dm, nwin * 4));
        CK(hipMalloc(&dsd, hsd.size() * 16));
        CK(hipMalloc(&dsc, hsc.size() * 4));
        CK(hipMalloc(&dfd, hfd.size() * 16));
        CK(hipMalloc(&dfc, hfc.size() * 4));
        CK(hipMemcpy(dm, hm.data(), nwin * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dsd, hsd.data(), hsd.size() * 16, hipMemcpyHostToDevice));
        CK(hipMemcpy(dsc, hsc.data(), hsc.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dfd, hfd.data(), hfd.size() * 16, hipMemcpyHostToDevice));
        CK(hipMemcpy(dfc, hfc.data(), hfc.size() * 4, hipMemcpyHostToDevice));
        // win holds encoded windows (ref); each decode rewrites the missing rows
        // with the originals, so the buffer must stay equal to ref
        CK(hipMemcpy(win, ref, bytes, hipMemcpyDeviceToDevice));
        for (int round = 0; round < 1; round++) {
            for (int gm : {4}) {
                const double ms = time_ms([&] { hipLaunchKernelGGL(tab_dec, cus * gm, 256, 0, 0, win, nwin, dm, dfd, dfc); });
                report("tab_dec(host plans)", gm, ms);
            }
#define DEC2(G, NT, U, PF, GS, GMS)                                                                          \
            for (int gm : GMS) {                                                                             \
                const double ms = time_ms([&] { hipLaunchKernelGGL((bs_dec2<G, NT, U, PF, GS>), cus * gm, NT, 0, 0, win, nwin, dm, dsd, dsc); }); \
                report("bs_dec2_G" #G "_" #NT "_U" #U "_pf" #PF "_gs" #GS, gm, ms);                           \
            }
            DEC2(6, 256, 2, true, false, (std::initializer_list<int>{2}))
#define DEC4(G, U, W, GMS)                                                                                   \
            for (int gm : GMS) {                                                                             \
                const double ms = time_ms([&] { hipLaunchKernelGGL((bs_dec3<G, U, W>), cus * gm, 256, 0, 0, win, nwin, dm, dsd, dsc); }); \
                report("bs_dec3_G" #G "_U" #U "_w" #W, gm, ms);                                             \
            }
            DEC4(6, 2, 1, (std::initializer_list<int>{2, 3, 4}))
            DEC4(6, 2, 4, (std::initializer_list<int>{4}))
            DEC4(6, 1, 4, (std::initializer_list<int>{4}))
            DEC4(3, 2, 4, (std::initializer_list<int>{4, 6}))
        }
    }
    printf("  {\"end\": true}\n]}\n");
    return 0;
}
