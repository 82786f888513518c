// win_probe.hip — HBM access patterns for the cfg3 window layout (k16 r4,
// 1200-B rows, 262,144 windows = 6.29 GB): which load/store pattern of the
// same bytes reaches the highest rate.  XOR-only combine (memory-side
// ceilings); the GF combine variants live in gf4_probe.hip.
//   rowwise  lane = (window, 16-B column), walks the 16 source rows (the
//            table kernels' pattern), U rows per load batch, 4 rows stored
//   flat     lane = (window, 16-B chunk c of the 4,800-B repair region),
//            reads chunks c, c + 300, c + 600, c + 900 of the sources
//   lds<G>   workgroup stages G windows' 19,200 source bytes in LDS with
//            global_load_lds_dwordx4 (contiguous 1 KiB per wave-instruction),
//            lanes then combine columns out of LDS and store rows
//   streams  16 separate input streams, 4 output streams (no windows)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/win_probe scripts/win_probe.hip
// Tuning aid, not part of the product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 *gptr_c;
typedef __attribute__((address_space(1))) u32x4 *gptr;

constexpr int K = 16, R = 4;

__device__ __forceinline__ u32x4 ld(const uint8_t *p) { return *(gptr_c)(p); }
__device__ __forceinline__ void st(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (gptr)(p)); }

// rowwise: slot s -> (w, col); persistent grid-stride
template <int U, int ST = 1>
__global__ __launch_bounds__(256) void rowwise(uint8_t *win, size_t nwin, uint32_t S, uint32_t stride) {
    const uint32_t ncol = S / 16;
    const size_t total = nwin * ncol, gt = (size_t)gridDim.x * 256;
    const size_t wb = (size_t)(K + R) * stride;
    for (size_t s = (size_t)blockIdx.x * 256 + threadIdx.x; s < total; s += gt) {
        const size_t w = s / ncol, c = s - w * ncol;
        uint8_t *b = win + w * wb + c * 16;
        u32x4 acc[R] = {};
        for (int j0 = 0; j0 < K; j0 += U) {
            u32x4 v[U];
#pragma unroll
            for (int t = 0; t < U; t++) v[t] = ld(b + (size_t)(j0 + t) * stride);
#pragma unroll
            for (int t = 0; t < U; t++) acc[(j0 + t) % R] ^= v[t];
        }
        if constexpr (ST == 1) {
#pragma unroll
            for (int o = 0; o < R; o++) st(b + (size_t)(K + o) * stride, acc[o]);
        } else if constexpr (ST == 2) {
#pragma unroll
            for (int o = 0; o < R; o++) *(gptr)(b + (size_t)(K + o) * stride) = acc[o];
        } else {
            u32x4 x = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
            if ((x.x ^ x.y ^ x.z ^ x.w) == 0x9e3779b9u) *(gptr)(b) = x;  // keep the loads live
        }
    }
}

// flat: unit = (w, chunk c of the repair region)
template <int ST = 1>
__global__ __launch_bounds__(256) void flat(uint8_t *win, size_t nwin, uint32_t S) {
    const uint32_t nch = R * S / 16;  // 300
    const size_t total = nwin * nch, gt = (size_t)gridDim.x * 256;
    const size_t wb = (size_t)(K + R) * S;
    for (size_t s = (size_t)blockIdx.x * 256 + threadIdx.x; s < total; s += gt) {
        const size_t w = s / nch, c = s - w * nch;
        uint8_t *b = win + w * wb + c * 16;
        u32x4 v[K / R];
#pragma unroll
        for (int t = 0; t < K / R; t++) v[t] = ld(b + (size_t)t * R * S);
        u32x4 x = v[0];
#pragma unroll
        for (int t = 1; t < K / R; t++) x ^= v[t];
        if constexpr (ST == 1) st(b + (size_t)K * S, x);
        else if ((x.x ^ x.y ^ x.z ^ x.w) == 0x9e3779b9u) *(gptr)(b) = x;
    }
}

// lds<G>: G windows per step staged by global_load_lds_dwordx4; one LDS buffer
// (occupancy gives the overlap)
template <int G>
__global__ __launch_bounds__(256) void ldsw(uint8_t *win, size_t nwin, uint32_t S) {
    extern __shared__ u32x4 lds[];  // G * K * S bytes
    const uint32_t ncol = S / 16;
    const uint32_t wsrc = K * S;                // 19,200 source bytes per window
    const size_t wb = (size_t)(K + R) * S;
    const uint32_t nchunk = G * wsrc / 16;      // 16-B chunks staged per step
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (size_t w0 = (size_t)blockIdx.x * G; w0 < nwin; w0 += (size_t)gridDim.x * G) {
        const int nb = (int)std::min((size_t)G, nwin - w0);
        // stage: chunk q = window q / (wsrc/16), offset inside its window
        for (uint32_t q0 = wv * 64; q0 < nchunk; q0 += 256) {
            const uint32_t q = q0 + lane;
            const uint32_t wl = q / (wsrc / 16), o = q - wl * (wsrc / 16);
            const uint8_t *src = win + (w0 + std::min<uint32_t>(wl, nb - 1)) * wb + o * 16;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(lds + q0), 16, 0, 0);
        }
        __syncthreads();
        for (uint32_t s = threadIdx.x; s < (uint32_t)nb * ncol; s += 256) {
            const uint32_t wl = s / ncol, c = s - wl * ncol;
            const u32x4 *b = lds + wl * (wsrc / 16) + c;
            u32x4 acc[R] = {};
#pragma unroll
            for (int j = 0; j < K; j++) acc[j % R] ^= b[j * ncol];
            uint8_t *o = win + (w0 + wl) * wb + (size_t)K * S + c * 16;
#pragma unroll
            for (int i = 0; i < R; i++) st(o + (size_t)i * S, acc[i]);
        }
        __syncthreads();
    }
}


// rowst<G>: rowwise loads, repairs gathered in LDS and stored contiguously
// (each window's 4,800-B repair region in 16-B chunks, consecutive lanes =
// consecutive chunks).  Workgroup = G whole windows, 75 G lanes rounded up to
// whole waves.
template <int G>
__global__ void rowst(uint8_t *win, size_t nwin, uint32_t S) {
    const uint32_t ncol = S / 16;
    const size_t wb = (size_t)(K + R) * S;
    __shared__ u32x4 out[G * R * 80];
    const uint32_t nt = blockDim.x;
    for (size_t w0 = (size_t)blockIdx.x * G; w0 < nwin; w0 += (size_t)gridDim.x * G) {
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        const uint32_t s = threadIdx.x;
        if (s < nb * ncol) {
            const uint32_t wl = s / ncol, c = s - wl * ncol;
            const uint8_t *b = win + (w0 + wl) * wb + c * 16;
            u32x4 acc[R] = {};
            for (int j0 = 0; j0 < K; j0 += 2) {
                const u32x4 v0 = ld(b + (size_t)j0 * S), v1 = ld(b + (size_t)(j0 + 1) * S);
                acc[j0 % R] ^= v0;
                acc[(j0 + 1) % R] ^= v1;
            }
#pragma unroll
            for (int o = 0; o < R; o++) out[(wl * R + o) * ncol + c] = acc[o];
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb * R * ncol; q += nt) {
            const uint32_t wl = q / (R * ncol), o = q - wl * (R * ncol);
            st(win + (w0 + wl) * wb + (size_t)K * S + o * 16, out[q]);
        }
        __syncthreads();
    }
}

// Decode shapes (cfg3: 4 of the 16 sources missing per window, all 4 repairs
// read): miss[w] = the 4 missing rows (ascending, packed 4 x 8 bits).
//   drow   lane = (w, c): 12 sources + 4 repairs loaded, 4 rows stored (the
//          table decode's pattern)
//   drowst G windows per workgroup, recovered rows gathered in LDS, each row
//          stored contiguously (EXT: widened to whole 128-B lines with the
//          neighbouring rows' bytes, kept in LDS by the lanes that loaded them)
__device__ __forceinline__ int miss_row(uint32_t m, int u) { return (m >> (8 * u)) & 0xFF; }

__device__ __forceinline__ void in_rows(uint32_t m, int (&rows)[K]) {
    uint32_t pm = 0xFFFFFu;
#pragma unroll
    for (int u = 0; u < 4; u++) pm &= ~(1u << miss_row(m, u));
#pragma unroll
    for (int j = 0; j < K; j++) {
        rows[j] = __builtin_ctz(pm);
        pm &= pm - 1;
    }
}

__global__ __launch_bounds__(256) void drow(uint8_t *win, size_t nwin, const uint32_t *miss) {
    constexpr uint32_t S = 1200, ncol = 75;
    const size_t total = nwin * ncol, gt = (size_t)gridDim.x * 256;
    const size_t wb = (size_t)(K + R) * S;
    for (size_t s = (size_t)blockIdx.x * 256 + threadIdx.x; s < total; s += gt) {
        const size_t w = s / ncol, c = s - w * ncol;
        const uint32_t m = miss[w];
        uint8_t *b = win + w * wb + c * 16;
        int rows[K];
        in_rows(m, rows);
        u32x4 acc[R] = {};
#pragma unroll
        for (int j0 = 0; j0 < K; j0 += 8) {
            u32x4 v[8];
#pragma unroll
            for (int t = 0; t < 8; t++) v[t] = ld(b + (size_t)rows[j0 + t] * S);
#pragma unroll
            for (int t = 0; t < 8; t++) acc[t % R] ^= v[t];
        }
#pragma unroll
        for (int o = 0; o < R; o++) st(b + (size_t)miss_row(m, o) * S, acc[o]);
    }
}

template <int G, bool EXT>
__global__ void drowst(uint8_t *win, size_t nwin, const uint32_t *miss) {
    constexpr uint32_t S = 1200, ncol = 75, NE = 7;  // edge columns kept per side
    const size_t wb = (size_t)(K + R) * S;
    __shared__ u32x4 out[G * R * ncol];
    __shared__ u32x4 edge[EXT ? G * (K + R) * 2 * NE : 1];  // [wl][row][side][col]
    __shared__ uint32_t s_miss[G];
    const uint32_t nt = blockDim.x;
    for (size_t w0 = (size_t)blockIdx.x * G; w0 < nwin; w0 += (size_t)gridDim.x * G) {
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        if (threadIdx.x < nb) s_miss[threadIdx.x] = miss[w0 + threadIdx.x];
        __syncthreads();
        const uint32_t s = threadIdx.x;
        if (s < nb * ncol) {
            const uint32_t wl = s / ncol, c = s - wl * ncol;
            const uint32_t m = s_miss[wl];
            const uint8_t *b = win + (w0 + wl) * wb + c * 16;
            const bool eg = EXT && (c < NE || c >= ncol - NE);
            const uint32_t ei = c < NE ? c : NE + (c - (ncol - NE));
            int rows[K];
            in_rows(m, rows);
            u32x4 acc[R] = {};
#pragma unroll
            for (int j0 = 0; j0 < K; j0 += 8) {
                u32x4 v[8];
#pragma unroll
                for (int t = 0; t < 8; t++) v[t] = ld(b + (size_t)rows[j0 + t] * S);
#pragma unroll
                for (int t = 0; t < 8; t++) {
                    acc[t % R] ^= v[t];
                    if (eg) edge[(wl * (K + R) + rows[j0 + t]) * 2 * NE + ei] = v[t];
                }
            }
#pragma unroll
            for (int o = 0; o < R; o++) {
                out[(wl * R + o) * ncol + c] = acc[o];
                if (eg) edge[(wl * (K + R) + miss_row(m, o)) * 2 * NE + ei] = acc[o];
            }
        }
        __syncthreads();
        if (!EXT) {
            for (uint32_t q = threadIdx.x; q < nb * R * ncol; q += nt) {
                const uint32_t wl = q / (R * ncol), o = q - wl * (R * ncol), uo = o / ncol, c = o - uo * ncol;
                st(win + (w0 + wl) * wb + (size_t)miss_row(s_miss[wl], uo) * S + c * 16, out[q]);
            }
        } else {
            // each recovered row widened to whole lines: 75 + 2 * 7 chunks at most per row
            constexpr uint32_t PER = ncol + 2 * NE;
            for (uint32_t q = threadIdx.x; q < nb * R * PER; q += nt) {
                const uint32_t wl = q / (R * PER), o = q - wl * (R * PER), uo = o / PER, t = o - uo * PER;
                const size_t w = w0 + wl;
                const int row = miss_row(s_miss[wl], uo);
                const uint64_t off0 = w * wb + (uint64_t)row * S;  // row start (win is 256-B aligned)
                const uint32_t pre = (uint32_t)(off0 & 127) / 16;
                const uint32_t endb = (uint32_t)((off0 + S) & 127);
                const uint32_t post = endb ? (128 - endb) / 16 : 0;
                const int rel = (int)t - (int)pre;
                if (t >= pre + ncol + post) continue;
                u32x4 v;
                if (rel >= 0 && rel < (int)ncol) {
                    v = out[(wl * R + uo) * ncol + rel];
                } else {
                    const int nrow = rel < 0 ? row - 1 : row + 1;
                    if (nrow < 0 || nrow >= K + R) continue;  // another window's bytes: leave the line partial
                    const int c = rel < 0 ? (int)ncol + rel : rel - (int)ncol;
                    const uint32_t ei = c < (int)NE ? (uint32_t)c : NE + (uint32_t)(c - (int)(ncol - NE));
                    v = edge[(wl * (K + R) + nrow) * 2 * NE + ei];
                }
                st(win + off0 + (int64_t)rel * 16, v);
            }
        }
        __syncthreads();
    }
}

// XCD-aware variants (the product kernels' mapping: units cut into 8
// contiguous regions, region b % 8 walked by workgroups b / 8, so neighbouring
// units share an L2)
struct XR { size_t cur, hi, step; };
__device__ __forceinline__ XR xr_make(size_t nunits) {
    const uint32_t nx = 8, bx = blockIdx.x % nx, bi = blockIdx.x / nx, nbx = gridDim.x / nx;
    const size_t lo = nunits * bx / nx, hi = nunits * (bx + 1) / nx;
    return {lo + bi, hi, nbx};
}
template <int U>
__global__ __launch_bounds__(256) void rowwise_x(uint8_t *win, size_t nwin, uint32_t S) {
    const uint32_t ncol = S / 16;
    const size_t total = nwin * ncol;
    const size_t wb = (size_t)(K + R) * S;
    for (XR xr = xr_make((total + 255) / 256); xr.cur < xr.hi; xr.cur += xr.step) {
        const size_t s = xr.cur * 256 + threadIdx.x;
        if (s >= total) continue;
        const size_t w = s / ncol, c = s - w * ncol;
        uint8_t *b = win + w * wb + c * 16;
        u32x4 acc[R] = {};
        for (int j0 = 0; j0 < K; j0 += U) {
            u32x4 v[U];
#pragma unroll
            for (int t = 0; t < U; t++) v[t] = ld(b + (size_t)(j0 + t) * S);
#pragma unroll
            for (int t = 0; t < U; t++) acc[(j0 + t) % R] ^= v[t];
        }
#pragma unroll
        for (int o = 0; o < R; o++) st(b + (size_t)(K + o) * S, acc[o]);
    }
}
template <int G>
__global__ void rowst_x(uint8_t *win, size_t nwin, uint32_t S) {
    const uint32_t ncol = S / 16;
    const size_t wb = (size_t)(K + R) * S;
    __shared__ u32x4 out[2][G * R * 80];
    const uint32_t nt = blockDim.x;
    int buf = 0;
    for (XR xr = xr_make((nwin + G - 1) / G); xr.cur < xr.hi; xr.cur += xr.step, buf ^= 1) {
        const size_t w0 = xr.cur * G;
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        const uint32_t s = threadIdx.x;
        if (s < nb * ncol) {
            const uint32_t wl = s / ncol, c = s - wl * ncol;
            const uint8_t *b = win + (w0 + wl) * wb + c * 16;
            u32x4 acc[R] = {};
            for (int j0 = 0; j0 < K; j0 += 2) {
                const u32x4 v0 = ld(b + (size_t)j0 * S), v1 = ld(b + (size_t)(j0 + 1) * S);
                acc[j0 % R] ^= v0;
                acc[(j0 + 1) % R] ^= v1;
            }
#pragma unroll
            for (int o = 0; o < R; o++) out[buf][(wl * R + o) * ncol + c] = acc[o];
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb * R * ncol; q += nt) {
            const uint32_t wl = q / (R * ncol), o = q - wl * (R * ncol);
            st(win + (w0 + wl) * wb + (size_t)K * S + o * 16, out[buf][q]);
        }
    }
}
__global__ __launch_bounds__(256) void drow_x(uint8_t *win, size_t nwin, const uint32_t *miss) {
    constexpr uint32_t S = 1200, ncol = 75;
    const size_t total = nwin * ncol;
    const size_t wb = (size_t)(K + R) * S;
    for (XR xr = xr_make((total + 255) / 256); xr.cur < xr.hi; xr.cur += xr.step) {
        const size_t s = xr.cur * 256 + threadIdx.x;
        if (s >= total) continue;
        const size_t w = s / ncol, c = s - w * ncol;
        const uint32_t m = miss[w];
        uint8_t *b = win + w * wb + c * 16;
        int rows[K];
        in_rows(m, rows);
        u32x4 acc[R] = {};
#pragma unroll
        for (int j0 = 0; j0 < K; j0 += 8) {
            u32x4 v[8];
#pragma unroll
            for (int t = 0; t < 8; t++) v[t] = ld(b + (size_t)rows[j0 + t] * S);
#pragma unroll
            for (int t = 0; t < 8; t++) acc[t % R] ^= v[t];
        }
#pragma unroll
        for (int o = 0; o < R; o++) st(b + (size_t)miss_row(m, o) * S, acc[o]);
    }
}

// rowsync_x: rowwise_x with a workgroup barrier before the stores (the waves
// store their pieces of the same rows at the same time; no LDS)
__global__ __launch_bounds__(256) void rowsync_x(uint8_t *win, size_t nwin, uint32_t S) {
    const uint32_t ncol = S / 16;
    const size_t total = nwin * ncol;
    const size_t wb = (size_t)(K + R) * S;
    for (XR xr = xr_make((total + 255) / 256); xr.cur < xr.hi; xr.cur += xr.step) {
        const size_t s = xr.cur * 256 + threadIdx.x;
        const bool live = s < total;
        const size_t ss = live ? s : total - 1;
        const size_t w = ss / ncol, c = ss - w * ncol;
        uint8_t *b = win + w * wb + c * 16;
        u32x4 acc[R] = {};
        for (int j0 = 0; j0 < K; j0 += 2) {
            const u32x4 v0 = ld(b + (size_t)j0 * S), v1 = ld(b + (size_t)(j0 + 1) * S);
            acc[j0 % R] ^= v0;
            acc[(j0 + 1) % R] ^= v1;
        }
        __syncthreads();
        if (live) {
#pragma unroll
            for (int o = 0; o < R; o++) st(b + (size_t)(K + o) * S, acc[o]);
        }
    }
}
// rowpass_x: per 256-slot pass, outputs to LDS, barrier, stored slot-major
// per output row (thread t stores slot (q % 256) of row q / 256)
__global__ __launch_bounds__(256) void rowpass_x(uint8_t *win, size_t nwin, uint32_t S) {
    const uint32_t ncol = S / 16;
    const size_t total = nwin * ncol;
    const size_t wb = (size_t)(K + R) * S;
    __shared__ u32x4 img[2][R * 256];
    int buf = 0;
    for (XR xr = xr_make((total + 255) / 256); xr.cur < xr.hi; xr.cur += xr.step, buf ^= 1) {
        const size_t s = xr.cur * 256 + threadIdx.x;
        const bool live = s < total;
        const size_t ss = live ? s : total - 1;
        const size_t w = ss / ncol, c = ss - w * ncol;
        uint8_t *b = win + w * wb + c * 16;
        u32x4 acc[R] = {};
        for (int j0 = 0; j0 < K; j0 += 2) {
            const u32x4 v0 = ld(b + (size_t)j0 * S), v1 = ld(b + (size_t)(j0 + 1) * S);
            acc[j0 % R] ^= v0;
            acc[(j0 + 1) % R] ^= v1;
        }
#pragma unroll
        for (int o = 0; o < R; o++) img[buf][o * 256 + threadIdx.x] = acc[o];
        __syncthreads();
        // window-row order over the pass: chunk q -> (window piece, row, col)
        const size_t sp0 = xr.cur * 256, sp1 = std::min(sp0 + 256, total);
        const size_t wa = sp0 / ncol;
        const uint32_t np = (uint32_t)(sp1 - sp0);
        for (uint32_t q = threadIdx.x; q < R * np; q += 256) {
            // pieces: window wa + i covers pass slots [lo_i, hi_i)
            uint32_t acc0 = 0, i = 0, lo = 0, len = 0;
            for (;; i++) {
                const size_t wlo = std::max(sp0, (wa + i) * ncol), whi = std::min(sp1, (wa + i + 1) * ncol);
                len = (uint32_t)(whi - wlo);
                lo = (uint32_t)(wlo - sp0);
                if (q < acc0 + R * len) break;
                acc0 += R * len;
            }
            const uint32_t rem = q - acc0, o = rem / len, t = rem - o * len;
            const size_t sl = sp0 + lo + t, w2 = sl / ncol, c2 = sl - w2 * ncol;
            st(win + w2 * wb + (size_t)(K + o) * S + c2 * 16, img[buf][o * 256 + lo + t]);
        }
    }
}

__global__ __launch_bounds__(256) void streams(const uint8_t *in, uint8_t *out, size_t n) {
    const size_t gt = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += gt) {
        u32x4 v[K];
#pragma unroll
        for (int t = 0; t < K; t++) v[t] = ld(in + (i + t * n) * 16);
#pragma unroll
        for (int o = 0; o < R; o++) {
            u32x4 x = {0, 0, 0, 0};
#pragma unroll
            for (int t = o; t < K; t += R) x ^= v[t];
            st(out + (i + o * n) * 16, x);
        }
    }
}

template <class F>
static double time_ms(F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 2; i++) launch();
    std::vector<float> ts;
    for (int i = 0; i < 7; i++) {
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

static int g_cus = 256;

template <class F>
static void sweep(const char *name, double bytes, F launch, std::initializer_list<int> gms) {
    printf("  {\"shape\": \"%s\", \"grids\": {", name);
    double best = 0;
    bool first = true;
    for (int gm : gms) {
        const double ms = time_ms([&] { launch(g_cus * gm); });
        const double tbs = bytes / (ms * 1e-3) / 1e12;
        printf("%s\"%d\": [%.4f, %.3f]", first ? "" : ", ", gm, ms, tbs);
        first = false;
        best = std::max(best, tbs);
    }
    printf("}, \"best_TBps\": %.3f},\n", best);
    fflush(stdout);
}

int main() {
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t nwin = 262144;
    const uint32_t S = 1200;
    const size_t bytes1200 = nwin * (K + R) * S;
    const size_t bytes1280 = nwin * (K + R) * 1280;
    uint8_t *win;
    CK(hipMalloc(&win, bytes1280));
    // random-ish contents (DVFS reads high on constant data)
    {
        std::vector<uint32_t> h(1 << 24);
        uint32_t x = 0x12345678u;
        for (auto &v : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = x; }
        for (size_t off = 0; off < bytes1280; off += h.size() * 4)
            CK(hipMemcpy(win + off, h.data(), std::min(h.size() * 4, bytes1280 - off), hipMemcpyHostToDevice));
    }
    const double alg = (double)bytes1200;
    printf("{\"cus\": %d, \"nwin\": %zu, \"alg_bytes\": %.0f, \"unit\": \"[ms, TB/s of algorithmic bytes]\", \"runs\": [\n",
           g_cus, nwin, alg);
    auto gms = {1, 2, 4, 8};
    // 4 distinct missing rows of 0..15 per window, ascending
    uint32_t *miss;
    {
        std::vector<uint32_t> h(nwin);
        uint32_t x = 0x9e3779b9u;
        for (size_t w = 0; w < nwin; w++) {
            uint32_t used = 0;
            int n = 0;
            while (n < 4) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; const int r = x & 15; if (!((used >> r) & 1)) { used |= 1u << r; n++; } }
            uint32_t m = 0; int u = 0;
            for (int r = 0; r < 16; r++) if ((used >> r) & 1) m |= (uint32_t)r << (8 * u++);
            h[w] = m;
        }
        CK(hipMalloc(&miss, nwin * 4));
        CK(hipMemcpy(miss, h.data(), nwin * 4, hipMemcpyHostToDevice));
    }
    sweep("rowwise_x_U2(encode)", alg, [&](int g) { hipLaunchKernelGGL((rowwise_x<2>), g, 256, 0, 0, win, nwin, S); }, {1, 2, 4});
    sweep("rowsync_x(encode)", alg, [&](int g) { hipLaunchKernelGGL(rowsync_x, g, 256, 0, 0, win, nwin, S); }, {1, 2, 4});
    sweep("rowpass_x(encode)", alg, [&](int g) { hipLaunchKernelGGL(rowpass_x, g, 256, 0, 0, win, nwin, S); }, {1, 2, 4});
    sweep("rowst_x_G3_256(encode)", alg, [&](int g) { hipLaunchKernelGGL((rowst_x<3>), g, 256, 0, 0, win, nwin, S); }, {1, 2, 4});
    printf("  {\"end\": true}\n]}\n");
    CK(hipFree(win));
    return 0;
}
