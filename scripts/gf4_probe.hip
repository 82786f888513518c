// gf4_probe.hip — cfg3 GF(2^8) k16 r4 encode (262,144 windows of 1200-B rows)
// with the table multiply, in the access patterns of win_probe.hip:
//   rowwise  the product kernel's shape: lane = (window, 16-B column), rows
//            loaded from HBM two at a time (PAIR folding), rows stored
//   staged   workgroup copies G windows' source rows into LDS with
//            global_load_lds_dwordx4 (each wave-instruction 1 KiB of contiguous
//            window bytes), then combines columns out of LDS; repairs stored per
//            row (ST 0) or gathered in LDS and stored contiguously (ST 1)
// Outputs are compared with rowwise's.  Tuning aid, not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -I quic-fec-eps_amd/csrc -o scripts/gf4_probe scripts/gf4_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "fec_spec.h"

using namespace fecgpu;

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
constexpr uint32_t S = 1200, NCOL = S / 16, WB = (K + R) * S, WSRC = K * S, WCH = WSRC / 16;

__device__ __forceinline__ u32x4 ldg(const uint8_t *p) { return *(gptr_c)(p); }
__device__ __forceinline__ void stg(uint8_t *p, u32x4 v) { __builtin_nontemporal_store(v, (gptr)(p)); }

struct Split {
    uint32_t a[4], b[4], c[4];
};
__device__ __forceinline__ Split split(u32x4 v) {
    Split s;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s.a[i] = v[i] & 0x07070707u;
        s.b[i] = (v[i] >> 3) & 0x07070707u;
        s.c[i] = (v[i] >> 6) & 0x03030303u;
    }
    return s;
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// acc ^= c0*x0 ^ c1*x1
__device__ __forceinline__ void gmac2(u32x4 &acc, const Split &s0, const Split &s1, uint4 ab0, uint32_t tc0, uint4 ab1,
                                      uint32_t tc1) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        uint32_t t = xor3(acc[i], __builtin_amdgcn_perm(ab0.y, ab0.x, s0.a[i]), __builtin_amdgcn_perm(ab0.w, ab0.z, s0.b[i]));
        t = xor3(t, __builtin_amdgcn_perm(tc0, tc0, s0.c[i]), __builtin_amdgcn_perm(ab1.y, ab1.x, s1.a[i]));
        acc[i] = xor3(t, __builtin_amdgcn_perm(ab1.w, ab1.z, s1.b[i]), __builtin_amdgcn_perm(tc1, tc1, s1.c[i]));
    }
}

// ---------------------------------------------------------------- rowwise ---
__global__ __launch_bounds__(256) void rowwise(uint8_t *win, size_t nwin, const uint4 *gab, const uint32_t *gc) {
    __shared__ uint4 tab[K * R];
    __shared__ uint32_t tc[K * R];
    if (threadIdx.x < K * R) { tab[threadIdx.x] = gab[threadIdx.x]; tc[threadIdx.x] = gc[threadIdx.x]; }
    __syncthreads();
    const size_t total = nwin * NCOL, gt = (size_t)gridDim.x * 256;
    for (size_t s = (size_t)blockIdx.x * 256 + threadIdx.x; s < total; s += gt) {
        const size_t w = s / NCOL, c = s - w * NCOL;
        uint8_t *b = win + w * WB + c * 16;
        u32x4 acc[R] = {};
        for (int j = 0; j < K; j += 2) {
            const u32x4 v0 = ldg(b + (size_t)j * S), v1 = ldg(b + (size_t)(j + 1) * S);
            const Split s0 = split(v0), s1 = split(v1);
            const int row = __builtin_amdgcn_readfirstlane(j * R);
#pragma unroll
            for (int m = 0; m < R; m++) gmac2(acc[m], s0, s1, tab[row + m], tc[row + m], tab[row + R + m], tc[row + R + m]);
        }
#pragma unroll
        for (int m = 0; m < R; m++) stg(b + (size_t)(K + m) * S, acc[m]);
    }
}

// ----------------------------------------------------------------- staged ---
// LDS: [image: G*WCH chunks rounded up to 64][out image: G*R*NCOL chunks if ST]
template <int G, int ST>
__global__ __launch_bounds__(256) void staged(uint8_t *win, size_t nwin, const uint4 *gab, const uint32_t *gc) {
    extern __shared__ u32x4 lds[];
    __shared__ uint4 tab[K * R];
    __shared__ uint32_t tc[K * R];
    constexpr uint32_t IMG = (G * WCH + 63) / 64 * 64;
    u32x4 *oimg = lds + IMG;
    if (threadIdx.x < K * R) { tab[threadIdx.x] = gab[threadIdx.x]; tc[threadIdx.x] = gc[threadIdx.x]; }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (size_t w0 = (size_t)blockIdx.x * G; w0 < nwin; w0 += (size_t)gridDim.x * G) {
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        const uint32_t nch = nb * WCH;
        uint8_t *wbase = win + w0 * WB;
        for (uint32_t q0 = wv * 64; q0 < nch; q0 += 256) {
            const uint32_t q = std::min(q0 + lane, nch - 1);
            const uint32_t wl = q / WCH, o = q - wl * WCH;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(wbase + wl * WB + o * 16),
                                             (__attribute__((address_space(3))) void *)(lds + q0), 16, 0, 0);
        }
        __syncthreads();
        const uint32_t ns = nb * NCOL;
        for (uint32_t s = threadIdx.x; s < ns; s += 256) {
            const uint32_t wl = s / NCOL, c = s - wl * NCOL;
            const u32x4 *b = lds + wl * WCH + c;
            u32x4 acc[R] = {};
#pragma unroll 2
            for (int j = 0; j < K; j += 2) {
                const Split s0 = split(b[j * NCOL]), s1 = split(b[(j + 1) * NCOL]);
                const int row = j * R;
#pragma unroll
                for (int m = 0; m < R; m++) gmac2(acc[m], s0, s1, tab[row + m], tc[row + m], tab[row + R + m], tc[row + R + m]);
            }
            if constexpr (ST == 0) {
                uint8_t *o = wbase + wl * WB + WSRC + c * 16;
#pragma unroll
                for (int m = 0; m < R; m++) stg(o + (size_t)m * S, acc[m]);
            } else {
#pragma unroll
                for (int m = 0; m < R; m++) oimg[(wl * R + m) * NCOL + c] = acc[m];
            }
        }
        __syncthreads();
        if constexpr (ST == 1) {
            const uint32_t no = nb * R * NCOL;
            for (uint32_t q = threadIdx.x; q < no; q += 256) {
                const uint32_t wl = q / (R * NCOL), o = q - wl * (R * NCOL);
                stg(wbase + wl * WB + WSRC + o * 16, oimg[q]);
            }
            // the next step's staging writes only the source image: no barrier needed
        }
    }
}

// ------------------------------------------------------------------ flatq ---
// One window per workgroup step, 320 threads (300 live).  Unit u = 75 jj + c
// (lane u): chunks at t * 4,800 + 16 u of the source region, i.e. rows 4t + jj
// at column c, so every load instruction covers contiguous window bytes.  The
// lane's 4 rows give partial repairs for the 4 outputs, exchanged through LDS:
// lane u then XORs the 4 partials of output i = u / 75, column c = u % 75 and
// stores chunk u of the repair region (contiguous again).
template <bool GF, bool PF, int W = 1>
__global__ __launch_bounds__(320) __attribute__((amdgpu_waves_per_eu(W, 8))) void flatq(uint8_t *win, size_t nwin, const uint4 *gab, const uint32_t *gc) {
    __shared__ uint4 tab[K * R];
    __shared__ uint32_t tc[K * R];
    __shared__ u32x4 part[4 * R * NCOL];  // [jj][i][c]
    if (threadIdx.x < K * R) { tab[threadIdx.x] = gab[threadIdx.x]; tc[threadIdx.x] = gc[threadIdx.x]; }
    __syncthreads();
    const uint32_t u = threadIdx.x;
    const bool live = u < R * NCOL;
    const uint32_t uu = live ? u : R * NCOL - 1;
    const uint32_t jj = uu / NCOL, c = uu - jj * NCOL;
    size_t w = blockIdx.x;
    u32x4 v[4];
    auto load = [&](size_t ww) {
        const uint8_t *b = win + ww * WB + uu * 16;
#pragma unroll
        for (int t = 0; t < 4; t++) v[t] = ldg(b + (size_t)t * R * S);
    };
    if (w < nwin) load(w);
    for (; w < nwin; w += gridDim.x) {
        u32x4 acc[R] = {};
        if constexpr (GF) {
#pragma unroll
            for (int t = 0; t < 4; t += 2) {
                const Split s0 = split(v[t]), s1 = split(v[t + 1]);
                const int r0 = (4 * t + jj) * R, r1 = (4 * (t + 1) + jj) * R;
#pragma unroll
                for (int m = 0; m < R; m++) gmac2(acc[m], s0, s1, tab[r0 + m], tc[r0 + m], tab[r1 + m], tc[r1 + m]);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 4; t++) acc[t] = v[t];
        }
        if (PF && w + gridDim.x < nwin) load(w + gridDim.x);
        if (live) {
#pragma unroll
            for (int m = 0; m < R; m++) part[(jj * R + m) * NCOL + c] = acc[m];
        }
        __syncthreads();
        if (live) {
            // output i = jj', column c': the same u read as (i, c)
            const u32x4 x = part[(0 * R + jj) * NCOL + c] ^ part[(1 * R + jj) * NCOL + c] ^
                            part[(2 * R + jj) * NCOL + c] ^ part[(3 * R + jj) * NCOL + c];
            stg(win + w * WB + WSRC + u * 16, x);
        }
        __syncthreads();
        if (!PF && w + gridDim.x < nwin) load(w + gridDim.x);
    }
}


// ---------------------------------------------------------------- staged2 ---
// G windows per group, NR source rows per stage (16 / NR stages per group);
// DB: two stage buffers, the next stage's global_load_lds issued right after
// the barrier that retires the current one, so it lands during the compute.
template <int G, int NR, bool DB>
__global__ __launch_bounds__(256) void staged2(uint8_t *win, size_t nwin, const uint4 *gab, const uint32_t *gc) {
    extern __shared__ u32x4 lds[];
    __shared__ uint4 tab[K * R];
    __shared__ uint32_t tc[K * R];
    constexpr uint32_t SCH = NR * NCOL;                 // chunks per window per stage
    constexpr uint32_t IMG = (G * SCH + 63) / 64 * 64;  // chunks per buffer
    constexpr int NST = K / NR;
    if (threadIdx.x < K * R) { tab[threadIdx.x] = gab[threadIdx.x]; tc[threadIdx.x] = gc[threadIdx.x]; }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t ngrp = (nwin + G - 1) / G;
    // steps: (group, stage) for this block's groups
    auto stage = [&](size_t gi, int st, u32x4 *buf) {
        const size_t w0 = gi * G;
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        const uint32_t nch = nb * SCH;
        uint8_t *wbase = win + w0 * WB + (size_t)st * NR * S;
        for (uint32_t q0 = wv * 64; q0 < nch; q0 += 256) {
            const uint32_t q = std::min(q0 + lane, nch - 1);
            const uint32_t wl = q / SCH, o = q - wl * SCH;
            __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(wbase + wl * WB + o * 16),
                                             (__attribute__((address_space(3))) void *)(buf + q0), 16, 0, 0);
        }
    };
    size_t gi = blockIdx.x;
    int st = 0;
    if (gi >= ngrp) return;
    __syncthreads();
    stage(gi, 0, lds);
    u32x4 acc[R] = {};
    int cur = 0;
    for (;;) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // next step
        size_t gn = gi;
        int sn = st + 1;
        if (sn == NST) { sn = 0; gn += gridDim.x; }
        const bool more = gn < ngrp;
        if (DB && more) stage(gn, sn, lds + (cur ^ 1) * IMG);
        const size_t w0 = gi * G;
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        const uint32_t s_ = threadIdx.x;
        const bool live = s_ < nb * NCOL;
        const uint32_t ss = live ? s_ : 0;
        const uint32_t wl = ss / NCOL, c = ss - wl * NCOL;
        const u32x4 *b = lds + cur * IMG + wl * SCH + c;
#pragma unroll 2
        for (int j = 0; j < NR; j += 2) {
            const Split s0 = split(b[j * NCOL]), s1 = split(b[(j + 1) * NCOL]);
            const int row = (st * NR + j) * R;
#pragma unroll
            for (int m = 0; m < R; m++) gmac2(acc[m], s0, s1, tab[row + m], tc[row + m], tab[row + R + m], tc[row + R + m]);
        }
        if (st == NST - 1) {
            if (live) {
                uint8_t *o = win + (w0 + wl) * WB + WSRC + c * 16;
#pragma unroll
                for (int m = 0; m < R; m++) stg(o + (size_t)m * S, acc[m]);
            }
#pragma unroll
            for (int m = 0; m < R; m++) acc[m] = u32x4{0, 0, 0, 0};
        }
        if (!more) break;
        if (!DB) {
            __syncthreads();
            stage(gn, sn, lds);
        } else {
            cur ^= 1;
        }
        gi = gn;
        st = sn;
    }
}

// rowst: rowwise loads and table multiply, the repairs gathered in LDS and
// stored contiguously (window by window); G whole windows per workgroup step
template <int G>
__global__ void rowst(uint8_t *win, size_t nwin, const uint4 *gab, const uint32_t *gc) {
    __shared__ uint4 tab[K * R];
    __shared__ uint32_t tc[K * R];
    __shared__ u32x4 out[G * R * NCOL];
    if (threadIdx.x < K * R) { tab[threadIdx.x] = gab[threadIdx.x]; tc[threadIdx.x] = gc[threadIdx.x]; }
    __syncthreads();
    const uint32_t nt = blockDim.x;
    for (size_t w0 = (size_t)blockIdx.x * G; w0 < nwin; w0 += (size_t)gridDim.x * G) {
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        const uint32_t s = threadIdx.x;
        if (s < nb * NCOL) {
            const uint32_t wl = s / NCOL, c = s - wl * NCOL;
            const uint8_t *b = win + (w0 + wl) * WB + c * 16;
            u32x4 acc[R] = {};
            for (int j = 0; j < K; j += 2) {
                const u32x4 v0 = ldg(b + (size_t)j * S), v1 = ldg(b + (size_t)(j + 1) * S);
                const Split s0 = split(v0), s1 = split(v1);
                const int row = j * R;
#pragma unroll
                for (int m = 0; m < R; m++) gmac2(acc[m], s0, s1, tab[row + m], tc[row + m], tab[row + R + m], tc[row + R + m]);
            }
#pragma unroll
            for (int m = 0; m < R; m++) out[(wl * R + m) * NCOL + c] = acc[m];
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb * R * NCOL; q += nt) {
            const uint32_t wl = q / (R * NCOL), o = q - wl * (R * NCOL);
            stg(win + (w0 + wl) * WB + WSRC + o * 16, out[q]);
        }
        __syncthreads();
    }
}

// rowst2: rowst with two LDS output images (one barrier per group) and a
// waves-per-EU floor W
template <int G, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8))) void rowst2(uint8_t *win, size_t nwin, const uint4 *gab, const uint32_t *gc) {
    __shared__ uint4 tab[K * R];
    __shared__ uint32_t tc[K * R];
    __shared__ u32x4 out[2][G * R * NCOL];
    if (threadIdx.x < K * R) { tab[threadIdx.x] = gab[threadIdx.x]; tc[threadIdx.x] = gc[threadIdx.x]; }
    __syncthreads();
    int buf = 0;
    for (size_t w0 = (size_t)blockIdx.x * G; w0 < nwin; w0 += (size_t)gridDim.x * G, buf ^= 1) {
        const uint32_t nb = (uint32_t)std::min((size_t)G, nwin - w0);
        const uint32_t s = threadIdx.x;
        if (s < nb * NCOL) {
            const uint32_t wl = s / NCOL, c = s - wl * NCOL;
            const uint8_t *b = win + (w0 + wl) * WB + c * 16;
            u32x4 acc[R] = {};
            for (int j = 0; j < K; j += 2) {
                const u32x4 v0 = ldg(b + (size_t)j * S), v1 = ldg(b + (size_t)(j + 1) * S);
                const Split s0 = split(v0), s1 = split(v1);
                const int row = j * R;
#pragma unroll
                for (int m = 0; m < R; m++) gmac2(acc[m], s0, s1, tab[row + m], tc[row + m], tab[row + R + m], tc[row + R + m]);
            }
#pragma unroll
            for (int m = 0; m < R; m++) out[buf][(wl * R + m) * NCOL + c] = acc[m];
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < nb * R * NCOL; q += 256) {
            const uint32_t wl = q / (R * NCOL), o = q - wl * (R * NCOL);
            stg(win + (w0 + wl) * WB + WSRC + o * 16, out[buf][q]);
        }
    }
}

__global__ void cmp(const u32x4 *a, const u32x4 *b, size_t n, unsigned long long *bad) {
    unsigned long long nb = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const u32x4 x = a[i], y = b[i];
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
    // Cauchy k16 r4 tables [j][i]
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
        hipLaunchKernelGGL(cmp, 4096, 256, 0, 0, (const u32x4 *)win, (const u32x4 *)ref, bytes / 16, bad);
        unsigned long long hb = 0;
        CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        printf("  {\"kernel\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"TBps\": %.3f, \"mismatch_chunks\": %llu},\n",
               name, gm, ms, alg / (ms * 1e-3) / 1e12, hb);
        fflush(stdout);
    };
    // reference output
    hipLaunchKernelGGL(rowwise, cus * 2, 256, 0, 0, win, nwin, gab, gc);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref, win, bytes, hipMemcpyDeviceToDevice));
    for (int round = 0; round < 2; round++) {
        for (int gm : {4}) {
            const double ms = time_ms([&] { hipLaunchKernelGGL(rowwise, cus * gm, 256, 0, 0, win, nwin, gab, gc); });
            report("rowwise", gm, ms);
        }
#define STAGED(G, ST, GMS)                                                                                      \
        {                                                                                                        \
            const size_t sh = ((G * WCH + 63) / 64 * 64 + (ST ? G * R * NCOL : 0)) * 16;                         \
            CK(hipFuncSetAttribute((const void *)staged<G, ST>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh)); \
            for (int gm : GMS) {                                                                                 \
                if ((size_t)gm * sh > 160 * 1024) continue;                                                      \
                const double ms = time_ms([&] { hipLaunchKernelGGL((staged<G, ST>), cus * gm, 256, sh, 0, win, nwin, gab, gc); }); \
                report("staged_G" #G "_st" #ST, gm, ms);                                                         \
            }                                                                                                    \
        }
        for (int gm : {4, 5, 8}) {
            const double ms = time_ms([&] { hipLaunchKernelGGL((rowst<3>), cus * gm, 256, 0, 0, win, nwin, gab, gc); });
            report("rowst_gf_G3_256", gm, ms);
        }
        for (int gm : {4, 5, 6, 8, 12}) {
            double ms = time_ms([&] { hipLaunchKernelGGL((rowst2<3, 1>), cus * gm, 256, 0, 0, win, nwin, gab, gc); });
            report("rowst2_G3_w1", gm, ms);
            ms = time_ms([&] { hipLaunchKernelGGL((rowst2<3, 6>), cus * gm, 256, 0, 0, win, nwin, gab, gc); });
            report("rowst2_G3_w6", gm, ms);
            ms = time_ms([&] { hipLaunchKernelGGL((rowst2<3, 8>), cus * gm, 256, 0, 0, win, nwin, gab, gc); });
            report("rowst2_G3_w8", gm, ms);
        }
    }
    printf("  {\"end\": true}\n]}\n");
    return 0;
}
