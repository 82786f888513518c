// mix_probe.hip — HBM ceilings for the read:write mixes of the FEC kernels
// (the denominators DESIGN.md §6 quotes beside the 8 TB/s spec).
//
// out_o = XOR of NIN input streams, NOUT output streams, 16 B per lane per
// access, U independent 16-B units per lane per iteration (more bytes in
// flight), grid-stride over the units; optional nontemporal loads / stores.
// Shapes: copy (1:1), read (8:0), XOR encode cfg2 (8:2), GF cfg3 (16:4), and
// the same mixes with the kernels' window layout (mix_win: k + r rows of S
// bytes per window, lanes on 16-B columns, sources read, repairs written).
// Streams are 512 MiB each (well past the 256 MiB Infinity Cache).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/mix_probe scripts/mix_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// streams: input t at in + t * n, output o at out + o * n (n units of 16 B each)
template <int NIN, int NOUT, int U, bool NT>
__global__ __launch_bounds__(256) void mix(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n,
                                           uint32_t *sink) {
    const size_t gt = (size_t)gridDim.x * 256;
    u32x4 keep = {0, 0, 0, 0};
    for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += gt * U) {
        u32x4 v[U][NIN];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = i0 + (size_t)u * 256;
#pragma unroll
            for (int t = 0; t < NIN; t++) v[u][t] = i < n ? ld<NT>(in + i + t * n) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = i0 + (size_t)u * 256;
            u32x4 x = v[u][0];
#pragma unroll
            for (int t = 1; t < NIN; t++) x ^= v[u][t];
            if (NOUT == 0) keep ^= x;
#pragma unroll
            for (int o = 0; o < NOUT; o++)
                if (i < n) st<NT>(out + i + o * n, x ^ (u32x4){(uint32_t)o, 0, 0, 0});
        }
    }
    if (NOUT == 0 && (keep.x ^ keep.y ^ keep.z ^ keep.w) == 0x12345678u) atomicAdd(sink, 1u);
}

// window layout: nwin windows of (K + R) rows of S bytes (S % 16 == 0), slot s
// = (window s / ncol, column s % ncol); rows 0..K-1 read, rows K.. written.
template <int K, int R, bool NT>
__global__ __launch_bounds__(256) void mix_win(u32x4 *__restrict__ win, size_t nwin, uint32_t S) {
    const uint32_t ncol = S / 16;
    const size_t total = nwin * ncol, gt = (size_t)gridDim.x * 256;
    for (size_t s = (size_t)blockIdx.x * 256 + threadIdx.x; s < total; s += gt) {
        const size_t w = s / ncol, c = s - w * ncol;
        u32x4 *b = win + w * (size_t)(K + R) * ncol + c;
        u32x4 v[K];
#pragma unroll
        for (int t = 0; t < K; t++) v[t] = ld<NT>(b + (size_t)t * ncol);
#pragma unroll
        for (int o = 0; o < R; o++) {
            u32x4 x = {0, 0, 0, 0};
#pragma unroll
            for (int t = o; t < K; t += R) x ^= v[t];
            st<true>(b + (size_t)(K + o) * ncol, x);
        }
    }
}

// split layout (SURVEY §8b encode_batch form): sources src[W][K][S], repairs
// rep[W][R][S] in their own array.  DEC: the decode shape instead — read the
// K - R present sources of src and the R repairs, write R recovered rows
// (the first R rows of each window) back into src.
template <int K, int R, bool DEC>
__global__ __launch_bounds__(256) void mix_split(u32x4 *__restrict__ src, u32x4 *__restrict__ rep, size_t nwin,
                                                 uint32_t S) {
    const uint32_t ncol = S / 16;
    const size_t total = nwin * ncol, gt = (size_t)gridDim.x * 256;
    for (size_t s = (size_t)blockIdx.x * 256 + threadIdx.x; s < total; s += gt) {
        const size_t w = s / ncol, c = s - w * ncol;
        u32x4 *b = src + w * (size_t)K * ncol + c;
        u32x4 *o = rep + w * (size_t)R * ncol + c;
        u32x4 v[K];
#pragma unroll
        for (int t = 0; t < K; t++) v[t] = (DEC && t < R) ? ld<false>(o + (size_t)t * ncol) : ld<false>(b + (size_t)t * ncol);
#pragma unroll
        for (int u = 0; u < R; u++) {
            u32x4 x = {0, 0, 0, 0};
#pragma unroll
            for (int t = u; t < K; t += R) x ^= v[t];
            st<true>((DEC ? b : o) + (size_t)u * ncol, x);
        }
    }
}

static int g_cus = 256;

template <class F>
static double time_ms(F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) launch();
    std::vector<float> ts;
    for (int i = 0; i < 9; i++) {
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

template <int NIN, int NOUT, int U, bool NT>
static void run_mix(const char *name, u32x4 *in, u32x4 *out, size_t n, uint32_t *sink) {
    double best = 0;
    int best_g = 0;
    printf("  {\"shape\": \"%s\", \"U\": %d, \"nt\": %d, \"grids\": {", name, U, (int)NT);
    bool first = true;
    for (int gm : {1, 2, 4, 8, 16}) {
        const int grid = g_cus * gm;
        const double ms = time_ms([&] { hipLaunchKernelGGL((mix<NIN, NOUT, U, NT>), grid, 256, 0, 0, in, out, n, sink); });
        const double tbs = (double)n * 16 * (NIN + NOUT) / (ms * 1e-3) / 1e12;
        printf("%s\"%d\": %.3f", first ? "" : ", ", gm, tbs);
        first = false;
        if (tbs > best) { best = tbs; best_g = gm; }
    }
    printf("}, \"best_TBps\": %.3f, \"best_blocks_per_cu\": %d},\n", best, best_g);
    fflush(stdout);
}

template <int K, int R, bool NT>
static void run_win(const char *name, u32x4 *win, size_t bytes, uint32_t S) {
    const size_t nwin = bytes / ((size_t)(K + R) * S);
    printf("  {\"shape\": \"%s\", \"S\": %u, \"nwin\": %zu, \"nt\": %d, \"grids\": {", name, S, nwin, (int)NT);
    double best = 0;
    bool first = true;
    for (int gm : {1, 2, 4, 8}) {
        const int grid = g_cus * gm;
        const double ms = time_ms([&] { hipLaunchKernelGGL((mix_win<K, R, NT>), grid, 256, 0, 0, win, nwin, S); });
        const double tbs = (double)nwin * (K + R) * S / (ms * 1e-3) / 1e12;
        printf("%s\"%d\": %.3f", first ? "" : ", ", gm, tbs);
        first = false;
        best = std::max(best, tbs);
    }
    printf("}, \"best_TBps\": %.3f},\n", best);
    fflush(stdout);
}

template <int K, int R, bool DEC>
static void run_split(const char *name, u32x4 *src, u32x4 *rep, size_t bytes, uint32_t S) {
    const size_t nwin = bytes / ((size_t)(K + R) * S);
    printf("  {\"shape\": \"%s\", \"S\": %u, \"nwin\": %zu, \"grids\": {", name, S, nwin);
    double best = 0;
    bool first = true;
    for (int gm : {1, 2, 4, 8}) {
        const int grid = g_cus * gm;
        const double ms = time_ms([&] { hipLaunchKernelGGL((mix_split<K, R, DEC>), grid, 256, 0, 0, src, rep, nwin, S); });
        const double tbs = (double)nwin * (K + R) * S / (ms * 1e-3) / 1e12;
        printf("%s\"%d\": %.3f", first ? "" : ", ", gm, tbs);
        first = false;
        best = std::max(best, tbs);
    }
    printf("}, \"best_TBps\": %.3f},\n", best);
    fflush(stdout);
}

int main() {
    const size_t per = (size_t)512 << 20;  // bytes per stream
    const size_t n = per / 16;
    u32x4 *in, *out;
    uint32_t *sink;
    CK(hipMalloc(&in, per * 16));
    CK(hipMalloc(&out, per * 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 0x5a, per * 16));
    CK(hipMemset(out, 0, per * 4));
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"cus\": %d, \"stream_MiB\": %zu, \"unit\": \"TB/s of bytes read + written\", \"runs\": [\n", g_cus,
           per >> 20);
    run_mix<1, 1, 1, false>("copy", in, out, n, sink);
    run_mix<1, 1, 2, false>("copy", in, out, n, sink);
    run_mix<1, 1, 4, false>("copy", in, out, n, sink);
    run_mix<1, 1, 4, true>("copy", in, out, n, sink);
    run_mix<8, 0, 1, false>("read8", in, out, n, sink);
    run_mix<8, 0, 2, false>("read8", in, out, n, sink);
    run_mix<8, 2, 1, false>("r8w2", in, out, n, sink);
    run_mix<8, 2, 2, false>("r8w2", in, out, n, sink);
    run_mix<8, 2, 1, true>("r8w2", in, out, n, sink);
    run_mix<16, 4, 1, false>("r16w4", in, out, n, sink);
    run_mix<16, 4, 1, true>("r16w4", in, out, n, sink);
    // the kernels' layout: windows of k + r rows, S = 1200 B (cfg2 / cfg3 shapes)
    run_win<8, 2, false>("win_k8r2", in, per * 16, 1200);
    run_win<8, 2, true>("win_k8r2", in, per * 16, 1200);
    run_win<16, 4, false>("win_k16r4", in, per * 16, 1200);
    // split layout: sources and repairs in separate arrays (encode_split form)
    run_split<8, 2, false>("split_enc_k8r2", in, out, per * 10, 1200);
    run_split<8, 2, true>("split_dec_k8r2", in, out, per * 10, 1200);
    run_split<16, 4, false>("split_enc_k16r4", in, out, per * 10, 1200);
    run_split<16, 4, true>("split_dec_k16r4", in, out, per * 10, 1200);
    printf("  {\"end\": true}\n]}\n");
    return 0;
}
