// layout_probe.hip — does the DRAM access pattern of the XOR encode matter?
// Same bytes, same cfg2 layout (65,536 windows x 10 symbols x 1200 B):
//   rows   : lane = 16-B column, reads the column of 8 source rows, writes 2
//            repair rows (the fecgpu kernel's pattern)
//   linear : lanes stream the windows' 9600-B source regions linearly and
//            the 2400-B repair regions linearly (what LDS staging would give)
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/layout_probe scripts/layout_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) { fprintf(stderr, "%s\n", hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr uint32_t NWIN = 65536, K = 8, R = 2, S = 1200, NCOL = S / 16, WB = (K + R) * S;

__global__ __launch_bounds__(256) void rows(uint8_t *win) {
    for (uint64_t s = blockIdx.x * 256ull + threadIdx.x; s < (uint64_t)NWIN * NCOL;
         s += (uint64_t)gridDim.x * 256) {
        const uint32_t w = s / NCOL, c = s % NCOL;
        uint8_t *b = win + (uint64_t)w * WB + c * 16;
        uint4 v[K];
#pragma unroll
        for (int j = 0; j < K; j++) v[j] = *(const uint4 *)(b + j * S);
        uint4 a0 = v[0], a1 = v[1];
#pragma unroll
        for (int j = 2; j < K; j += 2) {
            a0.x ^= v[j].x; a0.y ^= v[j].y; a0.z ^= v[j].z; a0.w ^= v[j].w;
            a1.x ^= v[j + 1].x; a1.y ^= v[j + 1].y; a1.z ^= v[j + 1].z; a1.w ^= v[j + 1].w;
        }
        *(uint4 *)(b + K * S) = a0;
        *(uint4 *)(b + (K + 1) * S) = a1;
    }
}

// linear: chunk c of the source stream (600 per window) and of the repair stream
// (150 per window); 4 source chunks per repair chunk, xor-folded.
// Each block owns a contiguous range of windows; it streams their source
// regions (consecutive lanes = consecutive 16-B chunks, U chunks in flight per
// lane) and then writes their repair regions the same way.
template <int U>
__global__ __launch_bounds__(256) void linear(uint8_t *win) {
    constexpr uint32_t SC = K * S / 16, RC = R * S / 16;  // 600, 150 chunks per window
    const uint32_t wpb = (NWIN + gridDim.x - 1) / gridDim.x;
    const uint32_t w0 = blockIdx.x * wpb, w1 = min(NWIN, w0 + wpb);
    uint4 a = make_uint4(0, 0, 0, 0);
    for (uint32_t w = w0; w < w1; w += 4) {  // 4 windows per step
        const uint32_t nw = min(4u, w1 - w);
        for (uint32_t c = threadIdx.x; c < nw * SC; c += 256 * U) {
            uint4 v[U];
#pragma unroll
            for (int t = 0; t < U; t++) {
                const uint32_t cc = min(c + t * 256, nw * SC - 1);
                v[t] = *(const uint4 *)(win + (uint64_t)(w + cc / SC) * WB + (cc % SC) * 16);
            }
#pragma unroll
            for (int t = 0; t < U; t++) { a.x ^= v[t].x; a.y ^= v[t].y; a.z ^= v[t].z; a.w ^= v[t].w; }
        }
        for (uint32_t c = threadIdx.x; c < nw * RC; c += 256)
            *(uint4 *)(win + (uint64_t)(w + c / RC) * WB + K * S + (c % RC) * 16) = a;
    }
}

template <class F>
double timeit(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    std::vector<float> ts;
    for (int i = 0; i < 15; i++) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    uint8_t *win;
    const size_t bytes = (size_t)NWIN * WB;
    CK(hipMalloc(&win, bytes));
    CK(hipMemset(win, 0x3c, bytes));
    const double alg = (double)NWIN * (K + R) * S;
    printf("{");
    for (int g : {2048, 4096, 8192}) {
        const double tr = timeit([&] { hipLaunchKernelGGL(rows, g, 256, 0, 0, win); });
        const double tl = timeit([&] { hipLaunchKernelGGL(linear<4>, g, 256, 0, 0, win); });
        printf("%s\"grid%d\": {\"rows_TBps\": %.3f, \"linear_TBps\": %.3f}", g == 2048 ? "" : ", ", g,
               alg / (tr * 1e-3) / 1e12, alg / (tl * 1e-3) / 1e12);
    }
    printf("}\n");
    return 0;
}
