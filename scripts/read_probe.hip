// read_probe.hip — what read rate can a kernel reach on this MI355X, and how?
//   reg<U>   : grid-stride global_load_dwordx4 into registers, U loads in flight
//              per lane per iteration (consecutive lanes = consecutive 16 B)
//   lds<U>   : global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave instruction)
//              into a per-wave LDS ring of U slots, then ds_read_b128 + xor
//   rw<U>    : reg<U> reads + one 16-B store per 4 loads (4:1 read:write)
// 4 GiB buffer, median of 10.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o scripts/read_probe scripts/read_probe.hip
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

template <int U>
__global__ __launch_bounds__(256) void reg(const uint4 *in, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    const size_t G = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += G * U) {
        uint4 v[U];
#pragma unroll
        for (int t = 0; t < U; t++) v[t] = in[min(i + t * G, n - 1)];
#pragma unroll
        for (int t = 0; t < U; t++) acc ^= v[t].x ^ v[t].y ^ v[t].z ^ v[t].w;
    }
    if (acc == 0x9e3779b9u) atomicAdd(sink, 1u);
}

template <int U>
__global__ __launch_bounds__(256) void rw(const uint4 *in, uint4 *out, size_t n) {
    const size_t G = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += G * U) {
        uint4 v[U];
#pragma unroll
        for (int t = 0; t < U; t++) v[t] = in[min(i + t * G, n - 1)];
        uint4 a = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int t = 0; t < U; t++) { a.x ^= v[t].x; a.y ^= v[t].y; a.z ^= v[t].z; a.w ^= v[t].w; }
        out[(i / 4) % (n / 4)] = a;  // one store per lane-iteration
    }
}

template <int U>
__global__ __launch_bounds__(256) void ldsdma(const uint4 *in, size_t n, uint32_t *sink) {
    __shared__ uint4 ring[4][U][64];  // per wave: U slots of 1 KiB
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t acc = 0;
    const size_t G = (size_t)gridDim.x * 256;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += G * U) {
#pragma unroll
        for (int t = 0; t < U; t++) {
            const uint4 *src = in + min(i + t * G, n - 1);
#if defined(__HIP_DEVICE_COMPILE__)
            __builtin_amdgcn_global_load_lds(src, &ring[wave][t][0], 16, 0, 0);
#else
            (void)src;
#endif
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int t = 0; t < U; t++) {
            const uint4 v = ring[wave][t][lane];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (acc == 0x9e3779b9u) atomicAdd(sink, 1u);
}

template <class F>
double timeit(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) f();
    std::vector<float> ts;
    for (int i = 0; i < 10; i++) {
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
    const size_t bytes = (size_t)4 << 30, n = bytes / 16;
    uint4 *in, *out;
    uint32_t *sink;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes / 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 0x11, bytes));
    auto rate = [&](double ms, double b) { return b / (ms * 1e-3) / 1e12; };
    printf("{");
    bool first = true;
    for (int g : {1024, 2048, 4096}) {
        printf("%s\"grid%d\": {", first ? "" : ", ", g);
        first = false;
        printf("\"reg2\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(reg<2>, g, 256, 0, 0, in, n, sink); }), bytes));
        printf("\"reg4\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(reg<4>, g, 256, 0, 0, in, n, sink); }), bytes));
        printf("\"reg8\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(reg<8>, g, 256, 0, 0, in, n, sink); }), bytes));
        printf("\"reg16\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(reg<16>, g, 256, 0, 0, in, n, sink); }), bytes));
        printf("\"lds4\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(ldsdma<4>, g, 256, 0, 0, in, n, sink); }), bytes));
        printf("\"lds8\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(ldsdma<8>, g, 256, 0, 0, in, n, sink); }), bytes));
        printf("\"lds16\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(ldsdma<16>, g, 256, 0, 0, in, n, sink); }), bytes));
        printf("\"rw4\": %.2f, ", rate(timeit([&] { hipLaunchKernelGGL(rw<4>, g, 256, 0, 0, in, out, n); }), bytes * 1.25));
        printf("\"rw8\": %.2f}", rate(timeit([&] { hipLaunchKernelGGL(rw<8>, g, 256, 0, 0, in, out, n); }), bytes * 1.125));
    }
    printf("}\n");
    return 0;
}
