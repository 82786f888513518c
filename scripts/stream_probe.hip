// stream_probe.hip — measured HBM ceilings for the read:write mixes of the FEC
// kernels (denominators beside the 8 TB/s spec).  Grid-stride dwordx4 streams:
//   read      : x = xor of N_IN input streams (result kept live)
//   r{N}w1    : out = xor of N input streams (N:1 read:write, XOR encode shape)
//   copy      : out = in
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/stream_probe scripts/stream_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

template <int NIN, bool WRITE>
__global__ __launch_bounds__(256) void stream(const uint4 *__restrict__ in, uint4 *__restrict__ out,
                                              size_t n, uint32_t *sink) {
    uint4 acc = make_uint4(0, 0, 0, 0);
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint4 v[NIN];
#pragma unroll
        for (int t = 0; t < NIN; t++) v[t] = in[i + t * n];
        uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int t = 0; t < NIN; t++) {
            x.x ^= v[t].x; x.y ^= v[t].y; x.z ^= v[t].z; x.w ^= v[t].w;
        }
        if (WRITE) out[i] = x;
        else { acc.x ^= x.x; acc.y ^= x.y; acc.z ^= x.z; acc.w ^= x.w; }
    }
    if (!WRITE && (acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) atomicAdd(sink, 1u);
}

template <int NIN, bool WRITE>
double run(const uint4 *in, uint4 *out, size_t n, uint32_t *sink, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; i++) hipLaunchKernelGGL((stream<NIN, WRITE>), grid, 256, 0, 0, in, out, n, sink);
    std::vector<float> ts;
    for (int i = 0; i < 10; i++) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((stream<NIN, WRITE>), grid, 256, 0, 0, in, out, n, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double bytes = (double)n * 16 * (NIN + (WRITE ? 1 : 0));
    return bytes / (ts[ts.size() / 2] * 1e-3) / 1e9;
}

int main() {
    const size_t per = (size_t)1 << 30;  // 1 GiB per stream
    const size_t n = per / 16;
    uint4 *in, *out;
    uint32_t *sink;
    CK(hipMalloc(&in, per * 8));
    CK(hipMalloc(&out, per));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 0x5a, per * 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"cus\": %d", cus);
    for (int gm : {4, 8, 16}) {
        const int grid = cus * gm;
        printf(", \"grid%d\": {\"read8\": %.1f, \"r8w1\": %.1f, \"r4w1\": %.1f, \"r2w1\": %.1f, \"copy\": %.1f}",
               gm, run<8, false>(in, out, n, sink, grid), run<8, true>(in, out, n, sink, grid),
               run<4, true>(in, out, n, sink, grid), run<2, true>(in, out, n, sink, grid),
               run<1, true>(in, out, n, sink, grid));
    }
    printf("}\n");
    return 0;
}
