// VALU issue-rate probe for the instructions of the GF multiply-accumulate
// (v_perm_b32, v_bitop3_b32, v_xor_b32, v_and_b32, v_lshrrev_b32): 16
// independent chains per lane, W waves per SIMD on every CU.  Prints
// wave-instructions per SIMD-cycle at the measured clock (s_memtime ticks at
// 100 MHz; the shader clock from wall time x assumed 2.4 GHz and from the
// in-kernel s_memrealtime).  Measurement aid for DESIGN.md §4, not product.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/valu_probe scripts/valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t *out, int iters, uint32_t seed) {
    uint32_t r[16];
#pragma unroll
    for (int i = 0; i < 16; i++) r[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
    const uint32_t b = seed ^ threadIdx.x, c = 0x07060504u ^ (seed & 0x03030303u);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if (OP == 0) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(r[i]) : "v"(b), "v"(c));
            if (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[i]) : "v"(b), "v"(c));
            if (OP == 2) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(b));
            if (OP == 3) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r[i]) : "v"(b));
            if (OP == 4) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(r[i]));
            if (OP == 5) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(r[i]) : "s"(b), "v"(c));
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= r[i];
    if (x == 0x12345678u) out[threadIdx.x] = x;
}

template <int OP>
static int run(const char *name, int cus, uint32_t *d) {
    const int iters = 4096;
    for (int w : {1, 2, 3, 4, 8}) {
        const int grid = cus * w;  // 256 threads = one wave per SIMD per block
        hipEvent_t e0, e1;
        CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
        probe<OP><<<grid, 256>>>(d, iters, 1);
        CHK(hipEventRecord(e0));
        probe<OP><<<grid, 256>>>(d, iters, 2);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
        const double winstr = (double)grid * 4 * iters * 16;       // wave-instructions
        const double per_simd = winstr / (cus * 4.0);
        const double cyc = ms * 1e-3 * 2.4e9;                       // at 2.4 GHz
        printf("%-14s waves/SIMD %d: %.3f ms  %.2f cycles per wave-instr per SIMD (2.4 GHz)\n",
               name, w, ms, cyc / per_simd);
        CHK(hipEventDestroy(e0)); CHK(hipEventDestroy(e1));
    }
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    printf("CUs %d\n", cus);
    uint32_t *d; CHK(hipMalloc(&d, 4096));
    if (run<0>("v_perm_b32", cus, d) || run<1>("v_bitop3_b32", cus, d) || run<2>("v_xor_b32", cus, d) ||
        run<3>("v_and_b32", cus, d) || run<4>("v_lshrrev_b32", cus, d) || run<5>("v_perm(sgpr)", cus, d))
        return 1;
    CHK(hipFree(d));
    return 0;
}
