// mfma_probe.hip — is GF(2^8) repair generation faster on the matrix cores?
//
// The code is a dense GF(2) bit-matrix product: output bit (i, b') of a byte
// position is the parity of sum_{j,b} M[(i,b'),(j,b)] * bit_b(S_j), M built
// from the multiply-by-C[i][j] maps.  This probe runs it on
// v_mfma_i32_32x32x32_i8 (M = 8r output bits, K = 8k input bits, N = byte
// positions) and checks it against a CPU encode:
//   * B operand from the data with shifts only: a lane holds, for one byte
//     position, a dword D of 4 rows (a 4x4 byte transpose of 4 loaded dwords);
//     D >> b has bit b of each row in the LSB of its byte, and the parity of
//     an integer sum depends only on the LSBs, so the garbage above is free.
//   * A operand: the coefficient bit matrices, 0/1 int8, staged in LDS.
//   * C: int32 counts; bit 0 is the GF(2) sum -> nibbles -> output bytes.
// Wave tile: 128 byte positions (32 lanes x 4 dwords-worth) of one window,
// all k rows, 8 outputs.  k = 32, r = 8 (config 4's code), S = 4096.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/mfma_probe scripts/mfma_probe.hip
//        (-DPROBE_NOLOAD: compute-only ceiling, outputs not meaningful)
// Measured on MI355X (r01, profiles/r01_mfma_probe.txt): both variants
// bit-exact; 32x32x32 1.79 TB/s of k+r rows (1 wave/SIMD: 222 VGPR + 128 AGPR),
// 16x16x64 with the next chunk's loads in flight 2.67 TB/s, and 2.74 TB/s
// with no loads at all — the MFMA issue is throttled by the bit-unpack /
// parity-extract VALU work around it, below the v_perm kernel's 3.7 TB/s.  So
// the product keeps the VALU path (DESIGN.md §4 "Why not MFMA").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int K = 32, R = 8, NG = K / 8;
constexpr uint32_t S = 4096, STRIDE = 4096, CH = 128, CPW = S / CH;

static uint8_t gexp[512], glog[256];
static void gf_init() {
    int x = 1;
    for (int i = 0; i < 255; i++) {
        gexp[i] = (uint8_t)x;
        glog[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) gexp[i] = gexp[i - 255];
}
static uint8_t gmul(uint8_t a, uint8_t b) { return (a && b) ? gexp[glog[a] + glog[b]] : 0; }
static uint8_t ginv(uint8_t a) { return gexp[255 - glog[a]]; }

__device__ __forceinline__ void transpose4(const uint32_t L[4], uint32_t D[4]) {
    const uint32_t x0 = __builtin_amdgcn_perm(L[1], L[0], 0x05010400u);
    const uint32_t x1 = __builtin_amdgcn_perm(L[1], L[0], 0x07030602u);
    const uint32_t y0 = __builtin_amdgcn_perm(L[3], L[2], 0x05010400u);
    const uint32_t y1 = __builtin_amdgcn_perm(L[3], L[2], 0x07030602u);
    D[0] = __builtin_amdgcn_perm(y0, x0, 0x05040100u);
    D[1] = __builtin_amdgcn_perm(y0, x0, 0x07060302u);
    D[2] = __builtin_amdgcn_perm(y1, x1, 0x05040100u);
    D[3] = __builtin_amdgcn_perm(y1, x1, 0x07060302u);
}

__device__ __forceinline__ uint32_t nibble(int c0, int c1, int c2, int c3) {
    return (uint32_t)(c0 & 1) | ((uint32_t)(c1 & 1) << 1) | ((uint32_t)(c2 & 1) << 2) |
           ((uint32_t)(c3 & 1) << 3);
}

// afrag[g][q][mb][lane]
__global__ __launch_bounds__(256) void mfma_encode(uint8_t *win, const v4i *afrag, uint64_t nchunks) {
    __shared__ v4i sA[NG * 2 * 2 * 64];
    for (int i = threadIdx.x; i < NG * 2 * 2 * 64; i += 256) sA[i] = afrag[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n = lane & 31, h = lane >> 5;
    const uint64_t wbytes = (uint64_t)(K + R) * STRIDE;
    for (uint64_t c = (uint64_t)blockIdx.x * 4 + wave; c < nchunks; c += (uint64_t)gridDim.x * 4) {
        const uint64_t w = c / CPW;
        const uint32_t base = (uint32_t)(c % CPW) * CH + 4u * n;
        const uint8_t *wp = win + w * wbytes + base;
        uint32_t L[NG][4];
#pragma unroll
        for (int g = 0; g < NG; g++)
#pragma unroll
            for (int i = 0; i < 4; i++) L[g][i] = *(const uint32_t *)(wp + (size_t)(8 * g + 4 * h + i) * STRIDE);
        v16i acc[4][2];
#pragma unroll
        for (int t = 0; t < 4; t++) acc[t][0] = acc[t][1] = (v16i){};
#pragma unroll
        for (int g = 0; g < NG; g++) {
            uint32_t D[4];
            transpose4(L[g], D);
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const v4i a0 = sA[((g * 2 + q) * 2 + 0) * 64 + lane];
                const v4i a1 = sA[((g * 2 + q) * 2 + 1) * 64 + lane];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const v4i b = {(int)(D[t] >> (4 * q)), (int)(D[t] >> (4 * q + 1)),
                                   (int)(D[t] >> (4 * q + 2)), (int)(D[t] >> (4 * q + 3))};
                    acc[t][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b, acc[t][0], 0, 0, 0);
                    acc[t][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b, acc[t][1], 0, 0, 0);
                }
            }
        }
        // lane (n, h): acc[t][mb][reg] = count for output mb*4 + (reg>>2), bit (reg&3) + 4h,
        // position 4n + t.  out[i]: byte t = that output's nibble at position 4n + t.
        uint32_t out[R];
#pragma unroll
        for (int mb = 0; mb < 2; mb++)
#pragma unroll
            for (int o = 0; o < 4; o++) {
                uint32_t v = 0;
#pragma unroll
                for (int t = 0; t < 4; t++)
                    v |= nibble(acc[t][mb][4 * o], acc[t][mb][4 * o + 1], acc[t][mb][4 * o + 2],
                                acc[t][mb][4 * o + 3]) << (8 * t);
                out[mb * 4 + o] = v;
            }
#pragma unroll
        for (int i = 0; i < R; i++) {
            const uint32_t other = (uint32_t)__shfl_xor((int)out[i], 32, 64);
            out[i] = h ? (other | (out[i] << 4)) : (out[i] | (other << 4));
        }
        uint8_t *op = win + w * wbytes + (size_t)K * STRIDE + base;
#pragma unroll
        for (int i = 0; i < 4; i++) *(uint32_t *)(op + (size_t)(4 * h + i) * STRIDE) = out[4 * h + i];
    }
}

// Variant 2: v_mfma_i32_16x16x64_i8.  Lane (c = l & 15, kg = l >> 4): element
// e = 4w + i <-> (row 8g + 4(kg >> 1) + i, bit 4(kg & 1) + w).  M-block mb =
// outputs 2mb, 2mb+1; C: lane holds rows 4kg..4kg+3 = output 2mb + (kg >> 1),
// bits 4(kg & 1)..+3.  Wave tile: 64 positions (16 lanes x 4) x all k rows,
// next chunk's rows loaded while this one multiplies.  afrag16[g][mb][lane].
typedef int v4c __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void mfma16_encode(uint8_t *win, const v4i *afrag, uint64_t nchunks) {
    __shared__ v4i sA[NG * 4 * 64];
    for (int i = threadIdx.x; i < NG * 4 * 64; i += 256) sA[i] = afrag[i];
    __syncthreads();
    constexpr uint32_t CH16 = 64, CPW16 = S / CH16;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, cl = lane & 15, kg = lane >> 4;
    const uint64_t wbytes = (uint64_t)(K + R) * STRIDE;
    const uint64_t step = (uint64_t)gridDim.x * 4;
    uint64_t c = (uint64_t)blockIdx.x * 4 + wave;
    auto load = [&](uint64_t ch, uint32_t (&L)[NG][4]) {
        const uint64_t cc = ch < nchunks ? ch : nchunks - 1;
        const uint8_t *wp = win + (cc / CPW16) * wbytes + (uint32_t)(cc % CPW16) * CH16 + 4u * cl;
#pragma unroll
        for (int g = 0; g < NG; g++)
#pragma unroll
            for (int i = 0; i < 4; i++)
                L[g][i] = *(const uint32_t *)(wp + (size_t)(8 * g + 4 * (kg >> 1) + i) * STRIDE);
    };
    uint32_t Ln[NG][4];
    if (c < nchunks) load(c, Ln);
    for (; c < nchunks; c += step) {
        uint32_t L[NG][4];
#pragma unroll
        for (int g = 0; g < NG; g++)
#pragma unroll
            for (int i = 0; i < 4; i++) L[g][i] = Ln[g][i];
#ifndef PROBE_NOLOAD
        load(c + step, Ln);  // next chunk in flight during the MFMAs
#else
#pragma unroll
        for (int g = 0; g < NG; g++)
#pragma unroll
            for (int i = 0; i < 4; i++) Ln[g][i] ^= (uint32_t)c;  // compute-only ceiling
#endif
        v4i acc[4][4];
#pragma unroll
        for (int t = 0; t < 4; t++)
#pragma unroll
            for (int mb = 0; mb < 4; mb++) acc[t][mb] = (v4i){};
#pragma unroll
        for (int g = 0; g < NG; g++) {
            uint32_t D[4];
            transpose4(L[g], D);
            const int sh = 4 * (kg & 1);
#pragma unroll
            for (int mb = 0; mb < 4; mb++) {
                const v4i a = sA[(g * 4 + mb) * 64 + lane];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const v4i b = {(int)(D[t] >> sh), (int)(D[t] >> (sh + 1)), (int)(D[t] >> (sh + 2)),
                                   (int)(D[t] >> (sh + 3))};
                    acc[t][mb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, acc[t][mb], 0, 0, 0);
                }
            }
        }
        uint32_t out[4];  // per mb: bytes t = nibbles of output 2mb + (kg >> 1)
#pragma unroll
        for (int mb = 0; mb < 4; mb++) {
            uint32_t v = 0;
#pragma unroll
            for (int t = 0; t < 4; t++) v |= nibble(acc[t][mb][0], acc[t][mb][1], acc[t][mb][2], acc[t][mb][3]) << (8 * t);
            const uint32_t other = (uint32_t)__shfl_xor((int)v, 16, 64);
            out[mb] = (kg & 1) ? (other | (v << 4)) : (v | (other << 4));
        }
        const uint64_t w = c / CPW16;
        uint8_t *op = win + w * wbytes + (size_t)K * STRIDE + (uint32_t)(c % CPW16) * CH16 + 4u * cl;
        // kg even stores mb 0,1; odd stores mb 2,3 (outputs 2mb + (kg >> 1))
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int mb = 2 * (kg & 1) + u;
            *(uint32_t *)(op + (size_t)(2 * mb + (kg >> 1)) * STRIDE) = out[mb];
        }
    }
}

int main() {
    gf_init();
    uint8_t C[R][K];
    for (int i = 0; i < R; i++)
        for (int j = 0; j < K; j++) C[i][j] = ginv((uint8_t)((K + i) ^ j));
    // A fragments: lane l, element e = 4w + i <-> (row 8g + 4h + i, bit 4q + w); row m = l & 31
    std::vector<int8_t> A((size_t)NG * 2 * 2 * 64 * 16);
    for (int g = 0; g < NG; g++)
        for (int q = 0; q < 2; q++)
            for (int mb = 0; mb < 2; mb++)
                for (int l = 0; l < 64; l++) {
                    const int m = l & 31, h = l >> 5, io = mb * 4 + (m >> 3), bp = m & 7;
                    for (int w = 0; w < 4; w++)
                        for (int i = 0; i < 4; i++) {
                            const int row = 8 * g + 4 * h + i, bit = 4 * q + w;
                            const uint8_t prod = gmul(C[io][row], (uint8_t)(1u << bit));
                            A[((((size_t)(g * 2 + q) * 2 + mb) * 64 + l) * 16) + 4 * w + i] =
                                (int8_t)((prod >> bp) & 1);
                        }
                }
    std::vector<int8_t> A16((size_t)NG * 4 * 64 * 16);
    for (int g = 0; g < NG; g++)
        for (int mb = 0; mb < 4; mb++)
            for (int l = 0; l < 64; l++) {
                const int m = l & 15, kg = l >> 4, io = 2 * mb + (m >> 3), bp = m & 7;
                for (int w = 0; w < 4; w++)
                    for (int i = 0; i < 4; i++) {
                        const int row = 8 * g + 4 * (kg >> 1) + i, bit = 4 * (kg & 1) + w;
                        const uint8_t prod = gmul(C[io][row], (uint8_t)(1u << bit));
                        A16[(((size_t)(g * 4 + mb) * 64 + l) * 16) + 4 * w + i] = (int8_t)((prod >> bp) & 1);
                    }
            }
    const uint64_t nwin = 16384;  // 16384 x 40 x 4096 = 2.7 GB
    const size_t wbytes = (size_t)(K + R) * STRIDE, total = nwin * wbytes;
    std::vector<uint8_t> h(total, 0);
    uint64_t s = 0x1234567;
    for (uint64_t w = 0; w < nwin; w++)
        for (int j = 0; j < K; j++) {
            uint8_t *p = &h[w * wbytes + (size_t)j * STRIDE];
            for (uint32_t b = 0; b < S; b += 8) {
                s = s * 6364136223846793005ull + 1442695040888963407ull;
                memcpy(p + b, &s, 8);
            }
        }
    uint8_t *d;
    v4i *da;
    CK(hipMalloc(&d, total));
    CK(hipMalloc(&da, A.size()));
    CK(hipMemcpy(d, h.data(), total, hipMemcpyHostToDevice));
    CK(hipMemcpy(da, A.data(), A.size(), hipMemcpyHostToDevice));
    v4i *da16;
    CK(hipMalloc(&da16, A16.size()));
    CK(hipMemcpy(da16, A16.data(), A16.size(), hipMemcpyHostToDevice));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int variant = getenv("PROBE_VARIANT") ? atoi(getenv("PROBE_VARIANT")) : 16;
    const uint64_t nchunks = nwin * (variant == 16 ? S / 64 : CPW);
    for (int bpc : {1, 2, 3, 4, 8}) {
        const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)cus * bpc, (nchunks + 3) / 4);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        auto run = [&]() {
            if (variant == 16) hipLaunchKernelGGL(mfma16_encode, dim3(grid), dim3(256), 0, 0, d, da16, nchunks);
            else hipLaunchKernelGGL(mfma_encode, dim3(grid), dim3(256), 0, 0, d, da, nchunks);
        };
        run();
        CK(hipDeviceSynchronize());
        std::vector<float> ms;
        for (int it = 0; it < 10; it++) {
            CK(hipEventRecord(e0));
            run();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double alg = (double)nwin * (K + R) * S;
        printf("variant %d blocks/CU %d: %.3f ms  %.2f TB/s alg (k+r rows), %.2f TB/s source\n", variant, bpc,
               ms[5], alg / ms[5] / 1e9, (double)nwin * K * S / ms[5] / 1e9);
    }
    // check a sample of windows against the CPU encode
    std::vector<uint8_t> got(total);
    CK(hipMemcpy(got.data(), d, total, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint64_t w = 0; w < nwin; w += 97)
        for (int i = 0; i < R; i++)
            for (uint32_t p = 0; p < S; p++) {
                uint8_t v = 0;
                for (int j = 0; j < K; j++) v ^= gmul(C[i][j], h[w * wbytes + (size_t)j * STRIDE + p]);
                if (got[w * wbytes + (size_t)(K + i) * STRIDE + p] != v && bad++ < 5)
                    printf("mismatch w %llu out %d pos %u: got %02x want %02x\n", (unsigned long long)w, i, p,
                           got[w * wbytes + (size_t)(K + i) * STRIDE + p], v);
            }
#ifdef PROBE_NOLOAD
    printf("verify: skipped (compute-only build)\n");
    return 0;
#else
    printf("verify: %s (%zu bad bytes)\n", bad ? "FAIL" : "ok", bad);
    return bad ? 3 : 0;
#endif
}
