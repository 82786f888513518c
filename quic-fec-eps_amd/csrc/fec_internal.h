// fec_internal.h — launch-side interface between the C ABI (fec_capi.cpp)
// and the gfx950 kernels (fec_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/fecgpu.h"
#include "fec_spec.h"

namespace fecgpu {

constexpr int kBlock = 256;   // 4 waves of 64
constexpr int kMaxWpb = 64;   // windows per workgroup (per-window header in static LDS)
constexpr int kMaxK = 64;
constexpr int kMaxR = 8;

// Geometry + decode inputs of one batch, passed by value as the kernel argument.
// Byte ranges [lo, lo + n) that symbol loads / stores of one launch may touch
// (FECGPU_CHECK builds; lo is an address, n == 0 = range unused).
struct ChkRange {
    uint64_t lo[2], n[2];
};

struct BatchArgs {
    uint8_t *win;
    const uint64_t *win_off;   // nullable: ragged windows
    const uint32_t *sym_len;   // nullable: every window S_all
    const uint64_t *present;   // decode
    uint8_t *status;           // decode
    const uint4 *enc_ab;       // encode tables [k][r] (TA lo/hi, TB lo/hi)
    const uint32_t *enc_c;     // encode tables [k][r] (TC)
    const uint8_t *coef;       // GF decode: parity rows P[r][k] of a non-Cauchy matrix (null: Cauchy)
    uint64_t nwin;
    uint64_t gmask[kMaxR];     // XOR: members of group g (bit j)
    uint64_t step_win;         // flat mode: (grid threads) / ncol
    uint32_t step_col;         // flat mode: (grid threads) % ncol
    uint32_t ncol;             // flat mode: 16-byte columns per symbol
    uint32_t nx;               // XCD regions (8, or 1 for tiny grids)
    uint32_t S_all;
    uint32_t stride;
    int k, r;
    int wpb;                   // group mode: windows per workgroup
    uint32_t win_lds;          // GF decode: LDS bytes per window region
    // Written symbols (repairs, recovered sources) go to p + out_delta for an
    // input address p: 0 in place; the host pipeline points it at the caller's
    // pinned host windows so outputs cross PCIe straight from the kernel.
    uint64_t out_delta;
    uint64_t out_wdelta;       // encode: + w * out_wdelta (split source / repair arrays)
    uint64_t wpitch;           // uniform layout: bytes from window w to w + 1 (0: (k + r) * stride)
    // ragged layout (win_off): symbol pitch of every window; 0 = packed
    // round_up(S_w, 16)
    uint32_t off_stride;
    ChkRange chk;              // FECGPU_CHECK builds: where this launch's symbols lie
};

struct LaunchPlan {
    bool flat;           // uniform S and stride: flat slot space
    int wpb;
    uint32_t lds_bytes;  // dynamic LDS per workgroup
    uint32_t win_lds;    // per-window region (GF decode)
    int grid_mult;       // resident blocks x grid_mult (tuning; 0 = automatic)
    int blocks_per_cu;   // persistent grid of CUs x blocks_per_cu (tuning; 0 = automatic)
    bool remote;         // windows in mapped host memory: one window per workgroup and
                         // deep load batches (PCIe latency, small batches)
    bool bitslice;       // GF encode by the bit-sliced kernel (compile-time matrix)
    int matrix;          // bitslice: the code's matrix (fecgpu_matrix)
};

// GF encode of (k, r, matrix) has a compiled bit-sliced kernel.
bool bitslice_supported(int k, int r, int matrix);

// Per-window LDS region of the GF decode kernel (fec_kernels.hip DecRegion):
// tables [k][R] uint4 (TA/TB) + [k][round_up(R, 4)] u32 (TC), input row byte
// offsets [round_up(k, 8)] u32, output row byte offsets [8] u32, input symbol
// list (64 B), output symbol list (16 B).
inline uint32_t gf_dec_win_lds(int k, int R) {
    const uint32_t r4 = (uint32_t)(R + 3) & ~3u, k8 = (uint32_t)(k + 7) & ~7u;
    return ((uint32_t)k * R * 16 + (uint32_t)k * r4 * 4 + k8 * 4 + 32 + 80 + 15) & ~15u;
}

hipError_t launch_encode(int scheme, const BatchArgs &a, const LaunchPlan &p, hipStream_t s);

// Library-internal entry (fec_conn.cpp): plan and launch one batch whose
// pointers the device can address (device memory or mapped pinned host
// memory) on `s`, on the ctx's device; asynchronous.  Geometry fields of `a`
// (win, win_off, sym_len, S_all, stride, off_stride, nwin, present, status)
// are the caller's; the rest is filled in.  dev: the device `s` belongs to
// (-1: the ctx's first device).
ssize_t launch_batch(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, BatchArgs &a,
                     hipStream_t s, bool remote = false, int dev = -1);
hipError_t launch_decode(int scheme, const BatchArgs &a, const LaunchPlan &p, hipStream_t s);

// FECGPU_CHECK builds: symbol accesses outside their launch's ChkRange since
// the last call (count, first offending address), then resets the record.
// Release builds: always {0, 0}.
hipError_t take_bounds_faults(uint64_t *count, uint64_t *first);

// Per-connection objects launch on a stream of the ctx's pool (fec_capi.cpp).
ssize_t ctx_conn_stream(fecgpu_ctx *ctx, int dev, hipStream_t *out);

// Pinned host blocks for per-connection objects: a block of exactly `bytes`
// from the ctx's cache of freed blocks, else a new hipHostMalloc; put returns
// it to the cache (up to "pinned_cache_mb"), else frees it.
ssize_t ctx_pinned_get(fecgpu_ctx *ctx, size_t bytes, void **host);
void ctx_pinned_put(fecgpu_ctx *ctx, void *host, size_t bytes);

struct SynthArgs {
    uint8_t *win;
    uint32_t *sym_len;
    uint64_t seed, w0, nwin;
    uint32_t L, stride;
    int k, r, workload;
};
hipError_t launch_synth(const SynthArgs &a, hipStream_t s);

struct EraseArgs {
    uint64_t *present;
    uint64_t seed, w0, nwin;
    int k, r, scheme, erasure;
};
hipError_t launch_erasure(const EraseArgs &a, hipStream_t s);

struct DigestArgs {
    const uint8_t *win;
    const uint32_t *sym_len;
    uint64_t *digest;
    uint64_t w0, nwin;
    uint32_t S_all, stride;
    int k, r;
};
hipError_t launch_digest(const DigestArgs &a, hipStream_t s);

}  // namespace fecgpu
