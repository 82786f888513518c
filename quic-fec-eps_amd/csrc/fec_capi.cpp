// fec_capi.cpp — C ABI (include/fecgpu.h) over the gfx950 kernels.
//
// Validation happens before any HIP call so argument errors are reported the
// same on hosts without a GPU.  There is no CPU fallback: without a device
// every compute entry point returns FECGPU_ERR_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/fecgpu.h"
#include "fec_internal.h"

using namespace fecgpu;


namespace {

thread_local std::string g_last_error;

ssize_t dev_err(hipError_t e, const char *what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return FECGPU_ERR_DEVICE;
}

#define HIP_TRY(expr, what)                          \
    do {                                             \
        hipError_t e_ = (expr);                      \
        if (e_ != hipSuccess) return dev_err(e_, what); \
    } while (0)

uint8_t host_gf_mul(uint8_t a, uint8_t b) {
    static constexpr GfTables t = make_gf_tables();
    if (!a || !b) return 0;
    return t.exp[t.log[a] + t.log[b]];
}
uint8_t host_gf_inv(uint8_t a) {
    static constexpr GfTables t = make_gf_tables();
    return t.exp[255 - t.log[a]];
}

struct EncTables {
    uint4 *ab = nullptr;
    uint32_t *c = nullptr;
    uint8_t *coef = nullptr;  // parity rows P[r][k] (non-Cauchy matrices: the decode plan reads them)
    uint32_t *bs = nullptr;   // plane masks [k][r][8] (runtime bit-sliced encode)
    uint8_t *rows = nullptr;  // parity rows P[r][k] of any matrix (the bit-sliced decode's plan)
};

uint8_t host_gf_pow(uint8_t a, int n) {  // a^n, 0^0 = 1
    static constexpr GfTables t = make_gf_tables();
    if (n == 0) return 1;
    if (a == 0) return 0;
    return t.exp[(t.log[a] * n) % 255];
}

// Parity rows P[i*k + j] of the code's systematic generator:
// Cauchy C[i][j] = inv((k+i) ^ j), the systematic Vandermonde matrix —
// V[i][j] = i^j over points 0..k+r-1 times the inverse of its top k x k block
// (Backblaze JavaReedSolomon / klauspost / reed-solomon-erasure construction) —
// or RFC 8681 RLC rows (fec_spec.h rlc_coefs).
void host_parity_rows(const fecgpu_code *code, std::vector<uint8_t> &P) {
    const int k = code->k, r = code->r;
    P.assign((size_t)r * k, 0);
    if (code->matrix == FECGPU_MATRIX_RLC) {  // RFC 8681 coefficients, one repair_key per row
        for (int i = 0; i < r; i++) rlc_coefs((uint32_t)code->rlc_key + i, k, code->rlc_dt, &P[(size_t)i * k]);
        return;
    }
    if (code->matrix == FECGPU_MATRIX_CAUCHY) {
        for (int i = 0; i < r; i++)
            for (int j = 0; j < k; j++) P[(size_t)i * k + j] = host_gf_inv((uint8_t)((k + i) ^ j));
        return;
    }
    // Gauss-Jordan inverse of the top block (distinct points: never singular)
    std::vector<uint8_t> M((size_t)k * 2 * k);
    for (int i = 0; i < k; i++)
        for (int j = 0; j < 2 * k; j++)
            M[(size_t)i * 2 * k + j] = j < k ? host_gf_pow((uint8_t)i, j) : (uint8_t)(j - k == i);
    for (int c = 0; c < k; c++) {
        int piv = c;
        while (!M[(size_t)piv * 2 * k + c]) piv++;
        if (piv != c)
            for (int j = 0; j < 2 * k; j++) std::swap(M[(size_t)piv * 2 * k + j], M[(size_t)c * 2 * k + j]);
        const uint8_t iv = host_gf_inv(M[(size_t)c * 2 * k + c]);
        for (int j = 0; j < 2 * k; j++) M[(size_t)c * 2 * k + j] = host_gf_mul(M[(size_t)c * 2 * k + j], iv);
        for (int i = 0; i < k; i++) {
            const uint8_t f = M[(size_t)i * 2 * k + c];
            if (i == c || !f) continue;
            for (int j = 0; j < 2 * k; j++) M[(size_t)i * 2 * k + j] ^= host_gf_mul(f, M[(size_t)c * 2 * k + j]);
        }
    }
    for (int i = 0; i < r; i++)
        for (int j = 0; j < k; j++) {
            uint8_t v = 0;
            for (int t = 0; t < k; t++)
                v ^= host_gf_mul(host_gf_pow((uint8_t)(k + i), t), M[(size_t)t * 2 * k + k + j]);
            P[(size_t)i * k + j] = v;
        }
}

constexpr int kPipeSlots = 3;

// Streams, events and device staging slots of the host-pointer pipeline.
struct HostPipe {
    int dev = 0;
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    hipEvent_t h2d_done[kPipeSlots] = {}, comp_done[kPipeSlots] = {}, d2h_done[kPipeSlots] = {};
    uint8_t *slot[kPipeSlots] = {};
    size_t slot_bytes = 0;
};

}  // namespace

struct fecgpu_ctx {
    std::vector<int> devs;
    std::mutex mu;
    // (device, k, r, matrix, rlc_key, rlc_dt) -> encode tables (and parity rows) on that device
    std::map<std::tuple<int, int, int, int, int, int>, EncTables> enc;
    // host-pointer staging per device
    std::map<int, std::pair<void *, size_t>> stage;
    // host-pointer pipelines, one per entry of devs (keyed by that index)
    std::map<int, HostPipe> pipes;
    // tuning knobs (fecgpu_ctx_set_tuning): 0 = automatic
    int grid_mult = 0;
    int blocks_per_cu = 0;
    int wpb_override = 0;
    // host pipeline: kernels store outputs straight into mapped pinned host
    // windows (bit 0 encode, bit 1 decode; bit 2: the kernels also read the
    // windows over PCIe, no H2D copy), chunk size in MiB.  cfg5 sweep (r01,
    // profiles/r01_cfg5_sweep.txt): decode zero-copy 12.2 ms vs 17.4 ms with
    // H2D + direct stores vs 26 ms with H2D + D2H; encode is H2D-bound either
    // way and its DMA copies beat kernel PCIe traffic (11.8 vs 12.5 ms).
    int host_direct = 6;
    int host_chunk_mb = 128;
    // GF encode by the bit-sliced kernel where the code has one (DESIGN.md §GF bit-slicing)
    int bitslice = 1;
    // per-connection encoders / decoders launch on a small pool of streams per
    // device owned by the ctx (round robin), not one stream per object: a
    // server holds thousands of connections, the GPU has few hardware queues
    int conn_nstreams = 4;
    uint32_t conn_rr = 0;
    std::map<int, std::vector<hipStream_t>> conn_streams;
    // pinned blocks freed by per-connection objects, by size, for the next ones
    std::multimap<size_t, void *> pinned_cache;
    size_t pinned_cached = 0;
    size_t pinned_cache_cap = (size_t)1 << 30;
    // bit-sliced encode in group mode: passes per group at the longest window
    int bs_passes = 8;
    // bit-sliced encode of short uniform rows with gathered stores
    // (gf_encode_bs_gs_kernel): 1 on, 0 the flat bit-sliced kernel
    int gs = 1;
    // GF decode of Cauchy k 16 r 4 on uniform short rows by the bit-sliced
    // syndrome kernel (gf_decode_bs_gs_kernel): 1 on, 0 the table decode
    int bsdec = 1;
    // wide decode (k + r > 64): stage 1 by plane picks skips the missing rows
    // (1, default) instead of reading the rows the plan zeroed (0)
    int wide_mask = 1;
    int sw_group = 4;  // sliding-window encode: repairs per combine job (1, 2, 4, 8)
    int sw_stream = kSwStreamDefault;  // sliding-window encode: 0 combine jobs, 1..5 streaming
                                       // (dwords per lane), kSwStreamAuto per symbol size
    int sw_long_min = kSwSmallE + 1;  // sliding-window decode: unknowns that force the long-system path
    uint64_t sw_log_entries = 0;      // long-system operation log: fixed size (tuning), 0 = automatic
    uint64_t sw_log_seen = 0;         // the largest log an overflow asked for on this ctx
    // FECGPU_CHECK builds: bytes taken off the end of every checked range, so a
    // test can see the checker fire on a correct kernel ("check_shrink")
    int check_shrink = 0;
    // fault injection for tests ("fault_launches"): the next N launches of the
    // sliding-window encoder objects fail with FECGPU_ERR_DEVICE, launching nothing
    int fault_launches = 0;
    // sliding-window calls: device scratch slots and the last call's end event, per device
    std::map<int, std::vector<std::pair<void *, size_t>>> sw_scratch;
    std::map<int, hipEvent_t> sw_event;
    std::map<int, SwSticky *> sw_sticky;  // asynchronous decodes' error flags, per device
    std::map<int, ChkRec *> chk_rec;      // FECGPU_CHECK builds: the index-checking kernels' fault record
    struct LbState {
        void *mem = nullptr;
        uint64_t nchunk = 0;
        uint32_t epoch = 0;
    };
    std::map<int, LbState> sw_lb;  // fused decode plan's look-back state, per device
    std::map<int, uint8_t *> rlc_tab;  // dense RFC 8681 coefficient table, per device (ctx_rlc_table)
    void *sw_host = nullptr;  // pinned staging of sliding-window decodes (ctx_sw_host)
    size_t sw_host_bytes = 0;
    // codes with k + r > 64: parity rows on each device, by (device, k, r, matrix, key, dt)
    std::map<std::tuple<int, int, int, int, int, int>, uint8_t *> wide_rows;
};

extern "C" {

int fecgpu_abi_version(void) { return FECGPU_ABI_VERSION; }

const char *fecgpu_strerror(ssize_t err) {
    switch (err) {
        case FECGPU_ERR_DONE: return "done";
        case FECGPU_ERR_BUFFER_TOO_SHORT: return "buffer too short";
        case FECGPU_ERR_INVALID_ARG: return "invalid argument";
        case FECGPU_ERR_UNSUPPORTED: return "unsupported";
        case FECGPU_ERR_DEVICE: return "device error";
        case FECGPU_ERR_UNRECOVERABLE: return "unrecoverable";
        case FECGPU_ERR_LIMIT: return "limit reached";
        default: return err >= 0 ? "ok" : "unknown error";
    }
}

const char *fecgpu_last_error(void) { return g_last_error.c_str(); }

ssize_t fecgpu_code_check(const fecgpu_code *code) {
    if (!code) return FECGPU_ERR_INVALID_ARG;
    if (code->scheme != FECGPU_SCHEME_XOR && code->scheme != FECGPU_SCHEME_GF256)
        return FECGPU_ERR_INVALID_ARG;
    if (code->framing != FECGPU_FRAMING_FIXED && code->framing != FECGPU_FRAMING_LENPREFIX)
        return FECGPU_ERR_INVALID_ARG;
    if (code->k < 1 || code->r < 1) return FECGPU_ERR_INVALID_ARG;
    if (code->k + code->r > (code->scheme == FECGPU_SCHEME_GF256 ? FECGPU_MAX_WIDE_N : FECGPU_MAX_K))
        return FECGPU_ERR_UNSUPPORTED;
    if (code->r > FECGPU_MAX_R) return FECGPU_ERR_UNSUPPORTED;
    if (code->scheme == FECGPU_SCHEME_XOR && code->r > code->k) return FECGPU_ERR_INVALID_ARG;
    if (code->scheme == FECGPU_SCHEME_GF256 && code->matrix != FECGPU_MATRIX_CAUCHY &&
        code->matrix != FECGPU_MATRIX_VANDERMONDE && code->matrix != FECGPU_MATRIX_RLC)
        return FECGPU_ERR_UNSUPPORTED;
    if (code->scheme == FECGPU_SCHEME_GF256 && code->matrix == FECGPU_MATRIX_RLC && code->rlc_dt > 15)
        return FECGPU_ERR_INVALID_ARG;
    if (code->poly != 0 && code->poly != 0x11D) return FECGPU_ERR_UNSUPPORTED;
    return 0;
}

}  // extern "C"

namespace fecgpu {
// Everything but the batch entry points takes codes of one 64-bit mask
ssize_t code_check_narrow(const fecgpu_code *code) {
    const ssize_t rc = fecgpu_code_check(code);
    if (rc) return rc;
    return code->k + code->r > FECGPU_MAX_K ? FECGPU_ERR_UNSUPPORTED : 0;
}
}  // namespace fecgpu

extern "C" {

ssize_t fecgpu_code_parity_rows(const fecgpu_code *code, uint8_t *out, size_t cap) {
    ssize_t rc = fecgpu_code_check(code);
    if (rc) return rc;
    const size_t n = (size_t)code->k * code->r;
    if (!out || cap < n) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (code->scheme == FECGPU_SCHEME_XOR) {
        for (int i = 0; i < code->r; i++)
            for (int j = 0; j < code->k; j++) out[(size_t)i * code->k + j] = (uint8_t)(j % code->r == i);
        return (ssize_t)n;
    }
    std::vector<uint8_t> P;
    host_parity_rows(code, P);
    std::memcpy(out, P.data(), n);
    return (ssize_t)n;
}

ssize_t fecgpu_ctx_new(const int *devs, int ndev, fecgpu_ctx **out) {
    if (!out || ndev < 0 || (ndev > 0 && !devs)) return FECGPU_ERR_INVALID_ARG;
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) {
        g_last_error = "no HIP device";
        return FECGPU_ERR_DEVICE;
    }
    auto *c = new fecgpu_ctx();
    if (ndev == 0) {
        int d = 0;
        HIP_TRY(hipGetDevice(&d), "hipGetDevice");
        c->devs.push_back(d);
    } else {
        for (int i = 0; i < ndev; i++) {
            if (devs[i] < 0 || devs[i] >= count) {
                delete c;
                return FECGPU_ERR_INVALID_ARG;
            }
            c->devs.push_back(devs[i]);
        }
    }
    *out = c;
    return 0;
}

ssize_t fecgpu_ctx_set_tuning(fecgpu_ctx *ctx, const char *key, int64_t value) {
    if (!ctx || !key) return FECGPU_ERR_INVALID_ARG;
    if (!std::strcmp(key, "grid_mult")) {
        if (value < 0 || value > 64) return FECGPU_ERR_INVALID_ARG;
        ctx->grid_mult = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "blocks_per_cu")) {
        if (value < 0 || value > 64) return FECGPU_ERR_INVALID_ARG;
        ctx->blocks_per_cu = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "host_direct")) {
        if (value < 0 || value > 7) return FECGPU_ERR_INVALID_ARG;
        ctx->host_direct = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "host_chunk_mb")) {
        if (value < 1 || value > 4096) return FECGPU_ERR_INVALID_ARG;
        ctx->host_chunk_mb = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "check_shrink")) {
        if (!FECGPU_CHECK) return FECGPU_ERR_UNSUPPORTED;  // release build: nothing is checked
        if (value < 0 || value > (1 << 20)) return FECGPU_ERR_INVALID_ARG;
        ctx->check_shrink = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "fault_launches")) {
        if (value < 0 || value > (1 << 20)) return FECGPU_ERR_INVALID_ARG;
        std::lock_guard<std::mutex> lk(ctx->mu);
        ctx->fault_launches = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "gs")) {
        if (value < 0 || value > 1) return FECGPU_ERR_INVALID_ARG;
        ctx->gs = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "bsdec")) {
        if (value < 0 || value > 1) return FECGPU_ERR_INVALID_ARG;
        ctx->bsdec = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "wide_mask")) {
        if (value < 0 || value > 1) return FECGPU_ERR_INVALID_ARG;
        ctx->wide_mask = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "bs_passes")) {
        if (value < 1 || value > 256) return FECGPU_ERR_INVALID_ARG;
        ctx->bs_passes = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "pinned_cache_mb")) {
        if (value < 0 || value > (1 << 20)) return FECGPU_ERR_INVALID_ARG;
        std::lock_guard<std::mutex> lk(ctx->mu);
        ctx->pinned_cache_cap = (size_t)value << 20;
        while (ctx->pinned_cached > ctx->pinned_cache_cap) {  // shrink now
            auto it = ctx->pinned_cache.begin();
            ctx->pinned_cached -= it->first;
            (void)hipHostFree(it->second);
            ctx->pinned_cache.erase(it);
        }
        return 0;
    }
    if (!std::strcmp(key, "conn_streams")) {
        if (value < 1 || value > 64) return FECGPU_ERR_INVALID_ARG;
        ctx->conn_nstreams = (int)value;  // objects created from now on
        return 0;
    }
    if (!std::strcmp(key, "sw_group")) {
        if (value != 1 && value != 2 && value != 4 && value != 8) return FECGPU_ERR_INVALID_ARG;
        ctx->sw_group = (int)value;  // calls and objects created from now on
        return 0;
    }
    if (!std::strcmp(key, "sw_stream")) {
        if (value < 0 || value > kSwStreamAuto) return FECGPU_ERR_INVALID_ARG;
        ctx->sw_stream = (int)value;  // calls and objects created from now on
        return 0;
    }
    if (!std::strcmp(key, "sw_long_min")) {
        if (value < 1 || value > (1 << 30)) return FECGPU_ERR_INVALID_ARG;
        ctx->sw_long_min = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "sw_log_entries")) {
        if (value < 0 || value > (1ll << 34)) return FECGPU_ERR_INVALID_ARG;
        ctx->sw_log_entries = (uint64_t)value;
        return 0;
    }
    if (!std::strcmp(key, "bitslice")) {
        if (value < 0 || value > 1) return FECGPU_ERR_INVALID_ARG;
        ctx->bitslice = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "wpb")) {
        if (value < 0 || value > kMaxWpb) return FECGPU_ERR_INVALID_ARG;
        ctx->wpb_override = (int)value;
        return 0;
    }
    return FECGPU_ERR_UNSUPPORTED;
}

void fecgpu_ctx_free(fecgpu_ctx *ctx) {
    if (!ctx) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto &kv : ctx->enc) {
        (void)hipSetDevice(std::get<0>(kv.first));
        (void)hipFree(kv.second.ab);
        (void)hipFree(kv.second.c);
        if (kv.second.rows) (void)hipFree(kv.second.rows);
        if (kv.second.bs) (void)hipFree(kv.second.bs);
    }
    for (auto &kv : ctx->stage) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second.first);
    }
    for (auto &kv : ctx->pinned_cache) (void)hipHostFree(kv.second);
    for (auto &kv : ctx->sw_scratch) {
        (void)hipSetDevice(kv.first);
        (void)hipDeviceSynchronize();
        for (auto &b : kv.second)
            if (b.first) (void)hipFree(b.first);
    }
    if (ctx->sw_host) (void)hipHostFree(ctx->sw_host);
    for (auto &kv : ctx->chk_rec) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
    }
    for (auto &kv : ctx->sw_sticky) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
    }
    for (auto &kv : ctx->sw_lb) {
        (void)hipSetDevice(kv.first);
        if (kv.second.mem) (void)hipFree(kv.second.mem);
    }
    for (auto &kv : ctx->rlc_tab) {
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
    }
    for (auto &kv : ctx->wide_rows) {
        (void)hipSetDevice(std::get<0>(kv.first));
        (void)hipFree(kv.second);
    }
    for (auto &kv : ctx->sw_event) {
        (void)hipSetDevice(kv.first);
        (void)hipEventDestroy(kv.second);
    }
    for (auto &kv : ctx->conn_streams) {
        (void)hipSetDevice(kv.first);
        for (hipStream_t st : kv.second) {
            (void)hipStreamSynchronize(st);
            (void)hipStreamDestroy(st);
        }
    }
    for (auto &kv : ctx->pipes) {
        HostPipe &hp = kv.second;
        (void)hipSetDevice(hp.dev);
        if (hp.h2d) (void)hipStreamSynchronize(hp.d2h);
        for (int i = 0; i < kPipeSlots; i++) {
            if (hp.slot[i]) (void)hipFree(hp.slot[i]);
            if (hp.h2d_done[i]) (void)hipEventDestroy(hp.h2d_done[i]);
            if (hp.comp_done[i]) (void)hipEventDestroy(hp.comp_done[i]);
            if (hp.d2h_done[i]) (void)hipEventDestroy(hp.d2h_done[i]);
        }
        if (hp.h2d) {
            (void)hipStreamDestroy(hp.h2d);
            (void)hipStreamDestroy(hp.comp);
            (void)hipStreamDestroy(hp.d2h);
        }
    }
    (void)hipSetDevice(cur);
    delete ctx;
}

ssize_t fecgpu_host_alloc(size_t bytes, void **out) {
    if (!out || bytes == 0) return FECGPU_ERR_INVALID_ARG;
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, bytes, hipHostMallocDefault), "hipHostMalloc");
    return 0;
}

void fecgpu_host_free(void *p) {
    if (p) (void)hipHostFree(p);
}

}  // extern "C"

namespace {

// Plane picks of the runtime-mask bit-sliced encode (fec_kernels.hip rbs4::) for parity rows P[r][k]: for source j, output i and output plane p,
// lo = the input planes q < 4 and hi = the planes q >= 4 (as bits q, q - 4)
// for which bit p of P[i][j] * 2^q is set; stored as the kernel's index format
// (kRbsDw4 dwords per 4 planes).  out: k * r * 2 * kRbsDw4 dwords.
void rbs_masks(const uint8_t *P, int k, int r, uint32_t *out) {
    static constexpr GfTables g = make_gf_tables();
    std::fill(out, out + (size_t)k * r * 2 * kRbsDw4, 0u);
    for (int j = 0; j < k; j++)
        for (int i = 0; i < r; i++) {
            const uint8_t c = P[(size_t)i * k + j];
            uint32_t *row = &out[((size_t)j * r + i) * 2 * kRbsDw4];  // this repair's 8 planes
            for (int p = 0; p < 8; p++) {
                uint32_t lo = 0, hi = 0;
                for (int q = 0; q < 8; q++) {
                    const uint8_t col = c ? g.exp[g.log[c] + q] : 0;
                    if ((col >> p) & 1) (q < 4 ? lo : hi) |= 1u << (q & 3);
                }
                // four-column units index register pairs (2 x index); bytes lo, hi
                // of plane p in dword p / 2
                row[p / 2] |= (lo * 2 | (hi * 2) << 8) << (16 * (p & 1));
            }
        }
}

// Encode tables for the code's parity rows on the current device, built once
// per ctx (and, for non-Cauchy matrices, the raw rows for the decode plan).
ssize_t get_enc_tables(fecgpu_ctx *ctx, const fecgpu_code *code, EncTables &out) {
    const int k = code->k, r = code->r;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    std::lock_guard<std::mutex> lk(ctx->mu);
    const bool rlc = code->matrix == FECGPU_MATRIX_RLC;
    auto key = std::make_tuple(dev, k, r, (int)code->matrix, rlc ? (int)code->rlc_key : 0,
                               rlc ? (int)code->rlc_dt : 0);
    auto it = ctx->enc.find(key);
    if (it != ctx->enc.end()) {
        out = it->second;
        return 0;
    }
    std::vector<uint8_t> P;
    host_parity_rows(code, P);
    std::vector<uint4> ab((size_t)k * r);
    std::vector<uint32_t> cc((size_t)k * r);
    for (int j = 0; j < k; j++)
        for (int i = 0; i < r; i++) {
            const CoefTab t = make_coef_tab(P[(size_t)i * k + j]);
            ab[(size_t)j * r + i] = make_uint4(t.a_lo, t.a_hi, t.b_lo, t.b_hi);
            cc[(size_t)j * r + i] = t.c;
        }
    EncTables t;
    HIP_TRY(hipMalloc(&t.ab, ab.size() * sizeof(uint4)), "hipMalloc");
    HIP_TRY(hipMalloc(&t.c, cc.size() * sizeof(uint32_t)), "hipMalloc");
    HIP_TRY(hipMemcpy(t.ab, ab.data(), ab.size() * sizeof(uint4), hipMemcpyHostToDevice), "hipMemcpy");
    HIP_TRY(hipMemcpy(t.c, cc.data(), cc.size() * sizeof(uint32_t), hipMemcpyHostToDevice), "hipMemcpy");
    {
        std::vector<uint32_t> m((size_t)k * r * 2 * kRbsDw4, 0);
        rbs_masks(P.data(), k, r, m.data());
        HIP_TRY(hipMalloc(&t.bs, m.size() * sizeof(uint32_t)), "hipMalloc");
        HIP_TRY(hipMemcpy(t.bs, m.data(), m.size() * sizeof(uint32_t), hipMemcpyHostToDevice), "hipMemcpy");
    }
    HIP_TRY(hipMalloc(&t.rows, P.size()), "hipMalloc");
    HIP_TRY(hipMemcpy(t.rows, P.data(), P.size(), hipMemcpyHostToDevice), "hipMemcpy");
    if (code->matrix != FECGPU_MATRIX_CAUCHY) t.coef = t.rows;
    ctx->enc[key] = t;
    out = t;
    return 0;
}

// Windows per workgroup: fill the 256 lanes with whole passes over the
// flattened column range while keeping the LDS footprint small enough for
// >= 4 workgroups per CU.
int choose_wpb(uint32_t ncol, uint32_t lds_per_win, uint32_t lds_budget) {
    int maxw = kMaxWpb;
    if (lds_per_win) maxw = std::max(1, std::min<int>(maxw, (int)(lds_budget / lds_per_win)));
    if (ncol == 0) return maxw;
    int best = 1;
    double best_u = -1;
    for (int w = 1; w <= maxw; w++) {
        const uint64_t slots = (uint64_t)w * ncol;
        const uint64_t passes = (slots + kBlock - 1) / kBlock;
        const double u = (double)slots / (double)(passes * kBlock);
        // prefer >= 2 passes per workgroup so setup is amortised
        const double score = u - (passes < 2 ? 0.05 : 0.0);
        if (score > best_u + 1e-9) {
            best_u = score;
            best = w;
        }
    }
    return best;
}

ssize_t validate_batch(const fecgpu_code *code, const void *win, const uint32_t *sym_len,
                       uint32_t sym_len_all, uint32_t stride, const uint64_t *win_off) {
    ssize_t rc = fecgpu_code_check(code);
    if (rc) return rc;
    if (!win) return FECGPU_ERR_INVALID_ARG;
    if (!win_off) {
        if (stride == 0 || (stride & 15)) return FECGPU_ERR_INVALID_ARG;
        if (!sym_len && sym_len_all > stride) return FECGPU_ERR_BUFFER_TOO_SHORT;
    } else if (stride) {  // ragged with a fixed symbol pitch
        if (stride & 15) return FECGPU_ERR_INVALID_ARG;
        if (!sym_len && sym_len_all > stride) return FECGPU_ERR_BUFFER_TOO_SHORT;
    }
    if (!sym_len && sym_len_all == 0) return FECGPU_ERR_INVALID_ARG;
    if (stride > FECGPU_MAX_SYMBOL || sym_len_all > FECGPU_MAX_SYMBOL) return FECGPU_ERR_UNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(win) & 15) != 0) return FECGPU_ERR_INVALID_ARG;
    return 0;
}

struct HostStage {
    // device copies for a host-pointer call
    uint8_t *win = nullptr;
    uint64_t *off = nullptr;
    uint32_t *len = nullptr;
    uint64_t *pres = nullptr;
    uint8_t *status = nullptr;
    size_t win_bytes = 0;
};

ssize_t stage_alloc(fecgpu_ctx *ctx, size_t bytes, void **p) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    auto &s = ctx->stage[dev];
    if (s.second < bytes) {
        if (s.first) HIP_TRY(hipFree(s.first), "hipFree");
        s.first = nullptr;
        s.second = 0;
        HIP_TRY(hipMalloc(&s.first, bytes), "hipMalloc staging");
        s.second = bytes;
    }
    *p = s.first;
    return 0;
}

size_t host_window_bytes(const fecgpu_code *code, const uint64_t *win_off, const uint32_t *sym_len,
                         uint32_t sym_len_all, uint32_t stride, uint64_t nwin) {
    const int n = code->k + code->r;
    if (!win_off) return (size_t)nwin * n * stride;
    size_t mx = 0;
    for (uint64_t w = 0; w < nwin; w++) {
        const uint32_t S = sym_len ? sym_len[w] : sym_len_all;
        mx = std::max(mx, (size_t)win_off[w] + (size_t)n * (stride ? stride : ((S + 15u) & ~15u)));
    }
    return mx;
}

ssize_t launch_device(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, BatchArgs &a,
                      hipStream_t s, bool remote = false);
ssize_t run_host_pipelined(fecgpu_ctx *ctx, int di, const fecgpu_code *code, bool decode,
                           uint8_t *win, const uint32_t *sym_len, uint32_t sym_len_all,
                           uint32_t stride, uint64_t nwin, const uint64_t *present,
                           uint8_t *status);

// Host-pointer batch over every device of the ctx: contiguous window ranges
// [d*n/D, (d+1)*n/D), one host thread per device, each with its own pipeline
// (windows are independent, nothing is exchanged).
ssize_t run_host_multi(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, uint8_t *win,
                       const uint32_t *sym_len, uint32_t sym_len_all, uint32_t stride,
                       uint64_t nwin, const uint64_t *present, uint8_t *status) {
    const int nd = (int)ctx->devs.size();
    if (nd == 1)
        return run_host_pipelined(ctx, 0, code, decode, win, sym_len, sym_len_all, stride, nwin,
                                  present, status);
    for (int d = 0; d < nd; d++) ctx->pipes[d].dev = ctx->devs[d];  // create entries up front
    const size_t wbytes = (size_t)(code->k + code->r) * stride;
    std::vector<ssize_t> rcs(nd, 0);
    std::vector<std::string> errs(nd);
    auto part = [&](int d) {
        const uint64_t lo = nwin * d / nd, hi = nwin * (d + 1) / nd;
        if (hi > lo)
            rcs[d] = run_host_pipelined(ctx, d, code, decode, win + lo * wbytes,
                                        sym_len ? sym_len + lo : nullptr, sym_len_all, stride, hi - lo,
                                        present ? present + lo : nullptr, status ? status + lo : nullptr);
        if (rcs[d] < 0) errs[d] = g_last_error;  // thread_local: carry it back
    };
    std::vector<std::thread> th;
    for (int d = 1; d < nd; d++) th.emplace_back(part, d);
    part(0);
    for (auto &t : th) t.join();
    for (int d = 0; d < nd; d++)
        if (rcs[d] < 0) {
            g_last_error = errs[d];
            return rcs[d];
        }
    return (ssize_t)nwin;
}

// GF codes with k + r > 64 (fec_wide.hip): device pointers, uniform stride.
// The parity rows go up once per code and device; the jobs, output lists and
// decode matrices live in a ctx scratch slot shared with the sliding-window
// calls (ordered by ctx_sw_begin / ctx_sw_end).
ssize_t run_wide(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, uint8_t *win, const uint64_t *win_off,
                 const uint32_t *sym_len, uint32_t sym_len_all, uint32_t stride, uint64_t nwin,
                 const uint64_t *present, uint8_t *status, uint32_t flags, hipStream_t s) {
    if (win_off || (flags & FECGPU_F_HOST_PTRS)) return FECGPU_ERR_UNSUPPORTED;
    const int k = code->k, r = code->r, n = k + r;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    uint8_t *P = nullptr;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        const auto key = std::make_tuple(dev, k, r, (int)code->matrix, (int)code->rlc_key, (int)code->rlc_dt);
        auto it = ctx->wide_rows.find(key);
        if (it == ctx->wide_rows.end()) {
            std::vector<uint8_t> rows;
            host_parity_rows(code, rows);
            // then [P | I] (r x (k + r)): the two-stage decode's syndrome block
            const size_t nP = rows.size();
            rows.resize(nP + (size_t)r * n);
            for (int i = 0; i < r; i++)
                for (int q = 0; q < n; q++)
                    rows[nP + (size_t)i * n + q] = q < k ? rows[(size_t)i * k + q] : (uint8_t)(q - k == i);
            // then the bit-sliced plane picks of P and of [P | I] (wide_masks)
            const size_t o_m = (rows.size() + 255) & ~size_t(255);
            std::vector<uint32_t> mP((size_t)k * r * 2 * kRbsDw4), mPI((size_t)n * r * 2 * kRbsDw4);
            rbs_masks(rows.data(), k, r, mP.data());
            rbs_masks(rows.data() + nP, n, r, mPI.data());
            rows.resize(o_m + (mP.size() + mPI.size()) * 4);
            std::memcpy(rows.data() + o_m, mP.data(), mP.size() * 4);
            std::memcpy(rows.data() + o_m + mP.size() * 4, mPI.data(), mPI.size() * 4);
            void *d = nullptr;
            HIP_TRY(hipMalloc(&d, rows.size()), "hipMalloc wide parity rows");
            HIP_TRY(hipMemcpy(d, rows.data(), rows.size(), hipMemcpyHostToDevice), "H2D wide parity rows");
            it = ctx->wide_rows.emplace(key, static_cast<uint8_t *>(d)).first;
        }
        P = it->second;
    }
    // per-window lengths: every window's columns up to the stride
    const uint32_t ncol = sym_len ? stride / 16u : (sym_len_all + 15u) / 16u;
    // plane picks (run_wide's row block: P, [P | I], then the picks of each)
    const uint32_t *mP = nullptr, *mPI = nullptr;
    if (ctx->bitslice && r >= 4) {
        const size_t o_m = ((size_t)r * k + (size_t)r * n + 255) & ~size_t(255);
        mP = reinterpret_cast<const uint32_t *>(P + o_m);
        mPI = mP + (size_t)k * r * 2 * kRbsDw4;
    }
    ssize_t rc = ctx_sw_begin(ctx, s);
    if (rc) return rc;
    ChkRec *chk = nullptr;
    rc = ctx_chk_record(ctx, &chk);
    if (rc) return rc;
    {
        // the two-stage decode (fec_wide.hip; plane picks when bitslice is on and r >= 4)
        const auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
        const size_t o_out = up(nwin * sizeof(CombJob)), o_coef = o_out + up(nwin * kMaxR * sizeof(uint64_t));
        const size_t coef_bytes = decode ? nwin * kMaxR * (size_t)kMaxR : 0;
        const size_t o_j1 = o_coef + up(coef_bytes), o_o1 = o_j1 + (decode ? up(nwin * sizeof(CombJob)) : 0);
        const size_t o_syn = o_o1 + (decode ? up(nwin * (size_t)r * sizeof(uint64_t)) : 0);
        const size_t total = o_syn + (decode ? nwin * (size_t)r * stride : 0);
        void *scratch = nullptr;
        rc = ctx_sw_scratch(ctx, 11, total, &scratch);
        if (rc) return rc;
        uint8_t *b = static_cast<uint8_t *>(scratch);
        HIP_TRY(launch_wide(win, present, status, P, nwin, stride, ncol, k, r, decode, reinterpret_cast<CombJob *>(b),
                            reinterpret_cast<uint64_t *>(b + o_out), b + o_coef, s,
                            reinterpret_cast<CombJob *>(b + o_j1), reinterpret_cast<uint64_t *>(b + o_o1), b + o_syn,
                            mP, decode ? mPI : nullptr, chk, ctx->wide_mask != 0),
                "wide batch launch");
    }
    rc = ctx_chk_finish(ctx, s, decode ? "wide decode" : "wide encode");  // FECGPU_CHECK builds (release: nothing)
    if (rc) return rc;
    rc = ctx_sw_end(ctx, s);
    if (rc) return rc;
    if (flags & FECGPU_F_SYNC) HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    return (ssize_t)nwin;
}

ssize_t run_batch(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, uint8_t *win,
                  const uint64_t *win_off, const uint32_t *sym_len, uint32_t sym_len_all,
                  uint32_t stride, uint64_t nwin, const uint64_t *present, uint8_t *status,
                  uint32_t flags, void *stream) {
    if (!ctx) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = validate_batch(code, win, sym_len, sym_len_all, stride, win_off);
    if (rc) return rc;
    if (decode && (!present || !status)) return FECGPU_ERR_INVALID_ARG;
    if (nwin == 0) return 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (code->k + code->r > FECGPU_MAX_K)
        return run_wide(ctx, code, decode, win, win_off, sym_len, sym_len_all, stride, nwin, present, status, flags,
                        s);

    // host pointers, uniform layout: chunked copy/compute pipeline on every device
    if ((flags & FECGPU_F_HOST_PTRS) && !win_off)
        return run_host_multi(ctx, code, decode, win, sym_len, sym_len_all, stride, nwin, present,
                              status);
    // host pointers, ragged layout: stage everything once, synchronously
    HostStage hs;
    int prev_dev = -1;
    if (flags & FECGPU_F_HOST_PTRS) {
        HIP_TRY(hipGetDevice(&prev_dev), "hipGetDevice");
        HIP_TRY(hipSetDevice(ctx->devs[0]), "hipSetDevice");
        hs.win_bytes = host_window_bytes(code, win_off, sym_len, sym_len_all, stride, nwin);
        const size_t o_off = (hs.win_bytes + 255) & ~size_t(255);
        const size_t o_len = o_off + (win_off ? ((nwin * 8 + 255) & ~size_t(255)) : 0);
        const size_t o_pres = o_len + (sym_len ? ((nwin * 4 + 255) & ~size_t(255)) : 0);
        const size_t o_stat = o_pres + (decode ? ((nwin * 8 + 255) & ~size_t(255)) : 0);
        const size_t total = o_stat + (decode ? nwin : 0) + 256;
        void *base = nullptr;
        rc = stage_alloc(ctx, total, &base);
        if (rc) return rc;
        uint8_t *b = static_cast<uint8_t *>(base);
        hs.win = b;
        HIP_TRY(hipMemcpyAsync(hs.win, win, hs.win_bytes, hipMemcpyHostToDevice, s), "H2D win");
        if (win_off) {
            hs.off = reinterpret_cast<uint64_t *>(b + o_off);
            HIP_TRY(hipMemcpyAsync(hs.off, win_off, nwin * 8, hipMemcpyHostToDevice, s), "H2D off");
        }
        if (sym_len) {
            hs.len = reinterpret_cast<uint32_t *>(b + o_len);
            HIP_TRY(hipMemcpyAsync(hs.len, sym_len, nwin * 4, hipMemcpyHostToDevice, s), "H2D len");
        }
        if (decode) {
            hs.pres = reinterpret_cast<uint64_t *>(b + o_pres);
            hs.status = b + o_stat;
            HIP_TRY(hipMemcpyAsync(hs.pres, present, nwin * 8, hipMemcpyHostToDevice, s), "H2D present");
        }
    }

    BatchArgs a{};
    a.win = hs.win ? hs.win : win;
    a.win_off = hs.win ? hs.off : win_off;
    a.sym_len = hs.win ? hs.len : sym_len;
    a.present = hs.win ? hs.pres : present;
    a.status = hs.win ? hs.status : status;
    a.nwin = nwin;
    a.S_all = sym_len_all;
    a.stride = stride;
    a.off_stride = win_off ? stride : 0;
    rc = launch_device(ctx, code, decode, a, s);
    if (rc) return rc;

    if (hs.win) {
        HIP_TRY(hipMemcpyAsync(win, hs.win, hs.win_bytes, hipMemcpyDeviceToHost, s), "D2H win");
        if (decode)
            HIP_TRY(hipMemcpyAsync(status, hs.status, nwin, hipMemcpyDeviceToHost, s), "D2H status");
        HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
        HIP_TRY(hipSetDevice(prev_dev), "hipSetDevice");
    } else if (flags & FECGPU_F_SYNC) {
        HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    }
    return (ssize_t)nwin;
}

#if FECGPU_CHECK
// The byte ranges a launch's symbol accesses may touch (BatchArgs::chk): the
// windows it reads (and writes in place), and the output rows when they are
// redirected (split repairs, outputs into mapped host windows).  Ragged
// windows are located from win_off (copied back: a debug build may wait).
ssize_t set_check_ranges(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, BatchArgs &a,
                         hipStream_t s) {
    const uint64_t k = code->k, r = code->r, n = a.nwin, base = reinterpret_cast<uint64_t>(a.win);
    const bool redirected = a.out_delta || a.out_wdelta;
    uint64_t lo = base, len;
    if (!a.win_off) {
        // in-place encode writes rows k..k+r-1 of the last window; redirected reads stop at row k
        len = (n - 1) * a.wpitch + ((!decode && redirected) ? k : k + r) * a.stride;
    } else {
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> sl(a.sym_len && !a.off_stride ? n : 0);
        HIP_TRY(hipMemcpyAsync(off.data(), a.win_off, n * 8, hipMemcpyDefault, s), "check: win_off");
        if (!sl.empty()) HIP_TRY(hipMemcpyAsync(sl.data(), a.sym_len, n * 4, hipMemcpyDefault, s), "check: sym_len");
        HIP_TRY(hipStreamSynchronize(s), "check: sync");
        int64_t mn = INT64_MAX, mx = INT64_MIN;
        for (uint64_t w = 0; w < n; w++) {
            uint64_t st = a.off_stride;
            if (!st) {
                const uint64_t S = std::min<uint64_t>(sl.empty() ? a.S_all : sl[w], FECGPU_MAX_SYMBOL);
                st = (S + 15) & ~uint64_t(15);
            }
            const int64_t o = (int64_t)off[w];
            mn = std::min(mn, o);
            mx = std::max(mx, o + (int64_t)((k + r) * st));
        }
        lo = base + (uint64_t)mn;
        len = (uint64_t)(mx - mn);
    }
    a.chk = ChkRange{};
    a.chk.lo[0] = lo;
    a.chk.n[0] = len;
    if (redirected) {
        if (decode) {  // recovered sources: rows 0..k-1 at + out_delta
            a.chk.lo[1] = lo + a.out_delta;
            a.chk.n[1] = len;
        } else {       // repairs: rows k..k+r-1 at + out_delta + w * out_wdelta
            a.chk.lo[1] = lo + a.out_delta + k * a.stride;
            a.chk.n[1] = (n - 1) * (a.wpitch + a.out_wdelta) + r * a.stride;
        }
    }
    for (int i = 0; i < kChkRanges; i++) a.chk.n[i] -= std::min<uint64_t>(a.chk.n[i], (uint64_t)ctx->check_shrink);
    return 0;
}
#endif

// Plan and launch one batch whose pointers are all device pointers.
ssize_t launch_device(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, BatchArgs &a,
                      hipStream_t s, bool remote) {
    ssize_t rc = 0;
    const int k = code->k, r = code->r, scheme = (int)code->scheme;
    const uint32_t *sym_len = a.sym_len;
    const uint64_t *win_off = a.win_off;
    const uint32_t sym_len_all = a.S_all, stride = a.stride;
    a.k = k;
    a.r = r;
    if (!a.wpitch) a.wpitch = (uint64_t)(k + r) * stride;
    for (int g = 0; g < kMaxR; g++) {
        uint64_t m = 0;
        if (g < r)
            for (int j = g; j < k; j += r) m |= 1ull << j;
        a.gmask[g] = m;
    }
    // column estimate for the windows-per-workgroup choice
    uint32_t ncol = 0;
    if (!sym_len) ncol = (sym_len_all + 15u) >> 4;
    else if (!win_off) ncol = stride >> 4;

    LaunchPlan p{};
    p.grid_mult = ctx->grid_mult;
    p.blocks_per_cu = ctx->blocks_per_cu;
    // XOR is pure streaming: HBM delivers most with few bytes in flight
    // (2 persistent workgroups per CU, ~8 MB chip-wide; scripts/read_probe.hip,
    // scripts/sweep.py).  GF kernels need full occupancy to hide VALU work.
    if (p.blocks_per_cu == 0 && p.grid_mult == 0 && scheme == FECGPU_SCHEME_XOR) p.blocks_per_cu = 2;
    // flat slot space when every window has the same geometry (GF decode
    // always plans per window in LDS, so it always runs in group mode)
    p.flat = !win_off && !sym_len && !(decode && scheme == FECGPU_SCHEME_GF256);
    a.ncol = (sym_len_all + 15u) >> 4;
    if (!decode) {
        if (scheme == FECGPU_SCHEME_GF256) {
            EncTables t;
            rc = get_enc_tables(ctx, code, t);
            if (rc) return rc;
            a.enc_ab = t.ab;
            a.enc_c = t.c;
            a.enc_bs = t.bs;
            p.lds_bytes = (uint32_t)(k * r * 20);
        }
        p.wpb = choose_wpb(ncol, 0, 0);
    } else {
        if (scheme == FECGPU_SCHEME_GF256) {
            EncTables t;
            rc = get_enc_tables(ctx, code, t);
            if (rc) return rc;
            a.coef = t.coef;  // non-Cauchy matrices: the plan reads the parity rows
            p.win_lds = gf_dec_win_lds(k, r);
            p.wpb = choose_wpb(ncol, p.win_lds, 40 * 1024);
            p.lds_bytes = p.win_lds * (uint32_t)p.wpb;
        } else {
            p.wpb = choose_wpb(ncol, 0, 0);
        }
    }
    // Per-window lengths (group mode): a group's last pass is partly idle by
    // half a pass on average, so give each group >= 16 passes at the longest
    // window (cfg4 encode: 5 -> 8 windows per group, -4 %, scripts/ab.py r01).
    if (sym_len && !win_off && ncol && !p.flat) {
        const int want = (int)((16u * kBlock + ncol - 1) / ncol);
        int cap = kMaxWpb;
        if (p.win_lds) cap = std::max(1, (int)((40u << 10) / p.win_lds));
        p.wpb = std::max(p.wpb, std::min(want, cap));
        if (p.win_lds) p.lds_bytes = p.win_lds * (uint32_t)p.wpb;
    }
    if (!decode && scheme == FECGPU_SCHEME_GF256 && !remote && ctx->bitslice &&
        bitslice_supported(k, r, (int)code->matrix)) {
        // column pairs in group mode; no tables.  Groups of >= 8 passes at the
        // longest window (a lane's unit is k sources x 32 B of heavy XOR work,
        // so a partly idle last pass costs more than in the table kernels).
        p.bitslice = true;
        p.matrix = (int)code->matrix;
        p.lds_bytes = 0;
        const uint32_t units = ncol ? (ncol + 1) / 2 : (uint32_t)((stride >> 4) + 1) / 2;
        const uint32_t want = (uint32_t)ctx->bs_passes * kBlock;
        p.wpb = units ? std::max(1, std::min<int>(kMaxWpb, (int)((want + units - 1) / units))) : kMaxWpb;
        // uniform short rows: whole windows per step, repairs stored through LDS
        // (gf_encode_bs_gs_kernel; both images within 64 KB), at the workgroups
        // the LDS allows (2 per CU at cfg3) unless a grid is forced
        if (p.flat && ctx->gs && ctx->wpb_override <= 0 && ncol && units <= (uint32_t)kBlock) {
            const uint32_t img = 2u * (uint32_t)r * ncol * 16u;  // one window, both images
            const uint32_t G = std::min<uint32_t>((uint32_t)kBlock / units, (64u << 10) / img);
            if (G >= 1) {
                p.bsgs = true;
                p.flat = false;
                p.wpb = (int)G;
                p.lds_bytes = G * img;
                if (p.grid_mult <= 0 && p.blocks_per_cu <= 0) p.grid_mult = 1;
            }
        }
    }
    else if (!decode && scheme == FECGPU_SCHEME_GF256 && !remote && ctx->bitslice && r >= kRbsMinR) {
        // no compiled masks for this code: the runtime-mask kernel, same unit
        // space and group sizing
        p.rbitslice = true;
        p.lds_bytes = 0;
        // units of kRbsCols columns (the group sizing above counted pairs)
        const uint32_t c16 = ncol ? ncol : stride >> 4;
        const uint32_t units = (c16 + kRbsCols - 1) / kRbsCols;
        const uint32_t want = (uint32_t)ctx->bs_passes * kBlock;
        p.wpb = units ? std::max(1, std::min<int>(kMaxWpb, (int)((want + units - 1) / units))) : kMaxWpb;
    }
    if (decode && scheme == FECGPU_SCHEME_GF256 && !remote && ctx->bsdec && ctx->bitslice && !win_off &&
        !sym_len && ncol && ctx->wpb_override <= 0 && bsdec_supported(k, r, (int)code->matrix)) {
        // whole windows per step, a lane per unit of two 16-B columns (at least
        // 3/4 of the lanes busy), the step's syndromes / recovered rows in one
        // LDS image within 64 KB, and the kernel's buffer resource over the
        // step's windows (G pitches < 2^31 B)
        const uint32_t units = (ncol + 1) / 2, nt = (uint32_t)kBsdBlock;
        const uint32_t G = std::min<uint32_t>(nt / std::max(units, 1u), nt / (uint32_t)(r * r));
        const uint32_t img = (uint32_t)r * ncol * 16u;
        if (units <= nt && G >= 1 && G * units * 4 >= 3u * nt && G * img <= (64u << 10) &&
            (uint64_t)G * a.wpitch < (1ull << 31)) {
            p.bsdec = true;
            p.wpb = (int)G;
            p.win_lds = 0;
            p.lds_bytes = bsd_lds_bytes(G, r, ncol);
            if (p.grid_mult <= 0 && p.blocks_per_cu <= 0) p.grid_mult = 1;
        }
    }
    if (remote) {  // PCIe-latency bound: as many workgroups as windows
        p.remote = true;
        p.flat = false;
        p.wpb = 1;
        if (p.win_lds) p.lds_bytes = p.win_lds;
    }
    if (ctx->wpb_override > 0 && !p.flat) {
        p.wpb = std::min(ctx->wpb_override, kMaxWpb);
        if (p.win_lds) {  // per-window decode regions must fit the workgroup's LDS
            p.wpb = std::max(1, std::min<int>(p.wpb, (int)((96u << 10) / p.win_lds)));
            p.lds_bytes = p.win_lds * (uint32_t)p.wpb;
        }
    }
    a.wpb = p.wpb;
    a.win_lds = p.win_lds;

#if FECGPU_CHECK
    rc = set_check_ranges(ctx, code, decode, a, s);
    if (rc) return rc;
#endif
    hipError_t e = decode ? launch_decode(scheme, a, p, s) : launch_encode(scheme, a, p, s);
    if (e != hipSuccess) return dev_err(e, decode ? "decode launch" : "encode launch");
#if FECGPU_CHECK
    HIP_TRY(hipStreamSynchronize(s), "check: sync");
    uint64_t nbad = 0, first = 0;
    HIP_TRY(take_bounds_faults(&nbad, &first), "check: read faults");
    if (nbad) {
        char msg[256];
        snprintf(msg, sizeof msg,
                 "bounds check: %s kernel made %llu symbol accesses outside its windows "
                 "(first at %#llx; windows [%#llx, +%llu))",
                 decode ? "decode" : "encode", (unsigned long long)nbad, (unsigned long long)first,
                 (unsigned long long)a.chk.lo[0], (unsigned long long)a.chk.n[0]);
        g_last_error = msg;
        return FECGPU_ERR_DEVICE;
    }
#endif
    return rc;
}

// Host-pointer batch with the uniform layout, pipelined:
// the windows are cut into ~64 MB chunks; chunk i's H2D copy (its own stream),
// kernel (compute stream) and D2H copy (its own stream) overlap with chunks
// i-1 and i+1 through three device staging slots and events.  Only the bytes
// each side needs cross PCIe: encode sends the k source rows and returns the r
// repair rows (2-D copies over the window pitch); decode sends whole windows
// and returns the k source rows plus status.  Pinned host memory
// (fecgpu_host_alloc) makes the copies asynchronous DMA.  When the caller's
// windows are pinned and mapped into the device's address space, the kernels
// store their outputs (repairs / recovered sources) straight into them over
// PCIe instead: decode then moves e rows per window device->host instead of
// k, and the D2H direction carries only the bytes that changed.
ssize_t run_host_pipelined(fecgpu_ctx *ctx, int di, const fecgpu_code *code, bool decode,
                           uint8_t *win, const uint32_t *sym_len, uint32_t sym_len_all,
                           uint32_t stride, uint64_t nwin, const uint64_t *present,
                           uint8_t *status) {
    const int k = code->k, r = code->r;
    const size_t wbytes = (size_t)(k + r) * stride;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev), "hipGetDevice");
    const int dev = ctx->devs[di];
    HIP_TRY(hipSetDevice(dev), "hipSetDevice");
    HostPipe &hp = ctx->pipes[di];
    hp.dev = dev;
    const uint64_t cw_max = std::max<uint64_t>(1, ((uint64_t)ctx->host_chunk_mb << 20) / wbytes);
    const size_t need = cw_max * wbytes;
    const size_t o_len = (need + 255) & ~size_t(255);
    const size_t o_pres = o_len + ((cw_max * 4 + 255) & ~size_t(255));
    const size_t o_stat = o_pres + ((cw_max * 8 + 255) & ~size_t(255));
    const size_t slot_bytes = o_stat + ((cw_max + 255) & ~size_t(255));
    if (!hp.h2d) {
        HIP_TRY(hipStreamCreateWithFlags(&hp.h2d, hipStreamNonBlocking), "stream");
        HIP_TRY(hipStreamCreateWithFlags(&hp.comp, hipStreamNonBlocking), "stream");
        HIP_TRY(hipStreamCreateWithFlags(&hp.d2h, hipStreamNonBlocking), "stream");
        for (int i = 0; i < kPipeSlots; i++) {
            HIP_TRY(hipEventCreateWithFlags(&hp.h2d_done[i], hipEventDisableTiming), "event");
            HIP_TRY(hipEventCreateWithFlags(&hp.comp_done[i], hipEventDisableTiming), "event");
            HIP_TRY(hipEventCreateWithFlags(&hp.d2h_done[i], hipEventDisableTiming), "event");
        }
    }
    if (hp.slot_bytes < slot_bytes) {
        HIP_TRY(hipDeviceSynchronize(), "sync");
        for (int i = 0; i < kPipeSlots; i++) {
            if (hp.slot[i]) HIP_TRY(hipFree(hp.slot[i]), "hipFree");
            hp.slot[i] = nullptr;
        }
        for (int i = 0; i < kPipeSlots; i++) HIP_TRY(hipMalloc(&hp.slot[i], slot_bytes), "hipMalloc slot");
        hp.slot_bytes = slot_bytes;
    }
    // device address of the caller's windows if they are mapped pinned memory
    uint8_t *hdev = nullptr;
    if (ctx->host_direct & (decode ? 2 : 1)) {
        hipPointerAttribute_t at{};
        void *dp = nullptr;
        if (hipPointerGetAttributes(&at, win) == hipSuccess && at.type == hipMemoryTypeHost &&
            hipHostGetDevicePointer(&dp, win, 0) == hipSuccess && dp)
            hdev = static_cast<uint8_t *>(dp);
        (void)hipGetLastError();  // a plain malloc pointer leaves an error behind
    }
    const bool zc = hdev && (ctx->host_direct & 4);
    const uint64_t nchunk = (nwin + cw_max - 1) / cw_max;
    for (uint64_t c = 0; c < nchunk; c++) {
        const int sl = (int)(c % kPipeSlots);
        const uint64_t w0 = c * cw_max, cw = std::min<uint64_t>(cw_max, nwin - w0);
        uint8_t *d = hp.slot[sl];
        uint8_t *h = win + w0 * wbytes;
        if (c >= (uint64_t)kPipeSlots) HIP_TRY(hipStreamWaitEvent(hp.h2d, hp.d2h_done[sl], 0), "wait");
        if (zc) {  // the kernel reads the host windows itself
            if (decode)
                HIP_TRY(hipMemcpyAsync(d + o_pres, present + w0, cw * 8, hipMemcpyHostToDevice, hp.h2d), "H2D");
        } else if (decode) {
            HIP_TRY(hipMemcpyAsync(d, h, cw * wbytes, hipMemcpyHostToDevice, hp.h2d), "H2D");
            HIP_TRY(hipMemcpyAsync(d + o_pres, present + w0, cw * 8, hipMemcpyHostToDevice, hp.h2d), "H2D");
        } else {
            HIP_TRY(hipMemcpy2DAsync(d, wbytes, h, wbytes, (size_t)k * stride, cw, hipMemcpyHostToDevice,
                                     hp.h2d), "H2D 2D");
        }
        if (sym_len)
            HIP_TRY(hipMemcpyAsync(d + o_len, sym_len + w0, cw * 4, hipMemcpyHostToDevice, hp.h2d), "H2D");
        HIP_TRY(hipEventRecord(hp.h2d_done[sl], hp.h2d), "record");
        HIP_TRY(hipStreamWaitEvent(hp.comp, hp.h2d_done[sl], 0), "wait");
        BatchArgs a{};
        a.win = zc ? hdev + w0 * wbytes : d;
        a.sym_len = sym_len ? reinterpret_cast<const uint32_t *>(d + o_len) : nullptr;
        a.present = decode ? reinterpret_cast<const uint64_t *>(d + o_pres) : nullptr;
        a.status = decode ? d + o_stat : nullptr;
        a.nwin = cw;
        a.S_all = sym_len_all;
        a.stride = stride;
        if (hdev && !zc) a.out_delta = reinterpret_cast<uint64_t>(hdev + w0 * wbytes) - reinterpret_cast<uint64_t>(d);
        ssize_t rc = launch_device(ctx, code, decode, a, hp.comp, zc);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(hp.comp_done[sl], hp.comp), "record");
        HIP_TRY(hipStreamWaitEvent(hp.d2h, hp.comp_done[sl], 0), "wait");
        if (hdev) {  // outputs already in host memory
            if (decode)
                HIP_TRY(hipMemcpyAsync(status + w0, d + o_stat, cw, hipMemcpyDeviceToHost, hp.d2h), "D2H");
        } else if (decode) {
            HIP_TRY(hipMemcpy2DAsync(h, wbytes, d, wbytes, (size_t)k * stride, cw, hipMemcpyDeviceToHost,
                                     hp.d2h), "D2H 2D");
            HIP_TRY(hipMemcpyAsync(status + w0, d + o_stat, cw, hipMemcpyDeviceToHost, hp.d2h), "D2H");
        } else {
            HIP_TRY(hipMemcpy2DAsync(h + (size_t)k * stride, wbytes, d + (size_t)k * stride, wbytes,
                                     (size_t)r * stride, cw, hipMemcpyDeviceToHost, hp.d2h), "D2H 2D");
        }
        HIP_TRY(hipEventRecord(hp.d2h_done[sl], hp.d2h), "record");
    }
    HIP_TRY(hipStreamSynchronize(hp.comp), "sync");
    HIP_TRY(hipStreamSynchronize(hp.d2h), "sync");
    HIP_TRY(hipSetDevice(prev), "hipSetDevice");
    return (ssize_t)nwin;
}

}  // namespace

namespace fecgpu {

ssize_t launch_batch(fecgpu_ctx *ctx, const fecgpu_code *code, bool decode, BatchArgs &a,
                     hipStream_t s, bool remote, int dev) {
    if (!ctx || !a.win) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = code_check_narrow(code);
    if (rc) return rc;
    if (a.nwin == 0) return 0;
    // the object's own device: its stream, pinned windows and tables live there
    const int d = dev >= 0 ? dev : ctx->devs[0];
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev), "hipGetDevice");
    if (prev != d) HIP_TRY(hipSetDevice(d), "hipSetDevice");
    rc = launch_device(ctx, code, decode, a, s, remote);
    if (prev != d) (void)hipSetDevice(prev);
    return rc;
}

}  // namespace fecgpu

namespace fecgpu {

// A stream of the ctx's per-connection pool on the current device (created on
// first use, round robin; freed with the ctx).
ssize_t ctx_conn_stream(fecgpu_ctx *ctx, int dev, hipStream_t *out) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::vector<hipStream_t> &v = ctx->conn_streams[dev];
    if ((int)v.size() < ctx->conn_nstreams) {
        hipStream_t st = nullptr;
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
        v.push_back(st);
        *out = st;
        return 0;
    }
    *out = v[ctx->conn_rr++ % v.size()];
    return 0;
}


ssize_t ctx_pinned_get(fecgpu_ctx *ctx, size_t bytes, void **host) {
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        auto it = ctx->pinned_cache.find(bytes);
        if (it != ctx->pinned_cache.end()) {
            *host = it->second;
            ctx->pinned_cached -= bytes;
            ctx->pinned_cache.erase(it);
            return 0;
        }
    }
    HIP_TRY(hipHostMalloc(host, bytes, hipHostMallocDefault), "hipHostMalloc");
    return 0;
}

ssize_t set_dev_error(hipError_t e, const char *what) { return dev_err(e, what); }

int choose_wpb_for(uint32_t ncol, uint32_t lds_per_unit, uint32_t lds_budget) {
    return choose_wpb(ncol, lds_per_unit, lds_budget);
}

int ctx_sw_group(const fecgpu_ctx *ctx) { return ctx->sw_group; }

int ctx_sw_stream(const fecgpu_ctx *ctx) { return ctx->sw_stream; }

int ctx_sw_long_min(const fecgpu_ctx *ctx) { return ctx->sw_long_min; }

uint64_t ctx_sw_log_entries(const fecgpu_ctx *ctx, uint64_t nsrc, uint64_t nrep) {
    if (ctx->sw_log_entries) return ctx->sw_log_entries;
    // a long system needs 2 (p + e + sum of its equations' unknowns) entries;
    // 8 per source and repair covers systems averaging ~3 unknowns per window
    return std::max<uint64_t>({(uint64_t)1 << 16, 8 * (nsrc + nrep), ctx->sw_log_seen});
}

void ctx_sw_log_grow(fecgpu_ctx *ctx, uint64_t entries) {
    if (!ctx->sw_log_entries) ctx->sw_log_seen = std::max(ctx->sw_log_seen, entries);
    else ctx->sw_log_entries = std::max(ctx->sw_log_entries, entries);
}

bool ctx_fault_take(fecgpu_ctx *ctx) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (ctx->fault_launches <= 0) return false;
    ctx->fault_launches--;
    g_last_error = "injected launch fault (tuning \"fault_launches\")";
    return true;
}

ssize_t ctx_sw_scratch(fecgpu_ctx *ctx, int slot, size_t bytes, void **p) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    std::vector<std::pair<void *, size_t>> &v = ctx->sw_scratch[dev];
    if ((int)v.size() <= slot) v.resize(slot + 1, {nullptr, 0});
    auto &b = v[slot];
    if (b.second < bytes) {
        const size_t want = std::max(bytes, b.second + b.second / 2);
        if (b.first) HIP_TRY(hipFree(b.first), "hipFree");
        b = {nullptr, 0};
        HIP_TRY(hipMalloc(&b.first, want), "hipMalloc sw scratch");
        b.second = want;
    }
    *p = b.first;
    return 0;
}

ssize_t ctx_sw_host(fecgpu_ctx *ctx, size_t bytes, void **p) {
    if (ctx->sw_host_bytes < bytes) {
        const size_t want = std::max(bytes, ctx->sw_host_bytes + ctx->sw_host_bytes / 2);
        if (ctx->sw_host) HIP_TRY(hipHostFree(ctx->sw_host), "hipHostFree");
        ctx->sw_host = nullptr;
        ctx->sw_host_bytes = 0;
        HIP_TRY(hipHostMalloc(&ctx->sw_host, want, hipHostMallocDefault), "hipHostMalloc sw staging");
        ctx->sw_host_bytes = want;
    }
    *p = ctx->sw_host;
    return 0;
}

ssize_t ctx_sw_sticky(fecgpu_ctx *ctx, SwSticky **p) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    SwSticky *&w = ctx->sw_sticky[dev];
    if (!w) {
        void *m = nullptr;
        HIP_TRY(hipMalloc(&m, sizeof(SwSticky)), "hipMalloc sw error flags");
        const hipError_t e = hipMemset(m, 0, sizeof(SwSticky));
        if (e != hipSuccess) {
            (void)hipFree(m);
            return dev_err(e, "hipMemset sw error flags");
        }
        w = static_cast<SwSticky *>(m);
    }
    *p = w;
    return 0;
}

ssize_t ctx_chk_record(fecgpu_ctx *ctx, ChkRec **p) {
    *p = nullptr;
    if (!FECGPU_CHECK) return 0;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    ChkRec *&w = ctx->chk_rec[dev];
    if (!w) {
        void *m = nullptr;
        HIP_TRY(hipMalloc(&m, sizeof(ChkRec)), "hipMalloc check record");
        const hipError_t e = hipMemset(m, 0, sizeof(ChkRec));
        if (e != hipSuccess) {
            (void)hipFree(m);
            return dev_err(e, "hipMemset check record");
        }
        w = static_cast<ChkRec *>(m);
    }
    *p = w;
    return 0;
}

ssize_t ctx_chk_finish(fecgpu_ctx *ctx, hipStream_t s, const char *what) {
    if (!FECGPU_CHECK) return 0;
    HIP_TRY(hipStreamSynchronize(s), "check: sync");
    ChkRec *d = nullptr;
    ssize_t rc = ctx_chk_record(ctx, &d);
    if (rc) return rc;
    ChkRec h{};
    HIP_TRY(hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost), "check: read record");
    if (h.bad) {
        const ChkRec z{};
        HIP_TRY(hipMemcpy(d, &z, sizeof(z), hipMemcpyHostToDevice), "check: reset record");
    }
    uint64_t nbad = 0, first = 0;
    HIP_TRY(take_bounds_faults(&nbad, &first), "check: read faults");
    if (!h.bad && !nbad) return 0;
    char msg[320];
    if (h.bad)
        snprintf(msg, sizeof msg, "bounds check: %s made %llu accesses outside their allocations (first: site %llu, index %llu)",
                 what, h.bad, h.first >> 48, h.first & 0xFFFFFFFFFFFFull);
    else
        snprintf(msg, sizeof msg, "bounds check: %s made %llu symbol accesses outside their rows (first at %#llx)", what,
                 (unsigned long long)nbad, (unsigned long long)first);
    g_last_error = msg;
    return FECGPU_ERR_DEVICE;
}

uint64_t ctx_check_shrink(const fecgpu_ctx *ctx) { return (uint64_t)ctx->check_shrink; }

ssize_t ctx_sw_lookback(fecgpu_ctx *ctx, uint64_t nchunk, SwLookback *lb, uint32_t *epoch) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    auto &st = ctx->sw_lb[dev];
    // layout: tickets (256 B), flags [cap] u32, aggregates [cap] and inclusive
    // prefixes [cap], 32 B (two uint4) per chunk each (fec_swdec.hip LbRec)
    auto bytes = [](uint64_t cap) { return 256 + cap * 4 + cap * 2 * kLbRecBytes; };
    if (st.nchunk < nchunk || st.epoch >= (1u << 29)) {
        const uint64_t cap = (std::max<uint64_t>(nchunk, std::max<uint64_t>(256, st.nchunk + st.nchunk / 2)) + 3) & ~3ull;
        if (st.mem) {
            HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
            HIP_TRY(hipFree(st.mem), "hipFree");
            st.mem = nullptr;
            st.nchunk = 0;
        }
        HIP_TRY(hipMalloc(&st.mem, bytes(cap)), "hipMalloc sw look-back");
        HIP_TRY(hipMemset(st.mem, 0, bytes(cap)), "hipMemset sw look-back");
        st.nchunk = cap;
        st.epoch = 0;
    }
    uint8_t *m = static_cast<uint8_t *>(st.mem);
    lb->ticket = reinterpret_cast<uint32_t *>(m);
    lb->flag = reinterpret_cast<uint32_t *>(m + 256);
    lb->agg = reinterpret_cast<uint4 *>(m + 256 + st.nchunk * 4);
    lb->inc = lb->agg + st.nchunk * (kLbRecBytes / sizeof(uint4));
    *epoch = ++st.epoch;
    return 0;
}

ssize_t ctx_rlc_table(fecgpu_ctx *ctx, hipStream_t s, const uint8_t **tab) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    uint8_t *&t = ctx->rlc_tab[dev];
    if (!t) {
        void *m = nullptr;
        HIP_TRY(hipMalloc(&m, kRlcTabBytes), "hipMalloc coefficient table");
        hipError_t e = launch_rlc_table(static_cast<uint8_t *>(m), s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            (void)hipFree(m);
            return dev_err(e, "coefficient table");
        }
        t = static_cast<uint8_t *>(m);
    }
    *tab = t;
    return 0;
}

ssize_t ctx_sw_wait(fecgpu_ctx *ctx) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    auto it = ctx->sw_event.find(dev);
    if (it != ctx->sw_event.end()) HIP_TRY(hipEventSynchronize(it->second), "hipEventSynchronize");
    return 0;
}

ssize_t ctx_sw_begin(fecgpu_ctx *ctx, hipStream_t s) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    auto it = ctx->sw_event.find(dev);
    if (it == ctx->sw_event.end()) {
        hipEvent_t ev = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
        HIP_TRY(hipEventRecord(ev, s), "hipEventRecord");
        ctx->sw_event[dev] = ev;
        return 0;
    }
    HIP_TRY(hipStreamWaitEvent(s, it->second, 0), "hipStreamWaitEvent");
    return 0;
}

ssize_t ctx_sw_end(fecgpu_ctx *ctx, hipStream_t s) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    HIP_TRY(hipEventRecord(ctx->sw_event[dev], s), "hipEventRecord");
    return 0;
}

void ctx_pinned_put(fecgpu_ctx *ctx, void *host, size_t bytes) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (ctx->pinned_cached + bytes <= ctx->pinned_cache_cap) {
        ctx->pinned_cache.emplace(bytes, host);
        ctx->pinned_cached += bytes;
        return;
    }
    (void)hipHostFree(host);
}

}  // namespace fecgpu

extern "C" {

ssize_t fecgpu_encode_batch(fecgpu_ctx *ctx, const fecgpu_code *code, uint8_t *win,
                            const uint64_t *win_off, const uint32_t *sym_len,
                            uint32_t sym_len_all, uint32_t stride, uint64_t nwin,
                            uint32_t flags, void *stream) {
    return run_batch(ctx, code, false, win, win_off, sym_len, sym_len_all, stride, nwin, nullptr,
                     nullptr, flags, stream);
}

ssize_t fecgpu_encode_split(fecgpu_ctx *ctx, const fecgpu_code *code, const uint8_t *src,
                            uint8_t *repair, const uint32_t *sym_len, uint32_t sym_len_all,
                            uint32_t stride, uint64_t nwin, uint32_t flags, void *stream) {
    if (!ctx || !repair) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = validate_batch(code, src, sym_len, sym_len_all, stride, nullptr);
    if (!rc) rc = code_check_narrow(code);
    if (rc) return rc;
    if ((reinterpret_cast<uintptr_t>(repair) & 15) != 0) return FECGPU_ERR_INVALID_ARG;
    if (flags & FECGPU_F_HOST_PTRS) return FECGPU_ERR_UNSUPPORTED;  // device pointers only
    if (nwin == 0) return 0;
    const uint64_t k = code->k, r = code->r;
    BatchArgs a{};
    // sources of window w at src + w*k*stride; its repair m lands at
    // repair + w*r*stride + m*stride = (source base) + (k + m)*stride + delta_w
    a.win = const_cast<uint8_t *>(src);  // never written: encode stores only repairs
    a.wpitch = k * stride;
    a.out_delta = reinterpret_cast<uint64_t>(repair) - reinterpret_cast<uint64_t>(src) - k * stride;
    a.out_wdelta = (r - k) * (uint64_t)stride;  // wraps when r < k
    a.sym_len = sym_len;
    a.nwin = nwin;
    a.S_all = sym_len_all;
    a.stride = stride;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    rc = launch_device(ctx, code, false, a, s);
    if (rc) return rc;
    if (flags & FECGPU_F_SYNC) HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    return (ssize_t)nwin;
}

ssize_t fecgpu_decode_batch(fecgpu_ctx *ctx, const fecgpu_code *code, uint8_t *win,
                            const uint64_t *win_off, const uint32_t *sym_len,
                            uint32_t sym_len_all, uint32_t stride, uint64_t nwin,
                            const uint64_t *present, uint8_t *status, uint32_t flags,
                            void *stream) {
    return run_batch(ctx, code, true, win, win_off, sym_len, sym_len_all, stride, nwin, present,
                     status, flags, stream);
}

ssize_t fecgpu_synth_batch(fecgpu_ctx *ctx, const fecgpu_code *code, int workload, uint64_t seed,
                           uint64_t w0, uint8_t *win, uint32_t *sym_len, uint32_t L,
                           uint32_t stride, uint64_t nwin, void *stream) {
    if (!ctx || !win) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = code_check_narrow(code);
    if (rc) return rc;
    if (workload != 0 && workload != 1) return FECGPU_ERR_INVALID_ARG;
    if (stride == 0 || (stride & 15)) return FECGPU_ERR_INVALID_ARG;
    if (workload == 0 && (L == 0 || L > stride)) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (workload == 1 && (stride < 9002 || !sym_len)) return FECGPU_ERR_BUFFER_TOO_SHORT;
    if (nwin > 0x7FFFFFFFull) return FECGPU_ERR_UNSUPPORTED;
    SynthArgs a{win, sym_len, seed, w0, nwin, L, stride, code->k, code->r, workload};
    hipError_t e = launch_synth(a, reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return dev_err(e, "synth launch");
    return (ssize_t)nwin;
}

ssize_t fecgpu_erasure_batch(fecgpu_ctx *ctx, const fecgpu_code *code, int erasure, uint64_t seed,
                             uint64_t w0, uint64_t *present, uint64_t nwin, void *stream) {
    if (!ctx || !present) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = code_check_narrow(code);
    if (rc) return rc;
    if (erasure < 0 || erasure > 2) return FECGPU_ERR_INVALID_ARG;
    EraseArgs a{present, seed, w0, nwin, code->k, code->r, (int)code->scheme, erasure};
    hipError_t e = launch_erasure(a, reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return dev_err(e, "erasure launch");
    return (ssize_t)nwin;
}

ssize_t fecgpu_digest_batch(fecgpu_ctx *ctx, const fecgpu_code *code, const uint8_t *win,
                            const uint32_t *sym_len, uint32_t sym_len_all, uint32_t stride,
                            uint64_t w0, uint64_t nwin, uint64_t *digest, void *stream) {
    if (!ctx || !win || !digest) return FECGPU_ERR_INVALID_ARG;
    ssize_t rc = code_check_narrow(code);
    if (rc) return rc;
    if (stride == 0 || (stride & 15)) return FECGPU_ERR_INVALID_ARG;
    if (!sym_len && (sym_len_all == 0 || sym_len_all > stride)) return FECGPU_ERR_INVALID_ARG;
    if (nwin > 0x7FFFFFFFull) return FECGPU_ERR_UNSUPPORTED;
    DigestArgs a{win, sym_len, digest, w0, nwin, sym_len_all, stride, code->k, code->r};
    hipError_t e = launch_digest(a, reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return dev_err(e, "digest launch");
    return (ssize_t)nwin;
}

}  // extern "C"
