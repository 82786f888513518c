// fec_internal.h — launch-side interface between the C ABI (fec_capi.cpp)
// and the gfx950 kernels (fec_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/fecgpu.h"
#include "fec_spec.h"

#ifndef FECGPU_CHECK
// Bounds-checked debug build (GPU AddressSanitizer is not available
// on this pool), lib/libfecgpu_check.so: every symbol load / store of the block
// kernels is checked against the byte ranges the host computed for the launch
// (ChkRange), and the sliding-window, wide and combine kernels check the
// indices of the rows, jobs, records and log entries they address against
// their allocations (CHK_IDX).  An access outside is not performed (loads
// give zero) and is recorded; the host fails the call with FECGPU_ERR_DEVICE.
#define FECGPU_CHECK 0
#endif

namespace fecgpu {

constexpr int kBlock = 256;   // 4 waves of 64
constexpr int kMaxWpb = 64;   // windows per workgroup (per-window header in static LDS)
constexpr int kMaxK = 64;
constexpr int kMaxR = 8;

// Geometry + decode inputs of one batch, passed by value as the kernel argument.
// Byte ranges [lo, lo + n) that symbol loads / stores of one launch may touch
// (FECGPU_CHECK builds; lo is an address, n == 0 = range unused).
constexpr int kChkRanges = 4;
struct ChkRange {
    uint64_t lo[kChkRanges], n[kChkRanges];
};

// FECGPU_CHECK builds: the fault record of the kernels that check indices
// (device memory, ctx_chk_record): faults, and the first one's site << 48 |
// index.  Release builds pass a null record and check nothing.
struct ChkRec {
    unsigned long long bad, first;
};
#if FECGPU_CHECK
__device__ __forceinline__ bool chk_index(ChkRec *rec, uint64_t i, uint64_t n, uint32_t site) {
    if (i < n) return true;
    if (rec) {
        atomicAdd(&rec->bad, 1ull);
        atomicCAS(&rec->first, 0ull, ((unsigned long long)site << 48) | (i & 0xFFFFFFFFFFFFull));
    }
    return false;
}
#define CHK_IDX(rec, i, n, site) ::fecgpu::chk_index((rec), (uint64_t)(i), (uint64_t)(n), (uint32_t)(site))
#else
#define CHK_IDX(rec, i, n, site) true
#endif

struct BatchArgs {
    uint8_t *win;
    const uint64_t *win_off;   // nullable: ragged windows
    const uint32_t *sym_len;   // nullable: every window S_all
    const uint64_t *present;   // decode
    uint8_t *status;           // decode
    const uint4 *enc_ab;       // encode tables [k][r] (TA lo/hi, TB lo/hi)
    const uint32_t *enc_c;     // encode tables [k][r] (TC)
    const uint8_t *coef;       // GF decode: parity rows P[r][k] of a non-Cauchy matrix (null: Cauchy)
    const uint32_t *enc_bs;    // runtime bit-sliced encode: plane indices [k][r][2][kRbsDw4]
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
    // runtime bit-sliced rows (launch_rbs_rows) of the wide decode's stage 1:
    // present words per window in `present` (0: every input row is read); an
    // absent row is read as zeros, with no memory access
    uint32_t pres_nw;
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
    bool rbitslice;      // GF encode by the runtime-mask bit-sliced kernel (any matrix)
    bool bsgs;           // bit-sliced encode with gathered stores (gf_encode_bs_gs_kernel)
    bool bsdec;          // GF decode by the bit-sliced syndrome kernel (gf_decode_bs_gs_kernel)
};

// GF encode of r parity rows goes to the runtime-mask bit-sliced kernel
// (fec_kernels.hip rbs::) when no compiled one exists: r >= this.
constexpr int kRbsMinR = 5;
// runtime bit-sliced encode: 16-B columns per lane (64 byte positions); its
// index table holds a byte per index, two planes per dword: kRbsDw4 dwords per
// 4 output planes (fec_kernels.hip rbs4::, fec_capi.cpp rbs_masks)
constexpr int kRbsCols = 4;
constexpr int kRbsDw4 = 2;

// GF encode of (k, r, matrix) has a compiled bit-sliced kernel.
bool bitslice_supported(int k, int r, int matrix);
// launch_rbs_rows with present masks reads through a raw buffer resource per
// wave over the windows its lanes touch: true when that span stays below 2^31 B
bool rbs_masked_ok(uint32_t ncol, uint64_t wpitch);
// GF decode of (k, r, matrix) has a bit-sliced syndrome kernel (gf_decode_bs_gs_kernel).
bool bsdec_supported(int k, int r, int matrix);
// bit-sliced syndrome decode: threads per workgroup; dynamic LDS of a workgroup taking G windows of
// ncol columns per step (fec_kernels.hip bsd::Lds): the image, then two
// buffers of solve tables (20 B per entry, r * r + 1 per window) and three
// words per window.  The plan uses r * r lanes per window: G * r * r <= threads.
constexpr int kBsdBlock = 512;
inline uint32_t bsd_lds_bytes(uint32_t G, int r, uint32_t ncol) {
    return G * (uint32_t)r * ncol * 16u + 2u * G * (uint32_t)(r * r + 1) * 20u + 6u * G * 4u;
}

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

// ---- sliding-window RLC (fecgpu_sw_*, fec_sw.cpp) ----------------------
// A combine job makes nout <= R output rows, each a GF(2^8) combination of
// nin contiguous input rows: repair generation (one output, the window's
// sources), decode syndromes (one output, xor of the received repair) and
// decode solves (up to 8 recovered sources from a system's syndromes).
struct CombJob {
    uint64_t in_off;    // input row q at in_base + in_off + q * stride
    uint64_t coef_off;  // coefficient bytes [nout][nin] at coef + coef_off
    uint64_t out_list;  // output u at out_base + outs[out_list + u]
    uint64_t xor_off;   // kNoXor, or every output ^= the row at xor_base + xor_off
    uint32_t nin, nout;
};
constexpr uint64_t kNoXor = ~0ull;
// CombJob::nout flag: the xor row is multiplied by the coefficient byte after
// the job's [nout][nin] block (output u: coef[nout * nin + u]) instead of
// added as is (a sliding-window decode's one-unknown system: syndrome and
// solve in one job, fec_swdec.hip small_solve)
constexpr uint32_t kCombXorScaled = 1u << 31;
constexpr int kSwMaxWindow = FECGPU_SW_MAX_WINDOW;
constexpr uint32_t kSwCoefPitch = 256;  // coefficient bytes per repair job

struct CombArgs {
    const CombJob *jobs;
    const uint8_t *coef;
    const uint64_t *outs;
    const uint8_t *in_base;
    uint8_t *out_base;
    const uint8_t *xor_base;
    uint64_t njobs;
    // optional device count of further jobs after the first njobs (grouped
    // encode's per-repair tail), at most extra_max; the grid covers the maximum
    const uint32_t *extra;
    uint64_t extra_max;
    int skip;                  // grouped encode jobs: skip zero coefficients (wave-uniform test)
    uint32_t ncol, stride;
    int wpb, nin_max, nout_max;
    uint32_t job_lds;
    uint32_t nx;
    // device-sized launch (decode): the job count is *extra alone, the widest
    // job *nin_dev (<= nin_max); each workgroup fits as many jobs as its
    // `budget` bytes of LDS hold at that width
    const uint32_t *nin_dev;
    int extra_shift;  // the device count counts 2^extra_shift units per job
    // device-sized launch: job groups dealt round-robin over every workgroup
    // instead of XCD-contiguous regions (a dense run of real jobs among empty
    // slots would otherwise land on one XCD)
    int interleave;
    // device-sized launch over mostly empty slots: each workgroup gathers the
    // non-empty jobs of its share (runs of kCombRun slots dealt round-robin)
    // into LDS and runs them in groups as large as `budget` holds
    int sparse;
    uint32_t budget;
    // nullable (sliding-window decode): the call's error bits; the launch does
    // nothing when a kSwErrStop bit is set (a bad header list or a failed
    // look-back recovers nothing)
    const uint32_t *err;
    ChkRange chk;  // FECGPU_CHECK builds: the arrays the jobs' rows lie in (inputs, xor rows, outputs)
    // every job has the same coefficient block (a block code's parity rows:
    // wide encode): [nout_max][nin_max] at coef, its tables built once per
    // workgroup and shared by the workgroup's jobs (job regions hold only their
    // output pointers), so more jobs fit a workgroup
    int shared_coef;
};
// sparse launches: slots per run (8 / 16 / 32 gave 0.201 / 0.198 / 0.208 ms per cfg7 decode call, r04)
constexpr uint32_t kCombRun = 16;
constexpr uint32_t kCombListLds = 256 * (uint32_t)sizeof(CombJob);   // sparse launches: one round's jobs
// LDS bytes per job of comb_kernel<R> at nin_max inputs
__host__ __device__ inline uint32_t comb_job_lds(int nin_max, int R) {
    const uint32_t rt = R == 1 ? 1u : (uint32_t)(R + 3) & ~3u;
    // nin_max input rows' tables plus one row for the xor row's multiplier
    return ((uint32_t)(nin_max + 1) * (16u * R + 4u * rt + 1u) + 8u * R + 8u + 15u) & ~15u;
}
// shared_coef launches: the shared tables, then a small region per job
__host__ __device__ inline uint32_t comb_shared_lds(int nin_max, int R) {
    const uint32_t rt = R == 1 ? 1u : (uint32_t)(R + 3) & ~3u;
    return ((uint32_t)nin_max * (16u * R + 4u * rt + 1u) + 15u) & ~15u;
}
__host__ __device__ inline uint32_t comb_job_small_lds(int R) {
    const uint32_t rt = R == 1 ? 1u : (uint32_t)(R + 3) & ~3u;
    return (16u * R + 4u * rt + 8u * (R + 1) + 15u) & ~15u;
}
hipError_t launch_comb(CombArgs a, int R, hipStream_t s);
// the runtime-mask bit-sliced encode over uniform windows of any k (fec_kernels.hip)
hipError_t launch_rbs_rows(uint8_t *win, uint64_t nwin, uint32_t ncol, uint32_t stride, uint64_t wpitch, int k,
                           int r, const uint32_t *masks, uint64_t out_delta, uint64_t out_wdelta, hipStream_t s,
                           const uint64_t *present = nullptr, uint32_t pres_nw = 0);
// GF block codes with k + r > 64 (fec_wide.hip): encode by the runtime-mask
// bit-sliced kernel (r >= 4) or a combine job per window; decode in two stages
// (syndromes of every repair with one coefficient block [P | I] for all
// windows, the missing sources' rows zeroed first; then x = T s per window over
// its r syndromes).  Scratch: stage-1 jobs [nwin], their outputs [nwin][r],
// syndrome rows [nwin][r][stride]; the parity-row block holds [P | I] after P.
hipError_t launch_wide(uint8_t *win, const uint64_t *present, uint8_t *status, const uint8_t *P_dev,
                       uint64_t nwin, uint32_t stride, uint32_t ncol, int k, int r, bool decode, CombJob *jobs,
                       uint64_t *outs, uint8_t *coef, hipStream_t s, CombJob *jobs1, uint64_t *outs1,
                       uint8_t *syn, const uint32_t *masks_P = nullptr, const uint32_t *masks_PI = nullptr,
                       ChkRec *chk = nullptr, bool mask_rows = true);

// encode: job t = repair t (coefficients at coef + t * kSwCoefPitch, output rep row t).
// group > 1: the repairs t0 = g * group .. t0 + group - 1 share job g when
// their windows fit in span_max sources together: one output per repair, the
// union of their windows as input rows, zero coefficients outside each window
// (at coef + t0 * kSwCoefPitch as [n][span]), so each source is loaded once
// per group instead of once per repair.  The repairs of groups that do not
// fit get one job each after the ngroups group jobs, counted in *tail
// (zeroed by the caller; sw_enc_jobs(nrep, group) jobs of room).
struct SwEncCoefArgs {
    const fecgpu_sw_repair *hdr;
    uint64_t nrep, nsrc;
    uint32_t stride;
    int max_window;
    int group, span_max;
    uint32_t *tail;
    CombJob *jobs;
    uint8_t *coef;
    uint64_t *outs;
    const uint8_t *rlc;  // nullable: the dense coefficient table (ctx_rlc_table)
};
hipError_t launch_sw_enc_coef(const SwEncCoefArgs &a, hipStream_t s);
// job slots of an encode's scratch (group jobs, per-repair tail, and a
// CombJob's room for the tail counter)
inline uint64_t sw_enc_jobs(uint64_t nrep, int group) {
    return group > 1 ? (nrep + group - 1) / group + nrep + 1 : nrep;
}

// Streaming encode (fec_swenc.hip): a workgroup takes a run of segments of
// up to kSwSeg consecutive repairs and streams each segment's source range
// once, every source multiplied into the accumulators of the repairs whose
// windows hold it.  Accumulator slot m of pass p carries the repairs
// p + m P, p + (m + A) P, ... of the segment in turn, which needs each window
// to start at or after the end of the one A P repairs before it (P = 1 and
// A = ceil(W / step) for a regular schedule; the workgroup picks the smallest
// P, then A <= kSwSlots, that its segment's headers allow).
constexpr int kSwSeg = 64;
constexpr int kSwSlots = 8;
constexpr int kSwStreamU = 8;  // sources per batch (a regular schedule's step divides it: whole batches)
struct SwStreamArgs {
    const uint8_t *src;
    uint8_t *rep;
    const fecgpu_sw_repair *hdr;
    uint64_t nsrc, nrep;
    uint32_t stride;
    uint32_t ncu;       // column units (C dwords each) of a symbol
    uint32_t cpass;     // column units per column pass (= block size)
    int max_window;     // table rows per repair
    int segcap;         // repairs per segment (<= kSwSeg)
    uint64_t nseg;      // segments; workgroup b takes [b nseg / grid, (b + 1) nseg / grid)
    uint32_t lds;       // dynamic LDS bytes
    const uint8_t *rlc;
    ChkRec *chk;        // FECGPU_CHECK builds: the fault record (release: null)  // nullable: the dense coefficient table (ctx_rlc_table)
};
// C: dwords per lane (1..5, dividing the row's dwords); LDS budget per workgroup in bytes
hipError_t launch_sw_stream(SwStreamArgs a, int C, uint32_t budget, hipStream_t s);
// LDS per streaming-encode repair: kSwStreamU zero tables and max_window
// tables (20 B each), coefficient bytes
inline uint32_t sw_stream_rep_lds(int max_window) {
    return (uint32_t)(max_window + kSwStreamU) * 20u + (uint32_t)max_window;
}
inline uint32_t sw_stream_lds(int segcap, int max_window) {
    return ((uint32_t)segcap * sw_stream_rep_lds(max_window) + kSwStreamU * 20u + 64u + 15u) & ~15u;
}

// ---- sliding-window decode, planned on the device (fec_swdec.hip) ----
// The lost sources are split into linked systems (two consecutive lost
// sources are linked when a received repair's window holds both).  A system
// of at most kSwSmallE unknowns and kSwSmallP equations is solved by one wave
// (Gauss-Jordan on [A | I]: solve jobs over its syndromes); a longer one by
// banded elimination (one wave plans it into an operation log, then waves
// replay the log over 256-byte column chunks of the data).
constexpr int kSwSmallE = 64;   // unknowns of a small system
constexpr int kSwSmallP = 96;   // equations (received repairs) of a small system
constexpr int kSwRows = 256;    // long systems: row slots (more rows alive at one column are reduced
                                // to a basis first: they span at most 255 columns, fec_swdec.hip)
constexpr int kSwPlanChunk = 2048;  // sources per block of the plan (one look-back launch; the
                                    // five-pass plan it replaced measured 0.236 vs 0.215 ms, r04)
// recovered sources per solve job (8, 4 or 2): the solve pass's critical path is
// its widest system's job, nin rows x outputs per lane (cfg7, r04: 4 gave 0.198
// vs 8 0.206 ms at 2 % loss, 1.70 vs 1.76 at 10 %)
constexpr int kSwSolveOut = 4;

// RFC 8681 coefficients at dt 15 depend on the repair key alone (a window takes
// a prefix of the key's sequence): the table holds every key's 255, one
// 256-byte row per key (byte 255 zero), 16 MiB per device (ctx_rlc_table)
constexpr uint32_t kRlcRow = 256;
constexpr uint64_t kRlcTabBytes = 65536ull * kRlcRow;
hipError_t launch_rlc_table(uint8_t *tab, hipStream_t s);

// SwDecCtr::err / SwSticky::err bits
constexpr uint32_t kSwErrHeader = 1u;    // a bad or unordered header: the call recovers nothing
constexpr uint32_t kSwErrCapacity = 2u;  // a long system's operation log (or the queue) did not fit:
                                         // that system stays lost (a larger log fixes it)
constexpr uint32_t kSwErrInternal = 4u;  // the plan's look-back gave up (never expected)
// the flags on which every launch after the plan stands down: the lost-list
// offsets and jobs would be built from a partial prefix (and stale scratch),
// and writing recovered rows from them could overwrite received ones
constexpr uint32_t kSwErrStop = kSwErrHeader | kSwErrInternal;
static_assert(kSwErrHeader == FECGPU_SW_ERR_HEADER && kSwErrCapacity == FECGPU_SW_ERR_CAPACITY &&
                  kSwErrInternal == FECGPU_SW_ERR_INTERNAL,
              "the public flags are the device's bits");
struct SwDecCtr {  // per call, written by the plan's last block
    uint32_t nlost, wmax, maxp, err;   // err: kSwErr* bits
    uint32_t pad3, nlong, npiv, recovered;  // queued long systems, pivot rows, recovered
    uint32_t maxin;                    // widest small-system solve (syndrome rows)
    uint32_t pad4;
    uint32_t nstart;                   // larger systems' first unknowns listed (starts)
    uint32_t pad0, pad1, pad2;
    unsigned long long nlog;           // long-system log entries
};
// one long system: lost[x0 .. x0 + e), candidate repairs [t_lo, t_hi); its
// forward / backward logs and first pivot row (set by the planner)
struct SwLong {
    uint32_t x0, e, t_lo, t_hi;
    unsigned long long fwd, bwd;
    uint32_t nfwd, nbwd, piv0, ok;
};
// a long system's operation: kind | slot a << 8 | slot b << 16, aux, a GF
// multiply table (CoefTab), aux2
struct SwOp {
    uint32_t op, aux;
    uint32_t tab[5];
    uint32_t aux2;
};
enum : uint32_t { kOpLoad = 1, kOpElim = 2, kOpStore = 3, kOpXBegin = 4, kOpXTerm = 5, kOpXEnd = 6, kOpXFree = 7,
                  kOpJump = 8 /* the log continues at aux | aux2 << 32 */ };
// Error flags of asynchronous decodes, OR-ed across calls on one device until
// read (fecgpu_sw_decode_errors); need = the largest log an overflow asked for
struct SwSticky {
    uint32_t err, pad;
    unsigned long long need;
};

struct SwDecArgs {
    const uint8_t *src_present, *rep_present;  // device
    const fecgpu_sw_repair *hdr;               // device
    uint8_t *stat;                             // [nsrc] out: 0 present / recovered, 1 lost
    uint64_t nsrc, nrep;
    uint32_t stride, S;
    int long_min;                              // systems with e >= long_min take the long path
    uint32_t *reach;                           // [nsrc + 1] rank[i] = lost sources before i
    uint32_t *rcnt;                            // [nsrc + 1] repfirst[i] = repairs starting before i
    uint32_t *lost, *reachL;                   // [nsrc] lost sources; prefix max of reach at each
    SwDecCtr *ctr;
    CombJob *syn_jobs;                         // [nrep] syndrome job of repair t (empty unless needed),
                                               // then [nsrc] the one-unknown systems' jobs by lost index
    uint64_t *syn_outs;                        // [nrep + nsrc]
    uint8_t *coef;                             // [nrep + nsrc][kSwCoefPitch]: syndrome coefficients
    CombJob *sol_jobs;                         // [nsrc] solve jobs of a small system in its unknowns' slots
    uint64_t *sol_outs;                        // [nsrc] their outputs (unknown x + d)
    uint8_t *sol_coef;                         // [nrep * kSwSmallE] coefficients (64 B per repair)
    SwLong *longs;                             // [long_cap]
    uint64_t long_cap;
    SwOp *log;                                 // [log_cap]
    uint64_t log_cap;
    uint32_t *synrow;                          // [nrep] long systems: syndrome row of repair t (~0: none)
    uint8_t *pivcoef;                          // [piv_cap][256] long systems: pivot rows' coefficients
    uint32_t *colpiv;                          // [nsrc] long systems: pivot row of column x (~0 free)
    uint32_t *pivhi;                           // [piv_cap] last unknown of each pivot row
    uint32_t *pivt;                            // [piv_cap] its repair index
    uint8_t *pivdata;                          // [piv_cap][stride] long systems: pivot rows' data
    uint64_t piv_cap;
    uint8_t *src;                              // the sources (replay writes recovered ones)
    const uint8_t *synd;                       // syndrome rows (g * stride)
    SwSticky *sticky;                          // nullable: asynchronous calls also raise errors here
    // plan: look-back state of the chunks, kept across
    // calls (ctx_sw_lookback): flags (epoch << 2 | state), aggregates, inclusive
    // prefixes, and the ticket counter that orders the chunks
    uint32_t *lb_flag;
    uint4 *lb_agg, *lb_inc;
    uint32_t *lb_ticket;  // [0] next chunk, [1] blocks done, [2] starts listed, [3] singles, [4] error bits
    uint32_t epoch;
    uint8_t *lkind;       // [nsrc] per lost index, from the plan: 0 member of a larger
                          // system, 1 recovered alone, 2 a larger system's first, 3 alone, lost
    uint32_t *starts;     // [nsrc] lost indices of the larger systems' first unknowns
                          // (ctr->nstart of them, in no particular order)
    const uint8_t *rlc;   // nullable: the dense coefficient table (kRlcRow bytes per repair key)
    uint64_t lb_cap;      // look-back records allocated (chunks)
    ChkRec *chk;          // FECGPU_CHECK builds: the fault record (release: null)
};
hipError_t launch_sw_dec_plan(const SwDecArgs &a, hipStream_t s);    // statuses, lost list, one-unknown systems
hipError_t launch_sw_dec_sys(const SwDecArgs &a, hipStream_t s);     // the larger systems
hipError_t launch_sw_dec_long(const SwDecArgs &a, hipStream_t s);    // long systems: logs, syndrome jobs
hipError_t launch_sw_dec_replay(const SwDecArgs &a, hipStream_t s);  // long systems: data

// fec_capi.cpp services for fec_sw.cpp: the thread's FECGPU_ERR_DEVICE text,
// the group-size choice of the block kernels, device scratch slots of the ctx
// (current device, grown on demand, contents not kept), and the ordering of
// sliding-window calls on one ctx (begin: `s` waits for the previous call's
// end; end: records it), which share that scratch.
ssize_t set_dev_error(hipError_t e, const char *what);
// Sliding-window encode launches on `s` with caller-owned device scratch:
// jobs (sw_enc_jobs(nrep, group) x sizeof(CombJob)), coefficients (nrep x
// kSwCoefPitch), output offsets (nrep x 8) (fec_sw.cpp; used by the
// per-connection encoder).  group: repairs per combine job (SwEncCoefArgs);
// hdr_host: a host-readable copy of hdr (nullable) that lets the launch skip
// the per-repair tail when every group fits.
ssize_t sw_encode_core(const uint8_t *src, uint64_t nsrc, uint8_t *rep, const fecgpu_sw_repair *hdr,
                       uint64_t nrep, int max_window, uint32_t S, uint32_t stride, void *jobs,
                       void *coef, void *outs, hipStream_t s, int group = 1,
                       const fecgpu_sw_repair *hdr_host = nullptr, int stream = 0, const uint8_t *rlc = nullptr,
                       ChkRec *chk = nullptr);
// the ctx's "sw_group" tuning (repairs per sliding-window encode job)
int ctx_sw_group(const fecgpu_ctx *ctx);
// the ctx's "sw_stream" tuning: 0 combine jobs, 1..5 the streaming encode
// with that many dwords per lane, kSwStreamAuto (default) chosen per symbol size
int ctx_sw_stream(const fecgpu_ctx *ctx);
constexpr int kSwStreamAuto = 6;
// the ctx's "sw_stream" default: 1 dword per lane (cfg7 A/B, r04: C = 1 / 2 /
// 3 / 4 / 5 gave 0.213 / 0.240 / 0.226 / 0.258 / 0.235 ms; the VALU, not the
// LDS table reads, bounds the kernel)
constexpr int kSwStreamDefault = 1;
int sw_stream_dwords(int stream, uint32_t S);
// "sw_long_min": systems of at least this many unknowns take the long-system
// path even when the small one would fit (default kSwSmallE + 1)
int ctx_sw_long_min(const fecgpu_ctx *ctx);
// entries of the long-system operation log a decode of nsrc / nrep reserves
// ("sw_log_entries" tuning, else grown past any overflow seen on this ctx)
uint64_t ctx_sw_log_entries(const fecgpu_ctx *ctx, uint64_t nsrc, uint64_t nrep);
void ctx_sw_log_grow(fecgpu_ctx *ctx, uint64_t entries);
// tests: true (and the thread's error text set) while the ctx's "fault_launches"
// count lasts, consuming one
bool ctx_fault_take(fecgpu_ctx *ctx);
int choose_wpb_for(uint32_t ncol, uint32_t lds_per_unit, uint32_t lds_budget);
ssize_t code_check_narrow(const fecgpu_code *code);  // fecgpu_code_check and k + r <= 64
ssize_t ctx_sw_scratch(fecgpu_ctx *ctx, int slot, size_t bytes, void **p);
// the ctx's pinned host staging block for sliding-window decodes (grown on
// demand; a decode synchronizes before returning, so the next may reuse it)
ssize_t ctx_sw_host(fecgpu_ctx *ctx, size_t bytes, void **p);
// FECGPU_CHECK builds: the current device's fault record of the index-checking
// kernels (allocated zeroed; release builds: null), and the end of a checked
// call: `s` synchronized, the record and the block kernels' symbol faults read
// and cleared, FECGPU_ERR_DEVICE (with the site) if any (release: nothing)
ssize_t ctx_chk_record(fecgpu_ctx *ctx, ChkRec **p);
ssize_t ctx_chk_finish(fecgpu_ctx *ctx, hipStream_t s, const char *what);
// bytes a test takes off the end of every checked range ("check_shrink")
uint64_t ctx_check_shrink(const fecgpu_ctx *ctx);
// the current device's sticky error word of asynchronous decodes (allocated zeroed)
ssize_t ctx_sw_sticky(fecgpu_ctx *ctx, SwSticky **p);
// Look-back state of the fused decode plan on the current device for nchunk
// chunks (zeroed when first allocated or grown): *epoch is this call's epoch
// (never 0; flags of earlier calls never match it).  ticket[0] hands out the
// chunks, ticket[1] counts finished blocks; the last block resets both, so
// every launch starts at 0.  Calls on one ctx are ordered (ctx_sw_begin), so
// one state per device serves them all.
struct SwLookback {
    uint32_t *flag, *ticket;
    uint4 *agg, *inc;  // kLbRecBytes per chunk each
};
constexpr uint64_t kLbRecBytes = 32;  // a chunk's look-back record: two uint4 (fec_swdec.hip LbRec)
ssize_t ctx_sw_lookback(fecgpu_ctx *ctx, uint64_t nchunk, SwLookback *lb, uint32_t *epoch);
// the current device's dense RFC 8681 coefficient table (kRlcTabBytes), drawn
// on `s` the first time and waited for once, so any stream may read it after
ssize_t ctx_rlc_table(fecgpu_ctx *ctx, hipStream_t s, const uint8_t **tab);
// waits until the current device's sliding-window calls issued so far have finished
ssize_t ctx_sw_wait(fecgpu_ctx *ctx);
ssize_t ctx_sw_begin(fecgpu_ctx *ctx, hipStream_t s);
ssize_t ctx_sw_end(fecgpu_ctx *ctx, hipStream_t s);

}  // namespace fecgpu
