/*
 * fecgpu.h — C ABI of the MI355X FEC engine (drop-in boundary).
 *
 * What each entry point replaces.  The reference fec branch
 * (holzingk/quic-fec-eps, /root/reference/README.md:7) is not mounted: no
 * Rust source exists here to cite by file:line.  The entry points below
 * replace the branch's FEC encoder / decoder / frame API named in
 * BASELINE.json "north_star" (the per-packet calls the quiche Connection
 * makes on send and recv: SURVEY.md §3 call stacks A and B), and follow
 * quiche's own C FFI conventions (opaque handles, caller-owned buffers,
 * ssize_t results with negative error codes).
 * INTEGRATION.md shows the Rust `extern "C"` block a maintainer adds to
 * call them.
 *
 * Coding contract: SURVEY.md Appendix A (field GF(2^8)/0x11D, systematic
 * Cauchy rows C[i][j] = inv((k+i) ^ j) or interleaved XOR groups j mod r,
 * FIXED or LENPREFIX framing).
 *
 * Batch layout (A.4): window w is (k + r) symbols, sources 0..k-1 then
 * repairs k..k+r-1.  With win_off == NULL window w starts at
 * win + w*(k+r)*stride and every symbol occupies `stride` bytes (multiple of
 * 16, >= S).  With win_off != NULL window w starts at win + win_off[w]
 * (64-bit wrap-around add, so offsets may reach below `win`) and its symbol
 * stride is `stride` when nonzero (S_w is clamped to it), else
 * round_up(S_w, 16) (windows packed).  S_w = sym_len[w], or sym_len_all
 * when sym_len == NULL.  Bytes [S_w, stride) of a symbol are padding: the
 * kernels compute on whole 16-byte columns, so padding of written symbols
 * holds the code applied to the inputs' padding (zero in, zero out).
 *
 * Pointers are device pointers (hipMalloc / torch) unless FECGPU_F_HOST_PTRS
 * is set, in which case every buffer argument is host memory and the call
 * stages through device memory owned by the ctx and returns synchronously.
 * `stream` is a hipStream_t (NULL = the default stream).  Device-pointer
 * calls are asynchronous on that stream unless FECGPU_F_SYNC is set.
 *
 * Threading: a ctx may be used by one thread at a time; distinct ctxs are
 * independent.  Errors are returned, never raised; there is no CPU fallback.
 */
#ifndef FECGPU_H
#define FECGPU_H

#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FECGPU_ABI_VERSION 5  /* 2: REPAIR frames carry nsrc; decoder limits / recovered queue;
                                 3: fecgpu_code.rlc_key / rlc_dt, FECGPU_MATRIX_RLC, sliding-window
                                    RLC (fecgpu_sw_*, SW frames, fecgpu_frame.key / dt);
                                 4: the nsrc-carrying REPAIR frame has its own type 0xfec4 (ABI 1's
                                    0xfec1 layout had no nsrc and is rejected, never misparsed);
                                    sliding-window decode without a system-size cap;
                                 5: fecgpu_sw_decode_errors (asynchronous decodes' error flags) */

/* errors (mirror quiche's QUICHE_ERR_DONE = -1, QUICHE_ERR_BUFFER_TOO_SHORT = -2 style) */
enum fecgpu_error {
    FECGPU_ERR_DONE = -1,             /* nothing to do / no more data */
    FECGPU_ERR_BUFFER_TOO_SHORT = -2, /* caller buffer too small */
    FECGPU_ERR_INVALID_ARG = -3,
    FECGPU_ERR_UNSUPPORTED = -4,      /* valid but not implemented (e.g. r > 8) */
    FECGPU_ERR_DEVICE = -5,           /* HIP error or no GPU */
    FECGPU_ERR_UNRECOVERABLE = -6,    /* too many erasures in a window */
    FECGPU_ERR_LIMIT = -7,            /* decoder: open-window limit reached (release windows) */
};

enum fecgpu_scheme { FECGPU_SCHEME_XOR = 0, FECGPU_SCHEME_GF256 = 1 };
/* GF(2^8) parity rows: CAUCHY C[i][j] = inv((k+i) ^ j) (ISA-L cauchy1 layout);
 * VANDERMONDE = rows k.. of V * inv(V[0..k)), V[i][j] = i^j (points 0..k+r-1):
 * the systematic matrix of Backblaze JavaReedSolomon, klauspost/reedsolomon
 * and the Rust crate reed-solomon-erasure.
 * RLC = random linear code of RFC 8681 (Sliding Window RLC FEC schemes, m = 8)
 * in block form: parity row i holds the coefficients that RFC 8681 §3.6
 * generate_coding_coefficients(repair_key = rlc_key + i, cc_nb = k, dt =
 * rlc_dt) draws from the RFC 8682 TinyMT32 PRNG.  Not MDS: a window whose
 * present repairs leave the missing sources' system singular is reported
 * unrecoverable (decode uses every present repair, pivoting). */
enum fecgpu_matrix { FECGPU_MATRIX_CAUCHY = 0, FECGPU_MATRIX_VANDERMONDE = 1, FECGPU_MATRIX_RLC = 2 };
enum fecgpu_framing { FECGPU_FRAMING_FIXED = 0, FECGPU_FRAMING_LENPREFIX = 1 };

/* per-window decode status */
enum fecgpu_status { FECGPU_STATUS_OK = 0, FECGPU_STATUS_UNRECOVERABLE = 1 };

#define FECGPU_F_HOST_PTRS 1u
#define FECGPU_F_SYNC 2u

#define FECGPU_MAX_K 64       /* k + r of the per-connection objects, XOR and the workload helpers */
#define FECGPU_MAX_WIDE_N 256 /* k + r of GF(2^8) codes through fecgpu_encode_batch / fecgpu_decode_batch */
#define FECGPU_MAX_R 8
#define FECGPU_MAX_SYMBOL (1u << 24) /* symbol length / pitch limit (QUIC packets are < 64 KiB) */

typedef struct fecgpu_code {
    uint32_t scheme;  /* enum fecgpu_scheme */
    uint32_t matrix;  /* enum fecgpu_matrix (GF256 only) */
    uint32_t framing; /* enum fecgpu_framing */
    uint16_t k;       /* source symbols per window, 1..64 */
    uint16_t r;       /* repair symbols per window, 1..8; k + r <= 64, or (GF(2^8), batch entry
                         points only) <= 256; XOR: r <= k */
    uint32_t poly;    /* field polynomial, 0x11D (0 = default) */
    uint16_t rlc_key; /* MATRIX_RLC: repair_key of parity row 0 (row i: rlc_key + i mod 2^16) */
    uint8_t rlc_dt;   /* MATRIX_RLC: RFC 8681 density threshold DT, 0..15 (15 = dense:
                         every coefficient nonzero; else nonzero w.p. (DT + 1) / 16) */
    uint8_t reserved; /* 0 */
} fecgpu_code;

typedef struct fecgpu_ctx fecgpu_ctx;
struct fecgpu_sw_repair;  /* sliding-window repair header, defined below */

int         fecgpu_abi_version(void);
const char *fecgpu_strerror(ssize_t err);
/* message of the last FECGPU_ERR_DEVICE on this thread ("" if none) */
const char *fecgpu_last_error(void);
/* 0 if the code is valid and supported, else a negative error */
ssize_t     fecgpu_code_check(const fecgpu_code *code);
/* The code's parity rows P[i*k + j] (i < r, j < k: repair i = sum_j P[i][j] *
 * source j over GF(2^8); XOR: 1 where j mod r == i) into out[0 .. r*k).  Host
 * only, no device.  Returns r*k, or BUFFER_TOO_SHORT / the code_check error. */
ssize_t     fecgpu_code_parity_rows(const fecgpu_code *code, uint8_t *out, size_t cap);

/* ctx over devs[0..ndev-1] (NULL/0 = current device).  Batches with device
 * pointers run on the current device (the one the pointers live on);
 * host-pointer batches with the uniform layout are split into contiguous
 * window ranges, one host thread and copy/compute pipeline per listed device
 * (windows are independent: nothing is exchanged between devices). */
ssize_t fecgpu_ctx_new(const int *devs, int ndev, fecgpu_ctx **out);
void    fecgpu_ctx_free(fecgpu_ctx *ctx);
/* Pinned (page-locked) host memory for FECGPU_F_HOST_PTRS buffers: with it the
 * host-pointer batches overlap H2D copies, kernels and D2H copies, and the
 * kernels store repairs / recovered sources straight into the (device-mapped)
 * host windows, so only changed rows cross PCIe device->host. */
ssize_t fecgpu_host_alloc(size_t bytes, void **out);
void    fecgpu_host_free(void *p);
/* Launch tuning knobs (0 = automatic): "grid_mult" (persistent grid =
 * resident workgroups x value), "blocks_per_cu" (persistent grid = CUs x
 * value), "wpb" (windows per workgroup, group mode); host pipeline:
 * "host_direct" (bit 0 encode, bit 1 decode: kernels write outputs into
 * mapped pinned host windows instead of D2H copies; bit 2: they also read the
 * windows over PCIe instead of H2D copies; default 6 = decode zero-copy),
 * "host_chunk_mb" (pipeline chunk, default 128); "bitslice" (1 default: GF
 * encode of a code with a compiled bit-sliced kernel — Cauchy or Vandermonde
 * rows, r = 8, k in {16, 24, 32} — uses it, and of any other code with r >= 5
 * the runtime-mask bit-sliced kernel; 0: the table multiply for every code);
 * "bsdec" (1 default: GF decode of Cauchy k 16 r 4 on uniform rows whose
 * windows fill a 512-thread workgroup — about 1-8 KiB — by the bit-sliced
 * syndrome kernel; 0: the table decode; the bytes are the same);
 * "wide_mask" (1 default: the decode of a code with k + r > 64 skips the
 * missing rows in its syndrome pass; 0: they are zeroed and read);
 * "sw_group" (sliding-window encode by combine jobs: consecutive repairs per
 * job, each source loaded once per group; 1, 2, 4 or 8, default 4);
 * "sw_stream" (sliding-window encode: 0 combine jobs, 1..5 the streaming
 * kernel with that many dwords of a symbol per lane, 6 chosen per symbol
 * size; default 1); "sw_long_min"
 * (sliding-window decode: linked systems of at least this many lost sources
 * take the banded long-system path, default 65 — systems of <= 64 lost
 * sources and <= 96 repairs are solved by one wave each); "sw_log_entries"
 * (the long-system operation log, default 8 x (sources + repairs));
 * "bs_passes" (bit-sliced encode on per-window lengths: 256-unit passes per
 * window group at the longest window, default 8); "conn_streams" (streams per
 * device shared round robin by the encoders / decoders created afterwards,
 * default 4, 1..64); "pinned_cache_mb" (pinned blocks that freed encoders /
 * decoders leave cached in the ctx for the next ones, default 1024). */
ssize_t fecgpu_ctx_set_tuning(fecgpu_ctx *ctx, const char *key, int64_t value);

/* ---- batch entry points (hot path) ---------------------------------- */

/* Repair generation: writes repairs k..k+r-1 of every
 * window from its sources.  Returns nwin or a negative error. */
ssize_t fecgpu_encode_batch(fecgpu_ctx *ctx, const fecgpu_code *code, uint8_t *win,
                            const uint64_t *win_off, const uint32_t *sym_len,
                            uint32_t sym_len_all, uint32_t stride, uint64_t nwin,
                            uint32_t flags, void *stream);

/* Repair generation with the sender's split layout (SURVEY §8b "encode_batch(
 * ctx, code, src, repair, sym_len, nwin, flags, stream)", A.4): sources of
 * window w in src[w][k][stride], repairs written to repair[w][r][stride]
 * (sources are only read).  Device pointers only (FECGPU_F_HOST_PTRS returns
 * FECGPU_ERR_UNSUPPORTED).  Returns nwin or a negative error. */
ssize_t fecgpu_encode_split(fecgpu_ctx *ctx, const fecgpu_code *code, const uint8_t *src,
                            uint8_t *repair, const uint32_t *sym_len, uint32_t sym_len_all,
                            uint32_t stride, uint64_t nwin, uint32_t flags, void *stream);

/* Recovery: present[w] bit i = symbol i received; codes
 * with k + r > 64 take ceil((k + r) / 64) words per window (bit i of window w
 * in word present[w * words + i / 64], bit i % 64), device pointers and a
 * uniform stride only; when r < 4, the "bitslice" knob is 0 or a wave's span
 * of windows reaches 2 GiB, their missing rows are zeroed and read (times
 * zero).  Missing sources are recovered in place; status[w] =
 * FECGPU_STATUS_*.  Otherwise symbols whose bit is clear are never read.  XOR recovers every group with
 * exactly one missing source and its repair, even when others are lost.
 * Returns nwin or a negative error. */
ssize_t fecgpu_decode_batch(fecgpu_ctx *ctx, const fecgpu_code *code, uint8_t *win,
                            const uint64_t *win_off, const uint32_t *sym_len,
                            uint32_t sym_len_all, uint32_t stride, uint64_t nwin,
                            const uint64_t *present, uint8_t *status, uint32_t flags,
                            void *stream);

/* ---- per-connection objects: the Connection's per-packet FEC API -------
 * (§3 call stacks A/B).  The sender appends every
 * protected payload as a source symbol and reads repair symbols back; the
 * receiver files sources and repairs by (window, index) and reads recovered
 * packets back.  Symbols are written once, straight into pinned host
 * windows the GPU maps (no staging copies): the sender fills `batch` windows
 * and launches their encode asynchronously while it fills the next ones; the
 * receiver files symbols into a pool of window slots and a flush decodes every
 * decodable window in one zero-copy launch (ragged layout, fixed pitch).
 * Caller buffers are plain host memory.  Objects launch on a small pool of
 * streams owned by their ctx (not one stream per connection), so they must be
 * freed before the ctx, and used from the ctx's thread. */
typedef struct fecgpu_encoder fecgpu_encoder;
typedef struct fecgpu_decoder fecgpu_decoder;

ssize_t fecgpu_encoder_new(fecgpu_ctx *ctx, const fecgpu_code *code, uint32_t max_len,
                           uint32_t batch, fecgpu_encoder **out);
void    fecgpu_encoder_free(fecgpu_encoder *enc);
/* Append one source packet; win and idx receive its window id and index.
 * Closing the k-th packet of a window queues it; `batch` queued windows are
 * encoded on the GPU.  FIXED framing: every packet of a window same length. */
ssize_t fecgpu_encoder_add_source(fecgpu_encoder *enc, const uint8_t *pkt, size_t len,
                                  uint64_t *win, uint16_t *idx);
/* Close the open window early (missing sources become empty/zero packets);
 * returns its window id, FECGPU_ERR_DONE if no window is open. */
ssize_t fecgpu_encoder_close_window(fecgpu_encoder *enc);
/* Encode every queued window now; returns the number encoded. */
ssize_t fecgpu_encoder_flush(fecgpu_encoder *enc);
/* fecgpu_encoder_flush for n encoders in ONE launch, waiting for it (same
 * ctx, code and max_len; INVALID_ARG otherwise, or if one is listed twice).
 * Returns the number of windows encoded. */
ssize_t fecgpu_encoder_flush_many(fecgpu_encoder *const *encs, size_t n);
/* Number of real sources (1..k) of closed window win: k unless the window was
 * closed early (close_window, window timeout), whose padding sources never go
 * on the wire.  Carried in the REPAIR frame (nsrc).  FECGPU_ERR_DONE if win is
 * not closed yet or released. */
ssize_t fecgpu_encoder_window_sources(fecgpu_encoder *enc, uint64_t win);
/* Copy repair i of window win (S bytes); FECGPU_ERR_DONE until encoded. */
ssize_t fecgpu_encoder_repair(fecgpu_encoder *enc, uint64_t win, uint16_t i, uint8_t *out,
                              size_t cap);
/* Drop an encoded window's buffers. */
ssize_t fecgpu_encoder_release(fecgpu_encoder *enc, uint64_t win);

ssize_t fecgpu_decoder_new(fecgpu_ctx *ctx, const fecgpu_code *code, uint32_t max_len,
                           uint32_t batch, fecgpu_decoder **out);
void    fecgpu_decoder_free(fecgpu_decoder *dec);
/* File a received source packet / repair symbol (repair length = S).  Every
 * batch*k filed symbols an automatic flush is launched without waiting; its
 * windows complete when a later call touches them (add, recovered, release),
 * at the next flush, or at a tick once the GPU is done. */
ssize_t fecgpu_decoder_add_source(fecgpu_decoder *dec, uint64_t win, uint16_t idx,
                                  const uint8_t *pkt, size_t len);
ssize_t fecgpu_decoder_add_repair(fecgpu_decoder *dec, uint64_t win, uint16_t idx,
                                  const uint8_t *sym, size_t len);
/* A REPAIR frame's nsrc < k: sources nsrc..k-1 of window win are padding
 * (empty / zero packets the sender never sent), so they count as received.
 * Idempotent; INVALID_ARG if a source >= nsrc was filed or nsrc differs from
 * an earlier call.  recovered() returns FECGPU_ERR_DONE for padding indices. */
ssize_t fecgpu_decoder_set_window_sources(fecgpu_decoder *dec, uint64_t win, uint16_t nsrc);
/* At most max_windows windows open (filed and not released) per decoder
 * (default 4096; 0 = no limit): a symbol of a further window is rejected with
 * FECGPU_ERR_LIMIT and nothing is pinned for it, so a peer cannot make the
 * receiver pin memory without bound.  The Connection releases delivered
 * windows (fecgpu_decoder_release) to make room. */
ssize_t fecgpu_decoder_set_max_windows(fecgpu_decoder *dec, uint64_t max_windows);
/* Decode every window that can now recover a missing source and wait for
 * it; returns the number of source packets recovered since the last flush or
 * tick returned, including those of automatic flushes completed in between
 * (inside add / recovered / release calls). */
ssize_t fecgpu_decoder_flush(fecgpu_decoder *dec);
/* fecgpu_decoder_flush for n decoders in ONE launch, waiting for it: a server
 * that flushes many connections at once pays one kernel, not n.  The decoders
 * must share ctx, code and max_len (INVALID_ARG otherwise, or if one is listed
 * twice).  Returns the number of source packets recovered over all of them. */
ssize_t fecgpu_decoder_flush_many(fecgpu_decoder *const *decs, size_t n);
/* Copy source packet idx of window win (received or recovered, de-framed);
 * returns its length, FECGPU_ERR_DONE if it is not available. */
ssize_t fecgpu_decoder_recovered(fecgpu_decoder *dec, uint64_t win, uint16_t idx, uint8_t *out,
                                 size_t cap);
/* Recovered packets in the order they were recovered: *win / *idx of the
 * oldest one not yet returned (skipping windows released since); returns 0,
 * or FECGPU_ERR_DONE when there is none.  Lets a Connection deliver recovered
 * packets without scanning its windows.  The queue holds at most
 * max(4096, k x max_windows) entries (oldest dropped first). */
ssize_t fecgpu_decoder_next_recovered(fecgpu_decoder *dec, uint64_t *win, uint16_t *idx);
ssize_t fecgpu_decoder_release(fecgpu_decoder *dec, uint64_t win);

/* Scheduling policy: bounds the time a packet waits for its
 * repairs / its recovery, on the caller's clock.  The Connection calls
 * *_tick(now_us) from its timer (and may call it on every packet); add calls
 * stamp windows with the latest `now_us` seen.  0 disables a timeout.
 *   window_timeout_us: the sender closes its open window this long after the
 *       window's first packet (missing sources become empty packets);
 *   batch_timeout_us : a partly filled batch is launched this long after its
 *       first window closed (sender), a flush runs this long after the first
 *       symbol filed since the last flush (receiver).
 * tick returns the number of windows launched (sender) or sources recovered
 * (receiver), or a negative error. */
typedef struct fecgpu_policy {
    uint64_t window_timeout_us;
    uint64_t batch_timeout_us;
} fecgpu_policy;

ssize_t fecgpu_encoder_set_policy(fecgpu_encoder *enc, const fecgpu_policy *policy);
ssize_t fecgpu_encoder_tick(fecgpu_encoder *enc, uint64_t now_us);
ssize_t fecgpu_decoder_set_policy(fecgpu_decoder *dec, const fecgpu_policy *policy);
ssize_t fecgpu_decoder_tick(fecgpu_decoder *dec, uint64_t now_us);

/* ---- FEC frames on the wire --------------------
 * QUIC varint-coded frames (RFC 9000 §16 integers):
 *   SOURCE_ID: type | window | index                    (next to a source payload)
 *   REPAIR   : type | window | k | r | nsrc | index | length | symbol bytes
 * nsrc = real sources of the window (fecgpu_encoder_window_sources), 1..k.
 * Frame types sit in QUIC's extension space.  Host-only, no device calls. */
#define FECGPU_FRAME_SOURCE_ID 0xfec0u
#define FECGPU_FRAME_REPAIR 0xfec4u /* 0xfec1 = the ABI-1 REPAIR without nsrc: not accepted */
/* sliding-window code (RFC 8681 FEC payload IDs):
 *   SW_SOURCE: type | esi                                  (next to a source payload)
 *   SW_REPAIR: type | fss | nss | repair_key | dt | length | symbol bytes */
#define FECGPU_FRAME_SW_SOURCE 0xfec2u
#define FECGPU_FRAME_SW_REPAIR 0xfec3u

typedef struct fecgpu_frame {
    uint64_t type;           /* FECGPU_FRAME_* */
    uint64_t win;            /* window id; SW_SOURCE: esi; SW_REPAIR: fss */
    uint16_t k, r;           /* REPAIR: code shape */
    uint16_t idx;            /* source index (SOURCE_ID) or repair index (REPAIR) */
    const uint8_t *payload;  /* REPAIR / SW_REPAIR: points into the parsed buffer */
    size_t payload_len;
    uint16_t nsrc;           /* REPAIR: real sources of the window, 1..k; SW_REPAIR: nss */
    uint16_t key;            /* SW_REPAIR: repair_key */
    uint8_t dt;              /* SW_REPAIR: DT */
} fecgpu_frame;

ssize_t fecgpu_frame_source_id_len(uint64_t win, uint16_t idx);
ssize_t fecgpu_frame_write_source_id(uint8_t *buf, size_t cap, uint64_t win, uint16_t idx);
ssize_t fecgpu_frame_repair_len(uint64_t win, uint16_t k, uint16_t r, uint16_t nsrc, uint16_t idx,
                                size_t sym_len);
ssize_t fecgpu_frame_write_repair(uint8_t *buf, size_t cap, uint64_t win, uint16_t k, uint16_t r,
                                  uint16_t nsrc, uint16_t idx, const uint8_t *sym, size_t sym_len);
/* REPAIR frame header only (every field up to and including length): the
 * symbol bytes follow from the caller's own buffer, e.g. as a second iovec of
 * a gather send straight from the pinned window row (zero-copy, §8f-4).
 * Returns the header length. */
ssize_t fecgpu_frame_write_repair_header(uint8_t *buf, size_t cap, uint64_t win, uint16_t k,
                                         uint16_t r, uint16_t nsrc, uint16_t idx, size_t sym_len);
/* sliding-window frames (hdr->fss is the absolute ESI of the window's first source) */
ssize_t fecgpu_frame_write_sw_source(uint8_t *buf, size_t cap, uint64_t esi);
ssize_t fecgpu_frame_write_sw_repair(uint8_t *buf, size_t cap, const struct fecgpu_sw_repair *hdr,
                                     const uint8_t *sym, size_t sym_len);
/* Parse one frame at buf; returns bytes consumed or a negative error
 * (BUFFER_TOO_SHORT on truncation, INVALID_ARG on an unknown type or bad field). */
ssize_t fecgpu_frame_parse(const uint8_t *buf, size_t len, fecgpu_frame *out);

/* ---- synthetic workload / verification (bench + tests) ---- */

/* Fill sources of windows w0..w0+nwin-1 on the device (workload 0: FIXED,
 * every packet L bytes; 1: mixed MTU 1200/9000, 10% shortened, LENPREFIX).
 * Writes sym_len[w] (device, may be NULL for workload 0).  stride must hold
 * the largest symbol (9002 for workload 1).  Device pointers only. */
ssize_t fecgpu_synth_batch(fecgpu_ctx *ctx, const fecgpu_code *code, int workload,
                           uint64_t seed, uint64_t w0, uint8_t *win, uint32_t *sym_len,
                           uint32_t L, uint32_t stride, uint64_t nwin, void *stream);

/* Erasure masks (0: none, 1: exactly r sources, 2: i.i.d. p = 0.1). */
ssize_t fecgpu_erasure_batch(fecgpu_ctx *ctx, const fecgpu_code *code, int erasure,
                             uint64_t seed, uint64_t w0, uint64_t *present, uint64_t nwin,
                             void *stream);

/* XOR-accumulates the batch digest into *digest
 * (device u64, caller zeroes it). */
ssize_t fecgpu_digest_batch(fecgpu_ctx *ctx, const fecgpu_code *code, const uint8_t *win,
                            const uint32_t *sym_len, uint32_t sym_len_all, uint32_t stride,
                            uint64_t w0, uint64_t nwin, uint64_t *digest, void *stream);

/* ---- sliding-window random linear code (RFC 8681, m = 8) --------------
 * SURVEY.md Appendix B q6 (window vs sliding-window coding).  Sources form a
 * stream: src[i] is source symbol i of the batch (i < nsrc), `stride` bytes
 * apart, S = sym_len bytes each (framing as A.3, done by the caller).  Repair
 * symbol t is the GF(2^8) combination of the nss sources of its encoding
 * window [fss, fss + nss) with the coefficients RFC 8681 §3.6 draws for
 * (repair_key, nss, dt) from the RFC 8682 TinyMT32 PRNG: the REPAIR frame of
 * RFC 8681 carries exactly these fields (repair_key, DT, NSS, FSS_ESI). */
#define FECGPU_SW_MAX_WINDOW 255 /* nss limit (sources per encoding window) */

typedef struct fecgpu_sw_repair {
    uint64_t fss;        /* first source of the encoding window (index into the batch) */
    uint16_t nss;        /* sources in the window, 1..FECGPU_SW_MAX_WINDOW */
    uint16_t key;        /* RFC 8681 repair_key */
    uint8_t  dt;         /* density threshold DT, 0..15 (15: every coefficient nonzero) */
    uint8_t  reserved[3];
} fecgpu_sw_repair;

/* The first sliding-window call (encode, decode or a per-connection
 * sliding-window object's launch) on a device draws the ctx's dense RFC 8681
 * coefficient table there (every repair_key's coefficients at DT 15, 16 MiB
 * of device memory): a hipMalloc and a wait on the caller's stream, once per
 * ctx and device.  Later calls are asynchronous as documented; a caller that
 * needs the first call asynchronous too makes a small synchronous one first.
 *
 * rep[t] (nrep rows of `stride` bytes) from the sources of hdr[t]'s window.
 * src, rep and hdr are device pointers (FECGPU_F_HOST_PTRS: host memory,
 * staged, synchronous).  max_window: the largest nss among the headers
 * (1..FECGPU_SW_MAX_WINDOW; 0 = FECGPU_SW_MAX_WINDOW), which sizes the
 * kernel's per-repair tables.  Device headers are not validated: a window
 * reaching past nsrc or longer than max_window is clipped, dt > 15 counts as
 * 15; host headers are checked (INVALID_ARG).  Returns nrep or a negative
 * error. */
ssize_t fecgpu_sw_encode(fecgpu_ctx *ctx, const uint8_t *src, uint64_t nsrc, uint8_t *rep,
                         const fecgpu_sw_repair *hdr, uint64_t nrep, uint32_t max_window,
                         uint32_t sym_len, uint32_t stride, uint32_t flags, void *stream);

/* Recovers lost sources in place.  The receiver's bookkeeping is host memory:
 * src_present[i] / rep_present[t] nonzero = received, hdr[t] the repairs'
 * headers (fss nondecreasing), src_status[i] out: 0 = present or recovered,
 * 1 = still lost.  src / rep are device pointers (FECGPU_F_HOST_PTRS: host).
 * Every lost source that the received repairs determine is recovered — the
 * result of one Gauss-Jordan elimination over all lost sources and all
 * received repairs, also where that system is rank deficient — with no limit
 * on how many lost sources the repairs link together.  The whole decode is
 * planned and run on the GPU (the bookkeeping is copied up, the statuses
 * down).  Synchronous on `stream`; returns the number of sources recovered,
 * or a negative error (INVALID_ARG for a bad or unordered header; nothing is
 * written then).  Nsrc and nrep < 2^32 - 256. */
ssize_t fecgpu_sw_decode(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *src_present, uint64_t nsrc,
                         const uint8_t *rep, const uint8_t *rep_present,
                         const fecgpu_sw_repair *hdr, uint64_t nrep, uint32_t sym_len,
                         uint32_t stride, uint8_t *src_status, uint32_t flags, void *stream);
/* The same decode with the receiver's bookkeeping on the device: src,
 * src_present, rep, rep_present, hdr and src_status are all device pointers
 * (FECGPU_F_HOST_PTRS is invalid).  Asynchronous on `stream` and returns 0,
 * the statuses valid once the stream reaches the end of the call; with
 * FECGPU_F_SYNC it waits and returns the number recovered, or INVALID_ARG if
 * a header is bad or out of order (the kernels check them; then nothing is
 * recovered and the statuses are the arrival flags).  A long linked system
 * whose operation log does not fit the ctx's reservation is retried larger
 * with FECGPU_F_SYNC; without it, that system stays lost and the call raises
 * FECGPU_SW_ERR_CAPACITY for fecgpu_sw_decode_errors (a bad header raises
 * FECGPU_SW_ERR_HEADER), so an asynchronous caller can tell an overflow from
 * a source the repairs do not determine (tuning "sw_log_entries"). */
ssize_t fecgpu_sw_decode_device(fecgpu_ctx *ctx, uint8_t *src, const uint8_t *src_present, uint64_t nsrc,
                                const uint8_t *rep, const uint8_t *rep_present,
                                const struct fecgpu_sw_repair *hdr, uint64_t nrep, uint32_t sym_len,
                                uint32_t stride, uint8_t *src_status, uint32_t flags, void *stream);

/* Error flags raised by asynchronous fecgpu_sw_decode_device calls on the
 * current device since the last query, OR-ed together: waits until every
 * sliding-window call issued on the ctx so far has finished, stores the flags
 * in *flags and clears them.  After FECGPU_SW_ERR_CAPACITY the ctx's later
 * calls reserve a log large enough for what overflowed (a synchronous decode
 * of the same inputs recovers what was left lost).  Returns 0 or a negative
 * error. */
#define FECGPU_SW_ERR_HEADER   1u /* a header was bad or out of order: that call recovered nothing */
#define FECGPU_SW_ERR_CAPACITY 2u /* a long system's operation log did not fit: its sources stayed lost */
#define FECGPU_SW_ERR_INTERNAL 4u /* the device plan's chunk look-back gave up (never expected): the call's
                                     results are not to be trusted; a synchronous retry reports it as
                                     FECGPU_ERR_DEVICE */
ssize_t fecgpu_sw_decode_errors(fecgpu_ctx *ctx, uint32_t *flags);

/* ---- sliding-window per-connection objects ----------------------------
 * The Connection's per-packet API for the sliding-window code (RFC 8681
 * semantics: encoding symbol size E fixed per session, ADU framing as A.3).
 * Sender: every protected payload gets the next ESI; after every `step`
 * sources a repair over the last `window` sources is scheduled (repair_key =
 * 0, 1, 2, ... mod 2^16); `batch` scheduled repairs are encoded in one
 * asynchronous launch (the kernel reads the sources from pinned host memory
 * the GPU maps; 4 launches' repairs held until read) and read back in order with
 * fecgpu_sw_encoder_next_repair for SW_REPAIR frames.  Receiver: files
 * sources by ESI and repairs by header, and a flush (automatic every `batch`
 * received repairs) runs fecgpu_sw_decode over its live span.  Sources more
 * than `span` behind the newest ESI are given up.  Objects must be freed
 * before their ctx and used from its thread. */
typedef struct fecgpu_sw_params {
    uint32_t framing;     /* FECGPU_FRAMING_FIXED (payload = symbol) or _LENPREFIX */
    uint32_t symbol_size; /* E bytes (LENPREFIX: 2 + the largest payload), <= 65537 */
    uint16_t window;      /* W: sources per encoding window, 1..FECGPU_SW_MAX_WINDOW */
    uint16_t step;        /* a repair after every `step` sources, >= 1 */
    uint8_t  dt;          /* RFC 8681 DT, 0..15 */
    uint8_t  reserved[3];
    uint32_t batch;       /* repairs per encode launch / per automatic decoder flush, >= 1 */
    uint32_t span;        /* receiver: sources kept behind the newest (0 = 16 x window +
                             5 x batch x step: the sender's 4 launch slots plus the filling
                             batch); repairs whose window starts before it are dropped
                             (add_repair returns FECGPU_ERR_DONE) */
} fecgpu_sw_params;

typedef struct fecgpu_sw_encoder fecgpu_sw_encoder;
typedef struct fecgpu_sw_decoder fecgpu_sw_decoder;

ssize_t fecgpu_sw_encoder_new(fecgpu_ctx *ctx, const fecgpu_sw_params *p, fecgpu_sw_encoder **out);
void    fecgpu_sw_encoder_free(fecgpu_sw_encoder *enc);
/* Append a source payload; *esi receives its ESI.  FECGPU_ERR_LIMIT (nothing
 * consumed) while every launch slot holds repairs not yet read. */
ssize_t fecgpu_sw_encoder_add_source(fecgpu_sw_encoder *enc, const uint8_t *pkt, size_t len,
                                     uint64_t *esi);
/* Launch the scheduled repairs (when a launch slot is free) and wait for
 * every launch; returns the number of repairs ready to read. */
ssize_t fecgpu_sw_encoder_flush(fecgpu_sw_encoder *enc);
/* The next encoded repair in order: header (absolute fss) and E bytes;
 * FECGPU_ERR_DONE if none is ready yet. */
ssize_t fecgpu_sw_encoder_next_repair(fecgpu_sw_encoder *enc, fecgpu_sw_repair *hdr, uint8_t *out,
                                      size_t cap);

ssize_t fecgpu_sw_decoder_new(fecgpu_ctx *ctx, const fecgpu_sw_params *p, fecgpu_sw_decoder **out);
void    fecgpu_sw_decoder_free(fecgpu_sw_decoder *dec);
ssize_t fecgpu_sw_decoder_add_source(fecgpu_sw_decoder *dec, uint64_t esi, const uint8_t *pkt,
                                     size_t len);
/* hdr->fss absolute; sym: E bytes.  INVALID_ARG (nothing changed) for a window
 * longer than the session's `window`; DONE if it starts behind the kept span. */
ssize_t fecgpu_sw_decoder_add_repair(fecgpu_sw_decoder *dec, const fecgpu_sw_repair *hdr,
                                     const uint8_t *sym, size_t len);
/* Decode now; returns the number of sources recovered (also queued for
 * fecgpu_sw_decoder_next_recovered). */
ssize_t fecgpu_sw_decoder_flush(fecgpu_sw_decoder *dec);
/* Payload of source esi (received or recovered, de-framed); FECGPU_ERR_DONE
 * if it is not available (lost, or given up). */
ssize_t fecgpu_sw_decoder_recovered(fecgpu_sw_decoder *dec, uint64_t esi, uint8_t *out, size_t cap);
ssize_t fecgpu_sw_decoder_next_recovered(fecgpu_sw_decoder *dec, uint64_t *esi);

#ifdef __cplusplus
}
#endif
#endif
